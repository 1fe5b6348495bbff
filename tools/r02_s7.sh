#!/bin/bash
# Session 7: buffer loads (32-bit offsets, no 64-bit address math) at 7 and 8
# waves/SIMD vs the in-tree global loads; headline + long-ray frames.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for A in buf buf8; do
  bash tools/ab_builds.sh $A "b4o1p5q0,b2o1p5q0" 3 "--frames 50" || exit 1
  bash tools/ab_builds.sh $A "b4o1p5q0" 2 "--tf-alpha 0.02 --frames 10" || exit 1
done
