#!/bin/bash
# Session 5: headline-kernel experiments (ablib/{reuse,morton,blk42}) vs the
# in-tree build, headline frame and long-ray frame.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for A in reuse morton blk42; do
  bash tools/ab_builds.sh $A "b4o1p5q0" 3 "--frames 50" > gpurun_out/s5_$A.txt || exit 1
  bash tools/ab_builds.sh $A "b4o1p5q0" 2 "--tf-alpha 0.02 --frames 10" >> gpurun_out/s5_$A.txt || exit 1
  cat gpurun_out/s5_$A.txt
done
