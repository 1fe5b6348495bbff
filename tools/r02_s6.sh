#!/bin/bash
# Session 6: 4-wave workgroups (16x16 pixel blocks share a CU's L1) vs one wave
# per workgroup, screen order (o0) and LPT (o1); headline + long-ray frames.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
export TMPDIR=/tmp
bash tools/ab_builds.sh wg4 "b4o0p0q0,b4o1p5q0" 3 "--frames 50" || exit 1
bash tools/ab_builds.sh wg4 "b4o0p0q0,b4o1p5q0" 2 "--tf-alpha 0.02 --frames 10" || exit 1
