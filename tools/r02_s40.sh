#!/bin/bash
# Session 40: headline march at 8 waves/SIMD (ablib/rc8) vs 7.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
export TMPDIR=/tmp
bash tools/ab_bench.sh rc8 ea "--steps 20 --warmup 5" 4 || exit 1
