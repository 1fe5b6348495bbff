#!/bin/bash
# Session 37: DOS march capped at 3 waves/SIMD (ablib/dos3) vs the compiler's choice (2 waves).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
export TMPDIR=/tmp
bash tools/ab_bench.sh dos3 dos "--renderer dos --steps 5 --warmup 1" 2 || exit 1
