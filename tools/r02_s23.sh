#!/bin/bash
# Session 23: cost probe: the headline march with every cell fetch served from LDS (wrong images).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
export TMPDIR=/tmp
bash tools/ab_bench.sh ldsprobe ldsp "--tf-alpha 0 --skip-min-pct 101 --steps 20 --warmup 5" 2 || exit 1
