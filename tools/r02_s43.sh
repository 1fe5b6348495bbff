#!/bin/bash
# Session 43: Phong register budgets: K=2 at 6 waves (ablib/ph6), K=4 at 4 waves (ablib/ph4).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
export TMPDIR=/tmp
bash tools/ab_bench.sh ph6 ph2 "--phong --batch 2 --steps 100 --warmup 20" 2 || exit 1
bash tools/ab_bench.sh ph4 ph4 "--phong --batch 4 --steps 100 --warmup 20" 2 || exit 1
