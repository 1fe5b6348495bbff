#!/bin/bash
# Session 18: A/B of the intra-batch cell reuse (ablib/reuse) vs the in-tree build, headline + long rays.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
export TMPDIR=/tmp
bash tools/ab_bench.sh reuse ea "--steps 100 --warmup 20" 3 || exit 1
bash tools/ab_bench.sh reuse long "--tf-alpha 0.02 --steps 20 --warmup 5" 2 || exit 1
