#!/bin/bash
# Session 32: iso marches, interleaved tile order (ablib/isow) vs XCD bands (tree).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for R in iso isodfs isoadapt; do
  bash tools/ab_bench.sh isow $R "--renderer $R --steps 20 --warmup 5" 2 || exit 1
done
