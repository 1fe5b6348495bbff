#!/bin/bash
# Session 56: iso marches, XCD column groups of 2 / 4 tiles vs interleaved (A/B).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for A in icg2 icg4; do
  for R in iso isodfs isoadapt; do
    bash tools/ab_bench.sh $A $R$A "--renderer $R --steps 20 --warmup 5" 2 || exit 1
  done
done
