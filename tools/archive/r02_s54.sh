#!/bin/bash
# Session 54: shaded marches (EBS, DOS), XCD column groups of 2 / 4 / 8 tiles vs 1 (A/B).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for A in cg2 cg4 cg8; do
  bash tools/ab_bench.sh $A ebs512$A "--renderer ebs --size 512 --steps 5 --warmup 1" 2 || exit 1
done
for A in cg2 cg4 cg8; do
  bash tools/ab_bench.sh $A dos$A "--renderer dos --steps 20 --warmup 3" 2 || exit 1
done
bash tools/ab_bench.sh cg4 ebs1024cg4 "--renderer ebs --steps 2 --warmup 1" 1 || exit 1
