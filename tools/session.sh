#!/bin/bash
# One GPU session of the current round (edited per session; the committed copy is
# the last one run).  Each GPU step has its own limit; the first failure ends the call.
# Round 5, s23: DOS cone-tap batching, sections per batch of the 1-ray stage (U1
# 2 / 8 against 4) and of the 3-ray stage (U3 3 against 2).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-r05_s23}
for v in dos_u1_2 dos_u1_8 dos_u3_3; do
  timeout -k 10 900 bash tools/ab_bench.sh $v ${T}_$v "--renderer dos --steps 5" 2 > gpurun_out/${T}_ab_$v.log 2>&1 || { tail -5 gpurun_out/${T}_ab_$v.log; exit 1; }
  tail -2 gpurun_out/${T}_ab_$v.log
done
