#!/bin/bash
# One GPU session of the current round (edited per session; the committed copy is
# the last one run).  Each GPU step has its own limit; the first failure ends the call.
# Round 5, s07: DOS flat-shade batching without register spills (A/B of builds).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-r05_s07}
for v in dos_s2u1 dos_s3u1; do
  timeout -k 10 900 bash tools/ab_bench.sh $v $v "--renderer dos --steps 5" 2 > gpurun_out/${T}_ab_$v.log 2>&1 || { tail -5 gpurun_out/${T}_ab_$v.log; exit 1; }
  tail -2 gpurun_out/${T}_ab_$v.log
done
# EBS flat shade: the vector-memory pipe split (TD work vs cache stall), TCP accesses, L2 misses
PMC_TIMEOUT=300 PMC_STEPS=2 bash tools/pmc_bench.sh ebs_td flat_shade_kernel "--renderer ebs --streams 1" \
  "TD_TD_BUSY TD_TC_STALL TA_TA_BUSY TA_ADDR_STALLED_BY_TC_CYCLES;TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum GRBM_GUI_ACTIVE;SQ_INSTS_VMEM_RD SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_WAIT_INST_ANY" > gpurun_out/${T}_pmc_ebs_td.log 2>&1 || { tail -5 gpurun_out/${T}_pmc_ebs_td.log; exit 1; }
cp gpurun_out/pmc_ebs_td/summary.json gpurun_out/${T}_pmc_ebs_td_summary.json
head -20 gpurun_out/${T}_pmc_ebs_td_summary.json
