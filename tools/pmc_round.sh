#!/bin/bash
# PMC counter passes (one rocprofv3 run per counter group; --pmc only with
# --kernel-trace, never with sys/runtime traces).  Workload: tools/ab_rc1pass.py
# single variant.  Output: gpurun_out/pmc/<group>/...
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
VAR=${1:-L1b4o1p5q0}
EXTRA=${2:-}
rm -rf gpurun_out/pmc; mkdir -p gpurun_out/pmc
rocprofv3 -L > gpurun_out/pmc/counters_list.txt 2>&1 || true
# counter groups: PMC_GROUPS="A B;C D;..." (one rocprofv3 pass per group)
DEFAULT_GROUPS="FETCH_SIZE;WRITE_SIZE;TCC_HIT_sum TCC_MISS_sum;SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS;SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU;SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS;TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum;GRBM_GUI_ACTIVE GRBM_COUNT"
IFS=';' read -ra GRPS <<< "${PMC_GROUPS:-$DEFAULT_GROUPS}"
i=0
for grp in "${GRPS[@]}"; do
  i=$((i+1))
  if [ -n "${PMC_CMD:-}" ]; then
    # PMC_CMD: another workload, e.g. "bench.py --renderer dos --no-cpu-baseline --steps 1 --warmup 0"
    timeout -k 10 ${PMC_TIMEOUT:-90} rocprofv3 --kernel-trace --pmc $grp -d gpurun_out/pmc/g$i -o pmc --output-format csv -- python3 $PMC_CMD > gpurun_out/pmc/g$i.log 2>&1
  else
    timeout -k 10 ${PMC_TIMEOUT:-90} rocprofv3 --kernel-trace --pmc $grp -d gpurun_out/pmc/g$i -o pmc --output-format csv -- python3 tools/ab_rc1pass.py --variants $VAR --rounds 1 --frames 5 $EXTRA > gpurun_out/pmc/g$i.log 2>&1
  fi
  rc=$?
  if [ $rc -ne 0 ]; then
    echo "group $grp failed (rc $rc)"; tail -5 gpurun_out/pmc/g$i.log
    # a crash, abort or time limit ends the call; a rejected counter does not
    case $rc in 124|134|137|139) exit $rc;; esac
  fi
done
python3 tools/pmc_summary.py gpurun_out/pmc ${KERNEL:-rc1pass} > gpurun_out/pmc/summary.json && cat gpurun_out/pmc/summary.json
