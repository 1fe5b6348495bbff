#!/bin/bash
# PMC counters of one bench.py workload, one rocprofv3 pass per counter group
# (--pmc only with --kernel-trace; a pass per group because rocprofv3 does not
# split counters over passes).  Summary: tools/pmc_summary.py.
#
#   tools/pmc_bench.sh NAME KERNEL "BENCH ARGS" ["GROUP;GROUP;..."]
#   e.g. tools/pmc_bench.sh ebs shaded_march_kernel "--renderer ebs"
#
# Output: gpurun_out/pmc_NAME/{gN/,gN.log,summary.json}.  A crash, abort or
# time limit ends the script (no retry); a rejected counter group is reported.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
NAME=$1; KERNEL=$2; ARGS=$3
GROUPS_DEFAULT="FETCH_SIZE;WRITE_SIZE;TCC_HIT_sum TCC_MISS_sum;SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_WAIT_INST_ANY;TD_TD_BUSY TD_TC_STALL TA_TA_BUSY TA_ADDR_STALLED_BY_TC_CYCLES;TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum;SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_WAVES;GRBM_GUI_ACTIVE GRBM_COUNT"
GRP_LIST=${4:-$GROUPS_DEFAULT}
OUT=gpurun_out/pmc_$NAME
rm -rf "$OUT"; mkdir -p "$OUT"
IFS=';' read -ra GRPS <<< "$GRP_LIST"
i=0
for grp in "${GRPS[@]}"; do
  i=$((i+1))
  timeout -k 10 -s KILL ${PMC_TIMEOUT:-180} rocprofv3 --kernel-trace --pmc $grp -d $OUT/g$i -o pmc \
    --output-format csv -- python3 bench.py $ARGS --no-cpu-baseline --steps ${PMC_STEPS:-3} --warmup 0 \
    --settle-ms 0 > $OUT/g$i.log 2>&1
  rc=$?
  if [ $rc -ne 0 ]; then
    echo "$NAME group '$grp' rc $rc"; tail -5 $OUT/g$i.log
    case $rc in 124|134|137|139) exit $rc;; esac
  fi
done
python3 tools/pmc_summary.py $OUT $KERNEL > $OUT/summary.json && head -c 1500 $OUT/summary.json; echo
