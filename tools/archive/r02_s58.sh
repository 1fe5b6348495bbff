#!/bin/bash
# Session 58: PMC of the pipelined EBS march with 4-column XCD groups at 1024^3 (traffic, L2 hits, issue counters; separate passes).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
export TMPDIR=/tmp
run_pmc() {   # $1 name, $2 groups, $3 bench args, $4 kernel
  local name=$1 groups=$2 args=$3 i=0
  rm -rf gpurun_out/pmc_$name; mkdir -p gpurun_out/pmc_$name
  IFS=';' read -ra GRPS <<< "$groups"
  for grp in "${GRPS[@]}"; do
    i=$((i+1))
    timeout -k 10 -s KILL 180 rocprofv3 --kernel-trace --pmc $grp -d gpurun_out/pmc_$name/g$i -o pmc --output-format csv -- python3 bench.py $args --no-cpu-baseline --steps 3 --warmup 0 --settle-ms 0 > gpurun_out/pmc_$name/g$i.log 2>&1
    rc=$?
    if [ $rc -ne 0 ]; then echo "$name group $grp rc $rc"; tail -5 gpurun_out/pmc_$name/g$i.log; exit $rc; fi
  done
  python3 tools/pmc_summary.py gpurun_out/pmc_$name $4 > gpurun_out/pmc_$name/summary.json && head -c 900 gpurun_out/pmc_$name/summary.json; echo
}
run_pmc ebscg4 "FETCH_SIZE;WRITE_SIZE;TCC_HIT_sum TCC_MISS_sum;SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_WAIT_INST_ANY;TA_TA_BUSY TD_TD_BUSY" "--renderer ebs" shaded_march_kernel || exit 1
