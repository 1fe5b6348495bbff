#!/bin/bash
# Round-2 measurement session: the long-ray line (bench --tf-alpha 0.02), its PMC
# traffic, PMC of the Phong frame, and the headline kernel-trace summary.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python bench.py --tf-alpha 0.02 --no-cpu-baseline --steps 50 > gpurun_out/r02_bench_longray.json 2> gpurun_out/r02_bench_longray.err || { tail -20 gpurun_out/r02_bench_longray.err; exit 1; }
cat gpurun_out/r02_bench_longray.json
run_pmc() {   # $1 name, $2 groups, $3 bench args
  local name=$1 groups=$2 args=$3 i=0
  rm -rf gpurun_out/pmc_$name; mkdir -p gpurun_out/pmc_$name
  IFS=';' read -ra GRPS <<< "$groups"
  for grp in "${GRPS[@]}"; do
    i=$((i+1))
    timeout -k 10 120 rocprofv3 --kernel-trace --pmc $grp -d gpurun_out/pmc_$name/g$i -o pmc --output-format csv -- python3 bench.py $args --no-cpu-baseline --steps 3 --warmup 0 --settle-ms 0 > gpurun_out/pmc_$name/g$i.log 2>&1
    rc=$?
    if [ $rc -ne 0 ]; then echo "$name group $grp rc $rc"; tail -5 gpurun_out/pmc_$name/g$i.log; case $rc in 124|134|137|139) exit $rc;; esac; fi
  done
  python3 tools/pmc_summary.py gpurun_out/pmc_$name ${KERNEL:-rc1pass_tile_kernel} > gpurun_out/pmc_$name/summary.json && cat gpurun_out/pmc_$name/summary.json | head -30
}
G="FETCH_SIZE;WRITE_SIZE;TCC_HIT_sum TCC_MISS_sum;SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_WAIT_INST_ANY;TD_TD_BUSY TD_TC_STALL TA_TA_BUSY TA_ADDR_STALLED_BY_TC_CYCLES;TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum;GRBM_GUI_ACTIVE GRBM_COUNT"
run_pmc longray "$G" "--tf-alpha 0.02" || exit 1
run_pmc phong "$G" "--phong" || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r02 -o trace --output-format csv -- python3 bench.py --no-cpu-baseline --steps 20 --warmup 5 --streams 1 > gpurun_out/r02_prof_bench.json 2> gpurun_out/r02_prof.err || { tail -20 gpurun_out/r02_prof.err; exit 1; }
find gpurun_out/prof_r02 -name "*stats*"
