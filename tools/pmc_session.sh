#!/bin/bash
# PMC records for bench.py's roofline: the bench line of each workload, then one
# rocprofv3 --pmc pass per counter group (tools/pmc_bench.sh), then the record
# (tools/pmc_record.py) keyed by workload, dominant kernel and library build.
#   bash tools/pmc_session.sh rc1pass phong dos ebs
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
export TMPDIR=/tmp
GRPS="FETCH_SIZE;WRITE_SIZE;TCC_HIT_sum TCC_MISS_sum;SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_WAIT_INST_ANY;TD_TD_BUSY TD_TC_STALL TA_TA_BUSY TA_ADDR_STALLED_BY_TC_CYCLES;TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum GRBM_GUI_ACTIVE"
for w in "$@"; do
  case $w in
    rc1pass) ARGS="--streams 1 --no-cadence"; K=rc1pass_tile_kernel; export PMC_GRID=5455872 PMC_STEPS=8; OUT=pmc_rc1pass.json;;   # 4 frames per launch x 21312 ordered slots (band_cap 130, bands of whole 4-slot groups) x 64
    phong)   ARGS="--streams 1 --phong --no-cadence"; K=rc1pass_tile_kernel; export PMC_GRID=5455872 PMC_STEPS=8; OUT=pmc_rc1pass_phong.json;;
    longray) ARGS="--streams 1 --tf-alpha 0.02 --no-cadence"; K=rc1pass_tile_kernel; export PMC_GRID=5455872 PMC_STEPS=8; OUT=pmc_rc1pass_longray.json;;
    dos)     ARGS="--renderer dos --streams 1"; K=flat_shade_kernel; unset PMC_GRID; export PMC_STEPS=3; OUT=pmc_dos.json;;
    ebs)     ARGS="--renderer ebs --streams 1"; K=flat_shade_kernel; unset PMC_GRID; export PMC_STEPS=3; OUT=pmc_ebs.json;;
  esac
  timeout -k 10 400 python3 bench.py $ARGS --no-cpu-baseline --steps $PMC_STEPS --warmup 1 > gpurun_out/pmcline_$w.json 2> gpurun_out/pmcline_$w.err || { tail -5 gpurun_out/pmcline_$w.err; exit 1; }
  PMC_TIMEOUT=${PMC_TIMEOUT:-240} bash tools/pmc_bench.sh $w $K "$ARGS" "$GRPS" > gpurun_out/pmc_$w.log 2>&1 || { tail -5 gpurun_out/pmc_$w.log; exit 1; }
  python3 tools/pmc_record.py gpurun_out/pmc_$w/summary.json gpurun_out/pmcline_$w.json gpurun_out/$OUT > /dev/null || exit 1
  python3 -c "import json; d=json.load(open('gpurun_out/$OUT')); print('$w', {k: d.get(k) for k in ('kernel_ns_avg_under_pmc','hbm_bytes_per_launch','tcc_hit_rate','td_busy_frac_per_cu','valu_issue_frac_per_simd','valu_per_sample')})"
done
