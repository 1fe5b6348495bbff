#!/bin/bash
# EBS session: config-5 bench line (1024^3 SAT + frame), the 512^3 line, PMC traffic at 1024^3.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python bench.py --renderer ebs > gpurun_out/r02_bench_ebs.json 2> gpurun_out/r02_bench_ebs.err || { tail -20 gpurun_out/r02_bench_ebs.err; exit 1; }
cat gpurun_out/r02_bench_ebs.json
timeout -k 10 300 python bench.py --renderer ebs --size 512 --no-cpu-baseline > gpurun_out/r02_bench_ebs512.json 2> gpurun_out/r02_bench_ebs512.err || { tail -20 gpurun_out/r02_bench_ebs512.err; exit 1; }
cat gpurun_out/r02_bench_ebs512.json
rm -rf gpurun_out/pmc_ebs; mkdir -p gpurun_out/pmc_ebs
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" "SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_WAIT_INST_ANY" "TD_TD_BUSY TA_TA_BUSY GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $grp -d gpurun_out/pmc_ebs/g$i -o pmc --output-format csv -- python3 bench.py --renderer ebs --no-cpu-baseline --steps 1 --warmup 0 --settle-ms 0 > gpurun_out/pmc_ebs/g$i.log 2>&1
  rc=$?; if [ $rc -ne 0 ]; then echo "group $grp rc $rc"; tail -5 gpurun_out/pmc_ebs/g$i.log; case $rc in 124|134|137|139) exit $rc;; esac; fi
done
python3 tools/pmc_summary.py gpurun_out/pmc_ebs "shaded_march_kernel<cvr::EbsShader" > gpurun_out/pmc_ebs/summary.json && cat gpurun_out/pmc_ebs/summary.json | head -20
