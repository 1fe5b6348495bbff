#!/bin/bash
# Session 50: half-box pipelined EBS chains: EBS/fullsize parity, the EBS bench at 1024^3 with the
# oracle band check, kernel-trace summary of the 512^3 EBS bench.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_ebs_gpu.py tests/test_fullsize_gpu.py -k "ebs or c5" -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r02_s50_tests.log 2>&1 || { tail -30 gpurun_out/r02_s50_tests.log; exit 1; }
tail -1 gpurun_out/r02_s50_tests.log
timeout -k 10 600 python bench.py --renderer ebs > gpurun_out/r02_s50_ebs.json 2> gpurun_out/r02_s50_ebs.err || { tail -20 gpurun_out/r02_s50_ebs.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/r02_s50_ebs.json')); print(d['ms_per_step'], d['value'], d['roofline']['kernel_ms'], d.get('parity'))"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/r02_s50_prof -o trace --output-format csv -- python3 bench.py --renderer ebs --size 512 --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/r02_s50_prof_bench.json 2> gpurun_out/r02_s50_prof.err || { tail -20 gpurun_out/r02_s50_prof.err; exit 1; }
grep shaded_march gpurun_out/r02_s50_prof/trace_kernel_stats.csv | awk -F'",' '{print $2}'
