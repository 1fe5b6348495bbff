#!/bin/bash
# Session 19: post-pass (pair staging, packed decimation sums) + DOS inside-box fast path:
# parity, bench --postpass, DOS A/B vs HEAD.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_postpass_gpu.py tests/test_dos_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r02_s19_tests.log 2>&1 || { tail -30 gpurun_out/r02_s19_tests.log; exit 1; }
tail -1 gpurun_out/r02_s19_tests.log
timeout -k 10 300 python bench.py --no-cpu-baseline --postpass --steps 50 --warmup 5 > gpurun_out/r02_s19_pp.json 2> gpurun_out/r02_s19_pp.err || { tail -5 gpurun_out/r02_s19_pp.err; exit 1; }
python3 -c "
import json; d=json.load(open('gpurun_out/r02_s19_pp.json'))
print([(f['mode'], f['kernel'], f['ms'], f['GB_s']) for f in d['postpass']['filters']])"
bash tools/ab_bench.sh prev dos "--renderer dos --steps 5 --warmup 1" 2 || exit 1
