#!/bin/bash
# Session 42: iso register budgets in tree: iso parity + bench lines.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_iso_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r02_s42_tests.log 2>&1 || { tail -30 gpurun_out/r02_s42_tests.log; exit 1; }
tail -1 gpurun_out/r02_s42_tests.log
for R in iso isodfs isoadapt; do
  timeout -k 10 300 python bench.py --renderer $R > gpurun_out/r02_s42_$R.json 2> gpurun_out/r02_s42_$R.err || { tail -5 gpurun_out/r02_s42_$R.err; exit 1; }
  python3 -c "
import json; d=json.load(open('gpurun_out/r02_s42_$R.json')); print('$R', d['ms_per_step'], d['roofline']['kernel_ms'], d['roofline']['frac'], d.get('parity',{}).get('bit_exact'))"
done
