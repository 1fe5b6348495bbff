#!/bin/bash
# Session 20: post-pass parity + kernel trace.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_postpass_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r02_s20_tests.log 2>&1 || { tail -30 gpurun_out/r02_s20_tests.log; exit 1; }
tail -1 gpurun_out/r02_s20_tests.log
timeout -k 10 300 python bench.py --no-cpu-baseline --postpass --steps 50 --warmup 5 > gpurun_out/r02_s20_pp.json 2> gpurun_out/r02_s20_pp.err || { tail -5 gpurun_out/r02_s20_pp.err; exit 1; }
python3 -c "
import json; d=json.load(open('gpurun_out/r02_s20_pp.json'))
print([(f['mode'], f['kernel'], f['ms'], f['GB_s']) for f in d['postpass']['filters']])"
bash tools/pp_probe.sh p5 new
