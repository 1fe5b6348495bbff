#!/bin/bash
# Session 30: alpha-first classification in tree: rc1pass / split / full-size parity + driver bench.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_rc1pass_gpu.py tests/test_split_gpu.py tests/test_fullsize_gpu.py tests/test_postpass_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r02_s30_tests.log 2>&1 || { tail -30 gpurun_out/r02_s30_tests.log; exit 1; }
tail -1 gpurun_out/r02_s30_tests.log
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r02_s30_bench.json 2> gpurun_out/r02_s30_bench.err || { tail -20 gpurun_out/r02_s30_bench.err; exit 1; }
python3 -c "
import json; d=json.load(open('gpurun_out/r02_s30_bench.json')); print(d['ms_per_step'], d['value'], d['roofline']['kernel_ms'], d['roofline']['frac'], d['parity']['bit_exact'])"
