#!/bin/bash
# Session 41: headline variant at 8 waves/SIMD in tree: rc1pass parity, A/B vs HEAD (driver command, long rays, orbit).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_rc1pass_gpu.py tests/test_split_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r02_s41_tests.log 2>&1 || { tail -30 gpurun_out/r02_s41_tests.log; exit 1; }
tail -1 gpurun_out/r02_s41_tests.log
bash tools/ab_bench.sh prev ea "--steps 20 --warmup 5" 3 || exit 1
bash tools/ab_bench.sh prev long "--tf-alpha 0.02 --steps 20 --warmup 5" 2 || exit 1
bash tools/ab_bench.sh prev orbit "--orbit --steps 48 --warmup 24" 2 || exit 1
