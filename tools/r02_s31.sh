#!/bin/bash
# Session 31: Phong with alpha-first classification (ablib/phalpha): parity with that build, A/B at K = 2 / 4.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
export TMPDIR=/tmp
CVR_LIB_OVERRIDE=ablib/phalpha/libcvr.so timeout -k 10 500 python -u -m pytest tests/test_rc1pass_gpu.py tests/test_fullsize_gpu.py -m gpu -x -q -k "phong or c3" --timeout 300 --timeout-method thread > gpurun_out/r02_s31_tests.log 2>&1 || { tail -30 gpurun_out/r02_s31_tests.log; exit 1; }
tail -1 gpurun_out/r02_s31_tests.log
bash tools/ab_bench.sh phalpha ph2 "--phong --batch 2 --steps 100 --warmup 20" 2 || exit 1
bash tools/ab_bench.sh phalpha ph4 "--phong --batch 4 --steps 100 --warmup 20" 2 || exit 1
