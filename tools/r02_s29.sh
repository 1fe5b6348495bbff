#!/bin/bash
# Session 29: alpha-first classification (ablib/alpha1): rc1pass parity with that build, A/B vs HEAD.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
export TMPDIR=/tmp
CVR_LIB_OVERRIDE=ablib/alpha1/libcvr.so timeout -k 10 500 python -u -m pytest tests/test_rc1pass_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r02_s29_tests.log 2>&1 || { tail -30 gpurun_out/r02_s29_tests.log; exit 1; }
tail -1 gpurun_out/r02_s29_tests.log
bash tools/ab_bench.sh alpha1 ea "--steps 100 --warmup 20" 3 || exit 1
bash tools/ab_bench.sh alpha1 long "--tf-alpha 0.02 --steps 20 --warmup 5" 2 || exit 1
