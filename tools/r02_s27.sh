#!/bin/bash
# Session 27: DOS border test from the exponent's sign: DOS parity (incl. full size), A/B vs HEAD.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_dos_gpu.py tests/test_fullsize_gpu.py -m gpu -x -q -k "dos or c4" --timeout 300 --timeout-method thread > gpurun_out/r02_s27_tests.log 2>&1 || { tail -30 gpurun_out/r02_s27_tests.log; exit 1; }
tail -1 gpurun_out/r02_s27_tests.log
bash tools/ab_bench.sh prev dos "--renderer dos --steps 5 --warmup 1" 2 || exit 1
