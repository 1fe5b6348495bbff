#!/bin/bash
# Session 38: DOS at 3 waves (parity with that build) and 4 waves; EBS at 3 waves (512^3).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
export TMPDIR=/tmp
CVR_LIB_OVERRIDE=ablib/dos3/libcvr.so timeout -k 10 500 python -u -m pytest tests/test_dos_gpu.py tests/test_fullsize_gpu.py -m gpu -x -q -k "dos or c4" --timeout 300 --timeout-method thread > gpurun_out/r02_s38_tests.log 2>&1 || { tail -30 gpurun_out/r02_s38_tests.log; exit 1; }
tail -1 gpurun_out/r02_s38_tests.log
bash tools/ab_bench.sh dos4 dos "--renderer dos --steps 5 --warmup 1" 1 || exit 1
bash tools/ab_bench.sh ebs3 ebs512 "--renderer ebs --size 512 --steps 5 --warmup 1" 2 || exit 1
