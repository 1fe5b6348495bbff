#!/bin/bash
# Session 52: EBS AO shells through the half-box pipeline: parity, A/B vs HEAD.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_ebs_gpu.py tests/test_fullsize_gpu.py -k "ebs or c5" -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r02_s52_tests.log 2>&1 || { tail -30 gpurun_out/r02_s52_tests.log; exit 1; }
tail -1 gpurun_out/r02_s52_tests.log
bash tools/ab_bench.sh prev ebs512ao "--renderer ebs --size 512 --steps 5 --warmup 1" 3 || exit 1
bash tools/ab_bench.sh prev ebs1024ao "--renderer ebs --steps 2 --warmup 1" 1 || exit 1
