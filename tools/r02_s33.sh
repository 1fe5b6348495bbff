#!/bin/bash
# Session 33: iso parity (interleaved default); DOS / EBS-512 interleaved tile order (ablib/shil) vs bands.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_iso_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r02_s33_tests.log 2>&1 || { tail -30 gpurun_out/r02_s33_tests.log; exit 1; }
tail -1 gpurun_out/r02_s33_tests.log
bash tools/ab_bench.sh shil dos "--renderer dos --steps 5 --warmup 1" 2 || exit 1
bash tools/ab_bench.sh shil ebs512 "--renderer ebs --size 512 --steps 5 --warmup 1" 2 || exit 1
