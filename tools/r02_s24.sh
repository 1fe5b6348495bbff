#!/bin/bash
# Session 24: packed-f32 lerps (trilerp y/z, TF classification): parity, A/B vs HEAD.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_rc1pass_gpu.py tests/test_dos_gpu.py tests/test_iso_gpu.py tests/test_ebs_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r02_s24_tests.log 2>&1 || { tail -30 gpurun_out/r02_s24_tests.log; exit 1; }
tail -1 gpurun_out/r02_s24_tests.log
bash tools/ab_bench.sh prev ea "--steps 100 --warmup 20" 3 || exit 1
bash tools/ab_bench.sh prev long "--tf-alpha 0.02 --steps 20 --warmup 5" 2 || exit 1
bash tools/ab_bench.sh prev phong "--phong --steps 100 --warmup 20" 2 || exit 1
