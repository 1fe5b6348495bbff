#!/bin/bash
# Session 12: deferred (wave-compacted) Blinn-Phong: Phong parity, then A/B vs HEAD (inline shading).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_rc1pass_gpu.py tests/test_fullsize_gpu.py -m gpu -x -q -k "phong" --timeout 300 --timeout-method thread > gpurun_out/r02_s12_tests.log 2>&1 || { tail -30 gpurun_out/r02_s12_tests.log; exit 1; }
tail -1 gpurun_out/r02_s12_tests.log
bash tools/ab_bench.sh prev phong2 "--phong --batch 2 --steps 100 --warmup 20" 2 || exit 1
bash tools/ab_bench.sh prev phong4 "--phong --batch 4 --steps 100 --warmup 20" 2 || exit 1
