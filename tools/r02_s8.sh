#!/bin/bash
# Session 8: buffer-load variant in-tree: rc1pass/full-size parity, A/B vs HEAD
# (ablib/prev), the driver's headline command.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_rc1pass_gpu.py tests/test_fullsize_gpu.py tests/test_split_gpu.py tests/test_postpass_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r02_s8_tests.log 2>&1 || { tail -30 gpurun_out/r02_s8_tests.log; exit 1; }
tail -1 gpurun_out/r02_s8_tests.log
bash tools/ab_builds.sh prev "b4o1p5q0" 3 "--frames 50" || exit 1
bash tools/ab_builds.sh prev "b4o1p5q0" 2 "--tf-alpha 0.02 --frames 10" || exit 1
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r02_bench_driver.json 2> gpurun_out/r02_bench_driver.err || { tail -20 gpurun_out/r02_bench_driver.err; exit 1; }
cat gpurun_out/r02_bench_driver.json
