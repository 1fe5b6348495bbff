#!/bin/bash
# Round-2 session: whole GPU suite, Phong A/B (ablib/base vs the in-tree build,
# batch 4 and 2), the driver's headline command.  Each GPU step has its own limit.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r02_gpu_all.log 2>&1 || { tail -30 gpurun_out/r02_gpu_all.log; exit 1; }
tail -2 gpurun_out/r02_gpu_all.log
bash tools/ab_builds.sh "${A:-base}" "b4o1p5q0,b2o1p5q0" 3 "--phong --frames 30" || exit 1
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r02_bench_driver.json 2> gpurun_out/r02_bench_driver.err || { tail -20 gpurun_out/r02_bench_driver.err; exit 1; }
cat gpurun_out/r02_bench_driver.json
