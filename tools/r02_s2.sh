#!/bin/bash
# Round-2 session 2: rc1pass/full-size parity, Phong K=2 occupancy A/B
# (ablib/k2 = no waves hint), the StepSize eval sweep, the Phong bench line.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_rc1pass_gpu.py tests/test_fullsize_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r02_s2_tests.log 2>&1 || { tail -30 gpurun_out/r02_s2_tests.log; exit 1; }
tail -1 gpurun_out/r02_s2_tests.log
bash tools/ab_builds.sh k2 "b2o1p5q0,b4o1p5q0" 3 "--phong --frames 30" || exit 1
timeout -k 10 400 python tools/eval_rc1pass.py --out gpurun_out/eval_rc1pass > gpurun_out/r02_eval_rc1pass.json 2> gpurun_out/r02_eval_rc1pass.err || { tail -20 gpurun_out/r02_eval_rc1pass.err; exit 1; }
timeout -k 10 300 python bench.py --phong --steps 50 --warmup 20 > gpurun_out/r02_bench_phong.json 2> gpurun_out/r02_bench_phong.err || { tail -20 gpurun_out/r02_bench_phong.err; exit 1; }
cat gpurun_out/r02_bench_phong.json
