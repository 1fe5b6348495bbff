#!/bin/bash
# Session 11 (re-entry): whole GPU suite, smoke, driver-command bench, Phong bench.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r02_s11_tests.log 2>&1 || { tail -30 gpurun_out/r02_s11_tests.log; exit 1; }
tail -1 gpurun_out/r02_s11_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r02_s11_smoke.log 2>&1 && tail -1 gpurun_out/r02_s11_smoke.log || exit 1
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r02_s11_bench.json 2> gpurun_out/r02_s11_bench.err || { tail -20 gpurun_out/r02_s11_bench.err; exit 1; }
cat gpurun_out/r02_s11_bench.json
timeout -k 10 400 python bench.py --phong --no-cpu-baseline > gpurun_out/r02_s11_phong.json 2> gpurun_out/r02_s11_phong.err || { tail -20 gpurun_out/r02_s11_phong.err; exit 1; }
cat gpurun_out/r02_s11_phong.json
