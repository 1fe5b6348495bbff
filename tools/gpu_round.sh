#!/bin/bash
# One GPU-box session: parity tests, smoke, bench, kernel-trace profile.
# Every GPU step has its own time limit; steps are chained with && so the
# first failure ends the call.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
export TMPDIR=/tmp
STEP=${1:-all}
nproc > gpurun_out/host_nproc.txt; lscpu > gpurun_out/host_lscpu.txt 2>&1 || true
if [ "$STEP" = "all" ] || [ "$STEP" = "test" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -rf --durations=15 --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/pytest_gpu.log; exit 1; }
  tail -3 gpurun_out/pytest_gpu.log
fi
if [ "$STEP" = "all" ] || [ "$STEP" = "bench" ]; then
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && tail -1 gpurun_out/smoke.log && \
  timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench.json 2> gpurun_out/bench.err && cat gpurun_out/bench.json || { echo "bench failed"; tail -20 gpurun_out/bench.err; exit 1; }
fi
if [ "$STEP" = "all" ] || [ "$STEP" = "prof" ]; then
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o trace --output-format csv -- python3 bench.py --no-cpu-baseline --no-cadence --streams 1 --steps 20 > gpurun_out/prof_bench.json 2> gpurun_out/prof.err || { echo "prof failed"; tail -20 gpurun_out/prof.err; exit 1; }
  find gpurun_out/prof -name "*stats*" | head
fi
