#!/bin/bash
# One GPU session of the current round (edited per session; the committed copy is
# the last one run).  Each GPU step has its own limit; the first failure ends the call.
# Round 5, s24: the GPU suite (with the band-cap multi-frame cases) and a kernel
# trace of the driver's exact command (3 render streams, 20 frames).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-r05_s24}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -rs --timeout 120 --timeout-method thread > gpurun_out/${T}_pytest_gpu_all.log 2>&1 || { tail -30 gpurun_out/${T}_pytest_gpu_all.log; exit 1; }
tail -3 gpurun_out/${T}_pytest_gpu_all.log
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_prof -o trace --output-format csv -- python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/${T}_driver_traced.json 2> gpurun_out/${T}_prof.err || { echo "prof failed"; tail -20 gpurun_out/${T}_prof.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/${T}_driver_traced.json')); print(d['ms_per_step'], d['roofline']['kernel_ms'], d['roofline']['frac'])"
find gpurun_out/${T}_prof -name "*kernel_stats.csv" | head -1
