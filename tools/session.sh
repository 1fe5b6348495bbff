#!/bin/bash
# One GPU session of the current round (edited per session; the committed copy is
# the last one run).  Each GPU step has its own limit; the first failure ends the call.
# Round 5, s19: the RCCL gather with several ranks on one GPU (rendering root at 2
# ranks, idle root at 3), with the skip reasons of the GPU suite.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-r05_s19}
timeout -k 10 400 python3 -u -m pytest -v -rs --timeout 180 --timeout-method thread tests/test_split_gpu.py -k "ranks_one_gpu" > gpurun_out/${T}_pytest_rccl.log 2>&1 || { tail -30 gpurun_out/${T}_pytest_rccl.log; exit 1; }
tail -8 gpurun_out/${T}_pytest_rccl.log
timeout -k 10 600 python3 -u -m pytest tests -m gpu -q -rs --timeout 120 --timeout-method thread > gpurun_out/${T}_pytest_gpu_all.log 2>&1 || { tail -30 gpurun_out/${T}_pytest_gpu_all.log; exit 1; }
tail -4 gpurun_out/${T}_pytest_gpu_all.log
