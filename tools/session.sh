#!/bin/bash
# One GPU session of the current round (edited per session; the committed copy is
# the last one run).  Each GPU step has its own limit; the first failure ends the call.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-r04_s17}
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_split_gpu.py tests/test_frames_gpu.py -m gpu > gpurun_out/${T}_pytest.log 2>&1; rc=$?; tail -3 gpurun_out/${T}_pytest.log; [ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" gpurun_out/${T}_pytest.log | head -20; exit 1; }
timeout -k 10 600 python -u tools/rank0_probe.py --nranks 8 --streams 4 --sets 16 --reserve-cus 0,32 --render-nranks 0,12,16,-1 --frames-per-launch 4 --frames 20,96 > gpurun_out/${T}_rank0.log 2>&1 || { tail -5 gpurun_out/${T}_rank0.log; exit 1; }
grep -v amdgpu.ids gpurun_out/${T}_rank0.log
timeout -k 10 400 python -u tools/rank0_probe.py --renderer dos --nranks 8 --streams 1,4 --frames-per-launch 1 --frames 8 > gpurun_out/${T}_rank0_dos.log 2>&1 || { tail -5 gpurun_out/${T}_rank0_dos.log; exit 1; }
grep -v amdgpu.ids gpurun_out/${T}_rank0_dos.log
timeout -k 10 500 python -u tools/rank0_probe.py --renderer ebs --nranks 8 --streams 1,4 --frames-per-launch 1 --frames 4 > gpurun_out/${T}_rank0_ebs.log 2>&1 || { tail -5 gpurun_out/${T}_rank0_ebs.log; exit 1; }
grep -v amdgpu.ids gpurun_out/${T}_rank0_ebs.log
