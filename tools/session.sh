#!/bin/bash
# One GPU session of the current round (edited per session; the committed copy is
# the last one run).  Each GPU step has its own limit; the first failure ends the call.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-r04_s15}
for p in copy unpack both; do
  timeout -k 10 300 python -u tools/rank0_probe.py --nranks 8 --streams 4 --frames-per-launch 4 --frames 96 --parts $p > gpurun_out/${T}_rank0_$p.log 2>&1 || { tail -5 gpurun_out/${T}_rank0_$p.log; exit 1; }
  grep -v amdgpu.ids gpurun_out/${T}_rank0_$p.log
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_prof -o rank0 --output-format csv -- python3 tools/rank0_probe.py --nranks 8 --streams 4 --frames-per-launch 4 --frames 96 > gpurun_out/${T}_rank0_prof.log 2>&1 || { tail -5 gpurun_out/${T}_rank0_prof.log; exit 1; }
find gpurun_out/${T}_prof -name "*kernel_stats*" -exec head -12 {} \;
