#!/bin/bash
# One GPU session of the current round (edited per session; the committed copy is
# the last one run).  Each GPU step has its own limit; the first failure ends the call.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-r04_s18}
bash tools/gpu_round.sh all || exit 1
for i in 1 2; do
  timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/${T}_driver$i.json 2> gpurun_out/${T}_driver$i.err || { tail -5 gpurun_out/${T}_driver$i.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/${T}_driver$i.json')); print('driver', d['ms_per_step'], d['value'], d['roofline']['kernel_ms'], d['roofline']['frac'])"
done
timeout -k 10 300 python -u tools/overlap_probe.py --hwq 32 --nranks 7 --streams 4 --frames 96 --frames-per-launch 4 > gpurun_out/${T}_split7.log 2>&1 || { tail -5 gpurun_out/${T}_split7.log; exit 1; }
timeout -k 10 300 python -u tools/overlap_probe.py --hwq 32 --nranks 7 --streams 4 --frames 20 --frames-per-launch 4 >> gpurun_out/${T}_split7.log 2>&1 || { tail -5 gpurun_out/${T}_split7.log; exit 1; }
grep -v amdgpu.ids gpurun_out/${T}_split7.log
timeout -k 10 300 python -u tools/host_overhead.py --frames 200 > gpurun_out/${T}_host.log 2>&1 || { tail -5 gpurun_out/${T}_host.log; exit 1; }
grep -v amdgpu.ids gpurun_out/${T}_host.log
