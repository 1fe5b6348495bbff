#!/bin/bash
# One GPU session of the current round (edited per session; the committed copy is
# the last one run).  Each GPU step has its own limit; the first failure ends the call.
# Round 5, s17: the spread of the driver's own command (20 frames after 5 warmup)
# on one box, against 200-frame runs.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-r05_s17}
out=gpurun_out/${T}_driver_spread.jsonl
: > $out
for i in 1 2 3 4 5 6; do
  timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/${T}_d$i.json 2> gpurun_out/${T}_d$i.err || { tail -5 gpurun_out/${T}_d$i.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/${T}_d$i.json')); print(json.dumps({'run':'d$i','ms':d['ms_per_step'],'kernel_ms':d['roofline']['kernel_ms'],'settle':d['config']['settle_frames']}))" | tee -a $out
done
for i in 1 2; do
  timeout -k 10 300 python3 bench.py --steps 200 --no-cpu-baseline --no-cadence > gpurun_out/${T}_l$i.json 2> gpurun_out/${T}_l$i.err || { tail -5 gpurun_out/${T}_l$i.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/${T}_l$i.json')); print(json.dumps({'run':'l$i','ms':d['ms_per_step'],'kernel_ms':d['roofline']['kernel_ms']}))" | tee -a $out
done
