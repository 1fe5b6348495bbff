#!/bin/bash
# One GPU session of the current round (edited per session; the committed copy is
# the last one run).  Each GPU step has its own limit; the first failure ends the call.
# Round 5, s26: Blinn-Phong schedule options (batch, band cap, boost, streams).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-r05_s26}
out=gpurun_out/${T}_phong_matrix.jsonl
: > $out
run() {  # tag, bench args
  local tag=$1; shift
  timeout -k 10 240 python3 bench.py --phong --no-cpu-baseline --no-cadence --steps 100 "$@" > gpurun_out/${T}_$tag.json 2> gpurun_out/${T}_$tag.err || { tail -5 gpurun_out/${T}_$tag.err; return 1; }
  python3 -c "
import json,sys; d=json.loads(open('gpurun_out/${T}_$tag.json').read().strip().splitlines()[-1])
print(json.dumps({'tag':'$tag','ms':d['ms_per_step'],'kernel_ms':d['roofline']['kernel_ms'],'opts':d['config'].get('options')}))" | tee -a $out
}
for rep in 1 2; do
  run base_$rep || exit 1
  run k4_$rep --batch 4 || exit 1
  run cap200_$rep --opt band_cap=200 || exit 1
  run boost0_$rep --opt boost=0 || exit 1
  run s4_$rep --streams 4 || exit 1
done
