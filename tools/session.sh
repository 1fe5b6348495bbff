#!/bin/bash
# One GPU session of the current round (edited per session; the committed copy is
# the last one run).  Each GPU step has its own limit; the first failure ends the call.
# Round 5, s27: the plugin cadence (one frame per call) against the priority
# boost of the longest tiles and the band cap.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-r05_s27}
out=gpurun_out/${T}_cadence.jsonl
: > $out
run() {  # tag, bench args
  local tag=$1; shift
  timeout -k 10 240 python3 bench.py --no-cpu-baseline --steps 20 "$@" > gpurun_out/${T}_$tag.json 2> gpurun_out/${T}_$tag.err || { tail -5 gpurun_out/${T}_$tag.err; return 1; }
  python3 -c "
import json,sys; d=json.loads(open('gpurun_out/${T}_$tag.json').read().strip().splitlines()[-1])
pc=d['plugin_cadence']
print(json.dumps({'tag':'$tag','static':[pc['static']['ms_per_frame'],pc['static']['kernel_ms_mean']],'orbit':[pc['orbit']['ms_per_frame'],pc['orbit']['kernel_ms_mean']],'opts':d['config'].get('options')}))" | tee -a $out
}
for rep in 1 2; do
  run base_$rep || exit 1
  run boost0_$rep --opt boost=0 || exit 1
  run boost20_$rep --opt boost=20 || exit 1
  run boost50_$rep --opt boost=50 || exit 1
  run cap200_$rep --opt band_cap=200 || exit 1
done
