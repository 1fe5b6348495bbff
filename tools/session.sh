#!/bin/bash
# One GPU session of the current round (edited per session; the committed copy is
# the last one run).  Each GPU step has its own limit; the first failure ends the call.
# Round 5, s13: schedule options around the new band cap (130): order rebuild
# interval, boost, frames per launch, streams; static view, 200 frames.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-r05_s13}
out=gpurun_out/${T}_matrix.jsonl
: > $out
run() {  # tag, bench args
  local tag=$1; shift
  timeout -k 10 240 python3 bench.py --no-cpu-baseline --no-cadence "$@" > gpurun_out/${T}_$tag.json 2> gpurun_out/${T}_$tag.err || { tail -5 gpurun_out/${T}_$tag.err; return 1; }
  python3 -c "
import json,sys; d=json.loads(open('gpurun_out/${T}_$tag.json').read().strip().splitlines()[-1])
print(json.dumps({'tag':'$tag','ms':d['ms_per_step'],'value':d['value'],'opts':d['config'].get('options'),'fpl':d['config'].get('frames_per_launch'),'streams':d['config'].get('render_streams')}))" | tee -a $out
}
for rep in 1 2; do
  run base_$rep --steps 200 || exit 1
  run oi16_$rep --steps 200 --opt order_interval=16 || exit 1
  run oi32_$rep --steps 200 --opt order_interval=32 || exit 1
  run boost0_$rep --steps 200 --opt boost=0 || exit 1
  run boost10_$rep --steps 200 --opt boost=10 || exit 1
  run fpl8_$rep --steps 200 --frames-per-launch 8 || exit 1
  run s4_$rep --steps 200 --streams 4 || exit 1
  run s2_$rep --steps 200 --streams 2 || exit 1
done
