#!/bin/bash
# One GPU session of the current round (edited per session; the committed copy is
# the last one run).  Each GPU step has its own limit; the first failure ends the call.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-r04_s27}
run() {   # name, bench args
  local name=$1; shift
  timeout -k 10 300 python bench.py "$@" > gpurun_out/${T}_$name.json 2> gpurun_out/${T}_$name.err || { tail -20 gpurun_out/${T}_$name.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/${T}_$name.json')); r=d['roofline']; print('$name', d['ms_per_step'], r['kernel_ms'], r['frac'], d['value'])"
}
for rep in 1 2; do for F in 20 96; do
timeout -k 10 300 python tools/overlap_probe.py --nranks 7,8 --frames-per-launch 4 --streams 4 --hwq 32 --frames $F --interleave 0,1 > gpurun_out/${T}_split_F${F}_$rep.jsonl 2> gpurun_out/${T}_split.err || { tail -20 gpurun_out/${T}_split.err; exit 1; }
cat gpurun_out/${T}_split_F${F}_$rep.jsonl | python3 -c "import sys,json; [print($F, d['nranks'], d['interleave'], d['max_ms'], d['mean_ms']) for d in map(json.loads, sys.stdin)]"
done; done
