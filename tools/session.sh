#!/bin/bash
# One GPU session of the current round (edited per session; the committed copy is
# the last one run).  Each GPU step has its own limit; the first failure ends the call.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-r04_s22}
run() {   # name, bench args
  local name=$1; shift
  timeout -k 10 300 python bench.py --no-cpu-baseline "$@" > gpurun_out/${T}_$name.json 2> gpurun_out/${T}_$name.err || { tail -20 gpurun_out/${T}_$name.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/${T}_$name.json')); r=d['roofline']; print('$name', d['ms_per_step'], r['kernel_ms'], d['value'])"
}
for rep in 1 2; do
for LS in 4:3 5:2 5:3 5:4 4:2 8:2; do
  L=${LS%:*}; S=${LS#*:}
  run L${L}s${S}_$rep --gpus 1 --steps 20 --warmup 5 --frames-per-launch $L --streams $S
done; done
