#!/bin/bash
# One GPU session of the current round (edited per session; the committed copy is
# the last one run).  Each GPU step has its own limit; the first failure ends the call.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-r04_s20}
run() {   # name, bench args
  local name=$1; shift
  timeout -k 10 400 python bench.py "$@" > gpurun_out/${T}_$name.json 2> gpurun_out/${T}_$name.err || { tail -20 gpurun_out/${T}_$name.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/${T}_$name.json')); r=d['roofline']; print('$name', d['ms_per_step'], r['kernel_ms'], d['value'], r['frac'], r.get('traffic'), r.get('traffic_frac'))"
}
run driver --gpus 1 --steps 20 --warmup 5
run phong --phong --no-cpu-baseline
run dos --renderer dos --no-cpu-baseline
run ebs --renderer ebs --no-cpu-baseline
run longray --tf-alpha 0.02 --no-cpu-baseline --steps 40
