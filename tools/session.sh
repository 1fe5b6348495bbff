#!/bin/bash
# One GPU session of the current round (edited per session; the committed copy is
# the last one run).  Each GPU step has its own limit; the first failure ends the call.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-r03}
env | grep -i "GPU_MAX\|HIP_\|HSA_" > gpurun_out/${T}_env.txt || true
run() {   # name, lib override ('' = in-tree), bench args
  local name=$1 lib=$2; shift 2
  if [ -n "$lib" ]; then export CVR_LIB_OVERRIDE=$lib; else unset CVR_LIB_OVERRIDE; fi
  timeout -k 10 300 python bench.py --no-cpu-baseline "$@" > gpurun_out/${T}_$name.json 2> gpurun_out/${T}_$name.err || { tail -20 gpurun_out/${T}_$name.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/${T}_$name.json')); print('$name', d['ms_per_step'], d['roofline']['kernel_ms'])"
}
for i in 1 2; do
  for q in 4 8; do
    run ea_q${q}_$i "" --hw-queues $q
    run phong_q${q}_$i "" --hw-queues $q --phong
    run iso_q${q}_$i "" --hw-queues $q --renderer iso
  done
done
