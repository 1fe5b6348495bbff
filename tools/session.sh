#!/bin/bash
# One GPU session of the current round (edited per session; the committed copy is
# the last one run).  Each GPU step has its own limit; the first failure ends the call.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-r03}
run() {   # name, lib override ('' = in-tree), bench args
  local name=$1 lib=$2; shift 2
  if [ -n "$lib" ]; then export CVR_LIB_OVERRIDE=$lib; else unset CVR_LIB_OVERRIDE; fi
  timeout -k 10 300 python bench.py --no-cpu-baseline "$@" > gpurun_out/${T}_$name.json 2> gpurun_out/${T}_$name.err || { tail -20 gpurun_out/${T}_$name.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/${T}_$name.json')); p=d.get('precompute',{}); print('$name', d['ms_per_step'], d['roofline']['kernel_ms'], p.get('sat_gpu_ms'), d.get('parity'))"
}
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_ebs_gpu.py tests/test_fullsize_gpu.py -m gpu -k "ebs or c5" > gpurun_out/${T}_pytest.log 2>&1; rc=$?; tail -3 gpurun_out/${T}_pytest.log; [ $rc -eq 0 ] || exit 1
run ebs "" --renderer ebs
