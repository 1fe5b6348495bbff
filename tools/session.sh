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
  python -c "import json; d=json.load(open('gpurun_out/${T}_$name.json')); print('$name', d['ms_per_step'], d['roofline']['kernel_ms'])"
}
CVR_LIB_OVERRIDE=ablib/dw5/libcvr.so timeout -k 10 400 python -u -m pytest tests/test_dos_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1 || { tail -30 gpurun_out/${T}_tests.log; exit 1; }
tail -1 gpurun_out/${T}_tests.log
for i in 1 2; do
  run w4_$i "" --renderer dos
  run w5_$i ablib/dw5/libcvr.so --renderer dos
  run w6_$i ablib/dw6/libcvr.so --renderer dos
done
