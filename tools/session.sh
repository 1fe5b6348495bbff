#!/bin/bash
# One GPU session of the current round (edited per session; the committed copy is
# the last one run).  Each GPU step has its own limit; the first failure ends the call.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-r04}
run() {   # name, bench args
  local name=$1; shift
  timeout -k 10 300 python bench.py --no-cpu-baseline "$@" > gpurun_out/${T}_$name.json 2> gpurun_out/${T}_$name.err || { tail -20 gpurun_out/${T}_$name.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/${T}_$name.json')); r=d['roofline']; print('$name', d['ms_per_step'], r['kernel_ms'], d['value'], r['frac'], d['config']['frames_in_flight'])"
}
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_dos_gpu.py tests/test_ebs_gpu.py tests/test_filter8_gpu.py tests/test_split_gpu.py -m gpu > gpurun_out/${T}_pytest.log 2>&1; rc=$?; tail -3 gpurun_out/${T}_pytest.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 600 python -u -m pytest -x -q --timeout 500 --timeout-method thread tests/test_fullsize_gpu.py -m gpu -k "c4 or c5" > gpurun_out/${T}_c45.log 2>&1; rc=$?; tail -3 gpurun_out/${T}_c45.log; [ $rc -eq 0 ] || exit 1
run dos --renderer dos
run dos_cs0 --renderer dos --cell-skip 0
run ebs --renderer ebs --steps 4
