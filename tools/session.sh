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
timeout -k 10 400 python -u -m pytest tests/test_split_gpu.py tests/test_rc1pass_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1 || { tail -30 gpurun_out/${T}_tests.log; exit 1; }
tail -1 gpurun_out/${T}_tests.log
for i in 1 2 3; do
  run head_$i ablib/head/libcvr.so
  run new_$i ""
done
run head_s1 ablib/head/libcvr.so --streams 1
run new_s1 "" --streams 1
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err || { tail -20 gpurun_out/${T}_bench.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/${T}_bench.json')); print('driver', d['ms_per_step'], d['value'], d['config']['hw_queues'], d['config']['frames_in_flight'])"
timeout -k 10 200 python tools/host_overhead.py > gpurun_out/${T}_host.log 2>&1 || { tail -10 gpurun_out/${T}_host.log; exit 1; }
tail -8 gpurun_out/${T}_host.log
