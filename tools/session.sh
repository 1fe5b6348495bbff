#!/bin/bash
# One GPU session of the current round (edited per session; the committed copy is
# the last one run).  Each GPU step has its own limit; the first failure ends the call.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-r04_s13}
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_frames_gpu.py tests/test_split_gpu.py -m gpu > gpurun_out/${T}_pytest.log 2>&1; rc=$?; tail -3 gpurun_out/${T}_pytest.log; [ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" gpurun_out/${T}_pytest.log | head -20; exit 1; }
run() {   # name, bench args
  local name=$1; shift
  timeout -k 10 300 python bench.py --no-cpu-baseline "$@" > gpurun_out/${T}_$name.json 2> gpurun_out/${T}_$name.err || { tail -20 gpurun_out/${T}_$name.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/${T}_$name.json')); r=d['roofline']; print('$name', d['ms_per_step'], r['kernel_ms'], d['value'], r['frac'], d['config']['frames_in_flight'])"
}
run driver1 --gpus 1 --steps 20 --warmup 5
run driver2 --gpus 1 --steps 20 --warmup 5
run driver3 --gpus 1 --steps 20 --warmup 5
run phong --phong
for v in ge5 ge4; do
  bash tools/ab_builds.sh $v b2o1p0q0 3 --phong > gpurun_out/${T}_ab_$v.log 2>&1 || { tail -5 gpurun_out/${T}_ab_$v.log; exit 1; }
  cat gpurun_out/${T}_ab_$v.log
done
