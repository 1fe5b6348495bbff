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
  python -c "import json; d=json.load(open('gpurun_out/${T}_$name.json')); r=d['roofline']; print('$name', d['ms_per_step'], r['kernel_ms'], d['value'], r['frac'], r.get('frac_fetched'), r.get('skipped_samples'))"
}
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu > gpurun_out/${T}_pytest.log 2>&1; rc=$?; tail -3 gpurun_out/${T}_pytest.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.log 2>&1 || exit 1
tail -1 gpurun_out/${T}_smoke.log
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/${T}_driver.json 2> gpurun_out/${T}_driver.err || exit 1
python -c "import json; d=json.load(open('gpurun_out/${T}_driver.json')); print('driver', d['ms_per_step'], d['value'], d['roofline']['frac'], d.get('parity'))"
run cs3 
run cs3_1s --streams 1
run cs0_1s --streams 1 --cell-skip 0
run phong --phong
run long --tf-alpha 0.02
run orbit --orbit
