#!/bin/bash
# One GPU session of the current round (edited per session; the committed copy is
# the last one run).  Each GPU step has its own limit; the first failure ends the call.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-r04_s25}
run() {   # name, bench args
  local name=$1; shift
  timeout -k 10 300 python bench.py "$@" > gpurun_out/${T}_$name.json 2> gpurun_out/${T}_$name.err || { tail -20 gpurun_out/${T}_$name.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/${T}_$name.json')); r=d['roofline']; print('$name', d['ms_per_step'], r['kernel_ms'], r['frac'], d['value'])"
}
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread --durations 5 > gpurun_out/${T}_pytest_gpu_all.log 2>&1 || { tail -30 gpurun_out/${T}_pytest_gpu_all.log; exit 1; }
tail -1 gpurun_out/${T}_pytest_gpu_all.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/${T}_smoke.log 2>&1 || { tail -20 gpurun_out/${T}_smoke.log; exit 1; }
tail -1 gpurun_out/${T}_smoke.log
bash tools/pmc_session.sh rc1pass phong longray dos ebs || exit 1
run driver
run phong --no-cpu-baseline --phong
run longray --no-cpu-baseline --tf-alpha 0.02
run dos --no-cpu-baseline --renderer dos
run ebs --no-cpu-baseline --renderer ebs
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_prof -o run -- python3 bench.py --no-cpu-baseline > gpurun_out/${T}_prof_bench.json 2> gpurun_out/${T}_prof.err || { tail -20 gpurun_out/${T}_prof.err; exit 1; }
echo prof done
# probe: a sample in its predecessor's cell reuses that load (CVR_CELL_REUSE build)
CVR_LIB_OVERRIDE=$PWD/cpp_volume_rendering_amd/lib/libcvr_reuse.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_frames_gpu.py tests/test_rc1pass_gpu.py > gpurun_out/${T}_reuse_tests.log 2>&1 || { tail -30 gpurun_out/${T}_reuse_tests.log; exit 1; }
tail -1 gpurun_out/${T}_reuse_tests.log
for rep in 1 2 3; do
  run base_$rep --no-cpu-baseline
  CVR_LIB_OVERRIDE=$PWD/cpp_volume_rendering_amd/lib/libcvr_reuse.so run reuse_$rep --no-cpu-baseline
done
