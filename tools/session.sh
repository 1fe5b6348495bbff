#!/bin/bash
# One GPU session of the current round (edited per session; the committed copy is
# the last one run).  Each GPU step has its own limit; the first failure ends the call.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-r05_s02}
# the state-race test on the round-4 library (expected to FAIL there: setters synchronised
# only the context stream), TF case only (a volume change there frees cells in use)
CVR_LIB_OVERRIDE=ablib/r04/libcvr.so timeout -k 10 120 python -u -m pytest tests/test_state_race_gpu.py -k "tf" -x -q --timeout 60 --timeout-method thread > gpurun_out/${T}_race_r04lib.log 2>&1; echo "r04 lib race test rc $?"; tail -3 gpurun_out/${T}_race_r04lib.log
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${T}_pytest_gpu_all.log 2>&1 || { tail -30 gpurun_out/${T}_pytest_gpu_all.log; exit 1; }
tail -2 gpurun_out/${T}_pytest_gpu_all.log
run() {   # name, bench args
  local name=$1; shift
  timeout -k 10 300 python bench.py "$@" > gpurun_out/${T}_$name.json 2> gpurun_out/${T}_$name.err || { tail -20 gpurun_out/${T}_$name.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/${T}_$name.json')); r=d['roofline']; print('$name', d['ms_per_step'], r['kernel_ms'], r.get('bound'), r['frac'], r.get('effective_frac'), d['value'], json.dumps(d.get('plugin_cadence', {}))[:700])"
}
# A/B: Blinn-Phong deferred (new) vs inline (round 4); DOS flat shading at 4 waves vs 5
timeout -k 10 900 bash tools/ab_bench.sh phong_inline phong "--phong --no-cadence" 2 > gpurun_out/${T}_ab_phong.log 2>&1 || { tail -5 gpurun_out/${T}_ab_phong.log; exit 1; }
tail -2 gpurun_out/${T}_ab_phong.log
timeout -k 10 900 bash tools/ab_bench.sh dos4 dos "--renderer dos --steps 5" 2 > gpurun_out/${T}_ab_dos.log 2>&1 || { tail -5 gpurun_out/${T}_ab_dos.log; exit 1; }
tail -2 gpurun_out/${T}_ab_dos.log
# the PMC records of this library (rc1pass 4-frame launches, Phong), then the bench line
timeout -k 10 1200 bash tools/pmc_session.sh rc1pass phong > gpurun_out/${T}_pmc_session.log 2>&1 || { tail -20 gpurun_out/${T}_pmc_session.log; exit 1; }
tail -3 gpurun_out/${T}_pmc_session.log
cp gpurun_out/pmc_rc1pass.json profiles/pmc_rc1pass.json
cp gpurun_out/pmc_rc1pass_phong.json profiles/pmc_rc1pass_phong.json
run driver --steps 20 --warmup 5
run phong --phong --no-cadence
