#!/bin/bash
# One GPU session of the current round (edited per session; the committed copy is
# the last one run).  Each GPU step has its own limit; the first failure ends the call.
# Round 5, s29: the library with the per-tile code (codec.hip) -- GPU suite, smoke, PMC records of every
# workload (bench.py uses a record only on the build it was counted on), bench lines,
# and the one-stream kernel trace of the headline.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-r05_s29}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${T}_pytest_gpu_all.log 2>&1 || { tail -30 gpurun_out/${T}_pytest_gpu_all.log; exit 1; }
tail -2 gpurun_out/${T}_pytest_gpu_all.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.log 2>&1 || { tail -10 gpurun_out/${T}_smoke.log; exit 1; }
tail -1 gpurun_out/${T}_smoke.log
timeout -k 10 2400 bash tools/pmc_session.sh rc1pass phong longray dos ebs > gpurun_out/${T}_pmc_session.log 2>&1 || { tail -20 gpurun_out/${T}_pmc_session.log; exit 1; }
tail -5 gpurun_out/${T}_pmc_session.log
for w in rc1pass rc1pass_phong rc1pass_longray dos ebs; do cp gpurun_out/pmc_$w.json profiles/pmc_$w.json; done
run() {   # name, bench args
  local name=$1; shift
  timeout -k 10 400 python bench.py "$@" > gpurun_out/${T}_$name.json 2> gpurun_out/${T}_$name.err || { tail -20 gpurun_out/${T}_$name.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/${T}_$name.json')); r=d['roofline']; print('$name', d['ms_per_step'], r['kernel_ms'], r.get('bound'), r['frac'], r.get('effective_frac'), d['value'], json.dumps({k: (v['ms_per_frame'], v['kernel_ms_mean']) for k, v in d.get('plugin_cadence', {}).items() if isinstance(v, dict)}))"
}
run driver --gpus 1 --steps 20 --warmup 5
run driver200
run phong --phong --no-cadence
run longray --tf-alpha 0.02 --no-cadence
run orbit --orbit --steps 96 --warmup 24 --no-cpu-baseline
run dos --renderer dos
run ebs --renderer ebs
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_prof -o trace --output-format csv -- python3 bench.py --no-cpu-baseline --no-cadence --streams 1 --steps 20 > gpurun_out/${T}_prof_bench.json 2> gpurun_out/${T}_prof.err || { echo "prof failed"; tail -20 gpurun_out/${T}_prof.err; exit 1; }
find gpurun_out/${T}_prof -name "*kernel_stats.csv" | head -1
