#!/bin/bash
# One GPU session of the current round (edited per session; the committed copy is
# the last one run).  Each GPU step has its own limit; the first failure ends the call.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-r05_s04}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${T}_pytest_gpu_all.log 2>&1 || { tail -30 gpurun_out/${T}_pytest_gpu_all.log; exit 1; }
tail -2 gpurun_out/${T}_pytest_gpu_all.log
# A/B: the x-lerps as one asm block (no s_nop hazard waits) vs four (round 4)
timeout -k 10 900 bash tools/ab_bench.sh tri_old ea "--steps 200 --warmup 20 --no-cadence" 3 > gpurun_out/${T}_ab_tri_ea.log 2>&1 || { tail -5 gpurun_out/${T}_ab_tri_ea.log; exit 1; }
tail -2 gpurun_out/${T}_ab_tri_ea.log
timeout -k 10 900 bash tools/ab_bench.sh tri_old ea1 "--steps 200 --warmup 20 --no-cadence --frames-per-launch 1 --streams 1" 2 > gpurun_out/${T}_ab_tri_ea1.log 2>&1 || { tail -5 gpurun_out/${T}_ab_tri_ea1.log; exit 1; }
tail -2 gpurun_out/${T}_ab_tri_ea1.log
timeout -k 10 900 bash tools/ab_bench.sh tri_old phong "--phong --no-cadence" 2 > gpurun_out/${T}_ab_tri_phong.log 2>&1 || { tail -5 gpurun_out/${T}_ab_tri_phong.log; exit 1; }
tail -2 gpurun_out/${T}_ab_tri_phong.log
timeout -k 10 900 bash tools/ab_bench.sh tri_old dos "--renderer dos --steps 5" 2 > gpurun_out/${T}_ab_tri_dos.log 2>&1 || { tail -5 gpurun_out/${T}_ab_tri_dos.log; exit 1; }
tail -2 gpurun_out/${T}_ab_tri_dos.log
# per-view kernel times over the 24 reference camera states (static vs orbit, LPT vs interleaved)
timeout -k 10 400 python tools/orbit_views.py --orders 1,2 --smooth 0,3,10 > gpurun_out/${T}_orbit_views.json 2> gpurun_out/${T}_orbit_views.err || { tail -5 gpurun_out/${T}_orbit_views.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/${T}_orbit_views.json')); print(d['modes'], d.get('smooth'))"
# plugin cadence (one frame per call, one stream) with the quad march for the longest
# tiles: a lone frame lasts as long as its longest tile (~110 us at ~0.28 us per batch)
for q in 0 1 3 6; do
  timeout -k 10 300 python bench.py --quad $q --steps 40 --warmup 10 --no-cpu-baseline > gpurun_out/${T}_cad_quad$q.json 2> gpurun_out/${T}_cad_quad$q.err || { tail -5 gpurun_out/${T}_cad_quad$q.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/${T}_cad_quad$q.json')); c=d['plugin_cadence']; print('quad $q', d['ms_per_step'], c['static']['ms_per_frame'], c['static']['kernel_ms_mean'], c['orbit']['ms_per_frame'], c['orbit']['kernel_ms_mean'], d.get('parity', {}).get('bit_exact'))"
done
