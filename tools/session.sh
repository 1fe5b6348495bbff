# round 6, session s29: several launch-order slots per one-wave workgroup (CVR_RC1_TPW 2 / 4) vs 1
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06_s29; mkdir -p $O
export CVR_LIB_OVERRIDE=ablib/t2/libcvr.so
timeout -k 10 400 python -u -m pytest tests/test_rc1pass_gpu.py tests/test_frames_gpu.py tests/test_split_gpu.py -x -q -rf --timeout 200 --timeout-method thread > $O/pytest_t2.log 2>&1 || { tail -20 $O/pytest_t2.log; exit 1; }
tail -1 $O/pytest_t2.log
for rep in 1 2; do
  for lib in cur t2 t4; do
    if [ $lib = cur ]; then unset CVR_LIB_OVERRIDE; else export CVR_LIB_OVERRIDE=ablib/$lib/libcvr.so; fi
    for mode in static orbit; do
      X=""; [ $mode = orbit ] && X="--orbit"
      timeout -k 10 200 python3 bench.py --no-cpu-baseline --steps 200 --warmup 10 $X > $O/${mode}_${lib}_r$rep.json 2>$O/${mode}_${lib}_r$rep.err || exit 1
      python3 -c "import json; d=json.loads(open('$O/${mode}_${lib}_r$rep.json').read().strip().splitlines()[-1]); pc=d.get('plugin_cadence') or {}; print('$mode $lib', d['ms_per_step'], d['value'], (pc.get('static') or {}).get('ms_per_frame'), (pc.get('orbit') or {}).get('ms_per_frame'))"
    done
  done
done
