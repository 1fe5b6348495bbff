#!/bin/bash
# Session 13: segment-parallel digital filter: post-pass parity, then bench --postpass A/B vs HEAD.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_postpass_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r02_s13_tests.log 2>&1 || { tail -30 gpurun_out/r02_s13_tests.log; exit 1; }
tail -1 gpurun_out/r02_s13_tests.log
for L in prev new; do
  if [ "$L" = prev ]; then export CVR_LIB_OVERRIDE=ablib/prev/libcvr.so; else unset CVR_LIB_OVERRIDE; fi
  timeout -k 10 300 python bench.py --no-cpu-baseline --postpass --steps 20 --warmup 5 > gpurun_out/r02_s13_pp_$L.json 2> gpurun_out/r02_s13_pp_$L.err || { tail -5 gpurun_out/r02_s13_pp_$L.err; exit 1; }
done
unset CVR_LIB_OVERRIDE
python3 - <<'PY'
import json
for L in ("prev", "new"):
    d = json.load(open(f"gpurun_out/r02_s13_pp_{L}.json"))
    print(L, [(f["mode"], f["kernel"], f["ms"], f["GB_s"]) for f in d["postpass"]["filters"]])
PY
