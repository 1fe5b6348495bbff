#!/bin/bash
# One GPU session of the current round (edited per session; the committed copy is
# the last one run).  Each GPU step has its own limit; the first failure ends the call.
# Round 5, s06: the prefetched march (option "prefetch") -- parity, then A/B.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-r05_s06}
timeout -k 10 300 python -u -m pytest tests/test_prefetch_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/${T}_pytest_prefetch.log 2>&1 || { tail -30 gpurun_out/${T}_pytest_prefetch.log; exit 1; }
tail -2 gpurun_out/${T}_pytest_prefetch.log
ab() {   # name, bench args (prefetch 0 / 1 alternated, 3 repeats)
  local name=$1; shift
  for rep in 1 2 3; do for pf in 0 1; do
    timeout -k 10 300 python bench.py --prefetch $pf --no-cpu-baseline "$@" > gpurun_out/${T}_${name}_pf${pf}_$rep.json 2> gpurun_out/${T}_${name}_pf${pf}_$rep.err || { tail -10 gpurun_out/${T}_${name}_pf${pf}_$rep.err; exit 1; }
  done; done
  python3 - "$name" <<'PY'
import json, sys
name = sys.argv[1]
for pf in (0, 1):
    rows = [json.load(open(f"gpurun_out/r05_s06_{name}_pf{pf}_{r}.json")) for r in (1, 2, 3)]
    cad = [d.get("plugin_cadence", {}).get("static", {}) for d in rows]
    print(name, "prefetch", pf, "ms/frame", [d["ms_per_step"] for d in rows], "kernel",
          [d["roofline"]["kernel_ms"] for d in rows], "cadence", [c.get("ms_per_frame") for c in cad],
          [c.get("kernel_ms_mean") for c in cad])
PY
}
ab driver --steps 200 --warmup 20
ab long --tf-alpha 0.02 --no-cadence --steps 40
ab orbit --orbit --steps 96 --warmup 24
