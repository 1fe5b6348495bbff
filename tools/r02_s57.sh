#!/bin/bash
# Session 57: check of the tree: whole GPU suite, smoke, driver-command bench, Phong bench,
# kernel-trace summary of the driver command (one stream).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r02_s57_tests.log 2>&1 || { tail -30 gpurun_out/r02_s57_tests.log; exit 1; }
tail -1 gpurun_out/r02_s57_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r02_s57_smoke.log 2>&1 && tail -1 gpurun_out/r02_s57_smoke.log || exit 1
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r02_s57_bench.json 2> gpurun_out/r02_s57_bench.err || { tail -20 gpurun_out/r02_s57_bench.err; exit 1; }
timeout -k 10 400 python bench.py --phong --no-cpu-baseline > gpurun_out/r02_s57_phong.json 2> gpurun_out/r02_s57_phong.err || { tail -20 gpurun_out/r02_s57_phong.err; exit 1; }
python3 - <<'PY'
import json
for n in ("bench", "phong"):
    d = json.load(open(f"gpurun_out/r02_s57_{n}.json"))
    print(n, d["ms_per_step"], d["value"], d["roofline"]["kernel_ms"], d["roofline"]["frac"], d.get("parity", {}).get("bit_exact"))
PY
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/r02_s57_prof -o trace --output-format csv -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --streams 1 --no-cpu-baseline > gpurun_out/r02_s57_prof_bench.json 2> gpurun_out/r02_s57_prof.err || { tail -20 gpurun_out/r02_s57_prof.err; exit 1; }
grep rc1pass_tile gpurun_out/r02_s57_prof/trace_kernel_stats.csv | awk -F'",' '{print $2}'
