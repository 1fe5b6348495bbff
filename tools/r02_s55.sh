#!/bin/bash
# Session 55: shaded marches with XCD column groups of 4: DOS/EBS parity (incl. split and full size), benches.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests/test_dos_gpu.py tests/test_ebs_gpu.py tests/test_split_gpu.py tests/test_fullsize_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r02_s55_tests.log 2>&1 || { tail -30 gpurun_out/r02_s55_tests.log; exit 1; }
tail -1 gpurun_out/r02_s55_tests.log
timeout -k 10 600 python bench.py --renderer ebs > gpurun_out/r02_s55_ebs.json 2> gpurun_out/r02_s55_ebs.err || { tail -20 gpurun_out/r02_s55_ebs.err; exit 1; }
timeout -k 10 600 python bench.py --renderer dos > gpurun_out/r02_s55_dos.json 2> gpurun_out/r02_s55_dos.err || { tail -20 gpurun_out/r02_s55_dos.err; exit 1; }
python3 - <<'PY'
import json
for n in ("ebs", "dos"):
    d = json.load(open(f"gpurun_out/r02_s55_{n}.json"))
    print(n, d["ms_per_step"], d["value"], d["roofline"]["kernel_ms"], d["roofline"]["frac"], d.get("parity", {}).get("bit_exact"))
PY
