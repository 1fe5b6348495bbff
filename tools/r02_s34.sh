#!/bin/bash
# Session 34: interleaved tile order in the shaded marches: DOS / EBS parity (incl. full size),
# bench lines for DOS (config 4), EBS 1024^3 (config 5), iso.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests/test_dos_gpu.py tests/test_ebs_gpu.py tests/test_fullsize_gpu.py -m gpu -x -q --timeout 400 --timeout-method thread > gpurun_out/r02_s34_tests.log 2>&1 || { tail -30 gpurun_out/r02_s34_tests.log; exit 1; }
tail -1 gpurun_out/r02_s34_tests.log
timeout -k 10 400 python bench.py --renderer dos --no-cpu-baseline > gpurun_out/r02_s34_dos.json 2> gpurun_out/r02_s34_dos.err || { tail -5 gpurun_out/r02_s34_dos.err; exit 1; }
timeout -k 10 600 python bench.py --renderer ebs --no-cpu-baseline > gpurun_out/r02_s34_ebs.json 2> gpurun_out/r02_s34_ebs.err || { tail -5 gpurun_out/r02_s34_ebs.err; exit 1; }
for R in iso isodfs isoadapt; do
  timeout -k 10 300 python bench.py --renderer $R --no-cpu-baseline > gpurun_out/r02_s34_$R.json 2> gpurun_out/r02_s34_$R.err || { tail -5 gpurun_out/r02_s34_$R.err; exit 1; }
done
python3 - <<'PY'
import json
for n in ("dos", "ebs", "iso", "isodfs", "isoadapt"):
    d = json.load(open(f"gpurun_out/r02_s34_{n}.json"))
    print(n, d["ms_per_step"], d["roofline"]["kernel_ms"], d["roofline"]["frac"], d.get("parity", {}).get("bit_exact"))
PY
