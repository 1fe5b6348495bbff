#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
for k in 9 1 2 3 4 0; do
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/epp/k$k -o t --output-format csv -- python3 tools/epi_phase.py $k > gpurun_out/epp_k$k.log 2>&1 || exit 1
  python3 - gpurun_out/epp/k$k $k <<'PY'
import csv, glob, sys
for f in glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True):
    d = sorted(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in csv.DictReader(open(f)) if "epilogue" in r["Kernel_Name"])
    print("stop", sys.argv[2], "epilogue median us", d[len(d)//2] / 1000, "n", len(d))
PY
done
