#!/bin/bash
# MAIN-to-MAIN launch gaps of the ray-march kernel for ab_rc1pass variants (rocprofv3 kernel trace).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
for v in "$@"; do
  timeout -k 10 120 rocprofv3 --kernel-trace -d gpurun_out/gap/$v -o t --output-format csv -- python3 tools/ab_rc1pass.py --variants $v --rounds 1 --frames 30 > gpurun_out/gap_$v.log 2>&1 || exit 1
  python3 - gpurun_out/gap/$v $v <<'PY'
import csv, glob, sys, statistics
f = glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True)[0]
rows = sorted((r for r in csv.DictReader(open(f)) if "rc1pass" in r["Kernel_Name"]), key=lambda r: int(r["Start_Timestamp"]))[-20:]
g = [(int(b["Start_Timestamp"]) - int(a["End_Timestamp"])) / 1000 for a, b in zip(rows, rows[1:])]
d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000 for r in rows]
print(sys.argv[2], "gap median %.1f us, kernel median %.1f us" % (statistics.median(g), statistics.median(d)))
PY
done
