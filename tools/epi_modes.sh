#!/bin/bash
# Epilogue kernel time per mode (sort+sum, sort only, sum only), rocprofv3 kernel trace.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
mkdir -p gpurun_out/epi
i=0
for m in "--variants b4o1p5q0" "--variants b4o1p5q0 --no-total" "--variants b4o0p0q0"; do
  i=$((i+1))
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/epi/m$i -o t --output-format csv -- python3 tools/ab_rc1pass.py $m --rounds 1 --frames 20 > gpurun_out/epi/m$i.log 2>&1 || exit 1
  echo "mode $i: $m"
  python3 - gpurun_out/epi/m$i <<'PY'
import csv, glob, sys
for f in glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "epilogue" in r["Name"] or "rc1pass" in r["Name"]:
            print("  ", r["Name"][:40], r["Calls"], r["AverageNs"])
PY
done
