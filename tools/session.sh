#!/bin/bash
# One GPU session of the current round (edited per session; the committed copy is
# the last one run).  Each GPU step has its own limit; the first failure ends the call.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-r03}
timeout -k 10 400 python -u -m pytest tests/test_dos_gpu.py tests/test_ebs_gpu.py tests/test_split_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1 || { tail -30 gpurun_out/${T}_tests.log; exit 1; }
tail -1 gpurun_out/${T}_tests.log
for r in dos ebs; do
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_prof_$r -o trace --output-format csv -- python3 bench.py --renderer $r --no-cpu-baseline --streams 1 --steps 3 > gpurun_out/${T}_prof_$r.json 2> gpurun_out/${T}_prof_$r.err || { echo "prof $r failed"; tail -20 gpurun_out/${T}_prof_$r.err; exit 1; }
  find gpurun_out/${T}_prof_$r -name "*kernel_stats.csv" -exec cp {} gpurun_out/${T}_${r}_kernel_stats.csv \;
  python - <<PY
import csv
for row in csv.DictReader(open('gpurun_out/${T}_${r}_kernel_stats.csv')):
    if 'flat' in row['Name'] or 'shaded' in row['Name']:
        print('$r', row['Name'][:60], round(float(row['AverageNs'])/1e6, 3))
PY
  timeout -k 10 400 python bench.py --renderer $r --no-cpu-baseline > gpurun_out/${T}_bench_$r.json 2> gpurun_out/${T}_bench_$r.err || { tail -20 gpurun_out/${T}_bench_$r.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/${T}_bench_$r.json')); print('$r', d['ms_per_step'], d['roofline']['kernel_ms'])"
done
timeout -k 10 300 python -u tools/overlap_probe.py --renderer dos --nranks 2,4,8 --tile 16 --frames 4 --streams 1 --out gpurun_out/${T}_split_dos.json > gpurun_out/${T}_split_dos.log 2>&1 || { tail -20 gpurun_out/${T}_split_dos.log; exit 1; }
grep '^{' gpurun_out/${T}_split_dos.log | cut -c1-200
timeout -k 10 400 python -u tools/overlap_probe.py --renderer ebs --nranks 2,4,8 --tile 16 --frames 2 --streams 1 --out gpurun_out/${T}_split_ebs.json > gpurun_out/${T}_split_ebs.log 2>&1 || { tail -20 gpurun_out/${T}_split_ebs.log; exit 1; }
grep '^{' gpurun_out/${T}_split_ebs.log | cut -c1-200
