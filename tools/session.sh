#!/bin/bash
# One GPU session of the current round (edited per session; the committed copy is
# the last one run).  Each GPU step has its own limit; the first failure ends the call.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-r03}
for q in 8 16; do
timeout -k 10 300 python -u tools/overlap_probe.py --hwq $q --nranks 8 --tile 16 --quad 0,10 --streams 4,6,8,12,16 --frames 48 --out gpurun_out/${T}_split_hwq$q.json > gpurun_out/${T}_split_hwq$q.log 2>&1 || { tail -20 gpurun_out/${T}_split_hwq$q.log; exit 1; }
grep '^{' gpurun_out/${T}_split_hwq$q.log | python -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l); print(d['hwq'], d['quad'], d['streams'], d['max_ms'], d['mean_ms'])"
done
