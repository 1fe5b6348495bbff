#!/bin/bash
# One GPU session of the current round (edited per session; the committed copy is
# the last one run).  Each GPU step has its own limit; the first failure ends the call.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-r03}
PMC_STEPS=24 PMC_TIMEOUT=120 bash tools/pmc_bench.sh rc1pass rc1pass_tile_kernel "--streams 1" > gpurun_out/${T}_pmc_rc1pass.log 2>&1 || { tail -20 gpurun_out/${T}_pmc_rc1pass.log; exit 1; }
PMC_STEPS=12 PMC_TIMEOUT=120 bash tools/pmc_bench.sh phong rc1pass_tile_kernel "--streams 1 --phong" > gpurun_out/${T}_pmc_phong.log 2>&1 || { tail -20 gpurun_out/${T}_pmc_phong.log; exit 1; }
find gpurun_out/pmc_rc1pass -name "*kernel_trace.csv" | head -1 | xargs -I{} python3 -c "
import csv, collections
c = collections.Counter(r['Grid_Size'] for r in csv.DictReader(open('{}')) if 'rc1pass_tile' in r['Kernel_Name'])
print(c)"
