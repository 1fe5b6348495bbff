#!/bin/bash
# One GPU session of the current round: the suites touched since the last run, then
# bench lines.  Each GPU step has its own limit; the first failure ends the call.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-r03}
timeout -k 10 500 python -u -m pytest tests/test_filter8_gpu.py tests/test_ebs_gpu.py tests/test_postpass_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1 || { tail -30 gpurun_out/${T}_tests.log; exit 1; }
tail -2 gpurun_out/${T}_tests.log
timeout -k 10 500 python -u -m pytest tests/test_fullsize_gpu.py -k c5 -x -q -s --timeout 450 --timeout-method thread > gpurun_out/${T}_c5.log 2>&1 || { tail -30 gpurun_out/${T}_c5.log; exit 1; }
grep -E "C5:|passed|failed" gpurun_out/${T}_c5.log
timeout -k 10 400 python bench.py --renderer ebs > gpurun_out/${T}_bench_ebs.json 2> gpurun_out/${T}_bench_ebs.err || { tail -20 gpurun_out/${T}_bench_ebs.err; exit 1; }
cat gpurun_out/${T}_bench_ebs.json
