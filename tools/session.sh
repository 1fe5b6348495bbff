#!/bin/bash
# One GPU session of the current round (edited per session; the committed copy is
# the last one run).  Each GPU step has its own limit; the first failure ends the call.
# Round 5, s25: the band-cap test (bands within the cap under the learned order).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-r05_s25}
timeout -k 10 300 python -u -m pytest -v --timeout 120 --timeout-method thread tests/test_rc1pass_gpu.py -k "band_cap" > gpurun_out/${T}_pytest_bandcap.log 2>&1 || { tail -30 gpurun_out/${T}_pytest_bandcap.log; exit 1; }
tail -6 gpurun_out/${T}_pytest_bandcap.log
