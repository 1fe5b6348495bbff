#!/bin/bash
# One GPU session of the current round (edited per session; the committed copy is
# the last one run).  Each GPU step has its own limit; the first failure ends the call.
# Round 5, s28: the per-tile code (codec.hip): GPU parity against the numpy
# restatement, and encode/decode cost and ratio on the headline's shares.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-r05_s28}
timeout -k 10 300 python -u -m pytest -v --timeout 120 --timeout-method thread tests/test_codec.py > gpurun_out/${T}_pytest_codec.log 2>&1 || { tail -30 gpurun_out/${T}_pytest_codec.log; exit 1; }
tail -3 gpurun_out/${T}_pytest_codec.log
timeout -k 10 300 python3 -u tools/codec_probe.py > gpurun_out/${T}_codec_probe.json 2> gpurun_out/${T}_codec_probe.err || { tail -5 gpurun_out/${T}_codec_probe.err; exit 1; }
cat gpurun_out/${T}_codec_probe.json
