#!/bin/bash
# One GPU session of the current round (edited per session; the committed copy is
# the last one run).  Each GPU step has its own limit; the first failure ends the call.
# Round 5, s20: shading passes of the Blinn-Phong march (probe build).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-r05_s20}
CVR_LIB_OVERRIDE=ablib/passprobe/libcvr.so timeout -k 10 300 python3 tools/phong_pass_probe.py > gpurun_out/${T}_phong_passes.json 2> gpurun_out/${T}_phong_passes.err || { tail -5 gpurun_out/${T}_phong_passes.err; exit 1; }
cat gpurun_out/${T}_phong_passes.json
