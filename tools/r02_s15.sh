#!/bin/bash
# Session 15: segment-parallel digital filter v2: parity, then kernel-trace vs HEAD and probes.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_postpass_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r02_s15_tests.log 2>&1 || { tail -30 gpurun_out/r02_s15_tests.log; exit 1; }
tail -1 gpurun_out/r02_s15_tests.log
bash tools/pp_probe.sh p2 prev new dprobe1 dprobe2
