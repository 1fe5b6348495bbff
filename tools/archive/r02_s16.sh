#!/bin/bash
# Session 16: digital filter diagnostics (per-workgroup unresolved-segment counts on the bench frames).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
export TMPDIR=/tmp
CVR_LIB_OVERRIDE=ablib/dstats/libcvr.so timeout -k 10 300 python bench.py --no-cpu-baseline --postpass --steps 1 --warmup 0 > gpurun_out/r02_s16_bench.json 2> gpurun_out/r02_s16.err; rc=$?
grep DSTAT gpurun_out/r02_s16_bench.json > gpurun_out/r02_s16_dstat.txt || true
wc -l gpurun_out/r02_s16_dstat.txt
exit $rc
