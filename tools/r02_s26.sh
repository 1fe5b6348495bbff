#!/bin/bash
# Session 26: per-rank cost at N = 8 / 4 by launch order (0 screen bands, 1 LPT, 2 interleaved).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
export TMPDIR=/tmp
export GPU_MAX_HW_QUEUES=8
for o in 0 1 2; do
  timeout -k 10 200 python tools/overlap_probe.py --nranks 8 --frames 96 --streams 4,6 --quads 0,10 --order $o | sed "s/^/order $o /" >> gpurun_out/r02_s26.txt 2>&1 || exit 1
  timeout -k 10 200 python tools/overlap_probe.py --nranks 4 --frames 96 --streams 4 --quads 0 --order $o | sed "s/^/order $o /" >> gpurun_out/r02_s26.txt 2>&1 || exit 1
done
cat gpurun_out/r02_s26.txt
