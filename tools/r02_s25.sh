#!/bin/bash
# Session 25: per-rank frame cost of the N-way screen split on one GPU, streams x quad share.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
export TMPDIR=/tmp
export GPU_MAX_HW_QUEUES=8
for n in 8 4 2; do
  timeout -k 10 200 python tools/overlap_probe.py --nranks $n --frames 96 --streams 1,4,6,8 --quads 0,10 >> gpurun_out/r02_s25_overlap.txt 2>&1 || exit 1
done
cat gpurun_out/r02_s25_overlap.txt
