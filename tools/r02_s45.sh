#!/bin/bash
# Session 45: per-rank cost at N = 8 (quad 10 %) with the quad variant at 8 waves (ablib/quad8) vs 7.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
export TMPDIR=/tmp
export GPU_MAX_HW_QUEUES=8
for rep in 1 2; do
  CVR_LIB_OVERRIDE=ablib/quad8/libcvr.so timeout -k 10 200 python tools/overlap_probe.py --nranks 8 --frames 96 --streams 4 --quads 10 | sed 's/^/quad8 /' || exit 1
  timeout -k 10 200 python tools/overlap_probe.py --nranks 8 --frames 96 --streams 4 --quads 0,10 | sed 's/^/tree  /' || exit 1
done
