#!/bin/bash
# Session 28: isodfs speculative multi-block skip: iso parity, A/B vs HEAD on ML and blobs.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
export TMPDIR=/tmp
true
true
bash tools/ab_bench.sh prev isodfs "--renderer isodfs --steps 20 --warmup 5" 2 || exit 1
bash tools/ab_bench.sh prev isodfsb "--renderer isodfs --field blobs --steps 20 --warmup 5" 2 || exit 1
