#!/bin/bash
# Session 36: shaded marches, scattered tile order (ablib/shhash) vs interleaved (tree).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
export TMPDIR=/tmp
bash tools/ab_bench.sh shhash dos "--renderer dos --steps 5 --warmup 1" 2 || exit 1
bash tools/ab_bench.sh shhash ebs512 "--renderer ebs --size 512 --steps 5 --warmup 1" 2 || exit 1
