#!/bin/bash
# Session 4: arithmetic self-test (rcp/sqrt/pow) + whole GPU suite; branch-free
# pow + exact fast normalize A/B (ablib/prev = before both) on Phong, DOS, iso.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r02_s4_gpu_all.log 2>&1 || { tail -30 gpurun_out/r02_s4_gpu_all.log; exit 1; }
tail -1 gpurun_out/r02_s4_gpu_all.log
bash tools/ab_builds.sh prev "b2o1p5q0" 3 "--phong --frames 30" || exit 1
bash tools/ab_bench.sh prev dos "--renderer dos --steps 5 --warmup 1" 2 || exit 1
bash tools/ab_bench.sh prev iso "--renderer iso --phong --steps 10 --warmup 2" 2 || exit 1
