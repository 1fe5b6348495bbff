#!/bin/bash
# Session 3: arithmetic self-test + whole GPU suite; exact fast normalize A/B
# (ablib/prev = before) on Phong, DOS, EBS 512^3 and iso.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_selftest_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r02_s3_gpu_all.log 2>&1 || { tail -30 gpurun_out/r02_s3_gpu_all.log; exit 1; }
tail -1 gpurun_out/r02_s3_gpu_all.log
bash tools/ab_builds.sh prev "b2o1p5q0" 3 "--phong --frames 30" || exit 1
bash tools/ab_bench.sh prev dos "--renderer dos --steps 5 --warmup 1" 2 || exit 1
bash tools/ab_bench.sh prev ebs512 "--renderer ebs --size 512 --steps 3 --warmup 1" 2 || exit 1
bash tools/ab_bench.sh prev iso "--renderer iso --steps 10 --warmup 2" 2 || exit 1
