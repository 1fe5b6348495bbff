#!/bin/bash
# Session 35: rc1pass launch order (1 LPT vs 2 interleaved) for EA and Phong.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for rep in 1 2; do
for args in "--tile-order 1" "--tile-order 2" "--phong --tile-order 1" "--phong --tile-order 2"; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --steps 100 --warmup 20 $args > gpurun_out/r02_s35.json 2> gpurun_out/r02_s35.err || { tail -5 gpurun_out/r02_s35.err; exit 1; }
  python3 -c "
import json; d=json.load(open('gpurun_out/r02_s35.json')); print('$args', d['ms_per_step'], d['roofline']['kernel_ms'])"
done
done
