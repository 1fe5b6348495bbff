#!/bin/bash
# Session 47: rc1pass batch K = 3 (56 VGPRs, 8 waves, no spills) vs K = 4 (64 VGPRs, 8 waves, 2 spilled).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for rep in 1 2 3; do
for args in "--batch 4" "--batch 3"; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --steps 20 --warmup 5 $args > gpurun_out/r02_s47.json 2> gpurun_out/r02_s47.err || { tail -5 gpurun_out/r02_s47.err; exit 1; }
  python3 -c "
import json; d=json.load(open('gpurun_out/r02_s47.json')); print('$args', d['ms_per_step'], d['roofline']['kernel_ms'])"
done
done
for args in "--batch 4" "--batch 3"; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --tf-alpha 0.02 --steps 20 --warmup 5 $args > gpurun_out/r02_s47.json 2> gpurun_out/r02_s47.err || { tail -5 gpurun_out/r02_s47.err; exit 1; }
  python3 -c "
import json; d=json.load(open('gpurun_out/r02_s47.json')); print('long $args', d['ms_per_step'], d['roofline']['kernel_ms'])"
done
