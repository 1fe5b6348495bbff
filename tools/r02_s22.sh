#!/bin/bash
# Session 22: frames in flight (render streams) 2/4/6/8 on the driver command.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for rep in 1 2; do
for S in 4 6 8 2; do
  timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --streams $S --no-cpu-baseline > gpurun_out/r02_s22_s${S}_$rep.json 2> gpurun_out/r02_s22_s$S.err || { tail -5 gpurun_out/r02_s22_s$S.err; exit 1; }
  python3 -c "
import json; d=json.load(open('gpurun_out/r02_s22_s${S}_$rep.json')); print($S, d['ms_per_step'], d['roofline']['kernel_ms'], d['value'])"
done
done
