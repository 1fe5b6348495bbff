#!/bin/bash
# Session 14: kernel-trace of bench --postpass, HEAD build vs working tree (digital filter kernels).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for L in prev new; do
  if [ "$L" = prev ]; then export CVR_LIB_OVERRIDE=ablib/prev/libcvr.so; else unset CVR_LIB_OVERRIDE; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r02_s14_$L -o trace --output-format csv -- python3 bench.py --no-cpu-baseline --postpass --steps 5 --warmup 1 > gpurun_out/r02_s14_$L.json 2> gpurun_out/r02_s14_$L.err || { tail -5 gpurun_out/r02_s14_$L.err; exit 1; }
done
unset CVR_LIB_OVERRIDE
for L in prev new; do
  f=$(find gpurun_out/r02_s14_$L -name "*kernel_stats.csv" | head -1)
  echo "== $L"; grep -i "digital\|downscale\|upscale" "$f" | cut -d, -f1-8
done
