#!/bin/bash
# One GPU session of the current round (edited per session; the committed copy is
# the last one run).  Each GPU step has its own limit; the first failure ends the call.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-r04_s10}
bash tools/gpu_round.sh all || exit 1
bash tools/ab_builds.sh phongfull b2o1p0q0 3 --phong > gpurun_out/${T}_ab_phong.log 2>&1 || { tail -5 gpurun_out/${T}_ab_phong.log; exit 1; }
cat gpurun_out/${T}_ab_phong.log
probe() {   # name, args...
  local name=$1; shift
  timeout -k 10 300 python -u tools/overlap_probe.py --hwq 32 --frames 96 "$@" > gpurun_out/${T}_split_$name.log 2>&1 || { tail -5 gpurun_out/${T}_split_$name.log; exit 1; }
  cat gpurun_out/${T}_split_$name.log
}
probe base --nranks 1,8 --streams 4,16
probe order0 --nranks 8 --streams 16 --tile-order 0
CVR_LIB_OVERRIDE=ablib/mf2/libcvr.so probe mf2 --nranks 1,8 --streams 4,8,16 --frames-per-launch 2
CVR_LIB_OVERRIDE=ablib/mf4/libcvr.so probe mf4 --nranks 1,8 --streams 4,8,16 --frames-per-launch 4
