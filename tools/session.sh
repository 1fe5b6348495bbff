#!/bin/bash
# One GPU session of the current round (edited per session; the committed copy is
# the last one run).  Each GPU step has its own limit; the first failure ends the call.
# Round 5, s21: 2 or 4 waves (tiles) per workgroup sharing one TF copy and one
# dispatch (CVR_RC1_WPG): rc1pass parity with the 4-wave build, then A/B of
# the previous library, 2 and 4 waves per workgroup against the new 1-wave build.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-r05_s21}
CVR_LIB_OVERRIDE=ablib/wpg4/libcvr.so timeout -k 10 900 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_rc1pass_gpu.py tests/test_frames_gpu.py > gpurun_out/${T}_pytest_wpg4.log 2>&1 || { tail -15 gpurun_out/${T}_pytest_wpg4.log; exit 1; }
tail -1 gpurun_out/${T}_pytest_wpg4.log
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_rc1pass_gpu.py tests/test_frames_gpu.py > gpurun_out/${T}_pytest_new.log 2>&1 || { tail -15 gpurun_out/${T}_pytest_new.log; exit 1; }
tail -1 gpurun_out/${T}_pytest_new.log
for v in prev wpg4 wpg2; do
  for spec in "static:--steps 200 --no-cadence" "orbit:--orbit --steps 200 --no-cadence"; do
    tag=${spec%%:*}; args=${spec#*:}
    timeout -k 10 900 bash tools/ab_bench.sh $v ${T}_${v}_$tag "$args" 2 > gpurun_out/${T}_ab_${v}_$tag.log 2>&1 || { tail -5 gpurun_out/${T}_ab_${v}_$tag.log; exit 1; }
    tail -2 gpurun_out/${T}_ab_${v}_$tag.log
  done
done
