# round 6, session s42: 16 frames per launch: exchange protocol (16-frame groups), multi-frame tests; then PMC records and the full round
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06_s42; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_exchange_gpu.py tests/test_frames_gpu.py -x -q -rf --timeout 200 --timeout-method thread > $O/pytest_16.log 2>&1 || { tail -30 $O/pytest_16.log; exit 1; }
tail -1 $O/pytest_16.log
bash tools/pmc_session.sh rc1pass phong longray dos ebs || exit 1
bash tools/gpu_round.sh all
