# round 6, session s30: group context error paths (member creation failure, host multi-frame)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06_s30; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_exchange_gpu.py -x -q -rf --timeout 200 --timeout-method thread > $O/pytest_exchange.log 2>&1 || { tail -30 $O/pytest_exchange.log; exit 1; }
tail -1 $O/pytest_exchange.log
