# round 6, session s34: exchange protocol at tile 32 and at 8-frame groups (the N >= 8 default)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06_s34; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_exchange_gpu.py -x -v -rf --timeout 200 --timeout-method thread > $O/pytest_exchange.log 2>&1 || { tail -30 $O/pytest_exchange.log; exit 1; }
grep -c PASSED $O/pytest_exchange.log; tail -1 $O/pytest_exchange.log
