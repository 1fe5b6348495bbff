# round 6, session s14: full GPU suite; the N = 8 share at 8 frames per launch
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06_s14; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -rf --durations=15 --timeout 300 --timeout-method thread > $O/pytest_gpu_all.log 2>&1 || exit 1
for rep in 1 2; do
  for st in 4 8; do
    timeout -k 10 200 python -u tools/exchange_probe.py --part A --ranks 8 --flp 8 --streams $st --sets 32 --frames 192 > $O/probeA_flp8_s${st}_r$rep.jsonl 2>&1 || exit 1
  done
done
export TMPDIR=/tmp
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/prof -o run -- python3 -u $GRAFT_REPO_ROOT/tools/exchange_probe.py --part B --ranks 8 --flp 8 --out $GRAFT_REPO_ROOT/$O/probeB_flp8.json > $GRAFT_REPO_ROOT/$O/probeB_flp8.log 2>&1 || exit 1
