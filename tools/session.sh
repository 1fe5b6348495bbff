# round 6, session s31: render streams for the driver's 20-frame command (3 = default) and 200 frames
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06_s31; mkdir -p $O
for rep in 1 2; do
  for st in 3 4 5 6; do
    for K in 20 200; do
      timeout -k 10 200 python3 bench.py --no-cpu-baseline --no-cadence --steps $K --warmup 5 --streams $st > $O/s${st}_k${K}_r$rep.json 2>$O/s${st}_k${K}_r$rep.err || exit 1
      python3 -c "import json; d=json.loads(open('$O/s${st}_k${K}_r$rep.json').read().strip().splitlines()[-1]); print('streams $st K $K', d['ms_per_step'])"
    done
  done
done
