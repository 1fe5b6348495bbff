# round 6, session s28: final bench lines of lib a3ef5d07 (PMC records installed): every workload
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06_s28; mkdir -p $O
run() { n=$1; shift; timeout -k 10 300 python3 bench.py "$@" > $O/$n.json 2>$O/$n.err || { tail -5 $O/$n.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/$n.json').read().strip().splitlines()[-1]); r=d['roofline']; print('$n', d['ms_per_step'], d['value'], r.get('bound'), r.get('frac'), r.get('traffic'))"; }
run driver --gpus 1 --steps 20 --warmup 5
run driver200 --no-cpu-baseline --no-cadence --steps 200 --warmup 10
run orbit --no-cpu-baseline --no-cadence --orbit --steps 200 --warmup 10
run phong --no-cpu-baseline --no-cadence --phong --steps 100 --warmup 10
run longray --no-cpu-baseline --no-cadence --tf-alpha 0.02 --steps 40 --warmup 4
run dos --renderer dos --steps 10 --warmup 2
run ebs --renderer ebs --steps 4 --warmup 1
