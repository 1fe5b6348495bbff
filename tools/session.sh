# round 6, session s37: kernel-trace summaries of every workload on the final library (one stream)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06_s37; mkdir -p $O
export TMPDIR=/tmp
run() { n=$1; shift; cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/$n -o run -- python3 -u $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --streams 1 "$@" > $GRAFT_REPO_ROOT/$O/$n.json 2> $GRAFT_REPO_ROOT/$O/$n.err || { tail -5 $GRAFT_REPO_ROOT/$O/$n.err; exit 1; }
  cd $GRAFT_REPO_ROOT; python3 -c "
import csv
rows=list(csv.DictReader(open('$O/$n/run_kernel_stats.csv')))
for r in rows[:3]: print('$n', r['Name'][:70], r['Calls'], round(float(r['AverageNs'])/1e6,4))"; }
run rc1pass --no-cadence --steps 40 --warmup 4
run phong --no-cadence --phong --steps 40 --warmup 4
run longray --no-cadence --tf-alpha 0.02 --steps 16 --warmup 2
run dos --renderer dos --steps 5 --warmup 1
run ebs --renderer ebs --steps 2 --warmup 1
