# round 6, session s33: the driver's command on the final library with its PMC records installed
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06_s33; mkdir -p $O
timeout -k 10 400 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
python3 -c "import json; d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1]); r=d['roofline']; print(d['ms_per_step'], d['value'], r['bound'], r['frac'], r['traffic'], d['config']['lib_sha16'])"
