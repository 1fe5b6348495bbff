# round 6, session s40: the driver's command and the DOS line with the final PMC records installed
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06_s40; mkdir -p $O
timeout -k 10 400 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
python3 -c "import json; d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1]); r=d['roofline']; print(d['ms_per_step'], d['value'], r['bound'], r['frac'], r['traffic'], d['config']['lib_sha16'])"
timeout -k 10 400 python3 bench.py --renderer dos --steps 10 --warmup 2 > $O/dos.json 2> $O/dos.err || { tail -5 $O/dos.err; exit 1; }
python3 -c "import json; d=json.loads(open('$O/dos.json').read().strip().splitlines()[-1]); r=d['roofline']; print(d['ms_per_step'], d['value'], r['bound'], r['frac'], r['traffic'])"
