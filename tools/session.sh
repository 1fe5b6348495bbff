# round 6, session s44: a 16-frame burst (the driver's short runs) of the N-way shares at 4 / 8 / 16 frames per launch
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06_s44; mkdir -p $O
for flp in 4 8 16; do
  timeout -k 10 300 python -u tools/exchange_probe.py --part A --ranks 2,4,8 --flp $flp --streams 4 --sets 16 --frames 16 > $O/burst_flp${flp}.jsonl 2>&1 || exit 1
  python3 -c "
import json
for l in open('$O/burst_flp${flp}.jsonl'):
    l=l.strip()
    if not l.startswith('{'): continue
    d=json.loads(l)
    if 'ms_per_frame' in d and d['encode']: print('burst16 flp $flp', d['nranks'], d['render_ranks'], d['ms_per_frame'])"
done
