#!/bin/bash
# One GPU session of the current round (edited per session; the committed copy is
# the last one run).  Each GPU step has its own limit; the first failure ends the call.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-r03}
timeout -k 10 400 python -u -m pytest tests/test_dos_gpu.py tests/test_ebs_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1 || { tail -30 gpurun_out/${T}_tests.log; exit 1; }
tail -2 gpurun_out/${T}_tests.log
for f in 0 1; do
  timeout -k 10 300 python bench.py --renderer dos --no-cpu-baseline --shade-flat $f > gpurun_out/${T}_dos_f$f.json 2> gpurun_out/${T}_dos_f$f.err || { tail -20 gpurun_out/${T}_dos_f$f.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/${T}_dos_f$f.json')); print('dos flat $f', d['ms_per_step'], d['roofline']['kernel_ms'], d['parity']['bit_exact'])"
done
for f in 0 1; do
  timeout -k 10 400 python bench.py --renderer ebs --no-cpu-baseline --shade-flat $f > gpurun_out/${T}_ebs_f$f.json 2> gpurun_out/${T}_ebs_f$f.err || { tail -20 gpurun_out/${T}_ebs_f$f.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/${T}_ebs_f$f.json')); print('ebs flat $f', d['ms_per_step'], d['roofline']['kernel_ms'], d['parity']['bit_exact'])"
done
timeout -k 10 300 python -u tools/overlap_probe.py --renderer dos --nranks 8 --tile 16 --frames 4 --streams 1 --out gpurun_out/${T}_split_dos.json > gpurun_out/${T}_split_dos.log 2>&1 || { tail -20 gpurun_out/${T}_split_dos.log; exit 1; }
grep '^{' gpurun_out/${T}_split_dos.log
timeout -k 10 400 python -u tools/overlap_probe.py --renderer ebs --nranks 8 --tile 16 --frames 2 --streams 1 --out gpurun_out/${T}_split_ebs.json > gpurun_out/${T}_split_ebs.log 2>&1 || { tail -20 gpurun_out/${T}_split_ebs.log; exit 1; }
grep '^{' gpurun_out/${T}_split_ebs.log
