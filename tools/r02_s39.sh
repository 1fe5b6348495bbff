#!/bin/bash
# Session 39: DOS at 3 waves/SIMD in tree: parity (incl. full size) + bench line + kernel-trace summary.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_dos_gpu.py tests/test_fullsize_gpu.py -m gpu -x -q -k "dos or c4" --timeout 300 --timeout-method thread > gpurun_out/r02_s39_tests.log 2>&1 || { tail -30 gpurun_out/r02_s39_tests.log; exit 1; }
tail -1 gpurun_out/r02_s39_tests.log
timeout -k 10 400 python bench.py --renderer dos > gpurun_out/r02_s39_dos.json 2> gpurun_out/r02_s39_dos.err || { tail -5 gpurun_out/r02_s39_dos.err; exit 1; }
python3 -c "
import json; d=json.load(open('gpurun_out/r02_s39_dos.json')); print(d['ms_per_step'], d['roofline']['kernel_ms'], d['roofline']['frac'], d.get('parity',{}).get('bit_exact'))"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/r02_s39_prof -o trace --output-format csv -- python3 bench.py --renderer dos --no-cpu-baseline --streams 1 --steps 5 --warmup 1 > gpurun_out/r02_s39_prof.json 2> gpurun_out/r02_s39_prof.err || { tail -5 gpurun_out/r02_s39_prof.err; exit 1; }
grep shaded_march gpurun_out/r02_s39_prof/trace_kernel_stats.csv | cut -c1-200
