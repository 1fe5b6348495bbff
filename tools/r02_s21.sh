#!/bin/bash
# Session 21: round-end check of the tree: whole GPU suite, smoke, driver-command bench,
# kernel-trace summary of the same command, post-pass bench.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r02_s21_tests.log 2>&1 || { tail -30 gpurun_out/r02_s21_tests.log; exit 1; }
tail -1 gpurun_out/r02_s21_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r02_s21_smoke.log 2>&1 && tail -1 gpurun_out/r02_s21_smoke.log || exit 1
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r02_s21_bench.json 2> gpurun_out/r02_s21_bench.err || { tail -20 gpurun_out/r02_s21_bench.err; exit 1; }
cat gpurun_out/r02_s21_bench.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/r02_s21_prof -o trace --output-format csv -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --streams 1 --no-cpu-baseline > gpurun_out/r02_s21_prof_bench.json 2> gpurun_out/r02_s21_prof.err || { tail -20 gpurun_out/r02_s21_prof.err; exit 1; }
find gpurun_out/r02_s21_prof -name "*kernel_stats.csv" | head -2
