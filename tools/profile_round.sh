#!/bin/bash
# Round profile evidence for one renderer workload: the bench line, a rocprofv3
# kernel-trace summary of the same command, and (rc1pass) HBM traffic from the
# FETCH_SIZE / WRITE_SIZE counters in separate --pmc passes.
# Usage: bash tools/profile_round.sh <tag> "<bench args>" [pmc]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
TAG=$1; ARGS=$2; PMC=${3:-}
OUT=gpurun_out/prof_$TAG
rm -rf $OUT; mkdir -p $OUT
nproc > $OUT/host_nproc.txt
timeout -k 10 400 python3 bench.py $ARGS > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed"; tail -20 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
# one render stream here: with frames in flight, launches overlap and a kernel's
# trace duration is no longer its own time (bench.py's kernel_ms is single-stream)
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/trace -o trace --output-format csv -- python3 bench.py $ARGS --no-cpu-baseline --streams 1 > $OUT/prof_bench.json 2> $OUT/prof.err || { echo "prof failed"; tail -20 $OUT/prof.err; exit 1; }
find $OUT/trace -name "*kernel_stats.csv" -exec cp {} $OUT/kernel_stats.csv \;
head -5 $OUT/kernel_stats.csv
if [ -n "$PMC" ]; then
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $c -d $OUT/pmc_$c -o pmc --output-format csv -- python3 bench.py $ARGS --no-cpu-baseline --steps 5 --warmup 1 > $OUT/pmc_$c.log 2>&1 || { echo "pmc $c failed"; tail -5 $OUT/pmc_$c.log; exit 1; }
  done
  ls -R $OUT | grep counter | head
fi
