#!/bin/bash
# Round-2 bench session: DOS parity after the tap counter, the driver's headline
# command, the orbit line and the DOS line.  Each GPU step has its own limit.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_dos_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r02_dos_tests.log 2>&1 || { tail -20 gpurun_out/r02_dos_tests.log; exit 1; }
tail -1 gpurun_out/r02_dos_tests.log
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r02_bench_driver.json 2> gpurun_out/r02_bench_driver.err || { tail -20 gpurun_out/r02_bench_driver.err; exit 1; }
cat gpurun_out/r02_bench_driver.json
timeout -k 10 300 python bench.py --orbit --steps 220 --no-cpu-baseline > gpurun_out/r02_bench_orbit.json 2> gpurun_out/r02_bench_orbit.err || { tail -20 gpurun_out/r02_bench_orbit.err; exit 1; }
cat gpurun_out/r02_bench_orbit.json
timeout -k 10 400 python bench.py --renderer dos --no-cpu-baseline > gpurun_out/r02_bench_dos.json 2> gpurun_out/r02_bench_dos.err || { tail -20 gpurun_out/r02_bench_dos.err; exit 1; }
cat gpurun_out/r02_bench_dos.json
