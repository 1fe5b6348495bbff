# round 6, session s38: DOS under native_exp (tolerance mode): gate tests and A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06_s38; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_tolerance_gpu.py tests/test_dos_gpu.py -x -q -rf --timeout 200 --timeout-method thread > $O/pytest_tol_dos.log 2>&1 || { tail -30 $O/pytest_tol_dos.log; exit 1; }
tail -1 $O/pytest_tol_dos.log
for rep in 1 2 3; do
  for nx in 0 1; do
    timeout -k 10 200 python3 bench.py --renderer dos --no-cpu-baseline --steps 10 --warmup 2 --opt native_exp=$nx > $O/dos_nx${nx}_r$rep.json 2>$O/dos_nx${nx}_r$rep.err || exit 1
    python3 -c "import json; d=json.loads(open('$O/dos_nx${nx}_r$rep.json').read().strip().splitlines()[-1]); print('dos native_exp $nx', d['ms_per_step'], d['roofline']['kernel_ms'])"
  done
done
