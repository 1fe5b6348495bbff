# round 6, session s35: flat shading with 2 / 4 / 8 waves (consecutive chunks) per workgroup, DOS and EBS
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06_s35; mkdir -p $O
export CVR_LIB_OVERRIDE=ablib/wpb4/libcvr.so
timeout -k 10 400 python -u -m pytest tests/test_dos_gpu.py tests/test_ebs_gpu.py -x -q -rf --timeout 200 --timeout-method thread > $O/pytest_wpb4.log 2>&1 || { tail -30 $O/pytest_wpb4.log; exit 1; }
tail -1 $O/pytest_wpb4.log
for rep in 1 2; do
  for lib in cur wpb2 wpb4 wpb8; do
    if [ $lib = cur ]; then unset CVR_LIB_OVERRIDE; else export CVR_LIB_OVERRIDE=ablib/$lib/libcvr.so; fi
    timeout -k 10 200 python3 bench.py --renderer dos --no-cpu-baseline --steps 10 --warmup 2 > $O/dos_${lib}_r$rep.json 2>$O/dos_${lib}_r$rep.err || exit 1
    python3 -c "import json; d=json.loads(open('$O/dos_${lib}_r$rep.json').read().strip().splitlines()[-1]); print('dos $lib', d['ms_per_step'], d['roofline']['kernel_ms'])"
  done
done
for lib in cur wpb4; do
  if [ $lib = cur ]; then unset CVR_LIB_OVERRIDE; else export CVR_LIB_OVERRIDE=ablib/$lib/libcvr.so; fi
  timeout -k 10 300 python3 bench.py --renderer ebs --no-cpu-baseline --steps 3 --warmup 1 > $O/ebs_${lib}.json 2>$O/ebs_${lib}.err || exit 1
  python3 -c "import json; d=json.loads(open('$O/ebs_${lib}.json').read().strip().splitlines()[-1]); print('ebs $lib', d['ms_per_step'], d['roofline']['kernel_ms'])"
done
