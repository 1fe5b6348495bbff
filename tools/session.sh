# round 6, session s22: DOS scalar loads for wave-uniform coarse taps (variant builds, mip >= 2/3/4)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06_s22; mkdir -p $O
export CVR_LIB_OVERRIDE=ablib/st3/libcvr.so
timeout -k 10 400 python -u -m pytest tests/test_dos_gpu.py tests/test_fullsize_gpu.py -x -q -rf --timeout 200 --timeout-method thread -k "dos or c4" > $O/pytest_dos_st3.log 2>&1 || exit 1
tail -1 $O/pytest_dos_st3.log
for rep in 1 2; do
  for lib in cur st2 st3 st4; do
    if [ $lib = cur ]; then unset CVR_LIB_OVERRIDE; else export CVR_LIB_OVERRIDE=ablib/$lib/libcvr.so; fi
    timeout -k 10 200 python3 bench.py --renderer dos --no-cpu-baseline --steps 10 --warmup 2 > $O/dos_${lib}_r$rep.json 2>$O/dos_${lib}_r$rep.err || exit 1
    python3 -c "import json; d=json.loads(open('$O/dos_${lib}_r$rep.json').read().strip().splitlines()[-1]); print('$lib', d['ms_per_step'], d['roofline']['kernel_ms'])"
  done
done
