# round 6, session s19: DOS shader force-inlined; 2x2x2-brick pyramid (variant build) vs x-fastest; filter_bits 8
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06_s19; mkdir -p $O
export CVR_LIB_OVERRIDE=ablib/brick/libcvr.so
timeout -k 10 300 python -u -m pytest tests/test_dos_gpu.py -x -q -rf --timeout 120 --timeout-method thread -k "bricked" > $O/pytest_brick.log 2>&1
tail -2 $O/pytest_brick.log
unset CVR_LIB_OVERRIDE
timeout -k 10 300 python -u -m pytest tests/test_dos_gpu.py -x -q -rf --timeout 120 --timeout-method thread -k "not bricked" > $O/pytest_dos.log 2>&1 || exit 1
tail -1 $O/pytest_dos.log
for rep in 1 2 3; do
  for lib in cur brick; do
    if [ $lib = cur ]; then unset CVR_LIB_OVERRIDE; L=0; else export CVR_LIB_OVERRIDE=ablib/brick/libcvr.so; L=1; fi
    timeout -k 10 200 python3 bench.py --renderer dos --no-cpu-baseline --steps 10 --warmup 2 --opt ext_layout=$L > $O/dos_${lib}_r$rep.json 2>$O/dos_${lib}_r$rep.err || exit 1
    python3 -c "import json; d=json.loads(open('$O/dos_${lib}_r$rep.json').read().strip().splitlines()[-1]); print('$lib', d['ms_per_step'], d['config']['lib_sha16'])"
  done
done
for lib in r05 cur; do
  if [ $lib = cur ]; then unset CVR_LIB_OVERRIDE; else export CVR_LIB_OVERRIDE=ablib/r05/libcvr.so; fi
  timeout -k 10 200 python3 bench.py --renderer dos --no-cpu-baseline --steps 5 --warmup 1 --opt filter_bits=8 > $O/dos_fb8_${lib}.json 2>$O/dos_fb8_${lib}.err || exit 1
  python3 -c "import json; d=json.loads(open('$O/dos_fb8_${lib}.json').read().strip().splitlines()[-1]); print('fb8 $lib', d['ms_per_step'], d['config']['lib_sha16'])"
done
