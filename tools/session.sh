# round 6, session s36: DOS cost probes: the border attenuation's exp as v_exp_f32, and no border at all (images differ)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06_s36; mkdir -p $O
for rep in 1 2; do
  for lib in cur nexp noborder; do
    if [ $lib = cur ]; then unset CVR_LIB_OVERRIDE; else export CVR_LIB_OVERRIDE=ablib/$lib/libcvr.so; fi
    timeout -k 10 200 python3 bench.py --renderer dos --no-cpu-baseline --steps 10 --warmup 2 > $O/dos_${lib}_r$rep.json 2>$O/dos_${lib}_r$rep.err || exit 1
    python3 -c "import json; d=json.loads(open('$O/dos_${lib}_r$rep.json').read().strip().splitlines()[-1]); print('dos $lib', d['ms_per_step'], d['roofline']['kernel_ms'])"
  done
done
