# DOS cost probes: the same bench on variant builds (images differ by design)
cd $GRAFT_REPO_ROOT
for v in "" noborder nofetch; do
  if [ -n "$v" ]; then export CVR_LIB_OVERRIDE=ablib/$v/libcvr.so; else unset CVR_LIB_OVERRIDE; fi
  timeout -k 10 200 python3 bench.py --renderer dos --no-cpu-baseline --steps 3 --warmup 1 --streams 1 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('$v', d['ms_per_step'], d['roofline']['kernel_ms'])" || exit 1
done
