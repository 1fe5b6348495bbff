#!/bin/bash
# Kernel-trace of bench --postpass for several library builds (ablib/<name> or "new"):
# mean duration of the post-pass kernels per build.  Usage: bash tools/pp_probe.sh tag lib1 lib2 ...
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=$1; shift
for L in "$@"; do
  if [ "$L" = new ]; then unset CVR_LIB_OVERRIDE; else export CVR_LIB_OVERRIDE=ablib/$L/libcvr.so; fi
  timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/pp_${TAG}_$L -o trace --output-format csv -- python3 bench.py --no-cpu-baseline --postpass --steps 5 --warmup 1 > gpurun_out/pp_${TAG}_$L.json 2> gpurun_out/pp_${TAG}_$L.err || { tail -5 gpurun_out/pp_${TAG}_$L.err; exit 1; }
done
unset CVR_LIB_OVERRIDE
python3 - "$TAG" "$@" <<'PY'
import csv, glob, sys, collections
tag, libs = sys.argv[1], sys.argv[2:]
for L in libs:
    f = glob.glob(f"gpurun_out/pp_{tag}_{L}/**/*kernel_trace.csv", recursive=True)[0]
    d = collections.defaultdict(list)
    for r in csv.DictReader(open(f)):
        n = r["Kernel_Name"]
        if "digital" in n or "scale" in n or "multisample" in n:
            key = n.replace("cvr::(anonymous namespace)::", "").split("(")[0] + f" g{r['Grid_Size_X']}"
            d[key].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000)
    print("==", L)
    for k, v in d.items():
        print(f"  {k:70s} n={len(v):3d} mean {sum(v)/len(v):8.1f} us")
PY
