#!/bin/bash
# A/B of two library builds through bench.py (kernel_ms of the renderer's march):
# alternates ablib/<A>/libcvr.so and the in-tree build, REPS times each.
# Usage: bash tools/ab_bench.sh <A> <tag> "<bench args>" [reps]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
A=$1; TAG=$2; ARGS=$3; REPS=${4:-2}
mkdir -p gpurun_out
for i in $(seq 1 "$REPS"); do
  for L in "$A" new; do
    if [ "$L" = new ]; then unset CVR_LIB_OVERRIDE; else export CVR_LIB_OVERRIDE=ablib/$A/libcvr.so; fi
    timeout -k 10 300 python bench.py --no-cpu-baseline $ARGS > gpurun_out/abx_${TAG}_${L}_$i.json 2> gpurun_out/abx_${TAG}_${L}_$i.err || { unset CVR_LIB_OVERRIDE; tail -5 gpurun_out/abx_${TAG}_${L}_$i.err; exit 1; }
    unset CVR_LIB_OVERRIDE
  done
done
python3 - "$A" "$TAG" "$REPS" <<'PY'
import json, sys
a, tag, reps = sys.argv[1], sys.argv[2], int(sys.argv[3])
for L in (a, "new"):
    ks, ms, ex = [], [], []
    for i in range(1, reps + 1):
        d = json.load(open(f"gpurun_out/abx_{tag}_{L}_{i}.json"))
        ks.append(d["roofline"]["kernel_ms"]); ms.append(d["ms_per_step"])
        ex.append(d.get("parity", {}).get("bit_exact"))
    print(tag, L, "kernel_ms", ks, "ms_per_step", ms, "bit_exact", ex)
PY
