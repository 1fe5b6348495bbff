#!/bin/bash
# A/B of two library builds in one GPU session: alternates runs of
# tools/ab_rc1pass.py on ablib/<A>/libcvr.so and the in-tree build.
# Usage: bash tools/ab_builds.sh <A name> "<variants>" [reps] [extra ab args]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
A=$1; VARS=$2; REPS=${3:-3}; EXTRA=${4:-}
mkdir -p gpurun_out
for i in $(seq 1 "$REPS"); do
  CVR_LIB_OVERRIDE=ablib/$A/libcvr.so timeout -k 10 120 python tools/ab_rc1pass.py --variants "$VARS" --rounds 3 $EXTRA > gpurun_out/abb_${A}_$i.json 2>/dev/null || exit 1
  timeout -k 10 120 python tools/ab_rc1pass.py --variants "$VARS" --rounds 3 $EXTRA > gpurun_out/abb_new_$i.json 2>/dev/null || exit 1
done
python3 - "$A" "$REPS" <<'PY'
import json, sys
a, reps = sys.argv[1], int(sys.argv[2])
for tag in (a, "new"):
    rows = {}
    for i in range(1, reps + 1):
        for r in json.load(open(f"gpurun_out/abb_{tag}_{i}.json"))["rows"]:
            rows.setdefault(r["variant"], []).append(r["median_ms"])
    print(tag, {k: sorted(v) for k, v in rows.items()})
PY
