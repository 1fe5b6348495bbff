set -o pipefail
for cfg in "k16:--keep 16" "k64:--keep 64" "k256:--keep 256" "all:" "q5k16:--quad 5 --keep 64"; do
  tag=${cfg%%:*}; args=${cfg#*:}
  timeout -k 10 120 python tools/tile_timeline.py --tag $tag $args > gpurun_out/tl_$tag.json 2>/dev/null || exit 1
done
python3 - <<'PY'
import json
for t in ["k16","k64","k256","all","q5k16"]:
    d=json.load(open("gpurun_out/tl_%s.json"%t))
    print(t, d["tiles"], d["span_us"], d["tile_dur_us"], d["us_per_iteration"], [(x["dur_us"],x["iters"]) for x in d["longest_tiles"][:4]])
PY
