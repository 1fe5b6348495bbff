#!/bin/bash
# Phong cost probes: ablib/p_{NOLOAD,NOMATH,BOTH} (gradient loads / shading math
# removed, images wrong by design) vs the in-tree build, plus the EA frame.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for P in NOLOAD NOMATH BOTH; do
  bash tools/ab_builds.sh p_$P "b2o1p5q0,b4o1p5q0" 2 "--phong --frames 30" > gpurun_out/probe_$P.txt || exit 1
  cat gpurun_out/probe_$P.txt
done
timeout -k 10 120 python tools/ab_rc1pass.py --variants b2o1p5q0,b4o1p5q0 --rounds 3 --frames 30 > gpurun_out/probe_EA.json || exit 1
python3 -c "import json; print('EA', [(r['variant'], r['median_ms']) for r in json.load(open('gpurun_out/probe_EA.json'))['rows']])"
