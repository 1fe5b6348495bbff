#!/bin/bash
# A/B session: ablib/<A> vs the in-tree build on the headline and long-ray frames.
# Usage: bash tools/ab_session.sh <A> [variants]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
A=$1; VARS=${2:-b4o1p5q0}
mkdir -p gpurun_out
bash tools/ab_builds.sh "$A" "$VARS" 3 "--frames 50" || exit 1
bash tools/ab_builds.sh "$A" "$VARS" 2 "--tf-alpha 0.02 --frames 10" || exit 1
