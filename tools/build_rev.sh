#!/bin/bash
# Build libcvr.so of git revision $1 into ablib/$2/libcvr.so (for A/B timing of
# two builds: CVR_LIB_OVERRIDE=ablib/$2/libcvr.so python tools/ab_rc1pass.py ...).
set -euo pipefail
REV=$1; NAME=$2
ROOT=$(cd "$(dirname "$0")/.." && pwd)
TMP=$(mktemp -d)
git -C "$ROOT" archive "$REV" include cpp_volume_rendering_amd/csrc | tar -x -C "$TMP"
make -s -C "$TMP/cpp_volume_rendering_amd/csrc" -j8 >/dev/null
mkdir -p "$ROOT/ablib/$NAME"
cp "$TMP/cpp_volume_rendering_amd/lib/libcvr.so" "$ROOT/ablib/$NAME/libcvr.so"
rm -rf "$TMP"
echo "ablib/$NAME/libcvr.so"
