#!/bin/bash
# Build the working tree's libcvr.so with extra compiler flags into
# ablib/<name>/libcvr.so (A/B timing: CVR_LIB_OVERRIDE=ablib/<name>/libcvr.so).
# Usage: bash tools/build_variant.sh <name> "<extra flags>"
set -euo pipefail
NAME=$1; EXTRA=$2
ROOT=$(cd "$(dirname "$0")/.." && pwd)
TMP=$(mktemp -d)
mkdir -p "$TMP/cpp_volume_rendering_amd"
cp -r "$ROOT/include" "$TMP/"
cp -r "$ROOT/cpp_volume_rendering_amd/csrc" "$TMP/cpp_volume_rendering_amd/"
rm -rf "$TMP/cpp_volume_rendering_amd/csrc/build"
make -s -C "$TMP/cpp_volume_rendering_amd/csrc" -j8 EXTRA="$EXTRA" >/dev/null
mkdir -p "$ROOT/ablib/$NAME"
cp "$TMP/cpp_volume_rendering_amd/lib/libcvr.so" "$ROOT/ablib/$NAME/libcvr.so"
rm -rf "$TMP"
echo "ablib/$NAME/libcvr.so"
