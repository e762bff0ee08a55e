#!/bin/bash
# Build an A/B arm of the native libraries with some sources taken from a git revision:
#   tools/ab_build_rev.sh OUT_DIR REV "file1.hip file2.hip ..."
# (the rest of the package as in the tree); puts libmlgate.so / libmlgate_torch.so in OUT_DIR
# for tools/ab_run.py --lib-dir.
set -eu
ROOT="$(cd "$(dirname "$0")/.." && pwd)"
OUT="$(mkdir -p "$1" && cd "$1" && pwd)"; REV="$2"; FILES="$3"
TMP="$(mktemp -d /tmp/abr_XXXX)"
mkdir -p "$TMP/pkg/mlgate"
cp -a "$ROOT/include" "$TMP/include"
cp -a "$ROOT/multi-level-indoor-slam_amd/csrc" "$TMP/pkg/csrc"
for f in $FILES; do git -C "$ROOT" show "$REV:multi-level-indoor-slam_amd/csrc/$f" > "$TMP/pkg/csrc/$f"; done
make -s -C "$TMP/pkg/csrc" -j8 > "$TMP/build.log" 2>&1 || { tail -20 "$TMP/build.log"; exit 1; }
cp "$TMP/pkg/mlgate/libmlgate.so" "$TMP/pkg/mlgate/libmlgate_torch.so" "$OUT/"
rm -rf "$TMP"
echo "built $OUT ($FILES at $REV)"
