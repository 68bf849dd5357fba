#!/usr/bin/env bash
# Build the library of a git revision into abl/librt_<name>.so, for a
# two-build A/B on one box (RT_AMD_LIB=abl/librt_<name>.so ...).
# usage: bash tools/build_rev.sh <name> [<rev>=HEAD]
set -e
NAME=${1:?name}; REV=${2:-HEAD}
ROOT=$(cd "$(dirname "$0")/.." && pwd)
WT=$(mktemp -d /tmp/rtrev.XXXXXX)
git -C "$ROOT" archive "$REV" raytracingstudy_amd/csrc include | tar -x -C "$WT"
make -s -C "$WT/raytracingstudy_amd/csrc" ../librt_amd.so 2>&1 | grep -v hip-link || true
mkdir -p "$ROOT/abl"
cp "$WT/raytracingstudy_amd/librt_amd.so" "$ROOT/abl/librt_$NAME.so"
rm -rf "$WT"
echo "built abl/librt_$NAME.so from $REV"
