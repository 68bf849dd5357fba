#!/usr/bin/env bash
# Build the working tree's library with extra device flags (e.g. an
# experiment's -D switch) into abl/librt_<name>.so, for tools/ab_libs2.sh.
# usage: bash tools/build_exp.sh <name> ["<extra devflags>"]
set -e
NAME=${1:?name}; FLAGS=${2:-}
ROOT=$(cd "$(dirname "$0")/.." && pwd)
WT=$(mktemp -d /tmp/rtexp.XXXXXX)
mkdir -p "$WT/raytracingstudy_amd"
cp -r "$ROOT/raytracingstudy_amd/csrc" "$WT/raytracingstudy_amd/"
cp -r "$ROOT/include" "$WT/"
rm -f "$WT"/raytracingstudy_amd/csrc/*.o
make -s -C "$WT/raytracingstudy_amd/csrc" ../librt_amd.so EXTRA_DEVFLAGS="$FLAGS" 2>&1 | grep -v hip-link || true
mkdir -p "$ROOT/abl"
cp "$WT/raytracingstudy_amd/librt_amd.so" "$ROOT/abl/librt_$NAME.so"
rm -rf "$WT"
echo "built abl/librt_$NAME.so ($FLAGS)"
