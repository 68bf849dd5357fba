#!/usr/bin/env bash
# Build the library with another machine-scheduler setting into abl/librt_<name>.so
# usage: bash tools/build_sched.sh <name> "<SCHED flags>"   (e.g. "" for the compiler default)
set -e
NAME=${1:?name}; SCHEDF=${2-}
ROOT=$(cd "$(dirname "$0")/.." && pwd)
WT=$(mktemp -d /tmp/rtsched.XXXXXX)
mkdir -p "$WT/raytracingstudy_amd" "$WT/include"
cp -r "$ROOT/raytracingstudy_amd/csrc" "$WT/raytracingstudy_amd/"
cp "$ROOT"/include/*.h "$ROOT"/include/*.hpp "$WT/include/"
rm -f "$WT"/raytracingstudy_amd/csrc/*.o
make -s -C "$WT/raytracingstudy_amd/csrc" ../librt_amd.so SCHED="$SCHEDF" 2>&1 | grep -v hip-link || true
mkdir -p "$ROOT/abl"
cp "$WT/raytracingstudy_amd/librt_amd.so" "$ROOT/abl/librt_$NAME.so"
rm -rf "$WT"
echo "built abl/librt_$NAME.so with SCHED=[$SCHEDF]"
