#!/usr/bin/env bash
# Build the library with extra device compiler flags into abl/librt_<name>.so
# (same-box A/B of code generation: RT_AMD_LIB=abl/librt_<name>.so ...).
# usage: bash tools/build_flags.sh <name> "<extra device flags>"
set -e
NAME=${1:?name}; FLAGS=${2:-}
ROOT=$(cd "$(dirname "$0")/.." && pwd)
WT=$(mktemp -d /tmp/rtflags.XXXXXX)
mkdir -p "$WT/raytracingstudy_amd" "$WT/include"
cp -r "$ROOT/raytracingstudy_amd/csrc" "$WT/raytracingstudy_amd/"
cp "$ROOT"/include/*.h "$ROOT"/include/*.hpp "$WT/include/"
rm -f "$WT"/raytracingstudy_amd/csrc/*.o
make -s -C "$WT/raytracingstudy_amd/csrc" ../librt_amd.so EXTRA_DEVFLAGS="$FLAGS"
mkdir -p "$ROOT/abl"
cp "$WT/raytracingstudy_amd/librt_amd.so" "$ROOT/abl/librt_$NAME.so"
rm -rf "$WT"
echo "built abl/librt_$NAME.so with [$FLAGS]"
