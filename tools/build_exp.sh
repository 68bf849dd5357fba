#!/usr/bin/env bash
# Build the working tree's library into abl/librt_<name>.so for an A/B
# (tools/ab_libs.sh), with extra device flags (an experiment's -D switch)
# and optional make variables (e.g. SCHED="" for the compiler's default
# machine scheduler).  For a git revision use tools/build_rev.sh.
# usage: bash tools/build_exp.sh <name> ["<extra devflags>"] ["<make VAR=value ...>"]
set -e
NAME=${1:?name}; FLAGS=${2:-}; MAKEVARS=${3:-}
ROOT=$(cd "$(dirname "$0")/.." && pwd)
WT=$(mktemp -d /tmp/rtexp.XXXXXX)
mkdir -p "$WT/raytracingstudy_amd"
cp -r "$ROOT/raytracingstudy_amd/csrc" "$WT/raytracingstudy_amd/"
cp -r "$ROOT/include" "$WT/"
rm -f "$WT"/raytracingstudy_amd/csrc/*.o
# shellcheck disable=SC2086
make -s -C "$WT/raytracingstudy_amd/csrc" ../librt_amd.so EXTRA_DEVFLAGS="$FLAGS" $MAKEVARS 2>&1 \
    | grep -v hip-link || true
mkdir -p "$ROOT/abl"
cp "$WT/raytracingstudy_amd/librt_amd.so" "$ROOT/abl/librt_$NAME.so"
rm -rf "$WT"
echo "built abl/librt_$NAME.so (devflags: $FLAGS; make: $MAKEVARS)"
