#!/usr/bin/env bash
# Build librt_amd.so at a git ref into build_ab/librt_<name>.so (for same-box A/B:
# RT_AMD_LIB=build_ab/librt_<name>.so python tools/variants.py ...).
# usage: bash tools/build_ref.sh <git-ref> [name]
set -e
REF=${1:?git ref}; NAME=${2:-$REF}
ROOT=$(cd "$(dirname "$0")/.." && pwd)
WT=$(mktemp -d /tmp/rtref.XXXXXX)
git -C "$ROOT" worktree add --detach "$WT" "$REF" >/dev/null 2>&1
make -s -C "$WT/raytracingstudy_amd/csrc" ../librt_amd.so
mkdir -p "$ROOT/build_ab"
cp "$WT/raytracingstudy_amd/librt_amd.so" "$ROOT/build_ab/librt_$NAME.so"
git -C "$ROOT" worktree remove --force "$WT"
echo "built build_ab/librt_$NAME.so from $REF"
