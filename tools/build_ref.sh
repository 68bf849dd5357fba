#!/usr/bin/env bash
# Build librt_amd.so at a git ref into abl/librt_<name>.so (for same-box A/B:
# RT_AMD_LIB=abl/librt_<name>.so python tools/variants.py ...).
# usage: bash tools/build_ref.sh <git-ref> [name]
set -e
REF=${1:?git ref}; NAME=${2:-$REF}
ROOT=$(cd "$(dirname "$0")/.." && pwd)
WT=$(mktemp -d /tmp/rtref.XXXXXX)
git -C "$ROOT" worktree add --detach "$WT" "$REF" >/dev/null 2>&1
make -s -C "$WT/raytracingstudy_amd/csrc" ../librt_amd.so
mkdir -p "$ROOT/abl"
cp "$WT/raytracingstudy_amd/librt_amd.so" "$ROOT/abl/librt_$NAME.so"
git -C "$ROOT" worktree remove --force "$WT"
echo "built abl/librt_$NAME.so from $REF"
