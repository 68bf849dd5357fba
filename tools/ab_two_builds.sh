#!/usr/bin/env bash
# Two-build A/B on the GPU box: the in-tree library against abl/librt_<base>.so
# (tools/build_rev.sh), in alternating processes, each timing plain frames
# with tools/variants.py.  usage: bash tools/ab_two_builds.sh <base> <log> [configs] [variant] [reps]
set -e -o pipefail
BASE=${1:?base}; LOG=${2:?log}; CFGS=${3:-c3,c5}; VAR=${4:-0}; REPS=${5:-2}
export TMPDIR=/tmp
for i in $(seq "$REPS"); do
  RT_AMD_LIB=abl/librt_$BASE.so timeout -k 10 200 python tools/variants.py --configs "$CFGS" \
      --variants "$VAR" --rounds 5 | sed "s/^/$BASE /" >> "$LOG"
  timeout -k 10 200 python tools/variants.py --configs "$CFGS" --variants "$VAR" --rounds 5 \
      | sed "s/^/new /" >> "$LOG"
done
