#!/usr/bin/env bash
# Alternating-process A/B of two prebuilt libraries abl/librt_<a>.so and abl/librt_<b>.so
# usage: bash tools/ab_libs2.sh <a> <b> <log> [configs] [reps]
set -e -o pipefail
A=${1:?a}; B=${2:?b}; LOG=${3:?log}; CFGS=${4:-c5}; REPS=${5:-3}
export TMPDIR=/tmp
for i in $(seq "$REPS"); do
  for L in "$A" "$B"; do
    RT_AMD_LIB=$PWD/abl/librt_$L.so timeout -k 10 200 python tools/variants.py --configs "$CFGS" \
        --variants 0 --rounds 5 | sed "s/^/$L /" >> "$LOG"
  done
done
