#!/usr/bin/env bash
# A/B of several builds on the multi-GPU share and the full frame
# (tools/share_cost.py), interleaved per repetition.  Run on the GPU box.
# usage: bash tools/ab_share.sh <log> <reps> <name>...   (abl/librt_<name>.so)
set -e -o pipefail
LOG=${1:?log}; REPS=${2:?reps}; shift 2
mkdir -p "$(dirname "$LOG")"
for i in $(seq "$REPS"); do
  for L in "$@"; do
    RT_AMD_LIB=abl/librt_$L.so timeout -k 10 120 python tools/share_cost.py 2>/dev/null \
        | sed "s/^/$L /" >> "$LOG"
  done
done
