#!/usr/bin/env bash
# A/B of the two-level wave queue (default build) against static XCD ranges
# with threshold stealing (abl/librt_static.so, RT_STEAL_FACTOR = 0 always,
# 2, 1000 ~never): variants.py on C3/C5d/C5 and share_cost.py, 2 reps.
set -o pipefail
OUT=${1:-gpurun_out/queue_ab}
mkdir -p "$OUT"
for rep in 1 2; do
  for v in twolevel:0 static:0 static:2 static:1000; do
    L=${v%%:*}; F=${v#*:}
    RT_STEAL_FACTOR=$F RT_AMD_LIB=abl/librt_$L.so timeout -k 10 300 python tools/variants.py \
        --configs c3,c5d,c5 --variants 0 --rounds 3 2>/dev/null | sed "s/^/$L:$F /" >> "$OUT/var.log" || exit 1
    RT_STEAL_FACTOR=$F RT_AMD_LIB=abl/librt_$L.so timeout -k 10 100 python tools/share_cost.py 2>/dev/null \
        | sed "s/^/$L:$F /" >> "$OUT/share.log" || exit 1
  done
done
