#!/usr/bin/env bash
# A/B of the wave queue's slot-size threshold (RT_SLOT_SB_MIN builds
# abl/librt_t<N>.so): 1/8 and 1/4 C3 shares with the full frame
# (tools/share_cost.py) and the C4 4- and 8-way shares (tools/shard_balance.py).
set -o pipefail
OUT=${1:?out}; shift
mkdir -p "$OUT"
for rep in 1 2; do
  for L in "$@"; do
    for n in 8 4; do
      RT_AMD_LIB=abl/librt_$L.so timeout -k 10 100 python tools/share_cost.py --n $n 2>/dev/null \
          | sed "s/^/$L /" >> "$OUT/share.log" || exit 1
    done
  done
done
for L in "$@"; do
  RT_AMD_LIB=abl/librt_$L.so timeout -k 10 200 python tools/shard_balance.py --config c4 --ranks 4,8 2>/dev/null \
      | tail -1 | sed "s/^/$L /" >> "$OUT/c4.log" || exit 1
done
