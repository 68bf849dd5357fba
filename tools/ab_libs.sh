#!/usr/bin/env bash
# A/B of several build_ab/librt_<name>.so builds, interleaved (c3, c5)
set -e -o pipefail
export TMPDIR=/tmp
LOG=gpurun_out/leaf_chunk_ab.log
mkdir -p gpurun_out
for i in 1 2 3; do
  for L in base ck3 ck4; do
    RT_AMD_LIB=build_ab/librt_$L.so timeout -k 10 200 python tools/variants.py --configs c3,c5 --variants 0 --rounds 5 | sed "s/^/$L /" >> $LOG
  done
done
