#!/usr/bin/env bash
set -o pipefail
mkdir -p gpurun_out/r03
RT_AMD_LIB=$PWD/abl/librt_bstats.so timeout -k 10 200 python -u tools/block_stats.py --configs c3,c5 --refill 63,16,62 > gpurun_out/r03/block_stats_refill.log 2>&1
echo "bstats rc=$?"
timeout -k 10 300 python -u tools/variants.py --configs c3,c5 --variants 0:0::63,0:0::62,0:0::56,0:0::4 --rounds 5 \
    > gpurun_out/r03/refill_ab2.log 2>&1
echo "ab rc=$?"
