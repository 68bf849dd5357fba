#!/usr/bin/env bash
set -o pipefail
mkdir -p gpurun_out/r03
# C5 levers: cell-table depth K (auto = 6), ticket size (opt bits 4..6: 1..4 -> 1,2,4,8 tiles)
timeout -k 10 400 python -u tools/variants.py --configs c5 --variants 0,0:0:5,0:0:7,0:16,0:32 --rounds 4 > gpurun_out/r03/c5_levers_ab.log 2>&1
echo "c5 rc=$?"
timeout -k 10 200 python -u tools/share_cost.py --config c3 --n 8 --rounds 7 > gpurun_out/r03/share_cost_head.log 2>&1
echo "share rc=$?"
