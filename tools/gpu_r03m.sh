#!/usr/bin/env bash
# Leaf-capacity A/B (interleaved in one process per config): cap 8 (default) vs 10, 12, 16, 24
set -o pipefail
mkdir -p gpurun_out/r03
timeout -k 10 240 python -u tools/variants.py --configs c3 --variants 0:0::8,0:0::10,0:0::12,0:0::16,0:0::24 --rounds 9 > gpurun_out/r03/cap_ab2.log 2>&1 &&
timeout -k 10 300 python -u tools/variants.py --configs c5,c5d --variants 0:0::8,0:0::12,0:0::16 --rounds 5 >> gpurun_out/r03/cap_ab2.log 2>&1
rc=$?; cat gpurun_out/r03/cap_ab2.log; exit $rc
