#!/usr/bin/env bash
# shadow-phase cost, walk block stats, bench tile-path checks after the pipeline refactor
set -o pipefail
mkdir -p gpurun_out/r03
timeout -k 10 240 python -u tools/phase_cost.py --configs c3,c5,c5d > gpurun_out/r03/phase_cost.log 2>&1
echo "phase rc=$?"
RT_AMD_LIB=$PWD/abl/librt_bstats.so timeout -k 10 200 python -u tools/block_stats.py --configs c3,c5 > gpurun_out/r03/block_stats.log 2>&1
echo "bstats rc=$?"
timeout -k 10 200 python -u bench.py --tiles --steps 30 --secondary= --cpu-baseline off > gpurun_out/r03/bench_tiles.json 2>&1
echo "tiles rc=$?"
timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 \
    bench.py --gpus 2 --backend gloo --same-device --steps 10 --warmup 2 --secondary= --cpu-baseline off > gpurun_out/r03/bench_gloo2.json 2>&1
echo "gloo2 rc=$?"
