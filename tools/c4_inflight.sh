#!/usr/bin/env bash
# C4 (3840x2160, 64 spp) on one GPU: the whole frame, and rank r's 1/8 share
# (--shard r/8, no gather) one frame at a time and with two frames in flight.
# usage (GPU box, repo root): bash tools/c4_inflight.sh > gpurun_out/c4_inflight.log
export TMPDIR=/tmp
B="timeout -k 10 300 python bench.py --config c4 --secondary '' --cpu-baseline off --steps 40 --warmup 4"
eval $B | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('full', d['ms_per_step'], d['config']['kernel_ms'])" || exit 1
for r in 0 3 7; do
  for F in 1 2; do
    eval $B --shard $r/8 --inflight $F | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('share $r/8 F=$F', d['ms_per_step'], d['config']['kernel_ms'])" || exit 1
  done
done
