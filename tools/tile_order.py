#!/usr/bin/env python3
"""Does a longest-first tile order shorten an N-way share?  (diagnostic)

    RT_AMD_LIB=abl/librt_timeline.so python tools/tile_order.py --n 8 --save order.json
    python tools/tile_order.py --n 8 --load order.json

With the timeline build: renders rank 0's share, sums the measured unit
durations per tile (in the wave queue a packed tile is one superblock, and XCD
range q takes list positions q, q + 8, ...), and writes the share sorted by
descending cost.  With any build and --load: times the share in list order
and in the sorted order (same tiles, same image).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

import raytracingstudy_amd as rt  # noqa: E402
from raytracingstudy_amd import tiles as T  # noqa: E402
from raytracingstudy_amd.camera import scene_pose  # noqa: E402

WAVE_WORDS = 65536 * 4


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c3")
    ap.add_argument("--n", type=int, default=8)
    ap.add_argument("--rank", type=int, default=0)
    ap.add_argument("--save", default="")
    ap.add_argument("--load", default="")
    ap.add_argument("--rounds", type=int, default=7)
    args = ap.parse_args()
    if args.save:
        fd, path = tempfile.mkstemp(suffix=".tl")
        os.close(fd)
        os.environ["RT_TIMELINE_FILE"] = path
    import torch
    cfg = rt.CONFIGS[args.config]
    sp, al = rt.configs.scene_spheres(cfg, rt.SEED)
    r = rt.KernelRenderer(cfg.width, cfg.height, mode="scene", spp=cfg.spp)
    r.resize(cfg.width, cfg.height)
    r.setPosition(scene_pose())
    r.set_scene(sp, al, max_depth=cfg.max_depth)
    ts = rt.configs.TILE_SIZE
    share = T.tiles_for_rank(cfg.width, cfg.height, args.rank, args.n, ts)
    slab = torch.zeros(len(share) * ts * ts * 4, dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()
    if args.save:
        r.render_tiles(share, ts, slab.data_ptr())
        open(path, "wb").close()
        r.render_tiles(share, ts, slab.data_ptr())
        r.synchronize()
        raw = np.fromfile(path, dtype=np.uint64).astype(np.int64)
        u = raw[WAVE_WORDS:].reshape(-1, 2)
        dur = np.where(u[:, 1] > 0, u[:, 1] - u[:, 0], 0)
        cost = dur[:len(share) * 4096].reshape(len(share), 4096)
        tile_cost = cost.sum(1) / 100.0          # us of wave time per tile
        tile_max = cost.max(1) / 100.0           # its longest unit
        order = np.argsort(-tile_max, kind="stable")
        # list position p goes to XCD range p % 8: deal the sorted tiles so
        # every range starts with its longest ones
        dealt = np.empty_like(order)
        per = [order[i::8] for i in range(8)]
        pos = 0
        for j in range(max(len(x) for x in per)):
            for q in range(8):
                if j < len(per[q]):
                    dealt[pos] = per[q][j]
                    pos += 1
        json.dump({"share": share.tolist(), "sorted": share[dealt].tolist(),
                   "tile_cost_us": tile_cost.tolist(), "tile_max_us": tile_max.tolist()},
                  open(args.save, "w"))
        print("saved", args.save, "max unit per tile us: top", np.sort(tile_max)[::-1][:8].round(1).tolist())
        os.unlink(path)
    if args.load:
        d = json.load(open(args.load))
        lists = {"list": np.asarray(d["share"], np.uint32), "longest_first": np.asarray(d["sorted"], np.uint32)}
        stream = torch.cuda.Stream()
        times = {k: [] for k in lists}
        for k, ids in lists.items():
            r.render_tiles(ids, ts, slab.data_ptr(), stream.cuda_stream)
        for _ in range(args.rounds):
            for k, ids in lists.items():
                e0 = torch.cuda.Event(enable_timing=True)
                e1 = torch.cuda.Event(enable_timing=True)
                e0.record(stream)
                r.render_tiles(ids, ts, slab.data_ptr(), stream.cuda_stream)
                e1.record(stream)
                e1.synchronize()
                times[k].append(e0.elapsed_time(e1))
        print(json.dumps({k: round(float(np.median(v)), 3) for k, v in times.items()}))
    r.close()


if __name__ == "__main__":
    main()
