#!/usr/bin/env python3
"""Each 64x64 tile rendered alone, on one GPU (diagnostic).

    python tools/tile_alone.py [--config c3] [--n 8]

A launch of one tile (4,096 wave units at 64 spp, fewer than the resident
waves) takes about as long as its slowest unit with little contention: the
latency floor of that tile.  Compared with an N-way share's time this says
whether the share's tail is set by a few long units (the share cannot end
before its slowest tile alone) or by the schedule.  Also times rank 0's share
as dealt, longest-alone-first, and without its slowest tiles.
"""
from __future__ import annotations

import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

import raytracingstudy_amd as rt  # noqa: E402
from raytracingstudy_amd import tiles as T  # noqa: E402
from raytracingstudy_amd.camera import scene_pose  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c3")
    ap.add_argument("--n", type=int, default=8)
    ap.add_argument("--rounds", type=int, default=3)
    args = ap.parse_args()
    import torch
    cfg = rt.CONFIGS[args.config]
    sp, al = rt.configs.scene_spheres(cfg, rt.SEED)
    r = rt.KernelRenderer(cfg.width, cfg.height, mode="scene", spp=cfg.spp)
    r.resize(cfg.width, cfg.height)
    r.setPosition(scene_pose())
    r.set_scene(sp, al, max_depth=cfg.max_depth)
    stream = torch.cuda.Stream()
    ts = rt.configs.TILE_SIZE
    tx, ty = T.tile_grid(cfg.width, cfg.height, ts)
    slab = torch.zeros(tx * ty * ts * ts * 4, dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()

    def timed(ids, rounds=args.rounds):
        ids = np.ascontiguousarray(ids, dtype=np.uint32)
        fn = lambda: r.render_tiles(ids, ts, slab.data_ptr(), stream.cuda_stream)  # noqa: E731
        fn()
        out = []
        for _ in range(rounds):
            e0 = torch.cuda.Event(enable_timing=True)
            e1 = torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            fn()
            e1.record(stream)
            e1.synchronize()
            out.append(e0.elapsed_time(e1))
        return float(min(out))

    alone = np.array([timed([t]) for t in range(tx * ty)])
    order = np.argsort(-alone)
    share = np.asarray(T.tiles_for_rank(cfg.width, cfg.height, 0, args.n, ts))
    sa = alone[share]
    res = {"config": args.config, "n": args.n, "tiles": int(tx * ty),
           "alone_ms": {"min": round(float(alone.min()), 4),
                        "p50": round(float(np.median(alone)), 4),
                        "p90": round(float(np.percentile(alone, 90)), 4),
                        "p99": round(float(np.percentile(alone, 99)), 4),
                        "max": round(float(alone.max()), 4)},
           "slowest_tiles": [[int(t), int(t % tx), int(t // tx), round(float(alone[t]), 4)]
                             for t in order[:12]],
           "share_tiles": int(len(share)),
           "share_alone_max_ms": round(float(sa.max()), 4),
           "share_ms": round(timed(share, 5), 4),
           "share_longest_first_ms": round(timed(share[np.argsort(-sa)], 5), 4),
           "full_ms": round(timed(np.arange(tx * ty), 3), 4)}
    for k in (1, 4, 8):
        keep = share[np.argsort(-sa)][k:]
        res[f"share_without_slowest_{k}_ms"] = round(timed(keep, 5), 4)
    res["alone_map"] = [round(float(a), 3) for a in alone]
    print(json.dumps(res))
    r.close()


if __name__ == "__main__":
    main()
