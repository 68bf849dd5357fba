#!/usr/bin/env python3
"""Where an N-way share's extra time goes, on one GPU (diagnostic).

    python tools/share_cost.py [--config c3] [--n 8]

Times rank 0's interleaved tile list once and concatenated with itself (a
fixed per-launch cost shows up as T(2x) < 2 T(1x)), and every contiguous
1/N band of tile rows (their sum against the full frame says whether the
excess is a property of small launches or of the interleaved plan).
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
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--opt", type=int, default=0, help="rt_config opt bits (A/B toggles)")
    args = ap.parse_args()
    import torch
    cfg = rt.CONFIGS[args.config]
    sp, al = rt.configs.scene_spheres(cfg, rt.SEED)
    r = rt.KernelRenderer(cfg.width, cfg.height, mode="scene", spp=cfg.spp, opt_off=args.opt)
    r.resize(cfg.width, cfg.height)
    r.setPosition(scene_pose())
    r.set_scene(sp, al, max_depth=cfg.max_depth, leaf_capacity=cfg.leaf_capacity)
    stream = torch.cuda.Stream()
    ts = rt.configs.TILE_SIZE
    tx, ty = T.tile_grid(cfg.width, cfg.height, ts)
    slab = torch.zeros(2 * tx * ty * ts * ts * 4, dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()

    def timed(fn):
        fn()
        fn()
        out = []
        for _ in range(args.rounds):
            e0 = torch.cuda.Event(enable_timing=True)
            e1 = torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            fn()
            e1.record(stream)
            e1.synchronize()
            out.append(e0.elapsed_time(e1))
        return round(float(np.median(out)), 3)

    def batched(fn, k=10):
        # k launches back to back, one event pair around all of them
        fn()
        torch.cuda.synchronize()
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for _ in range(k):
            fn()
        e1.record(stream)
        e1.synchronize()
        return round(e0.elapsed_time(e1) / k, 3)

    def tiles(ids):
        ids = np.ascontiguousarray(ids, dtype=np.uint32)
        return timed(lambda: r.render_tiles(ids, ts, slab.data_ptr(), stream.cuda_stream))

    res = {"config": args.config, "n": args.n, "opt": args.opt,
           "full_ms": timed(lambda: r.render(None, stream.cuda_stream))}
    share = T.tiles_for_rank(cfg.width, cfg.height, 0, args.n, ts)
    res["share_ms"] = tiles(share)
    res["share_twice_ms"] = tiles(np.concatenate([share, share]))
    res["share_batched_ms"] = batched(lambda: r.render_tiles(share, ts, slab.data_ptr(),
                                                             stream.cuda_stream))
    res["full_batched_ms"] = batched(lambda: r.render(None, stream.cuda_stream))
    bands = []
    for k in range(args.n):
        lo, hi = tx * ty * k // args.n, tx * ty * (k + 1) // args.n
        bands.append(tiles(np.arange(lo, hi)))
    res["band_ms"] = bands
    res["band_sum_ms"] = round(sum(bands), 3)
    res["all_tiles_ms"] = tiles(np.arange(tx * ty))
    print(json.dumps(res))
    r.close()


if __name__ == "__main__":
    main()
