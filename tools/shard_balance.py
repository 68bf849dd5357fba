#!/usr/bin/env python3
"""Per-rank cost of the multi-GPU tile plan, measured on one GPU.

    python tools/shard_balance.py [--config c3] [--ranks 2,4,8] [--rounds 3]

For each world size N, renders every rank's tile list (tiles.tiles_for_rank)
with one renderer and reports each rank's kernel time (HIP events, plain
frames): max/mean is the load imbalance a strong-scaling run pays, and
N * max vs the full frame is the projected scaling efficiency (kernel only).
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
    ap.add_argument("--ranks", default="2,4,8")
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--tile-size", type=int, default=rt.configs.TILE_SIZE)
    ap.add_argument("--opt", type=int, default=0, help="rt_config opt-off/A-B bits")
    ap.add_argument("--variant", type=int, default=0, help="scene-kernel variant (0 default)")
    ap.add_argument("--plan", default="interleave", choices=T.PLANS, help="tile plan")
    args = ap.parse_args()
    import torch
    cfg = rt.CONFIGS[args.config]
    sp, al = rt.configs.scene_spheres(cfg, rt.SEED)
    r = rt.KernelRenderer(cfg.width, cfg.height, mode="scene", spp=cfg.spp, opt_off=args.opt,
                          variant=args.variant)
    r.resize(cfg.width, cfg.height)
    r.setPosition(scene_pose())
    r.set_scene(sp, al, max_depth=cfg.max_depth)
    stream = torch.cuda.Stream()

    def timed(fn):
        fn()  # two untimed frames: the heavy-first list of this tile list is live
        fn()
        ts = []
        for _ in range(args.rounds):
            e0 = torch.cuda.Event(enable_timing=True)
            e1 = torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            fn()
            e1.record(stream)
            e1.synchronize()
            ts.append(e0.elapsed_time(e1))
        return float(np.median(ts))

    r.render(None, stream.cuda_stream)
    full = timed(lambda: r.render(None, stream.cuda_stream))
    out = {"config": args.config, "full_ms": round(full, 3), "tile_size": args.tile_size,
           "opt": args.opt, "variant": args.variant, "plan": args.plan}
    ts = args.tile_size
    for n in [int(x) for x in args.ranks.split(",")]:
        slab = torch.zeros(T.slab_tiles(cfg.width, cfg.height, n, ts, args.plan) * ts * ts * 4,
                           dtype=torch.uint8, device="cuda")
        torch.cuda.synchronize()
        per = []
        for k in range(n):
            ids = T.tiles_for_rank(cfg.width, cfg.height, k, n, ts, args.plan)
            r.render_tiles(ids, ts, slab.data_ptr(), stream.cuda_stream)
            per.append(timed(lambda: r.render_tiles(ids, ts, slab.data_ptr(), stream.cuda_stream)))
        # the same pixel count as one contiguous band of tile rows (locality check)
        tx, ty = T.tile_grid(cfg.width, cfg.height, ts)
        band = np.arange(0, (tx * ty + n - 1) // n, dtype=np.uint32)
        r.render_tiles(band, ts, slab.data_ptr(), stream.cuda_stream)
        band_ms = timed(lambda: r.render_tiles(band, ts, slab.data_ptr(), stream.cuda_stream))
        mx, mean = max(per), float(np.mean(per))
        out[f"n{n}"] = {"rank_ms": [round(x, 3) for x in per], "max_ms": round(mx, 3),
                        "imbalance_max_over_mean": round(mx / mean, 3),
                        "contiguous_band_ms": round(band_ms, 3),
                        "eff_vs_full_kernel": round(full / (n * mx), 3)}
        print(n, json.dumps(out[f"n{n}"]), flush=True)
    print(json.dumps(out))
    r.close()
    return 0


if __name__ == "__main__":
    sys.exit(main())
