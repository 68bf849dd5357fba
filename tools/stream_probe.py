#!/usr/bin/env python3
"""Concurrency of frames on several streams vs how the streams are made (diagnostic).

    python tools/stream_probe.py [--config c3] [--n 8]

Renders rank 0's 1/n tile share back to back, frame k on stream k mod F, for
F = 1..4, with the streams (a) taken from torch's pool after all renderers are
built (bench.py's order), (b) taken between renderer constructions
(tools/inflight.py's order), (c) high priority from the pool.  Frames that
overlap show up as ms/frame below the one-stream time.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

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
    ap.add_argument("--frames", type=int, default=40)
    args = ap.parse_args()
    import torch
    cfg = rt.CONFIGS[args.config]
    sp, al = rt.configs.scene_spheres(cfg, rt.SEED)
    ts = rt.configs.TILE_SIZE
    tx, ty = T.tile_grid(cfg.width, cfg.height, ts)
    share = np.ascontiguousarray(T.tiles_for_rank(cfg.width, cfg.height, 0, args.n, ts), np.uint32)

    def renderer():
        r = rt.KernelRenderer(cfg.width, cfg.height, mode="scene", spp=cfg.spp)
        r.resize(cfg.width, cfg.height)
        r.setPosition(scene_pose())
        r.set_scene(sp, al, max_depth=cfg.max_depth)
        return r

    def timed(rs, streams, outs):
        F = len(rs)

        def one(i):
            k = i % F
            rs[k].render_tiles(share, ts, outs[k].data_ptr(), streams[k].cuda_stream)
        for i in range(8):
            one(i)
        torch.cuda.synchronize()
        best = None
        for _ in range(3):
            t0 = time.perf_counter()
            for i in range(args.frames):
                one(i)
            torch.cuda.synchronize()
            ms = (time.perf_counter() - t0) * 1e3 / args.frames
            best = ms if best is None else min(best, ms)
        return round(best, 4)

    res = {"config": args.config, "n": args.n}
    for order in ("after", "between", "high"):
        for F in (1, 2, 3, 4):
            rs, streams = [], []
            for _ in range(F):
                rs.append(renderer())
                if order == "between":
                    streams.append(torch.cuda.Stream())
            if order == "after":
                streams = [torch.cuda.Stream() for _ in range(F)]
            elif order == "high":
                streams = [torch.cuda.Stream(priority=-1) for _ in range(F)]
            outs = [torch.zeros(tx * ty * ts * ts * 4, dtype=torch.uint8, device="cuda")
                    for _ in range(F)]
            res[f"{order}_f{F}_ms"] = timed(rs, streams, outs)
            for r in rs:
                r.close()
    print(json.dumps(res))


if __name__ == "__main__":
    main()
