#!/usr/bin/env python3
"""Frames in flight on one GPU (diagnostic).

    python tools/inflight.py [--config c3] [--n 8] [--frames 20]

A frame ends with a tail: its last waves run their longest units while the
rest of the GPU idles.  Two renderers (own counters and
queue heads, same scene) on two streams let frame k+1 start in frame k's
tail.  Times K frames back to back on one stream against K frames alternating
over two streams, for the whole frame and for rank 0's N-way tile share.
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
    ap.add_argument("--frames", type=int, default=20)
    ap.add_argument("--slots", type=int, default=2)
    args = ap.parse_args()
    import torch
    cfg = rt.CONFIGS[args.config]
    sp, al = rt.configs.scene_spheres(cfg, rt.SEED)
    rs, streams, outs = [], [], []
    ts = rt.configs.TILE_SIZE
    tx, ty = T.tile_grid(cfg.width, cfg.height, ts)
    for _ in range(args.slots):
        r = rt.KernelRenderer(cfg.width, cfg.height, mode="scene", spp=cfg.spp)
        r.resize(cfg.width, cfg.height)
        r.setPosition(scene_pose())
        r.set_scene(sp, al, max_depth=cfg.max_depth)
        rs.append(r)
        streams.append(torch.cuda.Stream())
        outs.append(torch.zeros(tx * ty * ts * ts * 4, dtype=torch.uint8, device="cuda"))
    share = np.ascontiguousarray(T.tiles_for_rank(cfg.width, cfg.height, 0, args.n, ts), np.uint32)
    torch.cuda.synchronize()

    def run(kind, slots):
        def one(i):
            k = i % slots
            if kind == "full":
                rs[k].render(outs[k].data_ptr(), streams[k].cuda_stream)
            else:
                rs[k].render_tiles(share, ts, outs[k].data_ptr(), streams[k].cuda_stream)
        for i in range(4):
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

    res = {"config": args.config, "n": args.n, "frames": args.frames}
    for kind in ("full", "share"):
        res[kind] = {"one_stream_ms": run(kind, 1)}
        for s in range(2, args.slots + 1):
            res[kind][f"{s}_streams_ms"] = run(kind, s)
    # images of overlapped frames are the plain frame's
    ref = torch.empty_like(outs[0])
    rs[0].render(ref.data_ptr(), streams[0].cuda_stream)
    torch.cuda.synchronize()
    for k in range(args.slots):
        rs[k].render(outs[k].data_ptr(), streams[k].cuda_stream)
    torch.cuda.synchronize()
    res["images_equal"] = all(bool(torch.equal(o[:ref.numel()], ref)) for o in outs)
    print(json.dumps(res))
    for r in rs:
        r.close()


if __name__ == "__main__":
    main()
