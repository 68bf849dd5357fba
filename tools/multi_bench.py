#!/usr/bin/env python3
"""Frame time of the C-ABI's multi-device handle (rt_create_multi) against a
single-device renderer, frames back to back (two in flight inside the handle).

    python tools/multi_bench.py [--config c3] [--frames 40] [--devices 0 | 0,1,...]

On a one-GPU box: --devices 0 is a 1-device RCCL communicator (every frame's
tiles go through ncclSend / ncclRecv to device 0 and one unpack); 0,0,...
rehearses the N-way plan with peer copies on one GPU.  Prints one JSON line
per handle: ms per frame (wall, host-timed over all frames) and the frame's
equality with the single renderer's.
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
from raytracingstudy_amd.camera import scene_pose  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c3")
    ap.add_argument("--frames", type=int, default=40)
    ap.add_argument("--devices", action="append", default=None,
                    help="comma-separated ordinals; repeat the flag for several handles")
    args = ap.parse_args()
    cfg = rt.CONFIGS[args.config]
    sp, al = rt.configs.scene_spheres(cfg, rt.SEED)
    handles = [None] + [[int(d) for d in s.split(",")] for s in (args.devices or ["0"])]
    ref = None
    for devs in handles:
        kw = {} if devs is None else {"devices": devs}
        with rt.KernelRenderer(cfg.width, cfg.height, mode="scene", spp=cfg.spp, **kw) as r:
            r.resize(cfg.width, cfg.height)
            r.setPosition(scene_pose())
            r.set_scene(sp, al, max_depth=cfg.max_depth, leaf_capacity=cfg.leaf_capacity)
            for _ in range(3):
                r.render()
            r.synchronize()
            t0 = time.perf_counter()
            for _ in range(args.frames):
                r.render()
            r.synchronize()
            ms = (time.perf_counter() - t0) / args.frames * 1e3
            img = r.readback()
            if ref is None:
                ref = img
            out = {"config": cfg.name, "handle": "single" if devs is None else r.multi_info(),
                   "frames": args.frames, "ms_per_frame": round(ms, 4),
                   "frame_equal_to_single": bool(np.array_equal(img, ref))}
            print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
