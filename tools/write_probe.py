#!/usr/bin/env python3
"""Render a few plain frames of one config at a chosen wave-queue ticket size
(where the HBM write bytes come from).

    python tools/write_probe.py --config c3 --chunk 3 --frames 4

--chunk k: 0 = automatic, k = 1..4 -> 2^(k-1) wave tiles per ticket (the
rt_config opt field kOptChunkShift).  Run under `rocprofv3 --pmc WRITE_SIZE`
(tools/write_bytes.sh) the per-dispatch bytes split into the framebuffer and
a part that scales with the number of queue tickets per frame, which this
script prints (tickets = wave tiles / tiles per ticket).
"""
from __future__ import annotations

import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c3")
    ap.add_argument("--chunk", type=int, default=0)
    ap.add_argument("--frames", type=int, default=4)
    ap.add_argument("--no-shadows", action="store_true",
                    help="primary rays only (RT_FLAG_NO_SHADOWS): tools/r6_gpu.sh pmcphase")
    args = ap.parse_args()
    import raytracingstudy_amd as rt
    from raytracingstudy_amd.camera import scene_pose
    c = rt.CONFIGS[args.config]
    sp, al = rt.configs.scene_spheres(c, rt.SEED)
    with rt.KernelRenderer(c.width, c.height, mode="scene", spp=c.spp,
                           opt_off=(args.chunk & 7) << 4, shadows=not args.no_shadows) as r:
        r.resize(c.width, c.height)
        r.setPosition(scene_pose())
        r.set_scene(sp, al, max_depth=c.max_depth, leaf_capacity=c.leaf_capacity)
        for _ in range(args.frames):
            r.render()
        r.synchronize()
    spw = min(c.spp, 64)
    g = 1
    while g < spw:
        g *= 2
    ppw = 64 // g
    lg = (ppw - 1).bit_length()
    tw, th = 1 << ((lg + 1) // 2), 1 << (lg // 2)
    units = -(-c.width // tw) * -(-c.height // th)
    rounds = -(-c.spp // spw)
    chunk = (1 << (args.chunk - 1)) if args.chunk else max(1, 4 // max(1, min(rounds, 4)))
    print(json.dumps({"config": c.name, "chunk_field": args.chunk, "tiles_per_ticket": chunk,
                      "wave_tiles": units, "tickets": -(-units // chunk),
                      "framebuffer_bytes": c.width * c.height * 4, "frames": args.frames}))


if __name__ == "__main__":
    main()
