#!/usr/bin/env python3
"""Time progressive-accumulation frames (RT_FLAG_PROGRESSIVE) of a config.

    python tools/prog_bench.py [--config c3] [--frames 6]
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
from raytracingstudy_amd.camera import scene_pose  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c3")
    ap.add_argument("--frames", type=int, default=6)
    args = ap.parse_args()
    import torch
    cfg = rt.CONFIGS[args.config]
    sp, al = rt.configs.scene_spheres(cfg, rt.SEED)
    r = rt.KernelRenderer(cfg.width, cfg.height, mode="scene", spp=cfg.spp, progressive=True)
    r.resize(cfg.width, cfg.height)
    r.setPosition(scene_pose())
    r.set_scene(sp, al, max_depth=cfg.max_depth)
    stream = torch.cuda.Stream()
    r.render(None, stream.cuda_stream)
    ms = []
    for _ in range(args.frames):
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        r.render(None, stream.cuda_stream)
        e1.record(stream)
        e1.synchronize()
        ms.append(e0.elapsed_time(e1))
    print(json.dumps({"config": args.config, "progressive_ms_median": round(float(np.median(ms)), 3),
                      "frames": args.frames}))
    r.close()


if __name__ == "__main__":
    main()
