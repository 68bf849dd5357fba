#!/usr/bin/env python3
"""Fixed costs of a scene launch (diagnostic).

    python tools/tiny_frames.py [--config c3]

Times (HIP events on the launch stream): windows of the headline frame of
1x1, 8x8, 64x64 and 256x256 pixels (a small frame whose intrinsic is the
1080p one shifted, so every pixel keeps its 1080p footprint), the same windows
aimed off the scene (every ray misses the root box: queue and launch cost
only), and the whole 1920x1080 frame aimed off the scene.
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
    args = ap.parse_args()
    import torch
    cfg = rt.CONFIGS[args.config]
    sp, al = rt.configs.scene_spheres(cfg, rt.SEED)
    big = rt.KernelRenderer(cfg.width, cfg.height, mode="scene", spp=cfg.spp)
    big.resize(cfg.width, cfg.height)
    _, K = big.camera()
    big.close()
    K = np.asarray(K, np.float32).reshape(3, 3)
    s = torch.cuda.Stream()

    def timed(w, h, px, py):
        r = rt.KernelRenderer(w, h, mode="scene", spp=cfg.spp)
        r.setPosition(scene_pose())
        r.set_scene(sp, al, max_depth=cfg.max_depth)
        k = K.copy()
        k[0, 2] -= px  # flat K[2] = cx, K[5] = cy
        k[1, 2] -= py
        r.setIntrinsic(k)
        out = torch.zeros(w * h * 4, dtype=torch.uint8, device="cuda")
        ts = []
        for _ in range(6):
            e0 = torch.cuda.Event(enable_timing=True)
            e1 = torch.cuda.Event(enable_timing=True)
            e0.record(s)
            r.render(out.data_ptr(), s.cuda_stream)
            e1.record(s)
            e1.synchronize()
            ts.append(e0.elapsed_time(e1) * 1e3)
        r.close()
        return round(float(np.median(ts[1:])), 1)

    res = {"config": args.config}
    for n in (1, 8, 64, 256):
        res[f"{n}x{n}_us"] = timed(n, n, 1000, 300)        # inside the sphere cloud's image
        res[f"{n}x{n}_off_us"] = timed(n, n, -100000, 300)  # every ray misses the root box
    res["full_off_us"] = timed(cfg.width, cfg.height, -100000, 0)
    res["full_us"] = timed(cfg.width, cfg.height, 0, 0)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
