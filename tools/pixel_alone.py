#!/usr/bin/env python3
"""One pixel's 64 samples alone on the GPU (diagnostic).

    python tools/pixel_alone.py --units gpurun_out/<dir>/units.npz [--config c3]

A 1x1 frame whose intrinsic puts pixel (px, py) of the full frame at (0, 0)
traces that pixel's footprint (its jitter hash differs: pixel id 0) as the
only wave unit of the launch, so the launch time is one unit's latency on an
otherwise idle GPU.  Compared with the same pixel's duration inside a full
frame (tools/timeline.py --dump) it separates a unit's intrinsic latency from
what its neighbours on the CU do for it.
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


def full_frame_durations(path, W, H):
    d = np.load(path)
    f = d["full"][0]
    nsx, nsy = (W + 63) // 64, (H + 63) // 64
    n = nsx * nsy * 4096
    uid = np.arange(n)
    sb, b, w = uid // 4096, (uid >> 6) & 63, uid & 63
    x = (sb % nsx) * 64 + (b % 8) * 8 + (w % 8)
    y = (sb // nsx) * 64 + (b // 8) * 8 + w // 8
    v = (x < W) & (y < H) & (f[:n, 1] > 0)
    img = np.zeros((H, W))
    img[y[v], x[v]] = (f[:n, 1][v] - f[:n, 0][v]) / 100.0
    return img


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c3")
    ap.add_argument("--units", required=True)
    ap.add_argument("--count", type=int, default=40)
    args = ap.parse_args()
    import torch
    cfg = rt.CONFIGS[args.config]
    img = full_frame_durations(args.units, cfg.width, cfg.height)
    sp, al = rt.configs.scene_spheres(cfg, rt.SEED)
    big = rt.KernelRenderer(cfg.width, cfg.height, mode="scene", spp=cfg.spp)
    big.resize(cfg.width, cfg.height)
    _, K = big.camera()
    big.close()
    r = rt.KernelRenderer(1, 1, mode="scene", spp=cfg.spp)
    r.setPosition(scene_pose())
    r.set_scene(sp, al, max_depth=cfg.max_depth)
    stream = torch.cuda.Stream()
    out = torch.zeros(4, dtype=torch.uint8, device="cuda")
    flat = img.reshape(-1)
    order = np.argsort(-flat)
    rng = np.random.default_rng(1)
    picks = list(order[:args.count]) + list(rng.choice(np.nonzero(flat > 0)[0], args.count))
    K = np.asarray(K, np.float32).reshape(3, 3).copy()

    def time_pixel(px, py):
        k = K.copy()
        k[0, 2] -= px  # flat K[2] = cx, K[5] = cy (oracle.c orc_get_ray)
        k[1, 2] -= py
        r.setIntrinsic(k)
        ts = []
        for _ in range(4):
            e0 = torch.cuda.Event(enable_timing=True)
            e1 = torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            r.render(out.data_ptr(), stream.cuda_stream)
            e1.record(stream)
            e1.synchronize()
            ts.append(e0.elapsed_time(e1) * 1e3)
        return float(min(ts[1:]))

    # empty-ish reference: a pixel that misses the root box
    empty_us = time_pixel(-5000, -5000)
    rows = []
    for p in picks:
        py, px = divmod(int(p), cfg.width)
        rows.append([px, py, round(float(flat[p]), 1), round(time_pixel(px, py), 1)])
    a = np.array(rows, float)
    top, rnd = a[:args.count], a[args.count:]
    res = {"config": args.config, "empty_launch_us": round(empty_us, 1),
           "slowest_in_frame": {"frame_us_median": float(np.median(top[:, 2])),
                                "alone_us_median": float(np.median(top[:, 3]))},
           "random": {"frame_us_median": float(np.median(rnd[:, 2])),
                      "alone_us_median": float(np.median(rnd[:, 3]))},
           "rows": rows}
    print(json.dumps(res))
    r.close()


if __name__ == "__main__":
    main()
