#!/usr/bin/env python3
"""How far can the reference BINARY's compat image differ from its source
semantics?  nvcc's default -fmad=true contracts getRay's sums
(include/camera.h:31-34) into FMAs; the oracle restates the source without
contraction.  This counts the RGBA8 bytes (and pixels) that differ between the
uncontracted image and the two possible contracted ones (oracle
orc_render_compat_fma, contract = 1 NVVM operand order, 2 the other), over the
standard poses and the 32 compat fuzz cameras of tests/test_gpu_parity.py, at
256x256 and 1920x1080.  CPU only (oracle); prints one JSON object.

    python tools/compat_fma_gap.py > profiles/r02/compat_fma_gap.json
"""
from __future__ import annotations

import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

import oracle  # noqa: E402
from raytracingstudy_amd.camera import (default_pose, display_pose,  # noqa: E402
                                        translation_pose)


def poses():
    out = {"default": default_pose(), "yawed": display_pose((0.3, 0.9, 2.5), 23.0, -11.0),
           "inside": translation_pose(0.64, 0.64, 0.64),
           "behind": translation_pose(0.64, 0.64, -3.0)}
    for seed in range(32):  # the compat fuzz cameras (test_compat_fuzz)
        g = np.random.default_rng(1000 + seed)
        g.integers(1, 300), g.integers(1, 200)
        if seed % 4 == 0:
            p = translation_pose(*(float(x) for x in g.choice([0.0, 0.64, 1.28, -1.0, 3.0], 3)))
        else:
            p = display_pose(tuple(g.uniform(-2.0, 3.3, 3)), float(g.uniform(-180, 180)),
                             float(g.uniform(-89, 89)))
        out[f"fuzz{seed}"] = p
    return out


def main():
    oracle.load()
    res = {"what": "RGBA8 bytes / pixels differing between the uncontracted compat image "
                   "and nvcc-style FMA-contracted getRay (oracle contract 1 and 2)",
           "sizes": {}}
    for (w, h) in [(256, 256), (1920, 1080)]:
        K = oracle.resize_intrinsic(w, h)
        per = {}
        tot = {1: [0, 0], 2: [0, 0]}
        for name, pose in poses().items():
            base = oracle.render_compat(w, h, pose, K)
            row = {}
            for c in (1, 2):
                img = oracle.render_compat_fma(w, h, pose, K, c)
                d = img != base
                nb, npx = int(d.sum()), int(d.any(-1).sum())
                tot[c][0] += nb
                tot[c][1] += npx
                row[f"contract{c}"] = {"bytes": nb, "pixels": npx,
                                       "max_abs": int(np.abs(img.astype(int) - base).max())}
            per[name] = row
        n_px = w * h * len(per)
        res["sizes"][f"{w}x{h}"] = {
            "poses": len(per), "pixels_total": n_px,
            "contract1": {"bytes": tot[1][0], "pixels": tot[1][1], "pixel_frac": tot[1][1] / n_px},
            "contract2": {"bytes": tot[2][0], "pixels": tot[2][1], "pixel_frac": tot[2][1] / n_px},
            "per_pose": per}
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
