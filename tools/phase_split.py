#!/usr/bin/env python3
"""Where a frame's time goes: primary walks vs shadow walks.

    python tools/phase_split.py [--configs c3,c5,c5d] [--rounds 5]

For each config, two renderers of the same scene and pose, one with shadow
rays (the config) and one without (RT_FLAG_NO_SHADOWS), render plain frames
in interleaved rounds (HIP events on one stream); the difference is the
shadow walks' share of the frame, with the ray counts of each.
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
    ap.add_argument("--configs", default="c3,c5,c5d")
    ap.add_argument("--rounds", type=int, default=5)
    args = ap.parse_args()
    import torch
    stream = torch.cuda.Stream()
    for name in args.configs.split(","):
        cfg = rt.CONFIGS[name]
        sp, al = rt.configs.scene_spheres(cfg, rt.SEED)
        rs = {}
        for shadows in (True, False):
            r = rt.KernelRenderer(cfg.width, cfg.height, mode="scene", spp=cfg.spp, shadows=shadows)
            r.resize(cfg.width, cfg.height)
            r.setPosition(scene_pose())
            r.set_scene(sp, al, max_depth=cfg.max_depth, leaf_capacity=cfg.leaf_capacity)
            r.render(stats=True)  # warm-up
            rs[shadows] = r
        stats = {k: rs[k].render(stats=True) for k in rs}
        times = {k: [] for k in rs}
        for _ in range(args.rounds):
            for k in rs:
                e0 = torch.cuda.Event(enable_timing=True)
                e1 = torch.cuda.Event(enable_timing=True)
                e0.record(stream)
                rs[k].render(None, stream.cuda_stream)
                e1.record(stream)
                e1.synchronize()
                times[k].append(e0.elapsed_time(e1))
        t_all = float(np.median(times[True]))
        t_prim = float(np.median(times[False]))
        st, sp0 = stats[True], stats[False]
        out = {"ms_with_shadows": round(t_all, 3), "ms_primary_only": round(t_prim, 3),
               "shadow_share": round(1.0 - t_prim / t_all, 3),
               "primary_rays": int(st.primary_rays), "shadow_rays": int(st.shadow_rays),
               "nodes_primary": int(sp0.nodes_visited), "prims_primary": int(sp0.prims_tested),
               "nodes_shadow": int(st.nodes_visited - sp0.nodes_visited),
               "prims_shadow": int(st.prims_tested - sp0.prims_tested)}
        for r in rs.values():
            r.close()
        print(name, json.dumps(out), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
