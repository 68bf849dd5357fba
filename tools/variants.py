#!/usr/bin/env python3
"""A/B the scene-kernel variants in ONE process (interleaved rounds).

    python tools/variants.py [--configs c2,c3] [--variants 1,2] [--rounds 3]

For each config, one renderer per variant renders the same frame; rounds are
interleaved (v1, v2, v1, v2, ...) and the kernel time (HIP events around
plain, counter-free frames) is reported as median/min.  Every variant's image must equal variant 1's
byte for byte (results are variant-independent by construction).
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
    ap.add_argument("--configs", default="c2,c3")
    ap.add_argument("--variants", default="1,2")
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--spp", type=int, default=0, help="override spp")
    args = ap.parse_args()
    # a variant spec is "V", "V:OPT", "V:OPT:T" or "V:OPT:T:CAP" (OPT = rt_config
    # opt bits, A/B toggles; T = cell-table depth: 0 off, 1..7, absent = chosen
    # from the tree; CAP = octree leaf capacity, absent = the config's)
    variants = args.variants.split(",")
    if len(set(variants)) != len(variants):
        ap.error("--variants: each spec at most once (rounds repeat them)")
    out = {}
    for name in args.configs.split(","):
        cfg = rt.CONFIGS[name]
        spp = args.spp or cfg.spp
        sp, al = rt.configs.scene_spheres(cfg, rt.SEED)
        rs = {}
        for v in variants:
            vv, _, rest = v.partition(":")
            oo, _, rest = rest.partition(":")
            tt, _, cc = rest.partition(":")
            r = rt.KernelRenderer(cfg.width, cfg.height, mode="scene", spp=spp, variant=int(vv),
                                  opt_off=int(oo or 0), cell_table=int(tt) if tt else None)
            r.resize(cfg.width, cfg.height)
            r.setPosition(scene_pose())
            info = r.set_scene(sp, al, max_depth=cfg.max_depth,
                               leaf_capacity=int(cc) if cc else cfg.leaf_capacity)
            r.cell_table_depth = info["cell_table_depth"]
            r.render(stats=True)  # warm-up
            rs[v] = r
        # timed frames are plain frames (no work counters), HIP events on a torch stream
        import torch
        stream = torch.cuda.Stream()
        times = {v: [] for v in variants}
        stats = {v: rs[v].render(stats=True) for v in variants}
        for _ in range(args.rounds):
            for v in variants:
                e0 = torch.cuda.Event(enable_timing=True)
                e1 = torch.cuda.Event(enable_timing=True)
                e0.record(stream)
                rs[v].render(None, stream.cuda_stream)
                e1.record(stream)
                e1.synchronize()
                times[v].append(e0.elapsed_time(e1))
        ref = rs[variants[0]].readback()
        res = {}
        for v in variants:
            img = rs[v].readback()
            st = stats[v]
            rays = st.primary_rays + st.shadow_rays
            med = float(np.median(times[v]))
            res[v] = {"ms_median": round(med, 3), "ms_min": round(min(times[v]), 3),
                      "Mrays_s": round(rays / med / 1e3, 1), "rays": int(rays),
                      "nodes_per_ray": round(st.nodes_visited / rays, 2),
                      "prims_per_ray": round(st.prims_tested / rays, 2),
                      "cell_table_depth": rs[v].cell_table_depth,
                      # across libraries (tools/ab_libs.sh): equal images, equal hashes
                      "image_sha1": __import__("hashlib").sha1(img.tobytes()).hexdigest()[:12],
                      "counters": [int(st.primary_rays), int(st.shadow_rays), int(st.nodes_visited),
                                   int(st.prims_tested)],
                      "image_equal_to_v%s" % variants[0]: bool(np.array_equal(img, ref))}
            rs[v].close()
        out[f"{name} spp{spp}"] = res
        print(name, json.dumps(res), flush=True)
    return 0 if all(r[v]["image_equal_to_v%s" % variants[0]] for r in out.values() for v in r) else 1


if __name__ == "__main__":
    sys.exit(main())
