#!/usr/bin/env python3
"""Time the octree builders: device (default) vs host (RT_FLAG_HOST_BUILD).

    python tools/build_bench.py [--configs c3,c5] [--reps 5]

Per config: median build_ms of repeated rebuilds (setOctree on the resident
scene; the device build reads the spheres already in HBM), tree sizes, and
whether both builders produced the same tree.
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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", default="c3,c5")
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--host-reps", type=int, default=2)
    args = ap.parse_args()
    out = {}
    for name in args.configs.split(","):
        cfg = rt.CONFIGS[name]
        sp, al = rt.configs.scene_spheres(cfg, rt.SEED)
        res = {}
        trees = {}
        for hb in (False, True):
            r = rt.KernelRenderer(64, 64, mode="scene", host_build=hb)
            info = r.set_scene(sp, al, max_depth=cfg.max_depth)
            times = [info["build_ms"]]
            for _ in range(args.host_reps if hb else args.reps):
                r.setOctree((0, 0, 0), (1.28, 1.28, 1.28), 1.28 / (1 << (cfg.max_depth or 7)))
                times.append(r.scene_info()["build_ms"])
            info = r.scene_info()
            trees[hb] = r.export_octree()
            key = "host" if hb else "device"
            res[key] = {"build_ms_median": round(float(np.median(times[1:])), 3),
                        "build_ms_first": round(times[0], 3),
                        "upload_ms": round(info["upload_ms"], 3)}
            res["tree"] = {k: info[k] for k in ("n_nodes", "n_leaves", "n_prim_refs",
                                                "max_depth", "depth_reached")}
            r.close()
        res["identical"] = all(np.array_equal(a, b) for a, b in zip(trees[False], trees[True]))
        res["speedup"] = round(res["host"]["build_ms_median"] / res["device"]["build_ms_median"], 1)
        out[name] = res
        print(name, json.dumps(res), flush=True)
    return 0 if all(v["identical"] for v in out.values()) else 1


if __name__ == "__main__":
    sys.exit(main())
