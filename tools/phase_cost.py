#!/usr/bin/env python3
"""Time of the shadow phase: plain frames with and without shadow rays.

    python tools/phase_cost.py --configs c3,c5 [--frames 5]

Per config: median kernel ms (HIP events on the renderer's stream) of plain
frames with shadows, without (RT_FLAG_NO_SHADOWS: the primary walk and
shading only), their difference, and the counted rays of both.
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def timed(rt, hip, r, frames):
    import numpy as np
    s = ctypes.c_void_p(r.stream_ptr())
    ev = [ctypes.c_void_p(), ctypes.c_void_p()]
    for e in ev:
        hip.hipEventCreate(ctypes.byref(e))
    ms = []
    r.render()
    r.synchronize()
    for _ in range(frames):
        hip.hipEventRecord(ev[0], s)
        r.render()
        hip.hipEventRecord(ev[1], s)
        hip.hipEventSynchronize(ev[1])
        t = ctypes.c_float()
        hip.hipEventElapsedTime(ctypes.byref(t), ev[0], ev[1])
        ms.append(t.value)
    for e in ev:
        hip.hipEventDestroy(e)
    return float(np.median(ms))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", default="c3,c5")
    ap.add_argument("--frames", type=int, default=5)
    args = ap.parse_args()
    import raytracingstudy_amd as rt
    from raytracingstudy_amd.camera import scene_pose
    rt._lib.load()
    hip = ctypes.CDLL("/opt/rocm/lib/libamdhip64.so")
    for name in args.configs.split(","):
        c = rt.CONFIGS[name]
        sp, al = rt.configs.scene_spheres(c, rt.SEED)
        res = {}
        for shadows in (True, False):
            with rt.KernelRenderer(c.width, c.height, mode="scene", spp=c.spp,
                                   shadows=shadows) as r:
                r.resize(c.width, c.height)
                r.setPosition(scene_pose())
                r.set_scene(sp, al, max_depth=c.max_depth)
                st = r.render(stats=True)
                res["on" if shadows else "off"] = {
                    "ms": round(timed(rt, hip, r, args.frames), 3),
                    "rays": st.primary_rays + st.shadow_rays, "shadow_rays": st.shadow_rays,
                    "nodes": st.nodes_visited, "prims": st.prims_tested}
        res["shadow_phase_ms"] = round(res["on"]["ms"] - res["off"]["ms"], 3)
        res["shadow_phase_frac"] = round(res["shadow_phase_ms"] / res["on"]["ms"], 4)
        print(name, json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
