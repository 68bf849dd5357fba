#!/usr/bin/env python3
"""Wave-execution counts of the walk's blocks (diagnostic build).

    bash tools/build_exp.sh bstats -DRT_BLOCK_STATS
    RT_AMD_LIB=abl/librt_bstats.so python tools/block_stats.py --configs c3,c5

One stats frame per config; the library appends, per frame, how many times a
wave executed each block of walk<> and the active lanes summed over those
executions (BlockStat in rt_params.h).  Printed per config: executions per
frame, per pixel-wave (one 64-sample round) and the mean active lanes.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

NAMES = ["iter", "jump", "jump_descend", "descend", "internal", "leaf", "leaf_chunk", "test",
         "sqrt", "accept", "exit", "pop", "walk", "phase", "iter_shadow", "test_shadow",
         "phase_shadow", "node_read", "node_reread", "exact_load", "past_end", "tie_load", "hit_idx",
         "shade_load", "chunk_shadow", "jump_descend_shadow",
         "lds_leaf"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", default="c3")
    ap.add_argument("--variant", type=int, default=0)
    args = ap.parse_args()
    import raytracingstudy_amd as rt
    from raytracingstudy_amd.camera import scene_pose
    out = {}
    for name in args.configs.split(","):
        c = rt.CONFIGS[name]
        fd, path = tempfile.mkstemp(suffix=".jsonl")
        os.close(fd)
        os.environ["RT_BLOCK_STATS_FILE"] = path
        sp, al = rt.configs.scene_spheres(c, rt.SEED)
        with rt.KernelRenderer(c.width, c.height, mode="scene", spp=c.spp, variant=args.variant) as r:
            r.resize(c.width, c.height)
            r.setPosition(scene_pose())
            r.set_scene(sp, al, max_depth=c.max_depth, leaf_capacity=c.leaf_capacity)
            st = r.render(stats=True)
        rec = json.loads(open(path).read().strip().splitlines()[-1])
        os.unlink(path)
        cnt = rec["counts"]
        waves = c.width * c.height * max(1, c.spp // 64) if c.spp >= 64 else None
        res = {"rays": st.primary_rays + st.shadow_rays, "primary": st.primary_rays,
               "shadow": st.shadow_rays, "nodes": st.nodes_visited, "prims": st.prims_tested,
               "blocks": {}}
        for i, n in enumerate(NAMES):
            ex, lanes = cnt[2 * i], cnt[2 * i + 1]
            res["blocks"][n] = {"exec": ex, "per_wave_round": round(ex / waves, 2) if waves else None,
                                "lanes": round(lanes / ex, 1) if ex else 0}
        out[name] = res
        print(name, f"v{args.variant}", json.dumps(res), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
