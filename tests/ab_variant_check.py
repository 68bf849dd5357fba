"""A/B-build parity job (run by tests/test_gpu_ab_variants.py in ONE child process).

Loads ``librt_amd_ab.so`` (RT_AMD_LIB, set by the caller) — the shipped kernels
plus the measured-and-rejected scene-kernel variants of DESIGN.md 5.1 — and
checks every A/B variant against the CPU oracle on small seeded scenes:
RGBA8 and radiance bit-exact, ray counters equal, node/prim counters equal
(the packet walk counts lane-node visits, so images and rays only there).
Prints one JSON line; exit status 0 iff everything matched.
"""
from __future__ import annotations

import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

import oracle  # noqa: E402
import raytracingstudy_amd as rt  # noqa: E402
from raytracingstudy_amd.camera import scene_pose  # noqa: E402

AB_VARIANTS = [1, 2, 3, 8, 9, 11, 12, 14, 15]
CASES = [  # n, w, h, spp, depth
    (1000, 160, 120, 1, 7),
    (20000, 128, 96, 2, 12),
    (20000, 64, 48, 64, 7),
    (5, 100, 70, 3, 7),
]


def main() -> int:
    oracle.load()
    assert os.path.basename(rt._lib.LIB_PATH) == "librt_amd_ab.so", rt._lib.LIB_PATH
    out, ok = {}, True
    for n, w, h, spp, depth in CASES:
        sp, al = rt.generate_spheres(n, rt.SEED)
        sc = oracle.Scene(sp, al, max_depth=depth)
        ref = None
        for v in AB_VARIANTS:
            with rt.KernelRenderer(w, h, mode="scene", spp=spp, radiance=True, variant=v) as r:
                r.resize(w, h)
                r.setPosition(scene_pose())
                r.set_scene(sp, al, max_depth=depth)
                st = r.render(stats=True)
                img, rad = r.readback(), r.readback_radiance()
                _, K = r.camera()
            if ref is None:
                ref = sc.render(w, h, scene_pose(), K, spp=spp)
            r8, r32, cnt = ref
            good = bool(np.array_equal(img, r8) and np.array_equal(rad, r32)
                        and (st.primary_rays, st.shadow_rays) == (int(cnt[0]), int(cnt[1])))
            if v != rt._lib.VARIANT_PACKET:
                good = good and (st.nodes_visited, st.prims_tested) == (int(cnt[2]), int(cnt[3]))
            out[f"n{n}_{w}x{h}_s{spp}_d{depth}_v{v}"] = good
            ok = ok and good
    print(json.dumps({"ok": ok, "cases": out}))
    return 0 if ok else 1


if __name__ == "__main__":
    sys.exit(main())
