"""Variant parity job: every scene-kernel variant of the loaded library against
the CPU oracle, with the padding after the last leaf list filled three ways.

Run in ONE child process (RT_AMD_LIB may select another build of the
library).  For every case x variant x pad fill it renders one stats frame and
compares RGBA8, the float4 radiance and the four work counters with the
oracle.  A mismatch is reported field by field: how many pixels differ and
the first one (with both values), the largest radiance difference, and the
counter deltas.  Prints one JSON line; exit status 0 iff everything matched.

    python tests/ab_variant_check.py [--variants 0,7,10,13] [--fills 0,1,2]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

import oracle  # noqa: E402
import raytracingstudy_amd as rt  # noqa: E402
from raytracingstudy_amd.camera import scene_pose  # noqa: E402

# the shipped variants: 0 = default for the spp, 7 = block-tile queue counting
# every frame, 10 = the spp < 8 default, 13 = the spp >= 8 default
SHIPPED_VARIANTS = [0, 4, 7, 10, 13]
CASES = [  # n, w, h, spp, depth
    (1000, 160, 120, 1, 7),
    (20000, 128, 96, 2, 12),
    (20000, 64, 48, 64, 7),
    (5, 100, 70, 3, 7),      # root leaf: every leaf chunk reads the padding
    (5, 64, 48, 64, 7),      # root leaf on the wave queue
    (9, 48, 40, 16, 7),      # one split: leaves at depth 1, the last one next to the pad
]


def poison(dev_ptr: int, nbytes: int) -> None:
    """Fill a device buffer with the 0xAB sentinel (the RT_FLAG_TEST_POISON
    pattern) before a call that writes only part of it, e.g. rt_unpack_tiles:
    a tile it skips then shows instead of the previous frame's pixels."""
    import ctypes
    hip = ctypes.CDLL("/opt/rocm/lib/libamdhip64.so")
    assert hip.hipMemset(ctypes.c_void_p(dev_ptr), 0xAB, ctypes.c_size_t(nbytes)) == 0
    assert hip.hipDeviceSynchronize() == 0


def diff_report(img, rad, st, ref) -> dict:
    """Which outputs differ from the oracle's, and how (empty dict: none)."""
    r8, r32, cnt = ref
    rep = {}
    bad = np.any(img != r8, axis=-1)
    if bad.any():
        ys, xs = np.nonzero(bad)
        y, x = int(ys[0]), int(xs[0])
        rep["rgba8"] = {"pixels": int(bad.sum()), "first": [x, y],
                        "got": img[y, x].tolist(), "want": r8[y, x].tolist()}
    dr = np.abs(rad.astype(np.float64) - r32.astype(np.float64))
    dr = np.where(np.isnan(dr), np.inf, dr)
    if (rad != r32).any():
        badr = np.any(rad != r32, axis=-1)
        ys, xs = np.nonzero(badr)
        y, x = int(ys[0]), int(xs[0])
        rep["radiance"] = {"pixels": int(badr.sum()), "max_abs": float(dr.max()), "first": [x, y],
                           "got": rad[y, x].tolist(), "want": r32[y, x].tolist()}
    got = (st.primary_rays, st.shadow_rays, st.nodes_visited, st.prims_tested)
    for name, g, w in zip(("primary", "shadow", "nodes", "prims"), got, cnt):
        if int(g) != int(w):
            rep[name] = {"got": int(g), "want": int(w), "delta": int(g) - int(w)}
    return rep


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--variants", default=",".join(map(str, SHIPPED_VARIANTS)))
    ap.add_argument("--fills", default="0,1,2")
    args = ap.parse_args()
    variants = [int(v) for v in args.variants.split(",")]
    fills = [int(f) for f in args.fills.split(",")]
    oracle.load()
    out, ok = {}, True
    for n, w, h, spp, depth in CASES:
        sp, al = rt.generate_spheres(n, rt.SEED)
        ref = None
        for v in variants:
            for fill in fills:
                with rt.KernelRenderer(w, h, mode="scene", spp=spp, radiance=True, variant=v,
                                       pad_fill=fill) as r:
                    r.resize(w, h)
                    r.setPosition(scene_pose())
                    r.set_scene(sp, al, max_depth=depth)
                    try:
                        st = r.render(stats=True)
                    except rt._lib.RtError as e:
                        out[f"n{n}_{w}x{h}_s{spp}_d{depth}_v{v}_f{fill}"] = {"error": str(e)}
                        ok = False
                        continue
                    img, rad = r.readback(), r.readback_radiance()
                    _, K = r.camera()
                if ref is None:
                    ref = oracle.Scene(sp, al, max_depth=depth).render(w, h, scene_pose(), K, spp=spp)
                rep = diff_report(img, rad, st, ref)
                out[f"n{n}_{w}x{h}_s{spp}_d{depth}_v{v}_f{fill}"] = rep or True
                ok = ok and not rep
    print(json.dumps({"ok": ok, "lib": os.path.basename(rt._lib.LIB_PATH), "cases": out}))
    return 0 if ok else 1


if __name__ == "__main__":
    sys.exit(main())
