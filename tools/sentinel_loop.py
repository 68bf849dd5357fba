"""The test_variants_independent_of_pad loop (every case x shipped variant x
pad fill: a fresh renderer, a plain frame, then a stats frame), repeated R
times in one process, with each renderer's framebuffer filled with a
sentinel (0xAB) before its first frame, so a block no wave rendered shows.
Prints every mismatch (plain frame and stats frame against the oracle) and
a summary line.  Round 5 found the wave-queue fault with it
(profiles/r05/wave_queue_claim_order.log).

    python tools/sentinel_loop.py [R=3]
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import numpy as np  # noqa: E402

import oracle  # noqa: E402
import raytracingstudy_amd as rt  # noqa: E402
import variant_check as vc  # noqa: E402
from raytracingstudy_amd.camera import scene_pose  # noqa: E402

R = int(sys.argv[1]) if len(sys.argv) > 1 else 3
import ctypes  # noqa: E402
hip = ctypes.CDLL("/opt/rocm/lib/libamdhip64.so")
oracle.load()
refs = {}
n_bad = n_all = 0
t0 = time.time()
for rep in range(R):
    for case in vc.CASES:
        n, w, h, spp, depth = case
        sp, al = rt.generate_spheres(n, rt.SEED)
        for v in vc.SHIPPED_VARIANTS:
            for fill in (0, 1, 2):
                with rt.KernelRenderer(w, h, mode="scene", spp=spp, radiance=True, variant=v,
                                       pad_fill=fill) as r:
                    r.resize(w, h)
                    r.setPosition(scene_pose())
                    r.set_scene(sp, al, max_depth=depth)
                    fb = r.framebuffer_ptr()
                    assert hip.hipMemset(ctypes.c_void_p(fb), 0xAB, ctypes.c_size_t(w * h * 4)) == 0
                    assert hip.hipDeviceSynchronize() == 0
                    r.render()
                    img0, rad0 = r.readback(), r.readback_radiance()
                    st = r.render(stats=True)
                    img, rad = r.readback(), r.readback_radiance()
                    _, K = r.camera()
                if case not in refs:
                    refs[case] = oracle.Scene(sp, al, max_depth=depth).render(
                        w, h, scene_pose(), K, spp=spp)
                ref = refs[case]
                n_all += 1
                rep0 = vc.diff_report(img0, rad0, st, ref)
                for k in ("primary", "shadow", "nodes", "prims"):
                    rep0.pop(k, None)
                rep1 = vc.diff_report(img, rad, st, ref)
                if rep0 or rep1:
                    n_bad += 1
                    d = np.any(img0 != ref[0], axis=-1)
                    rep0["sentinel_px"] = int(np.all(img0 == 0xAB, axis=-1).sum())
                    if d.any():
                        ys, xs = np.nonzero(d)
                        rep0["box"] = [int(xs.min()), int(xs.max()), int(ys.min()), int(ys.max())]
                    print(json.dumps({"rep": rep, "case": case, "v": v, "fill": fill,
                                      "plain": rep0, "stats": rep1}), flush=True)
    print(json.dumps({"rep": rep, "done": n_all, "bad": n_bad, "s": round(time.time() - t0, 1)}),
          flush=True)
print(json.dumps({"lib": os.path.basename(rt._lib.LIB_PATH), "renders": n_all, "bad": n_bad}))
