"""Fuzz soak: many more seeds of tests/test_gpu_parity.py's random scenes than
the suite runs (seeds FROM..TO), each rendered as a plain frame into a
sentinel-filled framebuffer and then as a stats frame, against the oracle
(RGBA8, radiance, the four counters).  Prints each mismatch and a summary.

    python tools/fuzz_soak.py [FROM=64] [TO=1064] [BUDGET_S=400]

Prints one line per seed (the box kills a silent run), and stops once the
time budget is spent.
"""
import ctypes
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
from test_gpu_parity import _fuzz_case  # noqa: E402

lo = int(sys.argv[1]) if len(sys.argv) > 1 else 64
hi = int(sys.argv[2]) if len(sys.argv) > 2 else 1064
budget = float(sys.argv[3]) if len(sys.argv) > 3 else 400.0
oracle.load()
# every frame sentinel-filled by the library too (RT_FLAG_TEST_POISON), stats
# frames included, as in the test suite (tests/conftest.py)
rt._lib.test_flags = rt._lib.RT_FLAG_TEST_POISON
hip = ctypes.CDLL("/opt/rocm/lib/libamdhip64.so")
bad, t0 = [], time.time()
done = 0
for seed in range(lo, hi):
    if time.time() - t0 > budget:
        break
    t1 = time.time()
    c = _fuzz_case(seed)
    # a tree past the builders' limits: the library refuses it (the oracle
    # aborts on it, so it is only built for trees the library accepts)
    refused = None
    with rt.KernelRenderer(c["w"], c["h"], mode="scene", spp=c["spp"]) as r:
        try:
            r.set_scene(c["sp"], c["al"], max_depth=c["depth"], leaf_capacity=c["leaf"])
        except rt._lib.RtError as ee:
            refused = str(ee)
    if refused is not None:
        done += 1
        print(json.dumps({"seed": seed, "ok": "too large" in refused, "refused": refused[:120],
                          "s": round(time.time() - t1, 2)}), flush=True)
        if "too large" not in refused:
            bad.append(seed)
        continue
    sc_ref = oracle.Scene(c["sp"], c["al"], max_depth=c["depth"], leaf_capacity=c["leaf"])
    with rt.KernelRenderer(c["w"], c["h"], mode="scene", spp=c["spp"], radiance=True,
                           shadows=c["shadows"], jitter=c["jitter"], light_dir=c["light"],
                           ambient=c["ambient"]) as r:
        r.resize(c["w"], c["h"])
        r.setPosition(c["pose"])
        r.set_scene(c["sp"], c["al"], max_depth=c["depth"], leaf_capacity=c["leaf"])
        fb = r.framebuffer_ptr()
        assert hip.hipMemset(ctypes.c_void_p(fb), 0xAB, ctypes.c_size_t(c["w"] * c["h"] * 4)) == 0
        assert hip.hipDeviceSynchronize() == 0
        r.render()
        img0 = r.readback()
        st = r.render(stats=True)
        img, rad = r.readback(), r.readback_radiance()
        _, K = r.camera()
    ref8, ref32, cnt = sc_ref.render(
        c["w"], c["h"], c["pose"], K, spp=c["spp"], jitter=c["jitter"], shadows=c["shadows"],
        light_dir=c["light"], ambient=c["ambient"])
    rep = {}
    if not np.array_equal(img0, ref8):
        rep["plain"] = int(np.any(img0 != ref8, axis=-1).sum())
    if not np.array_equal(img, ref8):
        rep["stats"] = int(np.any(img != ref8, axis=-1).sum())
    if not np.array_equal(rad, ref32):
        rep["radiance"] = int(np.any(rad != ref32, axis=-1).sum())
    got = (st.primary_rays, st.shadow_rays, st.nodes_visited, st.prims_tested)
    if tuple(int(g) for g in got) != tuple(int(x) for x in cnt):
        rep["counters"] = [int(g) - int(x) for g, x in zip(got, cnt)]
    if rep:
        bad.append(seed)
        print(json.dumps({"seed": seed, **rep}), flush=True)
    done += 1
    print(json.dumps({"seed": seed, "ok": not rep, "n": c["n"], "spp": c["spp"], "depth": c["depth"],
                      "leaf": c["leaf"], "s": round(time.time() - t1, 2)}), flush=True)
print(json.dumps({"lib": os.path.basename(rt._lib.LIB_PATH), "seeds": [lo, lo + done], "bad": bad,
                  "s": round(time.time() - t0, 1)}))
sys.exit(1 if bad else 0)
