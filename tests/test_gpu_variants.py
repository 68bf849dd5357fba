"""Every shipped scene-kernel variant (0, 7, 10, 13) renders the oracle's
images and counters whatever the padding after the last leaf list holds.

The leaf loads read one sphere past a leaf's end, which for the last leaf is
the kPrimPad tail (rt_params.h); its discriminant joins the leaf screen
unmasked (rt_kernels.hip, walk<> leaf).  rt_capi.cpp fills the tail; the
test-only pad_fill modes put NaN spheres or spheres covering the root box
there, which pass the screen and force the exact path.  Round 2's driver run
failed on case n5_100x70_s3_d7 of a since-removed variant (15, scalar leaf
loads); that input is case 4 below, on the product path.  Collected after
test_gpu_parity.py (tests/conftest.py).
"""
import os
import sys

import numpy as np
import pytest

import raytracingstudy_amd as rt

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import ab_variant_check as vc  # noqa: E402


def test_removed_variants_are_refused():
    # no GPU needed: rt_create validates the flags before touching a device
    with pytest.raises(rt._lib.RtError, match="variant not in this build"):
        rt.KernelRenderer(64, 48, mode="scene", spp=1, variant=rt._lib.VARIANT_REMOVED)


@pytest.mark.parametrize("chunk_bits", [5, 6, 7])
def test_oversized_ticket_field_is_refused(chunk_bits):
    # a ticket of 16..64 wave tiles could span half a block slot, and the
    # two-level queue's claim rule would never publish slot 1
    with pytest.raises(rt._lib.RtError, match="ticket size"):
        rt.KernelRenderer(64, 48, mode="scene", spp=64, opt_off=chunk_bits << 4)


def test_pad_fill_argument_checked():
    with pytest.raises(ValueError):
        rt.KernelRenderer(64, 48, mode="scene", spp=1, pad_fill=3)


@pytest.mark.gpu
@pytest.mark.parametrize("case", vc.CASES, ids=lambda c: "n%d_%dx%d_s%d_d%d" % c)
def test_variants_independent_of_pad(gpu, oracle, case):
    n, w, h, spp, depth = case
    sp, al = rt.generate_spheres(n, rt.SEED)
    ref = None
    bad = {}
    for v in vc.SHIPPED_VARIANTS:
        for fill in (0, 1, 2):
            with rt.KernelRenderer(w, h, mode="scene", spp=spp, radiance=True, variant=v,
                                   pad_fill=fill) as r:
                r.resize(w, h)
                r.setPosition(rt.camera.scene_pose())
                r.set_scene(sp, al, max_depth=depth)
                r.render()  # the plain (timed) build first, then a stats frame
                img0, rad0 = r.readback(), r.readback_radiance()
                st = r.render(stats=True)
                img, rad = r.readback(), r.readback_radiance()
                _, K = r.camera()
            if ref is None:
                ref = oracle.Scene(sp, al, max_depth=depth).render(w, h, rt.camera.scene_pose(), K,
                                                                   spp=spp)
            rep = vc.diff_report(img, rad, st, ref)
            if not (np.array_equal(img0, img) and np.array_equal(rad0, rad)):
                rep["plain_vs_stats"] = True
            if rep:
                bad[f"v{v}_f{fill}"] = rep
    assert not bad, bad

