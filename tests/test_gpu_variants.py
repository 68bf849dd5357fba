"""Every shipped scene-kernel variant (0, 4, 7, 10, 13) renders the oracle's
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
import variant_check as vc  # noqa: E402


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


@pytest.mark.gpu
@pytest.mark.parametrize("case", [(9, 48, 40, 16, 7), (20000, 128, 96, 2, 12)],
                         ids=lambda c: "n%d_%dx%d_s%d_d%d" % c)
@pytest.mark.parametrize("delay", [0, 30])
def test_wave_queue_claims_in_slot_order(gpu, oracle, case, delay, monkeypatch):
    """Every frame writes every pixel, even when XCD 0's first slot claim is
    held back (RT_TEST_CLAIM_DELAY: ~100 us of s_sleep before it) until the
    other claims of its first slots have been taken.  These frames hold 9
    and 6 blocks for 8 XCDs, so the level-1 counter runs out inside the
    first slots.  Claimed in ticket order (before round 5), slot 1's claim
    then took a real block and slot 0's came back empty; every wave of the
    XCD drew a slot-0 ticket and exited, and slot 1's block stayed
    unwritten (with the delay in every frame; without it in 13 of 1,800
    first frames of the pad-fill loop above,
    profiles/r05/wave_queue_claim_order.log).  The framebuffer is filled
    with a sentinel before every frame, so an unwritten block shows."""
    import ctypes
    n, w, h, spp, depth = case
    sp, al = rt.generate_spheres(n, rt.SEED)
    hip = ctypes.CDLL("/opt/rocm/lib/libamdhip64.so")
    monkeypatch.setenv("RT_TEST_CLAIM_DELAY", str(delay))  # read at rt_create
    want = None
    bad = []
    for i in range(12):
        with rt.KernelRenderer(w, h, mode="scene", spp=spp, radiance=True, variant=(0, 13)[i % 2],
                               pad_fill=i % 3) as r:
            r.resize(w, h)
            r.setPosition(rt.camera.scene_pose())
            r.set_scene(sp, al, max_depth=depth)
            if want is None:
                _, K = r.camera()
                want = oracle.Scene(sp, al, max_depth=depth).render(w, h, rt.camera.scene_pose(), K,
                                                                     spp=spp)[0]
            fb = r.framebuffer_ptr()
            for f in range(3):
                assert hip.hipMemset(ctypes.c_void_p(fb), 0xAB, ctypes.c_size_t(w * h * 4)) == 0
                assert hip.hipDeviceSynchronize() == 0
                r.render(stats=f == 2)
                img = r.readback()
                diff = np.any(img != want, axis=-1)
                if diff.any():
                    ys, xs = np.nonzero(diff)
                    bad.append({"renderer": i, "frame": f, "pixels": int(diff.sum()),
                                "box": [int(xs.min()), int(xs.max()), int(ys.min()), int(ys.max())],
                                "sentinel": int(np.all(img[diff] == 0xAB))})
    assert not bad, bad[:5]


@pytest.mark.gpu
@pytest.mark.parametrize("case", [(20000, 64, 48, 64, 7), (20000, 128, 96, 2, 12),
                                  (30000, 40, 30, 256, 12)],
                         ids=lambda c: "n%d_%dx%d_s%d_d%d" % c)
def test_lds_staging_on_and_off(gpu, oracle, case, monkeypatch):
    """LDS leaf staging changes which path reads a leaf's spheres, never what
    a frame computes: on (the default) and off (RT_LDS_STAGE=0, read when
    the scene is built), plain and stats frames give the oracle's image and
    counters.  (Since the 8-byte screens, RT_CAM8, the default build's walks
    stage no leaves, so here both settings read globally; the staging path
    is what RT_CAM8=0 builds run, parity-checked when they were the default,
    profiles/r06/pytest_*.log.)"""
    n, w, h, spp, depth = case
    sp, al = rt.generate_spheres(n, rt.SEED)
    out = {}
    for stage in ("0", "1"):
        monkeypatch.setenv("RT_LDS_STAGE", stage)
        with rt.KernelRenderer(w, h, mode="scene", spp=spp, radiance=True) as r:
            r.resize(w, h)
            r.setPosition(rt.camera.scene_pose())
            r.set_scene(sp, al, max_depth=depth)
            r.render()
            img0 = r.readback()
            st = r.render(stats=True)
            img, rad = r.readback(), r.readback_radiance()
            _, K = r.camera()
        out[stage] = (img0, img, rad, st)
    ref = oracle.Scene(sp, al, max_depth=depth).render(w, h, rt.camera.scene_pose(), K, spp=spp)
    for stage, (img0, img, rad, st) in out.items():
        rep = vc.diff_report(img, rad, st, ref)
        assert not rep, (stage, rep)
        assert np.array_equal(img0, img), stage


@pytest.mark.gpu
@pytest.mark.parametrize("case", [(20000, 64, 48, 64, 7, 12), (20000, 128, 96, 2, 12, 8),
                                  (30000, 40, 30, 256, 12, 10), (3000, 64, 48, 16, 7, 2)],
                         ids=lambda c: "n%d_%dx%d_s%d_d%d_cap%d" % c)
@pytest.mark.parametrize("pad_fill", [0, 1, 2])
def test_leaf_lines_packed_and_not(gpu, oracle, case, pad_fill, monkeypatch):
    """The line-packed leaf layout (RT_LEAF_PACK, read when the scene is
    built) moves leaf lists so that none straddles a cache line
    it fits in, leaving gaps filled like the kPrimPad tail.  Packed and
    back-to-back layouts give the oracle's image, radiance and counters, with
    any gap filling, and rt_export_octree returns the builders' compact tree
    either way (record for record the oracle's)."""
    n, w, h, spp, depth, cap = case
    sp, al = rt.generate_spheres(n, rt.SEED)
    out = {}
    for pack in ("0", "1"):
        monkeypatch.setenv("RT_LEAF_PACK", pack)
        with rt.KernelRenderer(w, h, mode="scene", spp=spp, radiance=True, pad_fill=pad_fill) as r:
            r.resize(w, h)
            r.setPosition(rt.camera.scene_pose())
            r.set_scene(sp, al, max_depth=depth, leaf_capacity=cap)
            r.render()
            img0 = r.readback()
            st = r.render(stats=True)
            img, rad = r.readback(), r.readback_radiance()
            tree = r.export_octree()
            _, K = r.camera()
        out[pack] = (img0, img, rad, st, tree)
    sc = oracle.Scene(sp, al, max_depth=depth, leaf_capacity=cap)
    ref = sc.render(w, h, rt.camera.scene_pose(), K, spp=spp)
    onodes, oidx = sc.export_bfs()
    for pack, (img0, img, rad, st, (nodes, psp, pidx)) in out.items():
        rep = vc.diff_report(img, rad, st, ref)
        assert not rep, (pack, rep)
        assert np.array_equal(img0, img), pack
        assert np.array_equal(nodes, onodes) and np.array_equal(pidx, oidx), pack
        assert np.array_equal(psp, sp[oidx]), pack


@pytest.mark.gpu
@pytest.mark.parametrize("spp", [64, 256])
def test_superblock_claim_order(gpu, oracle, spp, monkeypatch):
    """The superblock claim order (RT_SB_ORDER, read per frame: row-major or
    a Hilbert curve over the superblock grid) moves which XCD renders which
    64x64 region, never a pixel: 1024x768 is 192 superblocks, the smallest
    frame the queue claims in superblock slots; plain and stats frames give
    the same image and counters either way, and every 64th row is the
    oracle's."""
    n, w, h = 3000, 1024, 768
    sp, al = rt.generate_spheres(n, rt.SEED)
    out = {}
    for order in ("0", "1"):
        monkeypatch.setenv("RT_SB_ORDER", order)
        with rt.KernelRenderer(w, h, mode="scene", spp=spp, radiance=True) as r:
            r.resize(w, h)
            r.setPosition(rt.camera.scene_pose())
            r.set_scene(sp, al)
            r.render()
            img0 = r.readback()
            st = r.render(stats=True)
            img, rad = r.readback(), r.readback_radiance()
            _, K = r.camera()
        assert np.array_equal(img0, img), order
        out[order] = (img, rad, (st.primary_rays, st.shadow_rays, st.nodes_visited, st.prims_tested))
    assert np.array_equal(out["0"][0], out["1"][0]) and np.array_equal(out["0"][1], out["1"][1])
    assert out["0"][2] == out["1"][2]
    ref8, ref32, _ = oracle.Scene(sp, al).render(w, h, rt.camera.scene_pose(), K, spp=spp, row_step=64)
    rows = np.arange(0, h, 64)
    assert np.array_equal(out["1"][0][rows], ref8[rows]) and np.array_equal(out["1"][1][rows], ref32[rows])


@pytest.mark.gpu
@pytest.mark.parametrize("n,w,h,spp,jitter,tiles", [
    (30000, 70, 45, 256, None, False),   # four rounds (C5's shape), edge pixels
    (30000, 70, 45, 192, None, True),    # three rounds, packed tiles with off-image pixels
    (30000, 33, 20, 100, None, False),   # a partial second round
    (30000, 33, 20, 128, False, False),  # no jitter: every sample in one cell
    (30000, 20, 10, 320, None, False),   # five rounds: past the sorted path's four (unsorted)
])
def test_sorted_rounds_match_oracle(gpu, oracle, n, w, h, spp, jitter, tiles):
    """Quadrant-sorted rounds (spp 65..256): the samples are traced out of
    order, parked and summed in order; image, radiance and counters stay the
    oracle's, plain and stats frames alike."""
    import ctypes
    sp, al = rt.generate_spheres(n, rt.SEED)
    pose = rt.camera.scene_pose()
    with rt.KernelRenderer(w, h, mode="scene", spp=spp, radiance=True, jitter=jitter) as r:
        r.resize(w, h)
        r.setPosition(pose)
        r.set_scene(sp, al)
        r.render()
        img0, rad0 = r.readback(), r.readback_radiance()
        st = r.render(stats=True)
        img, rad = r.readback(), r.readback_radiance()
        _, K = r.camera()
        if tiles:
            ids = np.arange(((w + 63) // 64) * ((h + 63) // 64), dtype=np.uint32)[::-1].copy()
            hip = ctypes.CDLL("/opt/rocm/lib/libamdhip64.so")
            buf = ctypes.c_void_p()
            assert hip.hipMalloc(ctypes.byref(buf), ctypes.c_size_t(len(ids) * 64 * 64 * 4)) == 0
            try:
                r.render_tiles(ids, 64, buf.value)
                vc.poison(r.framebuffer_ptr(), w * h * 4)  # the fb holds img: hide nothing
                r.unpack_tiles(buf.value, ids, 64)
                assert np.array_equal(r.readback(), img)
            finally:
                hip.hipFree(buf)
    ref = oracle.Scene(sp, al).render(w, h, pose, K, spp=spp, jitter=jitter)
    rep = vc.diff_report(img, rad, st, ref)
    assert not rep, rep
    assert np.array_equal(img0, img) and np.array_equal(rad0, rad)


@pytest.mark.gpu
def test_sorted_rounds_progressive(gpu, oracle):
    """Progressive frames of 128 spp (two sorted rounds each) accumulate to
    the oracle's 384-spp image."""
    n, w, h = 30000, 40, 30
    sp, al = rt.generate_spheres(n, rt.SEED)
    pose = rt.camera.scene_pose()
    with rt.KernelRenderer(w, h, mode="scene", spp=128, progressive=True, radiance=True) as p:
        p.resize(w, h)
        p.setPosition(pose)
        p.set_scene(sp, al)
        for _ in range(3):
            p.render()
        img = p.readback()
        _, K = p.camera()
    ref8, _, _ = oracle.Scene(sp, al).render(w, h, pose, K, spp=384)
    assert np.array_equal(img, ref8)
