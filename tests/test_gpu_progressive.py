"""Progressive accumulation (RT_FLAG_PROGRESSIVE) on the GPU.

Frame k traces samples [k*spp, (k+1)*spp) and adds its round sums onto the
per-pixel sums kept in HBM; the image is their mean.  Parity: every frame is
bit-identical to the oracle's progressive frame (orc_render_scene_frame), and
K frames of 64 spp equal one 64*K-spp frame.  Accumulation restarts whenever
what the pixels show changes (pose, intrinsic, size, scene, tile list).
"""
import os
import sys

import numpy as np
import pytest

import raytracingstudy_amd as rt
from raytracingstudy_amd.camera import display_pose, scene_pose

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import variant_check as vc  # noqa: E402

pytestmark = pytest.mark.gpu

W, H = 96, 64


@pytest.fixture(scope="module")
def spheres():
    return rt.generate_spheres(20000, rt.SEED)


def _renderer(spheres, spp, progressive=True, w=W, h=H, variant=0):
    r = rt.KernelRenderer(w, h, mode="scene", spp=spp, radiance=True, progressive=progressive,
                          variant=variant)
    r.resize(w, h)
    r.setPosition(scene_pose())
    r.set_scene(*spheres)
    return r


@pytest.mark.parametrize("spp", [1, 4, 64, 96])
def test_progressive_frames_match_oracle(gpu, oracle, spheres, spp):
    s = oracle.Scene(*spheres)
    acc = np.zeros((H, W, 4), np.float32)
    with _renderer(spheres, spp) as r:
        pose, K = r.camera()
        for k in range(3):
            st = r.render(stats=True)
            assert st.samples_per_pixel == spp * (k + 1)
            img, rad, cnt = s.render(W, H, pose, K, spp=spp, frame=k, accum=acc)
            assert np.array_equal(r.readback(), img), k
            assert np.array_equal(r.readback_radiance(), rad), k
            assert st.primary_rays == cnt[0] and st.nodes_visited == cnt[2]
    s.close()


@pytest.mark.parametrize("variant", [0, 7, 13])
def test_three_64spp_frames_equal_one_192spp_frame(gpu, spheres, variant):
    # progressive frames always run the unified walk; the one-shot frame runs
    # the requested variant (all variants give identical images)
    with _renderer(spheres, 64, variant=variant) as p, \
            _renderer(spheres, 192, progressive=False, variant=variant) as one:
        for _ in range(3):
            p.render()
        one.render()
        assert np.array_equal(p.readback(), one.readback())
        assert np.array_equal(p.readback_radiance(), one.readback_radiance())


def test_same_pose_keeps_accumulating_new_pose_restarts(gpu, spheres):
    with _renderer(spheres, 4) as r, _renderer(spheres, 4, progressive=False) as fresh:
        r.render()
        r.setPosition(scene_pose())  # the Displayer sets the pose every frame
        st = r.render(stats=True)
        assert st.samples_per_pixel == 8
        moved = display_pose((0.6, 0.7, 2.3), 5.0, -3.0)
        r.setPosition(moved)
        st = r.render(stats=True)
        assert st.samples_per_pixel == 4
        fresh.setPosition(moved)
        fresh.render()
        assert np.array_equal(r.readback(), fresh.readback())


@pytest.mark.parametrize("change", ["intrinsic", "resize", "scene", "octree", "reset"])
def test_changes_restart_accumulation(gpu, spheres, change):
    with _renderer(spheres, 4) as r:
        r.render()
        r.render()
        if change == "intrinsic":
            _, K = r.camera()
            K = K.copy()
            K[0, 0] *= 1.01
            r.setIntrinsic(K)
        elif change == "resize":
            r.resize(W, H)
        elif change == "scene":
            r.set_scene(*spheres)
        elif change == "octree":
            r.setOctree((0, 0, 0), (1.28, 1.28, 1.28), 0.02)
        else:
            r.reset_accumulation()
        st = r.render(stats=True)
        assert st.samples_per_pixel == 4


def test_progressive_tiles_match_full_frame(gpu, spheres):
    import torch
    ts = 64
    ids = np.arange(((W + ts - 1) // ts) * ((H + ts - 1) // ts), dtype=np.uint32)
    with _renderer(spheres, 4) as full, _renderer(spheres, 4) as tiled:
        packed = torch.zeros(len(ids) * ts * ts * 4, dtype=torch.uint8, device="cuda")
        torch.cuda.synchronize()  # the renderer's stream does not order after torch's
        for k in range(3):
            full.render()
            st = tiled.render_tiles(ids, ts, packed.data_ptr(), stats=True)
            assert st.samples_per_pixel == 4 * (k + 1)
        vc.poison(tiled.framebuffer_ptr(), W * H * 4)  # a skipped tile shows
        tiled.unpack_tiles(packed.data_ptr(), ids, ts)
        assert np.array_equal(tiled.readback(), full.readback())
        # another tile list is another pixel set: starts over
        st = tiled.render_tiles(ids[:1], ts, packed.data_ptr(), stats=True)
        assert st.samples_per_pixel == 4
