"""GPU tests of the multi-device handle (rt_create_multi; SURVEY 8b B2 "device
ids", 8e E1): one process renders every frame across
several devices' renderers, tiles round-robin, slabs moved to devices[0] by
RCCL (one ncclCommInitAll communicator, grouped ncclSend / ncclRecv) or by
peer copies, one unpack.

The box has one GPU, so:
  * the RCCL transport runs as a 1-device communicator (device 0 sends its
    slab to itself through RCCL), bit-exact against the oracle;
  * the n-way plan runs as n renderers on device 0 (a repeated ordinal: the
    peer-copy transport, RCCL refuses a device twice), byte-identical to one
    renderer's whole frame, up to the C4 frame over 8 virtual devices.
"""
import ctypes

import numpy as np
import pytest

import raytracingstudy_amd as rt
from raytracingstudy_amd import _lib
from raytracingstudy_amd.camera import scene_pose

pytestmark = pytest.mark.gpu


def _scene_renderer(w, h, spp, sp, al, **kw):
    r = rt.KernelRenderer(w, h, mode="scene", spp=spp, **kw)
    r.resize(w, h)
    r.setPosition(scene_pose())
    r.set_scene(sp, al)
    return r


def _whole(w, h, spp, sp, al):
    with _scene_renderer(w, h, spp, sp, al) as r:
        st = r.render(stats=True)
        return r.readback(), st


def test_rccl_one_device_matches_oracle(gpu, oracle):
    """a 1-device communicator run of the RCCL path,
    bit-exact against the oracle, over both frame slots."""
    w, h, spp = 200, 130, 2
    sp, al = rt.generate_spheres(1000, rt.SEED)
    with _scene_renderer(w, h, spp, sp, al, devices=[0], transport="rccl") as r:
        info = r.multi_info()
        assert info["transport"] == "rccl" and info["devices"] == [0]
        _, K = r.camera()
        ref, _, cnt = oracle.Scene(sp, al).render(w, h, scene_pose(), K, spp=spp, radiance=False)
        st = r.render(stats=True)
        assert np.array_equal(r.readback(), ref)
        assert (st.primary_rays, st.shadow_rays) == (int(cnt[0]), int(cnt[1]))
        assert (st.nodes_visited, st.prims_tested) == (int(cnt[2]), int(cnt[3]))
        for _ in range(3):  # plain frames through both slots
            r.render()
        assert np.array_equal(r.readback(), ref)
        assert r.multi_info()["frames"] == 4


@pytest.mark.parametrize("n", [2, 3, 8])
def test_n_way_plan_on_one_device(gpu, n):
    """n renderers on device 0 (peer-copy transport): the assembled frame is
    byte-identical to one renderer's, with the counters summed over devices;
    a resize re-plans the tiles."""
    w, h, spp = 333, 197, 4
    sp, al = rt.generate_spheres(5000, rt.SEED)
    ref, st_ref = _whole(w, h, spp, sp, al)
    with _scene_renderer(w, h, spp, sp, al, devices=[0] * n) as r:
        info = r.multi_info()
        assert info["transport"] == "peer" and info["n_devices"] == n
        tiles = ((w + 63) // 64) * ((h + 63) // 64)
        assert info["slab_tiles"] == -(-tiles // n)
        st = r.render(stats=True)
        assert np.array_equal(r.readback(), ref)
        assert (st.primary_rays, st.shadow_rays, st.nodes_visited, st.prims_tested) == \
            (st_ref.primary_rays, st_ref.shadow_rays, st_ref.nodes_visited, st_ref.prims_tested)
        for _ in range(3):
            r.render()
        assert np.array_equal(r.readback(), ref)
        # resize: every device re-sizes, the plan and slabs follow
        r.resize(128, 200)
        r.setPosition(scene_pose())
        r.render()
        ref2, _ = _whole(128, 200, spp, sp, al)
        assert np.array_equal(r.readback(), ref2)


def test_c4_frame_over_8_virtual_devices(gpu):
    """SURVEY 8e's C4 (3840x2160, 64 spp, 100k spheres) as the native 8-device
    handle on one GPU: byte-identical to the whole-frame render."""
    cfg = rt.CONFIGS["c4"]
    sp, al = rt.configs.scene_spheres(cfg, rt.SEED)
    w, h = cfg.width, cfg.height

    def make(**kw):
        r = rt.KernelRenderer(w, h, mode="scene", spp=cfg.spp, **kw)
        r.resize(w, h)
        r.setPosition(scene_pose())
        r.set_scene(sp, al, max_depth=cfg.max_depth, leaf_capacity=cfg.leaf_capacity)
        return r

    with make() as r1:
        r1.render()
        ref = r1.readback()
    with make(devices=[0] * 8) as r8:
        r8.render()
        r8.render()
        assert np.array_equal(r8.readback(), ref)


def test_scene_from_device_is_broadcast(gpu):
    """rt_set_scene_device on a multi-device handle: the list on devices[0] is
    broadcast (RCCL ncclBroadcast, or peer copies) and every device builds it."""
    import torch
    w, h, spp = 160, 96, 2
    sp, al = rt.generate_spheres(3000, rt.SEED)
    ref, _ = _whole(w, h, spp, sp, al)
    dsp = torch.from_numpy(np.ascontiguousarray(sp, np.float32)).cuda()
    dal = torch.from_numpy(np.ascontiguousarray(al, np.uint32).view(np.int32)).cuda()
    torch.cuda.synchronize()
    for devs, tr in (([0], "rccl"), ([0, 0, 0], "peer")):
        with rt.KernelRenderer(w, h, mode="scene", spp=spp, devices=devs, transport=tr) as r:
            r.resize(w, h)
            r.setPosition(scene_pose())
            r.set_scene_device(dsp.data_ptr(), len(sp), dal.data_ptr())
            r.render()
            assert np.array_equal(r.readback(), ref), (devs, tr)


def test_progressive_and_display_on_multi(gpu, oracle):
    """Progressive frames accumulate per device (each device its own tiles);
    the display cycle maps, unpacks into the mapped buffer and unmaps."""
    import torch
    w, h, spp = 96, 64, 64
    sp, al = rt.generate_spheres(1000, rt.SEED)
    with _scene_renderer(w, h, spp, sp, al, progressive=True) as r1:
        for _ in range(3):
            r1.render()
        ref = r1.readback()
    with _scene_renderer(w, h, spp, sp, al, progressive=True, devices=[0, 0]) as r2:
        for _ in range(3):
            r2.render()
        assert np.array_equal(r2.readback(), ref)
    buf = torch.zeros(w * h * 4, dtype=torch.uint8, device="cuda")
    log = []
    with _scene_renderer(w, h, 2, sp, al, devices=[0, 0, 0, 0]) as r:
        _, K = r.camera()
        want, _, _ = oracle.Scene(sp, al).render(w, h, scene_pose(), K, spp=2, radiance=False)
        torch.cuda.synchronize()
        r.bind_display(lambda s: (log.append("map"), (buf.data_ptr(), w * h * 4))[1],
                       lambda s: log.append("unmap"))
        r.render()
        r.synchronize()
        assert log == ["map", "unmap"]
        assert np.array_equal(buf.cpu().numpy().reshape(h, w, 4), want)


def test_multi_refusals(gpu):
    lib = _lib.load()
    cfg = _lib.RtConfig()
    lib.rt_config_default(ctypes.byref(cfg))
    cfg.mode = _lib.RT_MODE_SCENE
    h = ctypes.c_void_p()
    devs = (ctypes.c_int32 * 2)(0, 0)
    # RCCL refuses a device twice in one communicator
    assert lib.rt_create_multi(ctypes.byref(cfg), devs, 2, _lib.RT_TRANSPORT_RCCL,
                               ctypes.byref(h)) == _lib.RT_E_INVALID
    assert b"distinct" in lib.rt_last_error(None)
    bad = (ctypes.c_int32 * 1)(rt.device_count())
    assert lib.rt_create_multi(ctypes.byref(cfg), bad, 1, 0, ctypes.byref(h)) == _lib.RT_E_INVALID
    assert lib.rt_create_multi(ctypes.byref(cfg), devs, 0, 0, ctypes.byref(h)) == _lib.RT_E_INVALID
    sp, al = rt.generate_spheres(100, rt.SEED)
    with _scene_renderer(64, 64, 1, sp, al, devices=[0, 0]) as r:
        with pytest.raises(_lib.RtError) as e:
            r.render_tiles([0], 64, r.framebuffer_ptr())
        assert e.value.code == _lib.RT_E_STATE
    with rt.KernelRenderer(64, 64, mode="scene", devices=[0]) as r:
        with pytest.raises(_lib.RtError) as e:
            r.render()  # no scene yet
        assert e.value.code == _lib.RT_E_NOSCENE
