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


def _free_bytes():
    import torch
    torch.cuda.synchronize()
    return torch.cuda.mem_get_info(0)[0]


def _create_multi(devs, transport, w=1920, h=1080, flags=0):
    lib = _lib.load()
    cfg = _lib.RtConfig()
    lib.rt_config_default(ctypes.byref(cfg))
    cfg.mode = _lib.RT_MODE_SCENE
    cfg.width, cfg.height, cfg.spp = w, h, 4
    cfg.flags = flags | _lib.test_flags
    h_ = ctypes.c_void_p()
    arr = (ctypes.c_int32 * len(devs))(*devs)
    st = lib.rt_create_multi(ctypes.byref(cfg), arr, len(devs), transport, ctypes.byref(h_))
    return st, h_


@pytest.mark.parametrize("fault,devs,transport,code,names", [
    ("create:2", [0, 0, 0], _lib.RT_TRANSPORT_PEER, _lib.RT_E_NOMEM, b"peer 2"),
    ("create:1", [0, 0], _lib.RT_TRANSPORT_PEER, _lib.RT_E_NOMEM, b"peer 1"),
    ("slab:1", [0, 0, 0], _lib.RT_TRANSPORT_PEER, _lib.RT_E_HIP, b"peer 1"),
    ("slab:0", [0], _lib.RT_TRANSPORT_RCCL, _lib.RT_E_HIP, b"peer 0"),
    ("comm", [0], _lib.RT_TRANSPORT_RCCL, _lib.RT_E_HIP, b"devices [0]"),
])
def test_multi_create_fault_injection(gpu, monkeypatch, fault, devs, transport, code, names):
    """a failure of peer k's renderer, of ncclCommInitAll
    or of a slab allocation fails rt_create_multi with the error, names the
    device in rt_last_error(NULL), returns no handle, and frees what the
    partial creation made (the b69acc2 path: peers after k never made).
    Repeated 6 times at 1080p (each attempt allocates tens of MB) with the
    device's free memory checked before and after."""
    lib = _lib.load()
    monkeypatch.setenv("RT_TEST_FAULT", fault)
    st, h = _create_multi(devs, transport)  # warm up allocator / RCCL state once
    assert st == code and not h.value
    before = _free_bytes()
    for _ in range(6):
        st, h = _create_multi(devs, transport)
        assert st == code, lib.rt_last_error(None)
        assert not h.value
        msg = lib.rt_last_error(None)
        assert names in msg, msg
        if fault != "comm":  # ncclCommInitAll names the device list instead
            assert b"device 0" in msg, msg
    assert before - _free_bytes() < 32 << 20, "device memory leaked by failed creations"
    monkeypatch.delenv("RT_TEST_FAULT")
    st, h = _create_multi(devs, transport)  # no fault: the same creation succeeds
    assert st == _lib.RT_OK, lib.rt_last_error(None)
    lib.rt_destroy(h)


def test_multi_peer_queue_error_is_reported(gpu, monkeypatch):
    """a peer whose frame flags its wave-queue error (a
    slot never published, so its slab is incomplete) makes rt_synchronize and
    rt_readback return RT_E_HIP naming that peer, as a single-device renderer
    does for itself; the next clean frame synchronizes without error."""
    monkeypatch.setenv("RT_TEST_FAULT", "queue:1")
    w, h, spp = 160, 96, 4
    sp, al = rt.generate_spheres(1000, rt.SEED)
    with _scene_renderer(w, h, spp, sp, al, devices=[0, 0, 0]) as r:
        r.render()
        with pytest.raises(_lib.RtError) as e:
            r.synchronize()
        assert e.value.code == _lib.RT_E_HIP and "peer 1" in str(e.value), str(e.value)
        r.render()
        with pytest.raises(_lib.RtError) as e:
            r.readback()
        assert e.value.code == _lib.RT_E_HIP and "peer 1" in str(e.value)
        st = r.render(stats=True)  # stats frames are not faulted: clean
        assert st.primary_rays == w * h * spp
        r.synchronize()


def test_multi_default_stream_and_timing(gpu):
    """with no stream the handle uses its own output stream
    on devices[0], not devices[0]'s render stream; rt_get_multi_timing gives
    every device's render time of the last frame and devices[0]'s delivery."""
    w, h, spp = 320, 200, 8
    sp, al = rt.generate_spheres(2000, rt.SEED)
    ref, _ = _whole(w, h, spp, sp, al)
    with _scene_renderer(w, h, spp, sp, al, devices=[0, 0]) as r:
        with pytest.raises(_lib.RtError) as e:
            r.multi_timing()  # no frame yet
        assert e.value.code == _lib.RT_E_STATE
        for _ in range(3):
            r.render()
        t = r.multi_timing()
        assert t["n_devices"] == 2 and t["frame"] == 2
        assert all(x > 0 for x in t["render_ms"]) and t["deliver_ms"] > 0
        assert np.array_equal(r.readback(), ref)
        out = r.stream_ptr()
        assert out and out != 0
    with _scene_renderer(w, h, spp, sp, al) as r1:
        with pytest.raises(_lib.RtError) as e:
            r1.multi_timing()
        assert e.value.code == _lib.RT_E_STATE


def test_multi_refuses_radiance_and_resize_keeps_frames(gpu):
    """RT_FLAG_RADIANCE is refused at creation; a resize
    waits for in-flight frames on the caller's stream before it frees them."""
    import torch
    st, h = _create_multi([0, 0], _lib.RT_TRANSPORT_PEER, w=64, h=64, flags=_lib.RT_FLAG_RADIANCE)
    assert st == _lib.RT_E_INVALID and b"RADIANCE" in _lib.load().rt_last_error(None)
    w, h, spp = 256, 160, 16
    sp, al = rt.generate_spheres(3000, rt.SEED)
    s = torch.cuda.Stream()
    with _scene_renderer(w, h, spp, sp, al, devices=[0, 0]) as r:
        for _ in range(2):
            r.render(None, s.cuda_stream)
        r.resize(96, 64)  # frames queued on s are still running
        r.setPosition(scene_pose())
        r.render()
        ref, _ = _whole(96, 64, spp, sp, al)
        assert np.array_equal(r.readback(), ref)


def test_bench_native_one_device(gpu):
    """`bench.py --gpus 1 --native` drives the C-ABI's
    multi-device handle as a 1-device RCCL communicator; its frame equals one
    renderer's whole frame and the line names the transport and device times."""
    import json
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    p = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "1", "--native",
                        "--config", "c2", "--steps", "5", "--warmup", "2"],
                       env=env, capture_output=True, text=True, timeout=240)
    assert p.returncode == 0, p.stderr[-3000:]
    line = json.loads(p.stdout.strip().splitlines()[-1])
    c = line["config"]
    assert line["n_gpus"] == 1 and c["transport"] == "rccl" and c["tiles_frame_check"] is True
    assert c["devices_seen"] >= 1 and len(c["device_render_ms"]) == 1
    assert line["value"] > 0 and line["roofline"]["frac"] > 0


def test_multi_refusals(gpu):
    lib = _lib.load()
    cfg = _lib.RtConfig()
    lib.rt_config_default(ctypes.byref(cfg))
    cfg.mode = _lib.RT_MODE_SCENE
    cfg.flags = _lib.test_flags
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
