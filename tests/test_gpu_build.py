"""Device octree builder (octree_build.hip) on the GPU.

The device-built tree must equal the oracle's tree record for record (nodes,
leaf lists, leaf sphere copies, root box, counts) and the host builder's
(RT_FLAG_HOST_BUILD), and frames rendered from it must equal frames rendered
from the host-built tree.  Scenes handed over in device memory
(rt_set_scene_device) must behave exactly like host scenes.
"""
import numpy as np
import pytest

import raytracingstudy_amd as rt
from raytracingstudy_amd.camera import scene_pose
from test_octree_build import CASE_NAMES, case

pytestmark = pytest.mark.gpu


def _renderer(w=64, h=48, spp=4, host_build=False):
    r = rt.KernelRenderer(w, h, mode="scene", spp=spp, host_build=host_build)
    r.resize(w, h)
    r.setPosition(scene_pose())
    return r


def _octree_kw(mn, mx, depth, cap):
    return dict(root_min=mn, root_max=mx, max_depth=depth, leaf_capacity=cap)


def _check_against_oracle(oracle, r, sp, al, mn, mx, depth, cap):
    info = r.scene_info()
    nodes, psp, idx = r.export_octree()
    s = oracle.Scene(sp, al, mn, mx, depth, cap)
    oi = s.info()
    onodes, oidx = s.export_bfs()
    rmin, rmax = s.root()
    s.close()
    assert (info["n_nodes"], info["n_leaves"], info["n_prim_refs"], info["depth_reached"]) == (
        oi["n_nodes"], oi["n_leaves"], oi["n_prim_refs"], oi["depth_reached"])
    assert np.array_equal(nodes, onodes)
    assert np.array_equal(idx, oidx)
    assert np.array_equal(psp, sp[idx].reshape(-1, 4))
    assert np.array_equal(np.float32(info["root_min"]), rmin)
    assert np.array_equal(np.float32(info["root_max"]), rmax)


@pytest.mark.parametrize("name", CASE_NAMES)
def test_device_build_matches_oracle(gpu, oracle, name):
    _, sp, al, mn, mx, depth, cap = case(name)
    kw = _octree_kw(mn, mx, depth, cap)
    if depth == 0:  # max_depth 0 at the API means "from resolution": ask for one cell
        kw["resolution"] = 4.0
    with _renderer() as r:
        info = r.set_scene(sp, al, **kw)
        assert info["max_depth"] == depth
        assert info["builder"] == "device"
        _check_against_oracle(oracle, r, sp, al, mn, mx, depth, cap)


def test_device_build_depth1_and_resolution(gpu, oracle):
    sp, al = rt.generate_spheres(1000, rt.SEED)
    with _renderer() as r:
        r.set_scene(sp, al, max_depth=1)
        _check_against_oracle(oracle, r, sp, al, (0, 0, 0), (1.28, 1.28, 1.28), 1, 8)
        # resolution 0.01 over 1.28 -> depth 7 (the reference's setOctree arguments)
        r.setOctree((0, 0, 0), (1.28, 1.28, 1.28), 0.01)
        assert r.scene_info()["max_depth"] == 7
        _check_against_oracle(oracle, r, sp, al, (0, 0, 0), (1.28, 1.28, 1.28), 7, 8)


@pytest.mark.parametrize("n,depth", [(100000, 7), (300000, 12)])
def test_device_build_equals_host_build_large(gpu, n, depth):
    sp, al = rt.generate_spheres(n, rt.SEED)
    with _renderer(host_build=True) as rh, _renderer() as rd:
        ih = rh.set_scene(sp, al, max_depth=depth)
        idv = rd.set_scene(sp, al, max_depth=depth)
        assert ih["builder"] == "host" and idv["builder"] == "device"
        for k in ("n_nodes", "n_leaves", "n_prim_refs", "depth_reached", "root_min", "root_max"):
            assert ih[k] == idv[k], k
        for a, b in zip(rh.export_octree(), rd.export_octree()):
            assert np.array_equal(a, b)


def test_frames_from_device_and_host_trees_identical(gpu):
    sp, al = rt.generate_spheres(20000, rt.SEED)
    imgs = []
    for hb in (False, True):
        with _renderer(160, 96, spp=8, host_build=hb) as r:
            r.set_scene(sp, al)
            st = r.render(stats=True)
            imgs.append((r.readback(), st.nodes_visited, st.prims_tested))
    assert np.array_equal(imgs[0][0], imgs[1][0])
    assert imgs[0][1:] == imgs[1][1:]


def test_scene_from_device_memory(gpu):
    import torch
    sp, al = rt.generate_spheres(5000, rt.SEED)
    dsp = torch.from_numpy(sp).cuda()
    dal = torch.from_numpy(al.view(np.int32)).cuda()
    stream = torch.cuda.current_stream()  # the stream that produced the tensors
    with _renderer() as ref, _renderer() as r:
        ref.set_scene(sp, al)
        ref.render()
        info = r.set_scene_device(dsp.data_ptr(), len(sp), dal.data_ptr(),
                                  stream=stream.cuda_stream)
        assert info["builder"] == "device" and info["n_spheres"] == 5000
        r.render()
        assert np.array_equal(r.readback(), ref.readback())
        for a, b in zip(r.export_octree(), ref.export_octree()):
            assert np.array_equal(a, b)
        # the renderer keeps its own copy: the caller's buffer may be reused
        dsp.zero_()
        r.render()
        assert np.array_equal(r.readback(), ref.readback())


def test_scene_from_device_memory_default_albedo_and_host_rebuild(gpu):
    import torch
    sp, _ = rt.generate_spheres(3000, 5)
    dsp = torch.from_numpy(sp).cuda()
    with _renderer() as ref, _renderer(host_build=True) as r:
        ref.set_scene(sp, None)
        ref.render()
        r.set_scene_device(dsp.data_ptr(), len(sp))  # host builder: downloads the spheres
        assert r.scene_info()["builder"] == "host"
        r.render()
        assert np.array_equal(r.readback(), ref.readback())
        r.setOctree((0, 0, 0), (1.28, 1.28, 1.28), 0.04)  # rebuild from the device copy
        ref.setOctree((0, 0, 0), (1.28, 1.28, 1.28), 0.04)
        for a, b in zip(r.export_octree(), ref.export_octree()):
            assert np.array_equal(a, b)


@pytest.mark.parametrize("bad", ["zero_radius", "nan_centre", "inf_radius"])
def test_invalid_device_spheres_rejected_scene_kept(gpu, bad):
    import torch
    sp, al = rt.generate_spheres(2000, rt.SEED)
    with _renderer() as r:
        r.set_scene(sp, al)
        r.render()
        before = r.readback()
        badsp = sp.copy()
        if bad == "zero_radius":
            badsp[1234, 3] = 0.0
        elif bad == "nan_centre":
            badsp[7, 1] = np.nan
        else:
            badsp[1999, 3] = np.inf
        d = torch.from_numpy(badsp).cuda()
        with pytest.raises(rt._lib.RtError) as e:
            r.set_scene_device(d.data_ptr(), len(badsp))
        assert e.value.code == rt._lib.RT_E_INVALID
        with pytest.raises(rt._lib.RtError):
            r.set_scene(badsp, al)
        r.render()
        assert np.array_equal(r.readback(), before)


def test_empty_device_scene_renders_background(gpu, oracle):
    with _renderer() as r:
        info = r.set_scene_device(0, 0)
        assert info["n_nodes"] == 1 and info["n_prim_refs"] == 0
        r.render()
        img = r.readback()
        s = oracle.Scene(np.zeros((0, 4), np.float32))
        pose, K = r.camera()
        ref, _, _ = s.render(64, 48, pose, K, spp=4)
        s.close()
        assert np.array_equal(img, ref)


def test_scene_file_renders_like_the_list(gpu, tmp_path):
    sp, al = rt.generate_spheres(4000, rt.SEED)
    p = str(tmp_path / "s.rtsph")
    rt.save_spheres(p, sp, al)
    with _renderer() as a, _renderer() as b:
        a.set_scene(sp, al)
        b.set_scene_file(p)
        a.render()
        b.render()
        assert np.array_equal(a.readback(), b.readback())
