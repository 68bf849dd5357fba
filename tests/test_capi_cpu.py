"""CPU tests of the product library: it loads, exports every symbol the C
header declares, and its host-side logic (scene generator, resize intrinsic,
argument validation) matches the oracle — no GPU compute here."""
import ctypes
import os
import re

import numpy as np
import pytest

import raytracingstudy_amd as rt
from raytracingstudy_amd import _lib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _declared_functions():
    src = open(os.path.join(ROOT, "include", "rt.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"^\s*(?:const\s+)?[\w\s\*]+?\b(rt_\w+)\s*\(", src, flags=re.M)))


def test_header_declares_expected_entry_points():
    names = _declared_functions()
    for must in ["rt_create", "rt_destroy", "rt_set_pose", "rt_set_intrinsic", "rt_resize",
                 "rt_set_scene", "rt_set_octree", "rt_render", "rt_render_tiles",
                 "rt_unpack_tiles", "rt_readback", "rt_last_error"]:
        assert must in names


def test_library_exports_every_declared_symbol():
    lib = _lib.load()
    names = _declared_functions()
    missing = [n for n in names if not hasattr(lib, n)]
    assert not missing, missing
    # the ctypes binding covers the whole header, too
    assert set(names) == set(_lib.SIGNATURES)


def test_abi_version():
    assert _lib.load().rt_abi_version() == 4


def test_library_has_gfx950_code_object():
    data = open(_lib.LIB_PATH, "rb").read()
    assert b"gfx950" in data


def test_generator_matches_oracle(oracle):
    for n in (0, 1, 7, 1000, 100_000):
        a_sp, a_al = rt.generate_spheres(n, rt.SEED)
        b_sp, b_al = oracle.generate_spheres(n, rt.SEED)
        assert np.array_equal(a_sp, b_sp) and np.array_equal(a_al, b_al)
    sp, _ = rt.generate_spheres(100_000, rt.SEED)
    assert sp[:, :3].min() >= 0 and sp[:, :3].max() < 1.28
    r = 0.02 * (1000 / 100_000) ** (1 / 3)
    assert sp[:, 3].min() >= 0.5 * r * 0.999 and sp[:, 3].max() < r * 1.001


@pytest.mark.parametrize("w,h", [(256, 256), (1920, 1080), (3840, 2160), (1, 1), (1281, 721)])
def test_resize_intrinsic_matches_oracle(oracle, w, h):
    assert np.array_equal(rt.resize_intrinsic(w, h), oracle.resize_intrinsic(w, h))


def test_known_focal_lengths():
    # f at C1 = 152.54446, C2 = 1144.0835, C4 = 2288.167
    assert abs(rt.resize_intrinsic(256, 256)[0, 0] - 152.54446) < 1e-4
    assert abs(rt.resize_intrinsic(1920, 1080)[0, 0] - 1144.0835) < 1e-3
    assert abs(rt.resize_intrinsic(3840, 2160)[0, 0] - 2288.167) < 1e-3
    K = rt.resize_intrinsic(1921, 1081)
    assert K[0, 2] == 960 and K[1, 2] == 540  # integer division, src/renderer.cu:168-169


def test_invalid_arguments_fail_loudly():
    lib = _lib.load()
    cfg = _lib.RtConfig()
    lib.rt_config_default(ctypes.byref(cfg))
    cfg.width = 0
    h = ctypes.c_void_p()
    assert lib.rt_create(ctypes.byref(cfg), ctypes.byref(h)) == _lib.RT_E_INVALID
    assert b"width" in lib.rt_last_error(None)
    with pytest.raises(_lib.RtError):
        rt.KernelRenderer(0, 10)
    with pytest.raises(KeyError):
        rt.KernelRenderer(10, 10, mode="bogus")


def test_create_without_gpu_is_an_error_not_a_crash():
    if rt.device_count() > 0:
        pytest.skip("a GPU is visible; covered by the gpu tests")
    with pytest.raises(_lib.RtError) as e:
        rt.KernelRenderer(64, 64)
    assert e.value.code == _lib.RT_E_HIP


def test_default_config_matches_reference():
    lib = _lib.load()
    cfg = _lib.RtConfig()
    lib.rt_config_default(ctypes.byref(cfg))
    assert (cfg.width, cfg.height) == (1280, 720)  # main.cpp:6
    p = _lib.RtOctreeParams()
    lib.rt_octree_params_default(ctypes.byref(p))
    assert list(p.min) == [0, 0, 0]
    assert np.allclose(list(p.max), [1.28] * 3)  # src/renderer.cu:134-136
    assert abs(p.resolution - 0.01) < 1e-9 and p.leaf_capacity == 8


def test_product_never_imports_oracle():
    """The product package must not reach the checker (no CPU fallback)."""
    pkg = os.path.join(ROOT, "raytracingstudy_amd")
    for dp, _, fs in os.walk(pkg):
        for f in fs:
            if f.endswith((".py", ".cpp", ".hip", ".h")):
                src = open(os.path.join(dp, f)).read()
                assert "import oracle" not in src and "liboracle" not in src, f
                assert "orc_" not in src, f


def test_gl_interop_header_compiles(tmp_path):
    """the Displayer-side PBO registration (include/rt_gl.hpp)
    and the resource-taking KernelRenderer compile against the GL and HIP headers."""
    import shutil
    import subprocess
    if not os.path.exists("/usr/include/GL/gl.h"):
        pytest.skip("no GL headers in this image")
    cxx = shutil.which("g++")
    r = subprocess.run([cxx, "-std=c++17", "-fsyntax-only", "-D__HIP_PLATFORM_AMD__",
                        "-I/opt/rocm/include", "-I" + os.path.join(ROOT, "include"),
                        os.path.join(ROOT, "tests", "native", "gl_interop_use.cpp")],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stderr


def test_committed_pmc_summary_feeds_the_bench_roofline():
    """bench.py reads profiles/pmc_latest.json (tools/pmc_traffic.py output) for
    the VALU-issue and HBM roofs.  It must be stamped with THIS build's kernel
    sources (re-run tools/profile.sh after every kernel change and copy the
    summary), or the round-end bench line falls back to the cache roof."""
    import bench
    from raytracingstudy_amd._lib import kernel_source_id
    path = os.path.join(ROOT, "profiles", "pmc_latest.json")
    import raytracingstudy_amd as rt
    ent, why = bench.load_pmc(path, "c3", 1, kernel_source_id(), rt.CONFIGS["c3"].leaf_capacity)
    assert ent is not None, why
    r = bench.roofline(ent["scene_kernel_avg_ns"] / 1e6, 182e9, ent, 1024)
    assert r["bound"] == "l2" and 0.0 < r["frac"] <= 1.0
    assert r["binding_unit"]["unit"] in ("scalar_issue", "valu_issue", "vmem_return")
    assert "scalar_issue" in r["roofs"] and "valu_issue" in r["roofs"]
    assert r["traffic"] and r["traffic"] > 0
    assert bench.load_pmc(path, "c4", 1, kernel_source_id())[0] is None  # not profiled
    assert bench.load_pmc(path, "c3", 2, kernel_source_id())[0] is None
