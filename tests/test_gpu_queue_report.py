"""Round 6: the test-only flags, the
sentinel framebuffer's negative control, and the report of an incomplete
frame on the reference caller's path.

* An incomplete frame (the wave queue's bounded slot wait gave up,
  rt_kernels.hip) stores its id into the renderer's pinned host word; the
  next rt_render reads it without a sync and returns RT_E_HIP, so the
  reference's Displayer, which renders into a mapped PBO every frame and never
  reads back (src/window/displayer.cpp:51-53), learns of it.  The fault is
  injected by RT_TEST_FAULT=queue:0 (the kernel itself stores the word).
* RT_TEST_* environment variables are honoured only with RT_FLAG_TEST_HOOKS.
* The negative control: the library built with round 4's wave-queue claim
  rule (tests/negctl/librt_claim_r4.so, `make -C raytracingstudy_amd/csrc`)
  loses a block when XCD 0's first claim is delayed; with RT_FLAG_TEST_POISON
  every such frame shows the sentinel, and the product library shows none.
"""
import ctypes
import json
import os
import subprocess
import sys

import numpy as np
import pytest

import raytracingstudy_amd as rt
from raytracingstudy_amd import _lib
from raytracingstudy_amd.camera import scene_pose

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
NEGCTL = os.path.join(ROOT, "tests", "negctl", "librt_claim_r4.so")


def _hip():
    return ctypes.CDLL("/opt/rocm/lib/libamdhip64.so")


def _renderer(w=96, h=64, spp=16, n=2000, **kw):
    sp, al = rt.generate_spheres(n, rt.SEED)
    r = rt.KernelRenderer(w, h, mode="scene", spp=spp, **kw)
    r.resize(w, h)
    r.setPosition(scene_pose())
    r.set_scene(sp, al)
    return r


def test_test_flags_match_the_header():
    src = open(os.path.join(ROOT, "include", "rt.h")).read()
    assert "RT_FLAG_TEST_HOOKS = 1u << 10" in src and _lib.RT_FLAG_TEST_HOOKS == 1 << 10
    assert "RT_FLAG_TEST_POISON = 1u << 11" in src and _lib.RT_FLAG_TEST_POISON == 1 << 11


def test_suite_renders_with_poison_and_hooks():
    # tests/conftest.py: every renderer of the suite carries both test flags
    assert _lib.test_flags == _lib.RT_FLAG_TEST_HOOKS | _lib.RT_FLAG_TEST_POISON


@pytest.mark.gpu
@pytest.mark.parametrize("spp", [16, 256, 1])
def test_incomplete_frame_reported_by_the_next_render(gpu, monkeypatch, spp):
    """RT_TEST_FAULT=queue:0: each plain frame reports itself incomplete.  The
    next rt_render (after the frame is done: the GL unmap is the Displayer's
    sync) returns RT_E_HIP naming it and renders nothing; a later frame's
    report reaches rt_synchronize; stats frames are not faulted."""
    monkeypatch.setenv("RT_TEST_FAULT", "queue:0")
    hip = _hip()
    with _renderer(spp=spp) as r:
        r.render()                     # frame 1: flags itself
        assert hip.hipDeviceSynchronize() == 0
        with pytest.raises(_lib.RtError) as e:
            r.render()                 # reports frame 1, queues nothing
        assert e.value.code == _lib.RT_E_HIP and "frame 1 " in str(e.value), str(e.value)
        r.render()                     # frame 2: renders (and flags itself)
        with pytest.raises(_lib.RtError) as e:
            r.synchronize()
        assert e.value.code == _lib.RT_E_HIP and "frame 2 " in str(e.value)
        r.synchronize()                # each report is given once
        st = r.render(stats=True)      # stats frames are not faulted
        assert st.primary_rays == 96 * 64 * spp
        r.render()                     # reported by readback this time
        with pytest.raises(_lib.RtError) as e:
            r.readback()
        assert "frame 4 " in str(e.value)
        r.readback()


@pytest.mark.gpu
def test_incomplete_frame_reported_on_the_display_path(gpu, oracle, monkeypatch):
    """The Displayer's cycle (rt_bind_display: map, render into the mapped
    buffer, unmap; no readback ever): the frame after an incomplete one
    returns RT_E_HIP from rt_render itself.  The faulted frame's pixels are
    still the oracle's (the injected fault marks the frame, it skips no work)."""
    import torch
    monkeypatch.setenv("RT_TEST_FAULT", "queue:0")
    w, h, spp = 96, 64, 16
    buf = torch.zeros(w * h * 4, dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()
    log = []
    with _renderer(w, h, spp) as r:
        r.bind_display(lambda s: (log.append("map"), (buf.data_ptr(), w * h * 4))[1],
                       lambda s: log.append("unmap"))
        r.render()
        torch.cuda.synchronize()
        _, K = r.camera()
        sp, al = rt.generate_spheres(2000, rt.SEED)
        want, _, _ = oracle.Scene(sp, al).render(w, h, scene_pose(), K, spp=spp, radiance=False)
        assert np.array_equal(buf.cpu().numpy().reshape(h, w, 4), want)
        with pytest.raises(_lib.RtError) as e:
            r.render()
        assert e.value.code == _lib.RT_E_HIP and "incomplete" in str(e.value)
        assert log == ["map", "unmap"]  # the reporting call mapped nothing


@pytest.mark.gpu
def test_test_hooks_need_the_flag(gpu, monkeypatch, capfd):
    """Without RT_FLAG_TEST_HOOKS a set RT_TEST_FAULT is ignored (and named on
    stderr once): a stray variable cannot fail a product renderer's frames."""
    monkeypatch.setenv("RT_TEST_FAULT", "queue:0")
    monkeypatch.setattr(_lib, "test_flags", _lib.RT_FLAG_TEST_POISON)
    hip = _hip()
    with _renderer() as r:
        r.render()
        assert hip.hipDeviceSynchronize() == 0
        r.render()
        r.synchronize()
    err = capfd.readouterr().err
    assert "RT_TEST_FAULT=queue:0 ignored" in err


_NEGCTL_SCRIPT = r"""
import json, sys
import numpy as np
sys.path.insert(0, sys.argv[1])
import raytracingstudy_amd as rt
from raytracingstudy_amd import _lib
from raytracingstudy_amd.camera import scene_pose
_lib.test_flags = _lib.RT_FLAG_TEST_HOOKS | _lib.RT_FLAG_TEST_POISON
n, w, h, spp = 9, 48, 40, 16
sp, al = rt.generate_spheres(n, rt.SEED)
frames = lost = 0
for i in range(4):
    with rt.KernelRenderer(w, h, mode="scene", spp=spp, variant=13) as r:
        r.resize(w, h)
        r.setPosition(scene_pose())
        r.set_scene(sp, al)
        for f in range(3):
            r.render()          # no memset of its own: only the library's poison
            img = r.readback()
            frames += 1
            sentinel = np.all(img == 0xAB, axis=-1)
            lost += int(sentinel.any())
print(json.dumps({"lib": _lib.LIB_PATH, "frames": frames, "frames_with_sentinel": lost}))
"""


def _negctl_run(lib_path):
    env = dict(os.environ, RT_TEST_CLAIM_DELAY="30")
    if lib_path:
        env["RT_AMD_LIB"] = lib_path
    else:
        env.pop("RT_AMD_LIB", None)
    p = subprocess.run([sys.executable, "-c", _NEGCTL_SCRIPT, ROOT], env=env, capture_output=True,
                       text=True, timeout=180)
    assert p.returncode == 0, p.stderr[-3000:]
    return json.loads(p.stdout.strip().splitlines()[-1])


@pytest.mark.gpu
def test_poison_sees_the_round4_claim_rule(gpu):
    """VERDICT r05 item 1's negative control: with XCD 0's first claim held
    back, round 4's claim rule leaves a block unrendered; RT_FLAG_TEST_POISON
    alone (no memset in the test) shows it as sentinel pixels.  The product
    library, under the same delay and poison, writes every pixel."""
    assert os.path.exists(NEGCTL), "build the control library: make -C raytracingstudy_amd/csrc"
    bad = _negctl_run(NEGCTL)
    assert bad["frames_with_sentinel"] > 0, bad
    good = _negctl_run(None)
    assert good["frames_with_sentinel"] == 0 and good["frames"] == 12, good
