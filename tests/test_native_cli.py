"""The native C++ host surface (include/rt_renderer.hpp) through rt_cli."""
import os
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CLI = os.path.join(ROOT, "raytracingstudy_amd", "rt_cli")
# every frame starts from a sentinel-filled framebuffer (RT_FLAG_TEST_POISON,
# VERDICT r05 item 1), as in the Python tests (tests/conftest.py)
POISON = "--test-poison"


def test_cli_built():
    assert os.access(CLI, os.X_OK)


def test_cli_fails_loudly_on_bad_args():
    r = subprocess.run([CLI, "--config", "nope"], capture_output=True, text=True)
    assert r.returncode == 2 and "unknown config" in r.stderr


@pytest.mark.gpu
def test_cli_compat_ppm_matches_known_answers(gpu, tmp_path):
    out = tmp_path / "c1.ppm"
    r = subprocess.run([CLI, "--config", "c1", "--frames", "1", "--out", str(out), POISON],
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    data = out.read_bytes()
    hdr = b"P6\n256 256\n255\n"
    assert data.startswith(hdr)
    rgb = np.frombuffer(data[len(hdr):], np.uint8).reshape(256, 256, 3)
    assert int((rgb == 255).all(-1).sum()) == 12996
    # byte sum of RGBA = RGB sum + 255 * pixels
    assert int(rgb.sum(dtype=np.int64)) + 255 * 256 * 256 == 38965473


@pytest.mark.gpu
def test_cli_scene_runs(gpu):
    r = subprocess.run([CLI, "--config", "c2", "--frames", "2", POISON], capture_output=True, text=True,
                       timeout=120)
    assert r.returncode == 0, r.stderr
    assert "Mrays/s" in r.stdout


@pytest.mark.gpu
def test_cli_scene_file_roundtrip_and_builders(gpu, tmp_path):
    # generate -> save -> reload; device and host builders give the same image
    f = tmp_path / "s.rtsph"
    outs = []
    for extra in (["--save-scene", str(f)], ["--scene", str(f)], ["--scene", str(f), "--host-build"]):
        o = tmp_path / ("img%d.ppm" % len(outs))
        r = subprocess.run([CLI, "--config", "c2", "--spheres", "3000", "--width", "160",
                            "--height", "120", "--frames", "1", "--out", str(o), POISON, *extra],
                           capture_output=True, text=True, timeout=120)
        assert r.returncode == 0, r.stderr
        assert ("host build" if "--host-build" in extra else "device build") in r.stdout
        assert "3000 spheres" in r.stdout
        outs.append(o.read_bytes())
    assert outs[0] == outs[1] == outs[2]


@pytest.mark.gpu
@pytest.mark.parametrize("gpus,same", [(2, True), (3, True), (1, False)])
def test_cli_multi_renderer_frame_equals_single(gpu, tmp_path, gpus, same):
    """rt_cli --gpus N: one process, the C-ABI's multi-device handle
    (rt_create_multi), rehearsed with all renderers on device 0
    (peer-copy transport), and as a 1-device RCCL communicator: the assembled
    frame equals the single-renderer frame byte for byte."""
    base = [CLI, "--config", "c3", "--spheres", "20000", "--width", "200", "--height", "150",
            "--spp", "8", "--frames", "2", POISON]
    one, many = tmp_path / "one.ppm", tmp_path / "many.ppm"
    r1 = subprocess.run(base + ["--out", str(one)], capture_output=True, text=True, timeout=120)
    assert r1.returncode == 0, r1.stderr
    rn = subprocess.run(base + ["--gpus", str(gpus)] + (["--same-device"] if same else []) +
                        ["--out", str(many)], capture_output=True, text=True, timeout=120)
    assert rn.returncode == 0, rn.stderr
    assert f"{gpus} devices" in rn.stdout
    assert ("transport peer" if same else "transport rccl") in rn.stdout
    assert one.read_bytes() == many.read_bytes()


@pytest.mark.gpu
def test_cli_panel_progressive_and_walk(gpu):
    """The stats panel (rt_camera.hpp) through the native driver: progressive
    frames accumulate spp while the camera stays put; walking restarts it."""
    base = [CLI, "--config", "c3", "--spheres", "20000", "--width", "160", "--height", "120",
            "--spp", "4", "--frames", "3", "--panel", "--progressive", POISON]
    r = subprocess.run(base, capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    spp = [int(l.split()[1]) for l in r.stdout.splitlines() if l.startswith("spp ")]
    assert spp == [4, 8, 12]
    assert "Mrays/s" in r.stdout and "GPUs 1" in r.stdout and "frames 3" in r.stdout
    r = subprocess.run(base + ["--walk"], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    spp = [int(l.split()[1]) for l in r.stdout.splitlines() if l.startswith("spp ")]
    assert spp == [4, 4, 4]  # every step moves the camera: accumulation restarts
