"""The native C++ host surface (include/rt_renderer.hpp) through rt_cli."""
import os
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CLI = os.path.join(ROOT, "raytracingstudy_amd", "rt_cli")


def test_cli_built():
    assert os.access(CLI, os.X_OK)


def test_cli_fails_loudly_on_bad_args():
    r = subprocess.run([CLI, "--config", "nope"], capture_output=True, text=True)
    assert r.returncode == 2 and "unknown config" in r.stderr


@pytest.mark.gpu
def test_cli_compat_ppm_matches_known_answers(gpu, tmp_path):
    out = tmp_path / "c1.ppm"
    r = subprocess.run([CLI, "--config", "c1", "--frames", "1", "--out", str(out)],
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
    r = subprocess.run([CLI, "--config", "c2", "--frames", "2"], capture_output=True, text=True,
                       timeout=120)
    assert r.returncode == 0, r.stderr
    assert "Mrays/s" in r.stdout
