"""Camera controls and stats panel: the Displayer's input
state machine (include/window/displayer.h:20-83) in C++ (include/rt_camera.hpp)
and Python (raytracingstudy_amd/controls.py), against each other and against
camera.display_pose (the same pose formula)."""
import os
import subprocess

import numpy as np
import pytest

from raytracingstudy_amd.camera import default_pose, display_pose
from raytracingstudy_amd.controls import CameraController, Keys, StatsPanel

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

SCRIPT = [("k", Keys()), ("k", Keys(w=True)), ("k", Keys(w=True, d=True)),
          ("b", (True, True, 100.0, 100.0)), ("m", (140.0, 90.0)), ("k", Keys()),
          ("m", (300.0, -400.0)), ("k", Keys(space=True)), ("b", (True, False, 0.0, 0.0)),
          ("m", (900.0, 900.0)), ("k", Keys(space=True, shift=True, a=True)),
          ("b", (True, True, 0.0, 0.0)), ("m", (-2000.0, 0.0)), ("k", Keys(s=True))]


def run_py():
    c = CameraController()
    poses = []
    for op, arg in SCRIPT:
        if op == "k":
            poses.append(c.process_input(arg))
        elif op == "b":
            c.mouse_button(*arg)
        else:
            c.mouse_move(*arg)
    return c, poses


def test_default_frame_is_the_displayer_default_pose():
    c = CameraController()
    assert np.allclose(c.process_input(Keys()), default_pose(), atol=1e-7)


def test_mouse_turn_wraps_and_clamps_like_the_displayer():
    c = CameraController()
    c.mouse_button(True, True, 0, 0)
    c.mouse_move(10, 0)          # yaw -= 3 -> 357 (wrapped)
    assert c.yaw == pytest.approx(357.0)
    c.mouse_move(10, -1000)      # pitch += 300 -> clamped 89
    assert c.pitch == 89.0
    c.mouse_button(True, False, 0, 0)
    c.mouse_move(500, 500)       # not controlling: no change
    assert (c.yaw, c.pitch) == (pytest.approx(357.0), 89.0)
    c.mouse_button(False, True, 0, 0)  # left button: ignored
    assert not c.control


def test_pose_matches_display_pose():
    c, _ = run_py()
    assert np.allclose(c.pose(), display_pose(tuple(c.pos), c.yaw, c.pitch), atol=1e-6)


def test_moves_follow_front_right_up():
    c = CameraController()
    for _ in range(10):
        c.process_input(Keys(w=True))
    assert np.allclose(c.pos, [0.0, 0.0, 2.9])
    c.process_input(Keys(d=True))
    assert np.allclose(c.pos, [0.01, 0.0, 2.9])
    c.process_input(Keys(space=True))
    assert np.allclose(c.pos, [0.01, 0.01, 2.9])


def test_cpp_controller_matches_python(tmp_path):
    exe = str(tmp_path / "camera_controls")
    subprocess.check_call(["g++", "-std=c++17", "-O2", "-o", exe,
                           os.path.join(ROOT, "tests", "native", "camera_controls.cpp"),
                           "-I" + os.path.join(ROOT, "include")])
    lines = []
    for op, arg in SCRIPT:
        if op == "k":
            lines.append("k " + " ".join(str(int(v)) for v in
                                         (arg.w, arg.a, arg.s, arg.d, arg.space, arg.shift)))
        elif op == "b":
            lines.append("b %d %d %f %f" % (int(arg[0]), int(arg[1]), arg[2], arg[3]))
        else:
            lines.append("m %f %f" % arg)
    out = subprocess.run([exe], input="\n".join(lines) + "\n", capture_output=True, text=True,
                         check=True).stdout.split("\n")
    cpp = [np.array(l.split(), np.float64).reshape(4, 4) for l in out if l.strip()]
    _, py = run_py()
    assert len(cpp) == len(py)
    for a, b in zip(cpp, py):
        assert np.allclose(a, b, atol=2e-5)  # C++ runs in float like glm, Python in double


def test_stats_panel_text():
    class S:
        primary_rays, shadow_rays, ms, samples_per_pixel = 132_710_400, 52_253_228, 15.6, 64
    p = StatsPanel()
    p.update(16.0, S(), 8)
    t = p.text()
    assert "FPS 62.5" in t and "frames 1" in t and "spp 64" in t and "GPUs 8" in t
    assert "Mrays/s 11856.6" in t
