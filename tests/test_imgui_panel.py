"""F4: the Displayer's ImGui panel (include/rt_imgui.hpp), headless, on the
reference's own ImGui core.

The reference draws "ui window" every frame (src/window/window.cpp:137-150):
elapsed time, FPS, frames and three drag widgets that edit the camera, whose
pose the next frame's processInput pushes to the renderer
(include/window/displayer.h:42-53).  tests/imgui_panel/panel_frames.cpp runs
that frame loop with no GL/GLFW backend against ImGui compiled from the sources
where they lie (/root/reference/imgui/{imgui,imgui_draw,imgui_widgets,
imgui_tables}.cpp, objects into build/imgui_panel/, never copied into the repo),
injects mouse drags, and reports the panel text (ImGui's own text log) and
every pose that reached rt_set_pose (a recording C-ABI stub: no GPU here).
Skipped where the reference tree is absent (the GPU box).
"""
import json
import os
import shutil
import subprocess

import numpy as np
import pytest

from raytracingstudy_amd.camera import display_pose

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
IMGUI = "/root/reference/imgui"
SOURCES = ("imgui", "imgui_draw", "imgui_widgets", "imgui_tables")
OUT = os.path.join(ROOT, "build", "imgui_panel")


def _build() -> str:
    os.makedirs(OUT, exist_ok=True)
    procs = []
    for name in SOURCES:
        src, obj = os.path.join(IMGUI, name + ".cpp"), os.path.join(OUT, name + ".o")
        if not os.path.exists(obj) or os.path.getmtime(obj) < os.path.getmtime(src):
            procs.append(subprocess.Popen(["g++", "-O1", "-c", src, "-I", IMGUI, "-o", obj]))
    assert all(p.wait() == 0 for p in procs), "compiling the reference's ImGui core failed"
    exe = os.path.join(OUT, "panel_frames")
    subprocess.run(["g++", "-O1", "-std=c++17", "-Wall", "-Werror",
                    os.path.join(ROOT, "tests", "imgui_panel", "panel_frames.cpp"),
                    *[os.path.join(OUT, n + ".o") for n in SOURCES],
                    "-I", IMGUI, "-I", os.path.join(ROOT, "include"), "-o", exe], check=True)
    return exe


@pytest.fixture(scope="module")
def frames():
    if not os.path.isdir(IMGUI) or shutil.which("g++") is None:
        pytest.skip("the reference's ImGui sources (or g++) are not present")
    out = subprocess.run([_build()], check=True, capture_output=True, text=True, timeout=120)
    return json.loads(out.stdout)


def _lines(text):
    return [ln.strip() for ln in text.strip().splitlines()]


def test_panel_text_mirrors_reference_window(frames):
    """window.cpp:140-145: the same labels and formats, plus the renderer's
    Mrays/s, spp and GPU count (rt_stats of the last frame)."""
    assert frames["imgui"].startswith("1.90")
    assert _lines(frames["text0"]) == [
        "Elapsed Time 0.064000",      # 4 frames x 16 ms
        "FPS 62.500000",
        "frames 4",
        "Mrays/s 2957.6",            # (320*240*64 + 1e6) rays / 2 ms
        "spp 64",
        "GPUs 8",
        "{ 0.000 } { 0.000 } { 3.000 } camera pos",   # displayer.h:89-94 defaults
        "{ 0.000 } camera yaw",
        "{ 0.000 } camera pitch",
    ]
    last = _lines(frames["text1"])
    assert last[2] == "frames %d" % frames["frames"]
    assert last[6:] == ["{ -0.500 } { 0.000 } { 3.000 } camera pos",
                        "{ 20.000 } camera yaw", "{ 89.000 } camera pitch"]


def test_panel_edits_reach_set_pose(frames):
    """Dragging yaw by 40 px (0.5 per px), pitch by 400 px (clamped at 89) and
    pos.x by -50 px (0.01 per px): each edit reaches rt_set_pose in the next
    frame as the Displayer's pose for the edited state."""
    assert frames["yaw"] == 20.0 and frames["pitch"] == 89.0
    assert frames["pos"] == [-0.5, 0.0, 3.0]
    assert frames["edits"] == 3
    tol = dict(rtol=0, atol=2e-6)
    np.testing.assert_allclose(np.array(frames["pose_after_yaw"]).reshape(4, 4),
                               display_pose((0, 0, 3), 20.0, 0.0), **tol)
    np.testing.assert_allclose(np.array(frames["pose_after_pitch"]).reshape(4, 4),
                               display_pose((0, 0, 3), 20.0, 89.0), **tol)
    np.testing.assert_allclose(np.array(frames["pose_after_pos"]).reshape(4, 4),
                               display_pose((-0.5, 0, 3), 20.0, 89.0), **tol)
    # every frame pushes its pose and renders once (window.cpp:101-102)
    assert frames["set_pose_calls"] == frames["renders"] == frames["frames"]
