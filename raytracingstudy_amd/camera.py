"""glm-free host camera helpers (column-major, glm ``m[c][r]`` indexing).

The reference builds the camera pose on the host in
``Displayer::processInput`` (``include/window/displayer.h:20-55``)::

    front = rotate(yaw, Y) * rotate(pitch, X) * vec4(0,0,-1,0)
    view  = inverse(lookAt(pos, pos + front, up)) * diag(1,-1,-1,1)

i.e. an OpenGL camera converted to the OpenCV (y-down, z-forward) convention
that ``Camera::getRay`` expects.  ``display_pose`` restates that in numpy
(float64 math, rounded to float32 at the end: glm runs it in float, so poses
with yaw/pitch not multiples of 90 degrees can differ in the last ulp; the
render path takes the pose as an explicit input, so goldens never depend on
this helper — SURVEY.md 8c C2).
"""
from __future__ import annotations

import math

import numpy as np

__all__ = ["default_pose", "scene_pose", "display_pose", "translation_pose"]


def translation_pose(x: float, y: float, z: float) -> np.ndarray:
    """Pose with rot = diag(1,-1,-1) (the Displayer's default orientation)."""
    p = np.zeros((4, 4), np.float32)
    p[0, 0] = 1.0
    p[1, 1] = -1.0
    p[2, 2] = -1.0
    p[3, :3] = (x, y, z)
    p[3, 3] = 1.0
    return p


def default_pose() -> np.ndarray:
    """Displayer default: position (0,0,3), yaw 0, pitch 0 (include/window/displayer.h:89-94)."""
    return translation_pose(0.0, 0.0, 3.0)


def scene_pose() -> np.ndarray:
    """SURVEY.md 8d camera: translation (0.64, 0.64, 2.2), rot diag(1,-1,-1)."""
    return translation_pose(0.64, 0.64, 2.2)


def display_pose(pos=(0.0, 0.0, 3.0), yaw_deg: float = 0.0, pitch_deg: float = 0.0,
                 up=(0.0, 1.0, 0.0)) -> np.ndarray:
    """include/window/displayer.h:42-52 without glm."""
    y, p = math.radians(yaw_deg), math.radians(pitch_deg)
    # rotate(yaw, Y) * rotate(pitch, X) * (0,0,-1)
    fx, fy, fz = 0.0, math.sin(p) * 1.0, -math.cos(p)
    front = np.array([math.cos(y) * fx + math.sin(y) * fz, fy, -math.sin(y) * fx + math.cos(y) * fz])
    eye = np.asarray(pos, np.float64)
    f = front / np.linalg.norm(front)
    s = np.cross(f, np.asarray(up, np.float64))
    s /= np.linalg.norm(s)
    u = np.cross(s, f)
    # inverse(lookAt) = camera-to-world with columns (s, u, -f, eye); then * diag(1,-1,-1,1)
    m = np.zeros((4, 4))  # [c][r]
    m[0, :3] = s
    m[1, :3] = -u
    m[2, :3] = f
    m[3, :3] = eye
    m[3, 3] = 1.0
    return m.astype(np.float32)
