"""Camera controls and stats panel of the reference's window, over the C-ABI.

Python mirror of ``include/rt_camera.hpp``: the Displayer's
input state machine (``include/window/displayer.h:20-83``) and the numbers of
its ImGui panel (``src/window/window.cpp:137-150``) plus the renderer's own
(Mrays/s, samples per pixel, GPUs).  A window toolkit reports key states and
mouse events; ``process_input`` moves the camera and pushes the pose through
``KernelRenderer.setPosition`` (rt_set_pose).
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field
from typing import Optional

import numpy as np

__all__ = ["Keys", "CameraController", "StatsPanel"]


@dataclass
class Keys:
    w: bool = False
    a: bool = False
    s: bool = False
    d: bool = False
    space: bool = False
    shift: bool = False


def _norm(v):
    return v / np.linalg.norm(v)


@dataclass
class CameraController:
    MOVE = 0.01  # displayer.h:22
    TURN = 0.3   # displayer.h:71
    pos: np.ndarray = field(default_factory=lambda: np.array([0.0, 0.0, 3.0]))
    front: np.ndarray = field(default_factory=lambda: np.array([0.0, 0.0, -1.0]))
    up: np.ndarray = field(default_factory=lambda: np.array([0.0, 1.0, 0.0]))
    yaw: float = 0.0
    pitch: float = 0.0
    control: bool = False
    prev_mouse: tuple = (0.0, 0.0)

    def process_input(self, keys: Keys, renderer=None) -> np.ndarray:
        """displayer.h:20-55: move along front / right / up, refresh front from
        yaw and pitch, return the pose (and set it on the renderer if given)."""
        if keys.w:
            self.pos = self.pos + self.MOVE * self.front
        if keys.s:
            self.pos = self.pos - self.MOVE * self.front
        right = _norm(np.cross(self.up, -self.front))
        if keys.d:
            self.pos = self.pos + self.MOVE * right
        if keys.a:
            self.pos = self.pos - self.MOVE * right
        cam_up = _norm(np.cross(-self.front, right))
        if keys.space:
            self.pos = self.pos + (-self.MOVE if keys.shift else self.MOVE) * cam_up
        ry, rp = math.radians(self.yaw), math.radians(self.pitch)
        self.front = np.array([math.sin(ry) * -math.cos(rp), math.sin(rp),
                               math.cos(ry) * -math.cos(rp)])
        p = self.pose()
        if renderer is not None:
            renderer.setPosition(p)
        return p

    def mouse_button(self, right_button: bool, press: bool, x: float, y: float) -> None:
        """displayer.h:57-67."""
        if not right_button:
            return
        if press:
            self.prev_mouse = (float(x), float(y))
            self.control = True
        else:
            self.control = False

    def mouse_move(self, x: float, y: float) -> None:
        """displayer.h:69-83: yaw wraps to [0, 360], pitch clamps to +-89."""
        if not self.control:
            return
        self.yaw -= (float(x) - self.prev_mouse[0]) * self.TURN
        self.pitch -= (float(y) - self.prev_mouse[1]) * self.TURN
        if self.yaw < 0.0:
            self.yaw += 360.0
        if self.yaw > 360.0:
            self.yaw -= 360.0
        self.pitch = min(89.0, max(-89.0, self.pitch))
        self.prev_mouse = (float(x), float(y))

    def pose(self) -> np.ndarray:
        """inverse(lookAt(pos, pos + front, up)) * diag(1,-1,-1,1), glm [c][r]."""
        f = _norm(self.front)
        s = _norm(np.cross(f, self.up))
        u = np.cross(s, f)
        m = np.zeros((4, 4))
        m[0, :3], m[1, :3], m[2, :3], m[3, :3] = s, -u, f, self.pos
        m[3, 3] = 1.0
        return m.astype(np.float32)


@dataclass
class StatsPanel:
    elapsed_s: float = 0.0
    fps: float = 0.0
    frames: int = 0
    mrays_s: float = 0.0
    spp: int = 0
    gpus: int = 1

    def update(self, frame_ms: float, stats, n_gpus: int = 1) -> None:
        """One call per frame with its wall time and the renderer's RtStats."""
        self.elapsed_s += frame_ms * 1e-3
        self.fps = 1e3 / frame_ms if frame_ms > 0 else 0.0
        self.frames += 1
        rays = stats.primary_rays + stats.shadow_rays
        self.mrays_s = rays / (stats.ms * 1e3) if stats.ms > 0 else 0.0
        self.spp = stats.samples_per_pixel
        self.gpus = n_gpus

    def text(self) -> str:
        return (f"Elapsed Time {self.elapsed_s:f}\nFPS {self.fps:f}\nframes {self.frames}\n"
                f"Mrays/s {self.mrays_s:.1f}\nspp {self.spp}\nGPUs {self.gpus}\n")
