"""TEST INFRASTRUCTURE ONLY — ctypes binding of the CPU oracle (liboracle.so).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
import this package, and only as the checker / the timed CPU baseline.  The
product path (raytracingstudy_amd) never imports it.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "liboracle.so")
_lib = None

_P = ctypes.c_void_p
_u32 = ctypes.c_uint32
_f = ctypes.c_float


def build() -> None:
    subprocess.check_call(["make", "-s", "-C", _HERE])


def load() -> ctypes.CDLL:
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        build()
    lib = ctypes.CDLL(LIB_PATH)
    sig = {
        "orc_resize_intrinsic": (None, [_u32, _u32, _P]),
        "orc_get_ray": (None, [_P, _P, _f, _f, _P]),
        "orc_hit_root_box": (ctypes.c_int, [_P, _P]),
        "orc_render_compat": (None, [_u32, _u32, _P, _P, _P]),
        "orc_render_compat_fma": (None, [_u32, _u32, _P, _P, ctypes.c_int, _P]),
        "orc_generate_spheres": (None, [_u32, _u32, _P, _P]),
        "orc_sample_hash": (_u32, [_u32, _u32, _u32, _u32]),
        "orc_scene_build": (_P, [_P, _P, _u32, _P, _P, _u32, _u32]),
        "orc_scene_free": (None, [_P]),
        "orc_scene_info": (None, [_P, _P]),
        "orc_depth_for_resolution": (_u32, [_P, _P, _f]),
        "orc_scene_root": (None, [_P, _P, _P]),
        "orc_scene_export_bfs": (None, [_P, _P, _P]),
        "orc_trace": (ctypes.c_int, [_P, _P, _P, _f, _f, ctypes.c_int, _P, _P, _P]),
        "orc_trace_brute": (ctypes.c_int, [_P, _P, _P, _f, _f, ctypes.c_int, _P, _P]),
        "orc_render_scene": (None, [_P, _u32, _u32, _P, _P, _u32, _u32, _u32, _P, _f, _u32, _u32,
                                    _u32, _u32, _u32, _u32, _P, _P, _P, ctypes.c_int]),
        "orc_render_scene_frame": (None, [_P, _u32, _u32, _P, _P, _u32, _u32, _u32, _P, _f, _u32,
                                          _u32, _u32, _u32, _u32, _u32, _u32, _P, _P, _P, _P,
                                          ctypes.c_int]),
        "orc_max_threads": (ctypes.c_int, []),
        "orc_cam_screen_check": (None, [_P, _P, _P, _P, _u32, ctypes.c_double, ctypes.c_double, _P]),
        "orc_cam8_screen_check": (None, [_P, _P, _u32, _P, _P, _P, _u32, ctypes.c_double, _P]),
        "orc_shd8_screen_check": (None, [_P, _P, _P, _P, _u32, ctypes.c_double, ctypes.c_double,
                                         ctypes.c_double, ctypes.c_double, _P]),
        "orc_shd_screen_check": (None, [_P, _P, _P, _P, _u32, ctypes.c_double, ctypes.c_double,
                                        ctypes.c_double, _P]),
    }
    for name, (res, args) in sig.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


def _p(a):
    return None if a is None else ctypes.c_void_p(a.ctypes.data)


def _f32(x, n=None):
    a = np.ascontiguousarray(np.asarray(x, np.float32).reshape(-1))
    if n is not None:
        assert a.size == n
    return a


def resize_intrinsic(w: int, h: int) -> np.ndarray:
    K = np.zeros(9, np.float32)
    load().orc_resize_intrinsic(w, h, _p(K))
    return K.reshape(3, 3)


def render_compat(w: int, h: int, pose, K) -> np.ndarray:
    out = np.zeros((h, w, 4), np.uint8)
    p, k = _f32(pose, 16), _f32(K, 9)  # keep the arrays alive across the call
    load().orc_render_compat(w, h, _p(p), _p(k), _p(out))
    return out


def render_compat_fma(w: int, h: int, pose, K, contract: int) -> np.ndarray:
    """The compat image with getRay's sums FMA-contracted as nvcc would
    (contract 1: NVVM operand order, 2: the other order, 0: none)."""
    out = np.zeros((h, w, 4), np.uint8)
    p, k = _f32(pose, 16), _f32(K, 9)
    load().orc_render_compat_fma(w, h, _p(p), _p(k), int(contract), _p(out))
    return out


def get_ray(pose, K, u: float, v: float) -> np.ndarray:
    d = np.zeros(3, np.float32)
    p, k = _f32(pose, 16), _f32(K, 9)
    load().orc_get_ray(_p(p), _p(k), u, v, _p(d))
    return d


def generate_spheres(n: int, seed: int):
    sp = np.zeros((max(n, 1), 4), np.float32)
    al = np.zeros(max(n, 1), np.uint32)
    load().orc_generate_spheres(n, seed, _p(sp), _p(al))
    return sp[:n], al[:n]


class Scene:
    """Oracle octree over spheres (same build spec as the product)."""

    def __init__(self, spheres, albedo=None, root_min=(0, 0, 0), root_max=(1.28, 1.28, 1.28),
                 max_depth: int = 7, leaf_capacity: int = 8):
        lib = load()
        self.sp = np.ascontiguousarray(spheres, np.float32).reshape(-1, 4)
        self.al = None if albedo is None else np.ascontiguousarray(albedo, np.uint32)
        self.rmin = _f32(root_min, 3)
        self.rmax = _f32(root_max, 3)
        self.max_depth = max_depth
        self._h = lib.orc_scene_build(_p(self.sp), _p(self.al), self.sp.shape[0], _p(self.rmin),
                                      _p(self.rmax), max_depth, leaf_capacity)

    def info(self) -> dict:
        a = np.zeros(4, np.uint32)
        load().orc_scene_info(self._h, _p(a))
        return {"n_nodes": int(a[0]), "n_leaves": int(a[1]), "n_prim_refs": int(a[2]),
                "depth_reached": int(a[3])}

    def root(self):
        a = np.zeros(3, np.float32)
        b = np.zeros(3, np.float32)
        load().orc_scene_root(self._h, _p(a), _p(b))
        return a, b

    def export_bfs(self):
        """(nodes (n,2) uint32, prim_idx (m,) uint32) in the product's record layout."""
        inf = self.info()
        nodes = np.zeros((max(inf["n_nodes"], 1), 2), np.uint32)
        idx = np.zeros(max(inf["n_prim_refs"], 1), np.uint32)
        load().orc_scene_export_bfs(self._h, _p(nodes), _p(idx))
        return nodes[:inf["n_nodes"]], idx[:inf["n_prim_refs"]]

    def trace(self, o, d, tmin=0.0, tmax=float("inf"), any_hit=False, brute=False):
        lib = load()
        t = ctypes.c_float()
        i = ctypes.c_uint32()
        cnt = np.zeros(4, np.uint64)
        oa, da = _f32(o, 3), _f32(d, 3)  # keep the arrays alive across the call
        if brute:
            h = lib.orc_trace_brute(self._h, _p(oa), _p(da), tmin, tmax,
                                    int(any_hit), ctypes.byref(t), ctypes.byref(i))
        else:
            h = lib.orc_trace(self._h, _p(oa), _p(da), tmin, tmax, int(any_hit),
                              ctypes.byref(t), ctypes.byref(i), _p(cnt))
        return (bool(h), t.value, i.value, cnt)

    def render(self, w, h, pose, K, spp=1, seed=0x2545F491, jitter=None, shadows=True,
               light_dir=(1.0, 1.0, -1.0), ambient=0.1, rect=None, row_step=1, row_phase=0,
               n_threads=0, radiance=True, frame=0, accum=None):
        """Returns (rgba8 (h,w,4), radiance (h,w,4) or None, counters[4]).
        Progressive: pass accum (h,w,4) float32 running sums (updated in place)
        and the frame index (0 starts over)."""
        if jitter is None:
            jitter = spp > 1
        flags = (1 if jitter else 0) | (0 if shadows else 8)
        x0, y0, x1, y1 = rect if rect is not None else (0, 0, w, h)
        out8 = np.zeros((h, w, 4), np.uint8)
        out32 = np.zeros((h, w, 4), np.float32) if radiance else None
        cnt = np.zeros(4, np.uint64)
        pa, ka, la = _f32(pose, 16), _f32(K, 9), _f32(light_dir, 3)  # alive across the call
        if accum is not None:
            assert accum.dtype == np.float32 and accum.shape == (h, w, 4) and accum.flags.c_contiguous
        load().orc_render_scene_frame(self._h, w, h, _p(pa), _p(ka), spp, seed,
                                      flags, _p(la), ambient, x0, y0, x1, y1,
                                      row_step, row_phase, frame, _p(accum), _p(out8), _p(out32),
                                      _p(cnt), n_threads)
        return out8, out32, cnt

    def close(self):
        if getattr(self, "_h", None):
            load().orc_scene_free(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def max_threads() -> int:
    return int(load().orc_max_threads())


def cam_screen_check(o, dirs, spheres, idx, slack_oc: float, slack_r: float):
    """Test-only check of the product's camera-relative screen (oracle.c
    orc_cam_screen_check): (exact-accepted pairs the screen rejects, pairs
    the screen passes, pairs the exact discriminant accepts)."""
    oa = _f32(o, 3)
    d = np.ascontiguousarray(dirs, np.float32).reshape(-1, 3)
    sp = np.ascontiguousarray(spheres, np.float32).reshape(-1, 4)
    ix = np.ascontiguousarray(idx, np.uint32).reshape(-1)
    assert ix.shape[0] == d.shape[0]
    out = np.zeros(3, np.uint64)
    load().orc_cam_screen_check(_p(oa), _p(d), _p(sp), _p(ix), d.shape[0], float(slack_oc),
                                float(slack_r), _p(out))
    return int(out[0]), int(out[1]), int(out[2])


def cam8_screen_check(o, B, ok: int, dirs, spheres, idx, shrink: float = 1.0):
    """Test-only check of the product's 8-byte image-plane screen (oracle.c
    orc_cam8_screen_check): (exact-accepted pairs the screen rejects, pairs
    the screen passes, pairs the exact discriminant accepts)."""
    oa = _f32(o, 3)
    ba = _f32(B, 9)
    d = np.ascontiguousarray(dirs, np.float32).reshape(-1, 3)
    sp = np.ascontiguousarray(spheres, np.float32).reshape(-1, 4)
    ix = np.ascontiguousarray(idx, np.uint32).reshape(-1)
    assert ix.shape[0] == d.shape[0]
    out = np.zeros(3, np.uint64)
    load().orc_cam8_screen_check(_p(oa), _p(ba), int(ok), _p(d), _p(sp), _p(ix), d.shape[0],
                                 float(shrink), _p(out))
    return int(out[0]), int(out[1]), int(out[2])


def shd8_screen_check(origins, L, spheres, idx, big_m: float, slack_m: float, grow: float,
                      shrink: float = 1.0):
    """Test-only check of the light-plane screen with per-sphere radii packed
    into 8-byte records (oracle.c orc_shd8_screen_check): (exact-accepted
    pairs the screen rejects, pairs passed, pairs the exact test accepts)."""
    o = np.ascontiguousarray(origins, np.float32).reshape(-1, 3)
    la = _f32(L, 3)
    sp = np.ascontiguousarray(spheres, np.float32).reshape(-1, 4)
    ix = np.ascontiguousarray(idx, np.uint32).reshape(-1)
    assert ix.shape[0] == o.shape[0]
    out = np.zeros(3, np.uint64)
    load().orc_shd8_screen_check(_p(o), _p(la), _p(sp), _p(ix), o.shape[0], float(big_m),
                                 float(slack_m), float(grow), float(shrink), _p(out))
    return int(out[0]), int(out[1]), int(out[2])


def shd_screen_check(origins, L, spheres, idx, big_m: float, slack_m: float, grow: float):
    """Test-only check of the product's light-plane shadow screen (oracle.c
    orc_shd_screen_check): (exact-accepted pairs the screen rejects, pairs
    the screen passes, pairs the exact discriminant accepts)."""
    o = np.ascontiguousarray(origins, np.float32).reshape(-1, 3)
    la = _f32(L, 3)
    sp = np.ascontiguousarray(spheres, np.float32).reshape(-1, 4)
    ix = np.ascontiguousarray(idx, np.uint32).reshape(-1)
    assert ix.shape[0] == o.shape[0]
    out = np.zeros(3, np.uint64)
    load().orc_shd_screen_check(_p(o), _p(la), _p(sp), _p(ix), o.shape[0], float(big_m),
                                float(slack_m), float(grow), _p(out))
    return int(out[0]), int(out[1]), int(out[2])
