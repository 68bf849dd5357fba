"""Host-side mirror of the reference's ``KernelRenderer`` over the C-ABI.

Reference interface (``include/renderer.cuh:25-50``)::

    KernelRenderer(cudaGraphicsResource_t cudaResource, int width, int height);
    void render();
    void resize(int width, int height);
    void setPosition(glm::mat4 pose);
    void setIntrinsic(glm::mat3 intrinsic);
    void setOctree(glm::vec3 min, glm::vec3 max, float resolution);

This class keeps those method names, argument meanings (glm column-major
matrices, pixel units) and call order, and adds what the reference left as
stubs: a real scene (``set_scene``), tiles for multi-GPU sharding, stats and
error reporting (the reference's methods return ``void`` and check nothing;
here a failing call raises ``RtError`` with the library's message).

Matrices are given in glm indexing: ``pose[c][r]`` is glm's ``m[c][r]`` (column
``c``, row ``r``), so ``pose[3][:3]`` is the camera origin
(``include/camera.h:43-46``) and ``K[0][2]``/``K[1][2]`` are cx/cy
(``include/camera.h:26-27``).  Flattening in C order yields glm's memory layout.
"""
from __future__ import annotations

import ctypes
from typing import Optional, Sequence

import numpy as np

from . import _lib
from ._lib import (RT_FLAG_HOST_BUILD, RT_FLAG_JITTER, RT_FLAG_NO_JITTER, RT_FLAG_NO_SHADOWS,
                   RT_FLAG_PROGRESSIVE, RT_FLAG_RADIANCE,
                   RT_MODE_COMPAT, RT_MODE_SCENE, RtConfig, RtOctreeParams, RtSceneInfo,
                   RtStats, check)

__all__ = ["KernelRenderer", "resize_intrinsic", "generate_spheres", "device_count",
           "save_spheres", "load_spheres"]

_MODES = {"compat": RT_MODE_COMPAT, "scene": RT_MODE_SCENE}


def _fptr(a: np.ndarray):
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_float))


def _vptr(a: Optional[np.ndarray]):
    return None if a is None else ctypes.c_void_p(a.ctypes.data)


def device_count() -> int:
    return int(_lib.load().rt_device_count())


def resize_intrinsic(width: int, height: int) -> np.ndarray:
    """K the reference's resize() sets (src/renderer.cu:162-170), glm [c][r] indexing."""
    K = np.zeros(9, np.float32)
    _lib.load().rt_resize_intrinsic(width, height, _fptr(K))
    return K.reshape(3, 3)


def generate_spheres(n: int, seed: int = 0x2545F491):
    """SURVEY.md 8d synthetic spheres: (n,4) float32 (cx,cy,cz,r) and (n,) uint32 albedo."""
    sp = np.zeros((max(n, 1), 4), np.float32)
    al = np.zeros(max(n, 1), np.uint32)
    check(_lib.load().rt_generate_spheres(n, seed, _vptr(sp), _vptr(al)))
    return sp[:n], al[:n]


def save_spheres(path: str, spheres: np.ndarray, albedo: Optional[np.ndarray] = None) -> None:
    """Write a binary sphere file (rt_save_spheres; format in DESIGN.md §4.1)."""
    sp = np.ascontiguousarray(spheres, np.float32).reshape(-1, 4)
    al = None if albedo is None else np.ascontiguousarray(albedo, np.uint32).reshape(-1)
    if al is not None and al.shape[0] != sp.shape[0]:
        raise ValueError("albedo must have one entry per sphere")
    check(_lib.load().rt_save_spheres(str(path).encode(), _vptr(sp), _vptr(al), sp.shape[0]))


def load_spheres(path: str):
    """Read a binary sphere file: ((n,4) float32 spheres, (n,) uint32 albedo)."""
    lib = _lib.load()
    n = ctypes.c_uint32(0)
    check(lib.rt_load_spheres(str(path).encode(), None, None, 0, ctypes.byref(n)))
    sp = np.zeros((max(n.value, 1), 4), np.float32)
    al = np.zeros(max(n.value, 1), np.uint32)
    check(lib.rt_load_spheres(str(path).encode(), _vptr(sp), _vptr(al), sp.shape[0],
                              ctypes.byref(n)))
    return sp[:n.value], al[:n.value]


def _octree_params(root_min, root_max, resolution, max_depth, leaf_capacity) -> RtOctreeParams:
    p = RtOctreeParams()
    for i in range(3):
        p.min[i] = float(root_min[i])
        p.max[i] = float(root_max[i])
    p.resolution = float(resolution)
    p.max_depth = int(max_depth)
    p.leaf_capacity = int(leaf_capacity)
    return p


class KernelRenderer:
    """MI355X renderer handle (one per thread / stream)."""

    def __init__(self, width: int, height: int, *, mode: str = "compat", spp: int = 1,
                 seed: int = 0x2545F491, device: int = -1, jitter: Optional[bool] = None,
                 shadows: bool = True, radiance: bool = False,
                 light_dir: Sequence[float] = (1.0, 1.0, -1.0), ambient: float = 0.1,
                 variant: int = 0, opt_off: int = 0, host_build: bool = False,
                 progressive: bool = False, cell_table: Optional[int] = None,
                 compat_fma: bool = False, pad_fill: int = 0,
                 devices: Optional[Sequence[int]] = None, transport: str = "auto"):
        """devices: render every frame across these HIP devices of this process
        (rt_create_multi: tiles round-robin, slabs gathered to devices[0] over
        RCCL or peer copies, one unpack); a repeated ordinal rehearses the plan
        on fewer GPUs.  transport: "auto", "rccl" or "peer"."""
        lib = _lib.load()
        cfg = RtConfig()
        lib.rt_config_default(ctypes.byref(cfg))
        cfg.width, cfg.height = int(width), int(height)
        cfg.spp = int(spp)
        cfg.seed = int(seed) & 0xFFFFFFFF
        cfg.device = int(device)
        cfg.mode = _MODES[mode]
        flags = 0
        if jitter is True:
            flags |= RT_FLAG_JITTER
        elif jitter is False:
            flags |= RT_FLAG_NO_JITTER
        if not shadows:
            flags |= RT_FLAG_NO_SHADOWS
        if radiance:
            flags |= RT_FLAG_RADIANCE
        if host_build:
            flags |= RT_FLAG_HOST_BUILD
        if progressive:
            flags |= RT_FLAG_PROGRESSIVE
        if compat_fma:
            flags |= _lib.RT_FLAG_COMPAT_FMA
        # pad_fill (test-only): 0 zeros, 1 NaN, 2 covering spheres after the last leaf list
        if not 0 <= int(pad_fill) <= 2:
            raise ValueError("pad_fill must be 0, 1 or 2")
        flags |= int(pad_fill) << _lib.RT_FLAG_PAD_FILL_SHIFT
        flags |= (int(variant) & 0xF) << _lib.RT_FLAG_VARIANT_SHIFT
        flags |= (int(opt_off) & 0xFF) << _lib.RT_FLAG_OPT_SHIFT
        # cell_table: None = depth chosen from the tree, 0 = no table, k = depth k
        if cell_table is not None:
            ct = _lib.RT_CELL_TABLE_OFF if int(cell_table) == 0 else int(cell_table)
            if not 1 <= ct <= 15:
                raise ValueError("cell_table must be None, 0 (off) or a depth 1..7")
            flags |= ct << _lib.RT_FLAG_CELL_TABLE_SHIFT
        cfg.flags = flags | _lib.test_flags
        for i in range(3):
            cfg.light_dir[i] = float(light_dir[i])
        cfg.ambient = float(ambient)
        self._lib = lib
        self.config = cfg
        self.mode = mode
        self.radiance = radiance
        h = ctypes.c_void_p()
        if devices is None:
            check(lib.rt_create(ctypes.byref(cfg), ctypes.byref(h)))
        else:
            tr = {"auto": _lib.RT_TRANSPORT_AUTO, "rccl": _lib.RT_TRANSPORT_RCCL,
                  "peer": _lib.RT_TRANSPORT_PEER}[transport]
            devs = (ctypes.c_int32 * len(devices))(*[int(d) for d in devices])
            check(lib.rt_create_multi(ctypes.byref(cfg), devs, len(devices), tr, ctypes.byref(h)))
        self._h = h
        self.width, self.height = int(width), int(height)

    # -- reference method names -------------------------------------------------
    def render(self, dev_ptr: Optional[int] = None, stream: Optional[int] = None,
               stats: bool = False) -> Optional[RtStats]:
        """render() (src/renderer.cu:143-153).  dev_ptr: a device RGBA8 buffer
        (e.g. the mapped GL PBO pointer) or None for the internal framebuffer."""
        st = RtStats() if stats else None
        check(self._lib.rt_render(self._h, ctypes.c_void_p(dev_ptr) if dev_ptr else None,
                                  ctypes.c_void_p(stream) if stream else None,
                                  ctypes.byref(st) if st is not None else None), self._h)
        return st

    def resize(self, width: int, height: int) -> None:
        """resize() (src/renderer.cu:155-187): new size + the FOV-80 intrinsic."""
        check(self._lib.rt_resize(self._h, int(width), int(height)), self._h)
        self.width, self.height = int(width), int(height)

    def setPosition(self, pose) -> None:
        """setPosition(glm::mat4) (src/renderer.cu:111-113, include/camera.h:43-46)."""
        p = np.ascontiguousarray(np.asarray(pose, np.float32).reshape(16))
        check(self._lib.rt_set_pose(self._h, _fptr(p)), self._h)

    def setIntrinsic(self, K) -> None:
        """setIntrinsic(glm::mat3) (src/renderer.cu:115-117)."""
        k = np.ascontiguousarray(np.asarray(K, np.float32).reshape(9))
        check(self._lib.rt_set_intrinsic(self._h, _fptr(k)), self._h)

    def setOctree(self, mn, mx, resolution: float) -> None:
        """setOctree(min, max, resolution) (include/renderer.cuh:35; undefined in
        the reference).  Rebuilds the octree of the current spheres."""
        a = np.asarray(mn, np.float32).reshape(3).copy()
        b = np.asarray(mx, np.float32).reshape(3).copy()
        check(self._lib.rt_set_octree(self._h, _fptr(a), _fptr(b), float(resolution)), self._h)

    # -- additions ------------------------------------------------------------
    def bind_display(self, map_fn=None, unmap_fn=None) -> None:
        """A display buffer mapped per frame (rt_bind_display): the
        reference's render() maps its PBO, renders into it and unmaps it
        (src/renderer.cu:145-151).  map_fn(stream) -> (device_ptr, nbytes) or
        None (failure); unmap_fn(stream) -> None, or False on failure.  Called
        with no arguments it unbinds (render into the internal framebuffer)."""
        if map_fn is None:
            self._display = None
            check(self._lib.rt_bind_display(self._h, None, None), self._h)
            return

        def _map(_user, stream, ptr, nbytes):
            try:
                got = map_fn(stream or 0)
            except Exception:  # an exception must not unwind through C
                return 1
            if got is None:
                return 1
            ptr[0], nbytes[0] = int(got[0]), int(got[1])
            return 0

        def _unmap(_user, stream):
            try:
                return 1 if unmap_fn(stream or 0) is False else 0
            except Exception:
                return 1

        ops = _lib.RtDisplayOps(_lib.DISPLAY_MAP(_map), _lib.DISPLAY_UNMAP(_unmap))
        self._display = ops  # the C side keeps raw function pointers: keep them alive
        check(self._lib.rt_bind_display(self._h, ctypes.byref(ops), None), self._h)

    def set_scene(self, spheres: np.ndarray, albedo: Optional[np.ndarray] = None, *,
                  root_min=(0.0, 0.0, 0.0), root_max=(1.28, 1.28, 1.28),
                  resolution: float = 0.01, max_depth: int = 0, leaf_capacity: int = 8) -> dict:
        sp = np.ascontiguousarray(spheres, np.float32).reshape(-1, 4)
        al = None if albedo is None else np.ascontiguousarray(albedo, np.uint32).reshape(-1)
        if al is not None and al.shape[0] != sp.shape[0]:
            raise ValueError("albedo must have one entry per sphere")
        p = _octree_params(root_min, root_max, resolution, max_depth, leaf_capacity)
        check(self._lib.rt_set_scene(self._h, _vptr(sp), _vptr(al), sp.shape[0], ctypes.byref(p)),
              self._h)
        return self.scene_info()

    def set_scene_device(self, spheres_ptr: int, n: int, albedo_ptr: Optional[int] = None, *,
                         stream: Optional[int] = None, root_min=(0.0, 0.0, 0.0),
                         root_max=(1.28, 1.28, 1.28), resolution: float = 0.01,
                         max_depth: int = 0, leaf_capacity: int = 8) -> dict:
        """Scene from a sphere list already in device memory (4*n float32 at
        spheres_ptr, n RGBA8 words at albedo_ptr); the octree is built on the GPU."""
        p = _octree_params(root_min, root_max, resolution, max_depth, leaf_capacity)
        check(self._lib.rt_set_scene_device(
            self._h, ctypes.c_void_p(spheres_ptr) if spheres_ptr else None,
            ctypes.c_void_p(albedo_ptr) if albedo_ptr else None, int(n), ctypes.byref(p),
            ctypes.c_void_p(stream) if stream else None), self._h)
        return self.scene_info()

    def set_scene_file(self, path: str, **octree) -> dict:
        """Load a binary sphere file (load_spheres) and make it the scene."""
        sp, al = load_spheres(path)
        return self.set_scene(sp, al, **octree)

    def export_octree(self):
        """The device octree as host arrays: nodes (n,2) uint32 records, prim_sp
        (m,4) float32, prim_idx (m,) uint32 (rt_export_octree)."""
        info = self.scene_info()
        nodes = np.zeros((max(info["n_nodes"], 1), 2), np.uint32)
        m = info["n_prim_refs"]
        sp = np.zeros((max(m, 1), 4), np.float32)
        idx = np.zeros(max(m, 1), np.uint32)
        check(self._lib.rt_export_octree(self._h, _vptr(nodes), _vptr(sp), _vptr(idx)), self._h)
        return nodes[:info["n_nodes"]], sp[:m], idx[:m]

    def scene_info(self) -> dict:
        info = RtSceneInfo()
        check(self._lib.rt_get_scene_info(self._h, ctypes.byref(info)), self._h)
        return info.as_dict()

    def multi_info(self) -> dict:
        """rt_get_multi_info: the devices, transport and tile plan of the handle
        (n_devices 1 for a single-device renderer)."""
        info = _lib.RtMultiInfo()
        check(self._lib.rt_get_multi_info(self._h, ctypes.byref(info)), self._h)
        return info.as_dict()

    def multi_timing(self) -> dict:
        """rt_get_multi_timing: per-device render ms of the last frame (HIP
        events on each device's render stream) and devices[0]'s delivery ms
        (its own tiles' end -> the frame unpacked).  Waits for the handle."""
        t = _lib.RtMultiTiming()
        check(self._lib.rt_get_multi_timing(self._h, ctypes.byref(t)), self._h)
        return t.as_dict()

    def camera(self):
        pose = np.zeros(16, np.float32)
        K = np.zeros(9, np.float32)
        check(self._lib.rt_get_camera(self._h, _fptr(pose), _fptr(K)), self._h)
        return pose.reshape(4, 4), K.reshape(3, 3)

    def render_tiles(self, tile_ids, tile_size: int, dev_ptr: int, stream: Optional[int] = None,
                     stats: bool = False) -> Optional[RtStats]:
        ids = np.ascontiguousarray(tile_ids, np.uint32)
        st = RtStats() if stats else None
        check(self._lib.rt_render_tiles(self._h, _vptr(ids), ids.shape[0], int(tile_size),
                                        ctypes.c_void_p(dev_ptr),
                                        ctypes.c_void_p(stream) if stream else None,
                                        ctypes.byref(st) if st is not None else None), self._h)
        return st

    def unpack_tiles(self, dev_packed: int, tile_ids, tile_size: int,
                     dev_rgba8: Optional[int] = None, stream: Optional[int] = None) -> None:
        ids = np.ascontiguousarray(tile_ids, np.uint32)
        check(self._lib.rt_unpack_tiles(self._h, ctypes.c_void_p(dev_packed), _vptr(ids),
                                        ids.shape[0], int(tile_size),
                                        ctypes.c_void_p(dev_rgba8) if dev_rgba8 else None,
                                        ctypes.c_void_p(stream) if stream else None), self._h)

    def reset_accumulation(self) -> None:
        """Progressive mode: the next frame starts from zero samples."""
        check(self._lib.rt_reset_accumulation(self._h), self._h)

    def synchronize(self) -> None:
        check(self._lib.rt_synchronize(self._h), self._h)

    def readback(self) -> np.ndarray:
        out = np.zeros((self.height, self.width, 4), np.uint8)
        check(self._lib.rt_readback(self._h, _vptr(out), None), self._h)
        return out

    def readback_radiance(self) -> np.ndarray:
        out = np.zeros((self.height, self.width, 4), np.float32)
        check(self._lib.rt_readback(self._h, None, _vptr(out)), self._h)
        return out

    def stream_ptr(self) -> int:
        """The renderer's own hipStream_t (what stream=None means)."""
        return int(self._lib.rt_stream(self._h) or 0)

    def framebuffer_ptr(self) -> int:
        return int(self._lib.rt_framebuffer(self._h) or 0)

    def close(self) -> None:
        if getattr(self, "_h", None):
            self._lib.rt_destroy(self._h)
            self._h = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
