"""ctypes binding of the C-ABI in ``include/rt.h`` (``librt_amd.so``).

The shared library is the product: the HIP kernels for gfx950 plus the host
runtime.  There is no fallback — if the library is missing or fails to load,
``load()`` raises, and every render entry point raises with the library's own
error message when a call fails.
"""
from __future__ import annotations

import ctypes
import os
import threading

_HERE = os.path.dirname(os.path.abspath(__file__))
# RT_AMD_LIB: load another build of the library (A/B of two builds on one box)
LIB_PATH = os.environ.get("RT_AMD_LIB") or os.path.join(_HERE, "librt_amd.so")

RT_OK = 0
RT_E_INVALID = -1
RT_E_HIP = -2
RT_E_NOMEM = -3
RT_E_NOSCENE = -4
RT_E_STATE = -5

RT_MODE_COMPAT = 0
RT_MODE_SCENE = 1

RT_FLAG_JITTER = 1 << 0
RT_FLAG_NO_JITTER = 1 << 1
RT_FLAG_RADIANCE = 1 << 2
RT_FLAG_NO_SHADOWS = 1 << 3
RT_FLAG_HOST_BUILD = 1 << 4
RT_FLAG_PROGRESSIVE = 1 << 5
RT_FLAG_COMPAT_FMA = 1 << 6
RT_BUILDER_DEVICE = 0
RT_BUILDER_HOST = 1
RT_TILE_SKIP = 0xFFFFFFFF  # rt_unpack_tiles: a padding slot, not copied
RT_FLAG_PAD_FILL_SHIFT = 8  # test-only: 0 zeros, 1 NaN, 2 covering spheres after the last leaf
RT_FLAG_TEST_HOOKS = 1 << 10   # test-only: honour the RT_TEST_* environment variables
RT_FLAG_TEST_POISON = 1 << 11  # test-only: sentinel-fill every frame's outputs first
RT_FLAG_VARIANT_SHIFT = 16
RT_FLAG_OPT_SHIFT = 20
RT_FLAG_CELL_TABLE_SHIFT = 28
RT_CELL_TABLE_OFF = 15
VARIANT_REMOVED = 2  # a removed variant number (the packet walk): rt_create refuses it
VARIANT_BLOCK = 7   # unified walk, block-tile queue (default for spp < 8)
VARIANT_WAVEQ = 13  # unified walk, per-wave per-XCD queues (default for spp >= 8)
VARIANT_WAVEQ_LOW = 4  # the same queue for spp < 8 (default for spp < 8 since round 4)
RT_TRANSPORT_AUTO = 0
RT_TRANSPORT_RCCL = 1
RT_TRANSPORT_PEER = 2
RT_MAX_DEVICES = 16

_f3 = ctypes.c_float * 3


class RtConfig(ctypes.Structure):
    _fields_ = [
        ("width", ctypes.c_uint32),
        ("height", ctypes.c_uint32),
        ("spp", ctypes.c_uint32),
        ("seed", ctypes.c_uint32),
        ("device", ctypes.c_int32),
        ("mode", ctypes.c_uint32),
        ("flags", ctypes.c_uint32),
        ("light_dir", _f3),
        ("ambient", ctypes.c_float),
    ]


class RtOctreeParams(ctypes.Structure):
    _fields_ = [
        ("min", _f3),
        ("max", _f3),
        ("resolution", ctypes.c_float),
        ("max_depth", ctypes.c_uint32),
        ("leaf_capacity", ctypes.c_uint32),
    ]


class RtStats(ctypes.Structure):
    _fields_ = [
        ("primary_rays", ctypes.c_uint64),
        ("shadow_rays", ctypes.c_uint64),
        ("nodes_visited", ctypes.c_uint64),
        ("prims_tested", ctypes.c_uint64),
        ("ms", ctypes.c_float),
        ("samples_per_pixel", ctypes.c_uint32),
    ]

    def as_dict(self) -> dict:
        return {f: getattr(self, f) for f, _ in self._fields_}


class RtSceneInfo(ctypes.Structure):
    _fields_ = [
        ("n_spheres", ctypes.c_uint32),
        ("n_nodes", ctypes.c_uint32),
        ("n_leaves", ctypes.c_uint32),
        ("n_prim_refs", ctypes.c_uint32),
        ("max_depth", ctypes.c_uint32),
        ("depth_reached", ctypes.c_uint32),
        ("node_bytes", ctypes.c_uint32),
        ("prim_bytes", ctypes.c_uint32),
        ("root_min", _f3),
        ("root_max", _f3),
        ("build_ms", ctypes.c_double),
        ("upload_ms", ctypes.c_double),
        ("builder", ctypes.c_uint32),
        ("cell_table_depth", ctypes.c_uint32),
    ]

    def as_dict(self) -> dict:
        d = {f: getattr(self, f) for f, _ in self._fields_}
        d["builder"] = "host" if self.builder == RT_BUILDER_HOST else "device"
        d["root_min"] = list(self.root_min)
        d["root_max"] = list(self.root_max)
        return d


# rt_display_ops: int map(void* user, void* stream, void** ptr, size_t* bytes),
# int unmap(void* user, void* stream)
DISPLAY_MAP = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p,
                               ctypes.POINTER(ctypes.c_void_p), ctypes.POINTER(ctypes.c_size_t))
DISPLAY_UNMAP = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p)


class RtMultiInfo(ctypes.Structure):
    _fields_ = [
        ("n_devices", ctypes.c_uint32),
        ("devices", ctypes.c_int32 * 16),
        ("transport", ctypes.c_uint32),
        ("tile_size", ctypes.c_uint32),
        ("slab_tiles", ctypes.c_uint32),
        ("frames_in_flight", ctypes.c_uint32),
        ("frames", ctypes.c_uint64),
    ]

    def as_dict(self) -> dict:
        n = int(self.n_devices)
        return {"n_devices": n, "devices": [int(self.devices[i]) for i in range(n)],
                "transport": {0: "single", 1: "rccl", 2: "peer"}.get(int(self.transport), "?"),
                "tile_size": int(self.tile_size), "slab_tiles": int(self.slab_tiles),
                "frames_in_flight": int(self.frames_in_flight), "frames": int(self.frames)}


class RtMultiTiming(ctypes.Structure):
    _fields_ = [
        ("n_devices", ctypes.c_uint32),
        ("frame", ctypes.c_uint64),
        ("render_ms", ctypes.c_float * 16),
        ("deliver_ms", ctypes.c_float),
    ]

    def as_dict(self) -> dict:
        n = int(self.n_devices)
        return {"n_devices": n, "frame": int(self.frame),
                "render_ms": [round(float(self.render_ms[i]), 4) for i in range(n)],
                "deliver_ms": round(float(self.deliver_ms), 4)}


class RtDisplayOps(ctypes.Structure):
    _fields_ = [("map", DISPLAY_MAP), ("unmap", DISPLAY_UNMAP)]


# every symbol declared in include/rt.h, with (restype, argtypes)
_P = ctypes.c_void_p
_u32 = ctypes.c_uint32
_int = ctypes.c_int
_fp = ctypes.POINTER(ctypes.c_float)
SIGNATURES = {
    "rt_abi_version": (_int, []),
    "rt_device_count": (_int, []),
    "rt_config_default": (None, [ctypes.POINTER(RtConfig)]),
    "rt_octree_params_default": (None, [ctypes.POINTER(RtOctreeParams)]),
    "rt_create": (_int, [ctypes.POINTER(RtConfig), ctypes.POINTER(_P)]),
    "rt_destroy": (_int, [_P]),
    "rt_set_pose": (_int, [_P, _fp]),
    "rt_set_intrinsic": (_int, [_P, _fp]),
    "rt_get_camera": (_int, [_P, _fp, _fp]),
    "rt_resize": (_int, [_P, _u32, _u32]),
    "rt_resize_intrinsic": (None, [_u32, _u32, _fp]),
    "rt_set_scene": (_int, [_P, _P, _P, _u32, ctypes.POINTER(RtOctreeParams)]),
    "rt_set_scene_device": (_int, [_P, _P, _P, _u32, ctypes.POINTER(RtOctreeParams), _P]),
    "rt_set_octree": (_int, [_P, _fp, _fp, ctypes.c_float]),
    "rt_get_scene_info": (_int, [_P, ctypes.POINTER(RtSceneInfo)]),
    "rt_export_octree": (_int, [_P, _P, _P, _P]),
    "rt_save_spheres": (_int, [ctypes.c_char_p, _P, _P, _u32]),
    "rt_load_spheres": (_int, [ctypes.c_char_p, _P, _P, _u32, ctypes.POINTER(_u32)]),
    "rt_generate_spheres": (_int, [_u32, _u32, _P, _P]),
    "rt_render": (_int, [_P, _P, _P, ctypes.POINTER(RtStats)]),
    "rt_bind_graphics_resource": (_int, [_P, _P]),
    "rt_bind_display": (_int, [_P, ctypes.POINTER(RtDisplayOps), _P]),
    "rt_render_tiles": (_int, [_P, _P, _u32, _u32, _P, _P, ctypes.POINTER(RtStats)]),
    "rt_unpack_tiles": (_int, [_P, _P, _P, _u32, _u32, _P, _P]),
    "rt_reset_accumulation": (_int, [_P]),
    "rt_synchronize": (_int, [_P]),
    "rt_readback": (_int, [_P, _P, _P]),
    "rt_framebuffer": (_P, [_P]),
    "rt_stream": (_P, [_P]),
    "rt_last_error": (ctypes.c_char_p, [_P]),
    "rt_create_multi": (_int, [ctypes.POINTER(RtConfig), ctypes.POINTER(ctypes.c_int32), _u32, _u32,
                               ctypes.POINTER(_P)]),
    "rt_get_multi_info": (_int, [_P, ctypes.POINTER(RtMultiInfo)]),
    "rt_get_multi_timing": (_int, [_P, ctypes.POINTER(RtMultiTiming)]),
}

_lock = threading.Lock()
_lib = None

# Flags OR-ed into every renderer's rt_config by KernelRenderer.  0 in the
# product; the test suite sets RT_FLAG_TEST_HOOKS | RT_FLAG_TEST_POISON
# (tests/conftest.py), so every frame it renders starts from a sentinel-filled
# framebuffer and the RT_TEST_* hooks are honoured.
test_flags = 0

# the sources the scene kernel's machine code is built from (device code and
# its compile flags): a PMC summary is valid for a build iff its stamp matches
KERNEL_SOURCES = ("csrc/rt_kernels.hip", "csrc/rt_params.h", "csrc/Makefile")


def kernel_source_id() -> str:
    """sha256 (first 16 hex digits) of KERNEL_SOURCES with comments and
    whitespace removed: stamps profiles/ PMC summaries (tools/pmc_traffic.py)
    so bench.py uses counters only for the kernel code they were collected on."""
    import hashlib
    import re
    h = hashlib.sha256()
    for rel in KERNEL_SOURCES:
        with open(os.path.join(_HERE, rel), encoding="utf-8") as f:
            src = f.read()
        # code only: comments and layout do not change the machine code
        src = re.sub(r"/\*.*?\*/", " ", src, flags=re.S)
        src = re.sub(r"//[^\n]*", " ", src)
        if rel.endswith("Makefile"):
            src = re.sub(r"#[^\n]*", " ", src)
        src = " ".join(src.split())
        h.update(rel.encode() + b"\0" + src.encode())
    return h.hexdigest()[:16]


class RtError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"rt error {code}: {msg}")
        self.code = code


def load() -> ctypes.CDLL:
    """Load librt_amd.so (raises if it is missing: there is no fallback)."""
    global _lib
    with _lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(LIB_PATH):
            raise ImportError(
                f"{LIB_PATH} is missing: build it with `python -c 'import __graft_entry__ as g; g.build()'`"
                " (or `make -C raytracingstudy_amd/csrc`); the render path has no CPU fallback")
        lib = ctypes.CDLL(LIB_PATH, mode=ctypes.RTLD_GLOBAL)
        for name, (res, args) in SIGNATURES.items():
            # an RT_AMD_LIB override (A/B against an older build) may predate
            # some entry points; the in-tree library must export all of them
            if os.environ.get("RT_AMD_LIB") and not hasattr(lib, name):
                continue
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        _lib = lib
        return lib


def check(code: int, handle=None) -> None:
    if code != RT_OK:
        lib = load()
        msg = lib.rt_last_error(handle)
        raise RtError(code, msg.decode() if msg else "")
