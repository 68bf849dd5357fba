"""MI355X-native render path of randomwons/RayTracingStudy.

The product is ``librt_amd.so`` (hand-written HIP kernels for gfx950 behind
the C-ABI in ``include/rt.h``); this package is its host-side mirror of the
reference's ``KernelRenderer`` interface plus the multi-GPU tile plan.
"""
from .configs import CONFIGS, SEED, RenderConfig
from .renderer import (KernelRenderer, device_count, generate_spheres, load_spheres,
                       resize_intrinsic, save_spheres)
from .camera import default_pose, display_pose, scene_pose, translation_pose
from . import tiles

__all__ = [
    "KernelRenderer", "device_count", "generate_spheres", "resize_intrinsic",
    "save_spheres", "load_spheres",
    "default_pose", "display_pose", "scene_pose", "translation_pose",
    "CONFIGS", "SEED", "RenderConfig", "tiles",
]
