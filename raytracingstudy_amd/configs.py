"""BASELINE.json configs C1-C5 as plain data."""
from __future__ import annotations

from dataclasses import dataclass

SEED = 0x2545F491


@dataclass(frozen=True)
class RenderConfig:
    name: str
    width: int
    height: int
    spp: int
    n_spheres: int  # 0 = compat scene (root box only)
    max_depth: int  # octree depth limit (0: from the reference's resolution 0.01 -> 7)
    gpus: int
    mode: str
    note: str

    @property
    def pixels(self) -> int:
        return self.width * self.height


CONFIGS = {
    "c1": RenderConfig("c1", 256, 256, 1, 0, 7, 0, "compat",
                       "reference-compat root box, CPU scalar loop (plumbing)"),
    "c2": RenderConfig("c2", 1920, 1080, 1, 1_000, 7, 1, "scene", "1 spp, ~1k-sphere octree"),
    "c3": RenderConfig("c3", 1920, 1080, 64, 100_000, 7, 1, "scene",
                       "64 spp Monte-Carlo accumulate, ~100k spheres (headline)"),
    "c4": RenderConfig("c4", 3840, 2160, 64, 100_000, 7, 8, "scene",
                       "64 spp, 100k spheres, 64x64 tiles across 8 GPUs + RCCL gather"),
    "c5": RenderConfig("c5", 1920, 1080, 256, 1_000_000, 12, 1, "scene",
                       "256 spp, 1M spheres, depth-12 octree (compaction stress)"),
}

LIGHT_DIR = (1.0, 1.0, -1.0)  # direction the light travels (normalize(1,1,-1))
AMBIENT = 0.1
LEAF_CAPACITY = 8
TILE_SIZE = 64
