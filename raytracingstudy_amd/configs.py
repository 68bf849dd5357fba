"""BASELINE.json configs C1-C5 as plain data."""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np

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
    scene: str = "uniform"  # sphere generator: "uniform"  or "clustered"
    # Octree leaf capacity.  A build parameter, not part of the image: every
    # capacity gives the same pixels (nearest hit = min t then min index;
    # shadow = any hit), only the work counters move.  Measured in one process
    # per config (profiles/r03/cap_ab*.log): C3 8.82 ms at 8 -> 8.61 at 12
    # (10: 8.64, 16: 8.64, 24: 9.75; 2-6 slower), C5 54.9 -> 51.9.  C5d takes
    # 10, the largest capacity whose tree still reaches depth 12 (at 11 and 12
    # it stops at 11, and the config exists for depth 12): 26.28 -> 25.71 ms
    # (c5d_cap.log).  C2 keeps 8: 0.154 ms against 0.156 at 12 (c2_cap_ab.log).
    leaf_capacity: int = 8

    @property
    def pixels(self) -> int:
        return self.width * self.height


CONFIGS = {
    "c1": RenderConfig("c1", 256, 256, 1, 0, 7, 0, "compat",
                       "reference-compat root box, CPU scalar loop (plumbing)"),
    "c2": RenderConfig("c2", 1920, 1080, 1, 1_000, 7, 1, "scene", "1 spp, ~1k-sphere octree"),
    "c3": RenderConfig("c3", 1920, 1080, 64, 100_000, 7, 1, "scene",
                       "64 spp Monte-Carlo accumulate, ~100k spheres (headline)",
                       leaf_capacity=12),
    "c4": RenderConfig("c4", 3840, 2160, 64, 100_000, 7, 8, "scene",
                       "64 spp, 100k spheres, 64x64 tiles across 8 GPUs + RCCL gather",
                       leaf_capacity=12),
    "c5": RenderConfig("c5", 1920, 1080, 256, 1_000_000, 12, 1, "scene",
                       "256 spp, 1M spheres, depth-12 octree (compaction stress)",
                       leaf_capacity=12),
    # C5 with a tree that actually reaches depth 12 (BASELINE config 5 "deep
    # (depth-12) octree"): uniform centres stop splitting at depth 8, so the
    # same 1M spheres are drawn around 64 clusters (clustered_spheres)
    "c5d": RenderConfig("c5d", 1920, 1080, 256, 1_000_000, 12, 1, "scene",
                        "256 spp, 1M clustered spheres, octree reaching depth 12", "clustered",
                        leaf_capacity=10),
}


def clustered_spheres(n: int, seed: int = SEED, clusters: int = 64, sigma: float = 0.03):
    """n spheres around `clusters` Gaussian clusters (sd `sigma`) whose centres
    are uniform in [0.15, 1.13]^3, clipped to the root box; radii and albedo
    as SURVEY 8d D2 (0.02 (1000/n)^(1/3) U[0.5, 1]).  numpy PCG64 from `seed`:
    the same arrays on every machine.  At 1M spheres the octree (max depth 12)
    reaches depth 12 at leaf capacity 8 (1.74 M nodes, 5.8 M leaf references)
    and 10 (1.24 M, 4.9 M; the benchmarked one), not at 11 or 12."""
    g = np.random.default_rng(seed)
    centres = g.uniform(0.15, 1.13, (clusters, 3))
    which = g.integers(0, clusters, n)
    c = np.clip(centres[which] + g.normal(0.0, sigma, (n, 3)), 0.0, 1.28)
    r = 0.02 * (1000.0 / max(n, 1)) ** (1.0 / 3.0) * g.uniform(0.5, 1.0, n)
    sp = np.ascontiguousarray(np.concatenate([c, r[:, None]], 1), dtype=np.float32)
    al = (g.integers(0, 1 << 24, n, dtype=np.uint32) | np.uint32(0xFF000000)).astype(np.uint32)
    return sp, al


def scene_spheres(cfg: "RenderConfig", seed: int = SEED):
    """The sphere list of a config (its generator, its count)."""
    if cfg.scene == "clustered":
        return clustered_spheres(cfg.n_spheres, seed)
    from .renderer import generate_spheres
    return generate_spheres(cfg.n_spheres, seed)

LIGHT_DIR = (1.0, 1.0, -1.0)  # direction the light travels (normalize(1,1,-1))
AMBIENT = 0.1
LEAF_CAPACITY = 8  # the C-ABI default (rt_octree_params); configs may set their own
TILE_SIZE = 64
