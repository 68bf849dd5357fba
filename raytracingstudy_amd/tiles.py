"""Image-tile partition of one frame over ranks.

64x64 tiles, row-major ids over ceil(W/64) x ceil(H/64), dealt round-robin
(tile t -> rank t % R).  Interleaving balances the load because the scene
sits in the middle of the image.  Each rank renders its tiles into one packed
slab (``rt_render_tiles``); all slabs have the same size (padded to the
largest rank's tile count) so the gather is one equal-size collective.
"""
from __future__ import annotations

import numpy as np

__all__ = ["tile_grid", "tiles_for_rank", "slab_tiles", "pack_reference", "unpack_host", "TILE_SKIP"]

TILE_SKIP = 0xFFFFFFFF  # include/rt.h RT_TILE_SKIP: a padding slot of a gathered slab


def tile_grid(width: int, height: int, ts: int = 64):
    return (width + ts - 1) // ts, (height + ts - 1) // ts


PLANS = ("interleave", "latin")


def tiles_for_rank(width: int, height: int, rank: int, world: int, ts: int = 64,
                   plan: str = "interleave") -> np.ndarray:
    """Tile ids of one rank.

    interleave: tile t -> rank t % R (row-major ids).
    latin: the tile grid is cut into an R x R grid of compact regions and rank r
      takes region (i, (i + r) mod R) of every region row i, so it gets one
      region per region row and per region column.  The load is as
      interleaved as above, but a rank's share is R compact pieces (L2
      locality), listed region by region.
    """
    tx, ty = tile_grid(width, height, ts)
    if plan == "interleave":
        return np.arange(rank, tx * ty, world, dtype=np.uint32)
    if plan != "latin":
        raise ValueError(f"unknown tile plan {plan!r}")
    out = []
    for i in range(world):
        j = (i + rank) % world
        r0, r1 = ty * i // world, ty * (i + 1) // world
        c0, c1 = tx * j // world, tx * (j + 1) // world
        for row in range(r0, r1):
            out.extend(range(row * tx + c0, row * tx + c1))
    return np.asarray(out, dtype=np.uint32)


def slab_tiles(width: int, height: int, world: int, ts: int = 64,
               plan: str = "interleave") -> int:
    """Tile slots per rank in the equal-size gather (max over ranks)."""
    tx, ty = tile_grid(width, height, ts)
    if plan == "interleave":
        return (tx * ty + world - 1) // world
    return max(len(tiles_for_rank(width, height, k, world, ts, plan)) for k in range(world))


def pack_reference(img: np.ndarray, tile_ids, ts: int = 64) -> np.ndarray:
    """Host restatement of the packed layout (for tests): (n, ts, ts, 4) uint8."""
    H, W = img.shape[:2]
    tx, _ = tile_grid(W, H, ts)
    out = np.zeros((len(tile_ids), ts, ts, img.shape[2]), img.dtype)
    for k, t in enumerate(np.asarray(tile_ids, np.int64)):
        x0, y0 = (t % tx) * ts, (t // tx) * ts
        blk = img[y0:y0 + ts, x0:x0 + ts]
        out[k, :blk.shape[0], :blk.shape[1]] = blk
    return out


def unpack_host(packed: np.ndarray, tile_ids, width: int, height: int, ts: int = 64,
                out: np.ndarray | None = None) -> np.ndarray:
    """Host restatement of rt_unpack_tiles (for tests and CPU-only ranks)."""
    tx, _ = tile_grid(width, height, ts)
    if out is None:
        out = np.zeros((height, width, packed.shape[-1]), packed.dtype)
    packed = packed.reshape(-1, ts, ts, packed.shape[-1])
    for k, t in enumerate(np.asarray(tile_ids, np.int64)):
        if t == TILE_SKIP:
            continue
        x0, y0 = (t % tx) * ts, (t // tx) * ts
        h, w = min(ts, height - y0), min(ts, width - x0)
        out[y0:y0 + h, x0:x0 + w] = packed[k, :h, :w]
    return out
