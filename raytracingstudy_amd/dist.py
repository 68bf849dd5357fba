"""Multi-GPU frame sharding: one process per GPU, tiles + gather to rank 0.

SURVEY.md 8e: 64x64 tiles dealt round-robin over R ranks; each rank renders
its tiles into a packed slab (``rt_render_tiles``); rank 0 gathers the
equal-size slabs over RCCL (``torch.distributed.gather``: on the nccl backend
each peer's slab travels over its own xGMI link to rank 0) and scatters them
into the frame (``rt_unpack_tiles``).  The scene is replicated: every rank
builds it from the same seed, so there is no broadcast.

The class is backend-agnostic: the GPU path passes CUDA tensors and the
renderer's unpack kernel; the CPU tests use gloo with host tensors.
"""
from __future__ import annotations

from typing import Callable, List, Optional

import numpy as np

from . import tiles as T

__all__ = ["TileSharder", "TileFramePipeline", "rank_timing_report"]


class TileSharder:
    def __init__(self, width: int, height: int, rank: int, world: int, tile_size: int = 64,
                 channels: int = 4):
        self.width, self.height = int(width), int(height)
        self.rank, self.world = int(rank), int(world)
        self.ts = int(tile_size)
        self.channels = channels
        self.all_ids: List[np.ndarray] = [T.tiles_for_rank(width, height, k, world, tile_size)
                                          for k in range(world)]
        self.ids = self.all_ids[self.rank]
        self.slab_tiles = T.slab_tiles(width, height, world, tile_size)
        self.slab_elems = self.slab_tiles * self.ts * self.ts * channels
        # every rank's ids padded to the slab size with RT_TILE_SKIP: the
        # gathered slabs, end to end in one buffer, unpack in ONE call
        self.all_ids_padded = np.full(self.world * self.slab_tiles, T.TILE_SKIP, np.uint32)
        for k, ids in enumerate(self.all_ids):
            self.all_ids_padded[k * self.slab_tiles:k * self.slab_tiles + len(ids)] = ids

    def new_slab(self, torch_mod, device=None, dtype=None):
        """Zeroed packed slab for this rank (uint8 RGBA by default)."""
        dtype = dtype if dtype is not None else torch_mod.uint8
        return torch_mod.zeros(self.slab_elems, dtype=dtype, device=device)

    def gather(self, slab, group=None, slot: int = 0, async_op: bool = False):
        """Equal-size gather of every rank's slab to rank 0; returns the list on rank 0.
        The receive buffers are allocated once per `slot` (one per frame in
        flight) and reused every frame.  async_op: return (list, work), where
        work.wait() orders the caller's current stream after the collective
        (None when nothing is left to wait for)."""
        if self.world == 1:
            return ([slab], None) if async_op else [slab]
        import torch
        import torch.distributed as dist
        # gloo moves host tensors only: device slabs are staged through host
        # memory (rehearsal of the multi-rank path; RCCL gathers device slabs)
        staged = slab.is_cuda and dist.get_backend(group) == "gloo"
        src = slab.cpu() if staged else slab
        out = None
        if self.rank == 0:
            key = (tuple(src.shape), src.dtype, src.device)
            bufs = self.__dict__.setdefault("_recv_bufs", {})
            if slot not in bufs or bufs[slot][0] != key:
                # the receive slabs are views of ONE buffer (unpack_fused)
                buf = torch.empty((self.world,) + tuple(src.shape), dtype=src.dtype,
                                  device=src.device)
                bufs[slot] = (key, buf, list(buf.unbind(0)))
            out = bufs[slot][2]
        work = dist.gather(src, out, dst=0, group=group, async_op=async_op and not staged)
        if staged and out is not None:
            out = [t.to(slab.device) for t in out]
        return (out, work) if async_op else out

    def unpack_fused(self, gathered, unpack_fn: Callable[[object, np.ndarray], None]) -> None:
        """Rank 0: ONE unpack_fn(buffer, all_ids_padded) call over every rank's
        slab, end to end in one contiguous buffer (padding slots are
        RT_TILE_SKIP), instead of one call per rank."""
        if self.rank != 0:
            return
        import torch
        for _, buf, _ in getattr(self, "_recv_bufs", {}).values():
            if gathered[0].data_ptr() == buf.data_ptr():
                break
        else:
            buf = torch.stack(list(gathered))  # staged (gloo) slabs: make them contiguous
        unpack_fn(buf, self.all_ids_padded)

    def unpack(self, gathered, unpack_fn: Callable[[object, np.ndarray], None]) -> None:
        """Rank 0: call unpack_fn(slab_k, tile_ids_k) for every rank's slab."""
        if self.rank != 0:
            return
        for k in range(self.world):
            unpack_fn(gathered[k], self.all_ids[k])

    def unpack_host(self, gathered, out: Optional[np.ndarray] = None) -> np.ndarray:
        """CPU restatement of the unpack (tests / host-only ranks)."""
        if out is None:
            out = np.zeros((self.height, self.width, self.channels), np.uint8)
        for k in range(self.world):
            ids = self.all_ids[k]
            packed = np.asarray(gathered[k].cpu().numpy()).reshape(-1, self.ts, self.ts, self.channels)
            T.unpack_host(packed[:len(ids)], ids, self.width, self.height, self.ts, out)
        return out


class TileFramePipeline:
    """One step of the multi-GPU tile path, with F frames in flight: exactly
    what bench.py times on every rank, and what tests/test_tiles_dist.py
    drives with gloo on CPU.

    Frame i uses slot k = i mod F (its own renderer, stream, slab, receive
    buffer and frame).  step(i):
      1. ``render(k, slab_k)``: this rank's tiles into slot k's packed slab;
      2. ``sharder.gather(slab_k, slot=k, async_op=True)``: the equal-size
         slabs to rank 0 (on the nccl backend RCCL's stream waits for the
         render on slot k's stream);
      3. ``work.wait()``: slot k's stream waits for the gather, so rank 0's
         unpack and every rank's next render into slab k come after it;
      4. rank 0: ONE ``unpack(k, buffer, ids)`` over all ranks' slabs
         (``TileSharder.unpack_fused``, padding slots skipped).
    ``stream(k)`` returns a context manager that makes slot k's stream
    current (``torch.cuda.stream``), or None on CPU.  ``gather=False``
    renders only (a local projection of one rank's share, no collective).
    ``on_render(k, phase)`` is called with phase 0 / 1 right before / after
    the render call, and with phase 2 once the step's gather and unpack are
    enqueued (bench.py records its HIP events there: 0 -> 1 is the render,
    1 -> 2 the gather + unpack as slot k's stream sees them).
    """

    def __init__(self, sharder: TileSharder, slabs, render: Callable, unpack: Callable,
                 stream: Optional[Callable] = None, gather: bool = True,
                 on_render: Optional[Callable] = None, group=None):
        self.sharder = sharder
        self.slabs = list(slabs)
        self.frames_in_flight = len(self.slabs)
        self.render = render
        self.unpack = unpack
        self.stream = stream
        self.do_gather = gather
        self.on_render = on_render
        self.group = group
        self.last_work = None  # the collective's Work of the last step (tests)

    def step(self, i: int) -> None:
        k = i % self.frames_in_flight
        ctx = self.stream(k) if self.stream is not None else None
        if ctx is not None:
            with ctx:
                self._step(k)
        else:
            self._step(k)

    def _step(self, k: int) -> None:
        slab = self.slabs[k]
        if self.on_render is not None:
            self.on_render(k, 0)
        self.render(k, slab)
        if self.on_render is not None:
            self.on_render(k, 1)
        if not self.do_gather:
            return
        gathered, work = self.sharder.gather(slab, group=self.group, slot=k, async_op=True)
        self.last_work = work
        if work is not None:
            work.wait()
        self.sharder.unpack_fused(gathered, lambda buf, ids: self.unpack(k, buf, ids))
        if self.on_render is not None:
            self.on_render(k, 2)


def rank_timing_report(render_ms: float, gather_unpack_ms: float, share_ms: float,
                       whole_ms: Optional[float] = None, group=None) -> Optional[dict]:
    """Per-rank timings of the tile path, collected on rank 0 (VERDICT r03
    item 4: the N>1 bench line explains itself).  Every rank passes
      render_ms        its mean render span over the timed frames (HIP events
                       on the slot stream; with frames in flight a span also
                       covers the other slot's overlapping kernels),
      gather_unpack_ms its mean span from render end to the step's end (the
                       gather, plus the fused unpack on rank 0),
      share_ms         its tiles rendered alone, one frame at a time (the clean
                       per-rank kernel time),
    and rank 0 the whole frame rendered alone (whole_ms).  Returns, on rank 0,
    {ranks_seen, render_ms {min, max}, share_ms {min, max}, gather_unpack_ms
    {rank0, max}, ideal_share_ms = whole_ms / ranks, slowest_share_over_ideal};
    None elsewhere.  Outside any timed region (one all_gather_object)."""
    import torch.distributed as dist
    world = dist.get_world_size(group) if dist.is_initialized() else 1
    rank = dist.get_rank(group) if dist.is_initialized() else 0
    mine = [float(render_ms), float(gather_unpack_ms), float(share_ms)]
    if world > 1:
        allv: list = [None] * world
        dist.all_gather_object(allv, mine, group=group)
    else:
        allv = [mine]
    if rank != 0:
        return None
    rend = [v[0] for v in allv]
    gu = [v[1] for v in allv]
    sh = [v[2] for v in allv]
    out = {"ranks_seen": world,
           "render_ms": {"min": round(min(rend), 4), "max": round(max(rend), 4)},
           "share_ms": {"min": round(min(sh), 4), "max": round(max(sh), 4)},
           "gather_unpack_ms": {"rank0": round(gu[0], 4), "max": round(max(gu), 4)},
           "per_rank": [{"render_ms": round(a, 4), "gather_unpack_ms": round(b, 4),
                         "share_ms": round(c, 4)} for a, b, c in allv]}
    if whole_ms:
        ideal = float(whole_ms) / world
        out["whole_frame_ms"] = round(float(whole_ms), 4)
        out["ideal_share_ms"] = round(ideal, 4)
        out["slowest_share_over_ideal"] = round(max(sh) / ideal, 4)
    return out
