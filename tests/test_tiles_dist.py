"""Tile partition, pack/unpack, and the N>1 gather path on CPU (gloo, world 2).

The GPU ranks render with rt_render_tiles and unpack with rt_unpack_tiles;
here the CPU oracle stands in as each rank's renderer (test only), so the
plan + packed layout + torch.distributed gather + unpack are exercised
end to end and must reproduce the single-rank frame byte for byte.
"""
import os
import socket

import numpy as np
import pytest

from raytracingstudy_amd import tiles as T
from raytracingstudy_amd.dist import TileSharder


@pytest.mark.parametrize("w,h,world", [(1920, 1080, 1), (1920, 1080, 2), (1920, 1080, 8),
                                       (3840, 2160, 8), (100, 70, 3), (64, 64, 4)])
def test_partition_covers_each_tile_once(w, h, world):
    tx, ty = T.tile_grid(w, h)
    ids = np.concatenate([T.tiles_for_rank(w, h, r, world) for r in range(world)])
    assert sorted(ids.tolist()) == list(range(tx * ty))
    counts = [len(T.tiles_for_rank(w, h, r, world)) for r in range(world)]
    assert max(counts) - min(counts) <= 1
    assert T.slab_tiles(w, h, world) == max(counts)


def test_c4_tile_geometry():
    # 3840x2160 -> 60 x 34 = 2040 tiles, last row 48 px tall
    assert T.tile_grid(3840, 2160) == (60, 34)
    assert 2160 - 33 * 64 == 48


def test_pack_unpack_roundtrip():
    rng = np.random.default_rng(0)
    img = rng.integers(0, 256, (70, 100, 4), dtype=np.uint8)
    ids = np.array([3, 0, 2, 1], np.uint32)  # 2 x 2 tiles over 100 x 70
    packed = T.pack_reference(img, ids)
    out = np.zeros_like(img)
    T.unpack_host(packed, ids, 100, 70, out=out)
    tx, _ = T.tile_grid(100, 70)
    for t in ids:
        x0, y0 = (t % tx) * 64, (t // tx) * 64
        assert np.array_equal(out[y0:y0 + 64, x0:x0 + 64], img[y0:y0 + 64, x0:x0 + 64])
    # edge tiles are zero-padded in the packed slab
    k = list(ids).index(3)  # bottom-right tile: 36 x 6 valid pixels
    assert not packed[k, 6:].any() and not packed[k, :, 36:].any()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rank_main(rank, world, port, w, h, spp, q):
    import torch
    import torch.distributed as dist

    import oracle
    from raytracingstudy_amd.configs import SEED
    from raytracingstudy_amd.camera import scene_pose

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    sh = TileSharder(w, h, rank, world)
    sp, al = oracle.generate_spheres(1000, SEED)
    sc = oracle.Scene(sp, al)
    K = oracle.resize_intrinsic(w, h)
    # this rank's tiles (oracle stands in for rt_render_tiles on CPU)
    slab = sh.new_slab(torch)
    view = slab.numpy().reshape(sh.slab_tiles, 64, 64, 4)
    tx, _ = T.tile_grid(w, h)
    for k, t in enumerate(sh.ids):
        x0, y0 = int(t % tx) * 64, int(t // tx) * 64
        img, _, _ = sc.render(w, h, scene_pose(), K, spp=spp, rect=(x0, y0, x0 + 64, y0 + 64),
                              radiance=False)
        blk = img[y0:y0 + 64, x0:x0 + 64]
        view[k, :blk.shape[0], :blk.shape[1]] = blk
    gathered = sh.gather(slab)
    if rank == 0:
        per_rank = sh.unpack_host(gathered)
        # the bench's fused unpack: all slabs end to end, padding slots skipped
        fused = {}
        sh.unpack_fused(gathered, lambda buf, ids: fused.setdefault(
            "img", T.unpack_host(buf.numpy().reshape(-1, 64, 64, 4), ids, w, h)))
        assert np.array_equal(fused["img"], per_rank)
    # bench.py's timed step itself (dist.TileFramePipeline): 2 frames in
    # flight, each slot its own slab, receive buffer and frame; the gather is
    # asynchronous (gloo runs host tensors async: a real Work object), then
    # work.wait(), then one fused unpack on rank 0
    from raytracingstudy_amd.dist import TileFramePipeline
    slabs = [slab, sh.new_slab(torch)]
    frames = [np.zeros((h, w, 4), np.uint8) for _ in slabs]
    rendered = []

    def render(k, sl):
        sl.copy_(slab)  # this rank's tiles (the oracle's, above)
        rendered.append(k)

    def unpack(k, buf, ids):
        T.unpack_host(buf.numpy().reshape(-1, 64, 64, 4), ids, w, h, out=frames[k])

    phases = []
    pipe = TileFramePipeline(sh, slabs, render, unpack, on_render=lambda k, ph: phases.append((k, ph)))
    works = []
    for i in range(3):
        pipe.step(i)
        works.append(pipe.last_work)
    assert rendered == [0, 1, 0]
    # bench.py's event hooks: before / after the render, and after gather + unpack
    assert phases == [(0, 0), (0, 1), (0, 2), (1, 0), (1, 1), (1, 2), (0, 0), (0, 1), (0, 2)]
    # the per-rank timings bench.py adds to an N>1 line
    from raytracingstudy_amd.dist import rank_timing_report
    rep = rank_timing_report(1.0 + rank, 0.25 * (rank + 1), 1.1 + 0.1 * rank,
                             whole_ms=8.0 if rank == 0 else None)
    if rank == 0:
        assert rep["ranks_seen"] == world
        assert rep["render_ms"] == {"min": 1.0, "max": 1.0 + (world - 1)}
        assert rep["gather_unpack_ms"]["rank0"] == 0.25
        assert rep["gather_unpack_ms"]["max"] == 0.25 * world
        assert rep["share_ms"]["max"] == round(1.1 + 0.1 * (world - 1), 4)
        assert rep["ideal_share_ms"] == round(8.0 / world, 4)
        assert rep["slowest_share_over_ideal"] == round((1.1 + 0.1 * (world - 1)) / (8.0 / world), 4)
        assert len(rep["per_rank"]) == world
    else:
        assert rep is None
    assert all(wk is not None and hasattr(wk, "wait") for wk in works)
    if rank == 0:
        recv = sh.__dict__["_recv_bufs"]
        assert recv[0][1].data_ptr() != recv[1][1].data_ptr()  # one receive buffer per slot
        for f in frames:
            assert np.array_equal(f, per_rank)
        q.put(per_rank)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 5])  # 12 tiles: 5 ranks leave padding slots
def test_gloo_world2_gather_reproduces_frame(oracle, world):
    import torch.multiprocessing as mp
    from raytracingstudy_amd.configs import SEED
    from raytracingstudy_amd.camera import scene_pose

    w, h, spp = 200, 130, 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank_main, args=(r, world, port, w, h, spp, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = q.get(timeout=120)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    sp, al = oracle.generate_spheres(1000, SEED)
    ref, _, _ = oracle.Scene(sp, al).render(w, h, scene_pose(), oracle.resize_intrinsic(w, h),
                                            spp=spp, radiance=False)
    assert np.array_equal(got, ref)


@pytest.mark.parametrize("w,h,world", [(1920, 1080, 2), (1920, 1080, 4), (1920, 1080, 8),
                                       (3840, 2160, 8), (100, 70, 3)])
def test_latin_plan_partitions_the_frame(w, h, world):
    # every tile exactly once; each rank gets one region per region row/column
    ids = [T.tiles_for_rank(w, h, k, world, 64, "latin") for k in range(world)]
    tx, ty = T.tile_grid(w, h)
    assert np.array_equal(np.sort(np.concatenate(ids)), np.arange(tx * ty))
    assert T.slab_tiles(w, h, world, 64, "latin") == max(len(x) for x in ids)
