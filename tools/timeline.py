#!/usr/bin/env python3
"""Per-wave timeline of the wave-queue scene kernel (diagnostic build).

    bash tools/build_exp.sh timeline -DRT_TIMELINE
    RT_AMD_LIB=abl/librt_timeline.so python tools/timeline.py [--config c3] [--n 8]

Renders the full frame and rank 0's N-way share a few times; every frame's
per-wave {start, first empty range, exit, units} (100 MHz wall clock) is
summarised: the span, when the queues first ran dry, how long the last waves
ran after that, and how many waves were still busy over the tail.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

import raytracingstudy_amd as rt  # noqa: E402
from raytracingstudy_amd import tiles as T  # noqa: E402
from raytracingstudy_amd.camera import scene_pose  # noqa: E402


WAVE_WORDS = 65536 * 4


def unit_gaps(u: np.ndarray) -> dict:
    """Per wave (column 2's low 16 bits: workgroup * 4 + wave), the idle time
    between one unit's end and the same wave's next unit's start: the
    scheduler's cost per unit (dequeue, barriers, the pixel epilogue)."""
    if u.shape[1] < 3 or not len(u):
        return {}
    wid = (u[:, 2] & 0xFFFF).astype(np.int64)
    order = np.lexsort((u[:, 0], wid))
    w, s, e = wid[order], u[order, 0], u[order, 1]
    same = w[1:] == w[:-1]
    gaps = (s[1:] - e[:-1])[same] / 100.0
    if not len(gaps):
        return {}
    return {"gap_us": {p: round(float(np.percentile(gaps, q)), 2) for p, q in
                       (("p10", 10), ("p50", 50), ("p90", 90), ("p99", 99))},
            "gap_mean_us": round(float(gaps.mean()), 3), "gaps": int(len(gaps))}


def summarise_units(u: np.ndarray, t0: int, span_us: float) -> dict:
    u = u[u[:, 1] > 0]
    if not len(u):
        return {"units": 0}  # this path records no per-unit times
    gaps = unit_gaps(u)
    st = (u[:, 0] - t0) / 100.0
    du = (u[:, 1] - u[:, 0]) / 100.0
    en = st + du
    dec = np.minimum((st / span_us * 10).astype(int), 9)
    late = en > 0.9 * span_us
    return {"units": int(len(u)),
            "dur_us": {p: round(float(np.percentile(du, q)), 1)
                       for p, q in (("p0.1", 0.1), ("p1", 1), ("p10", 10), ("p50", 50), ("p90", 90),
                                    ("p99", 99), ("p99.9", 99.9))},
            "dur_max_us": round(float(du.max()), 1), "dur_mean_us": round(float(du.mean()), 2),
            "mean_dur_by_start_decile": [round(float(du[dec == i].mean()), 1) if (dec == i).any()
                                         else None for i in range(10)],
            "units_ending_last_10pct": int(late.sum()),
            "their_dur_p50_max_us": [round(float(np.median(du[late])), 1) if late.any() else 0,
                                     round(float(du[late].max()), 1) if late.any() else 0],
            "their_start_min_us": round(float(st[late].min()), 1) if late.any() else 0,
            # share of the waves' launch span spent inside units (the rest:
            # ramp, scheduling gaps, tail)
            "in_unit_share": (round(float(du.sum()) / (len(np.unique(u[:, 2] & 0xFFFF)) * span_us), 3)
                              if u.shape[1] > 2 else None),
            **gaps}


def summarise(rec: np.ndarray, unit_rec: np.ndarray) -> dict:
    rec = rec[rec[:, 2] > 0]
    t0 = rec[:, 0].min()
    start, empty, end, units = [(rec[:, i] - (t0 if i < 3 else 0)) / (100.0 if i < 3 else 1)
                                for i in range(4)]  # us
    empty = np.where(rec[:, 1] > 0, empty, end)
    first_dry = float(empty.min())
    span = float(end.max())
    busy = lambda t: int(((start <= t) & (end > t)).sum())  # noqa: E731
    return {"waves": int(len(rec)), "span_us": round(span, 1),
            "start_spread_us": round(float(start.max()), 1),
            "first_dry_us": round(first_dry, 1),
            "end_pcts_us": [round(float(np.percentile(end, p)), 1) for p in (1, 10, 50, 90, 99, 100)],
            "tail_us": round(span - first_dry, 1),
            "busy_at": {f"{f:.2f}": busy(f * span) for f in (0.5, 0.8, 0.9, 0.95, 0.98)},
            "units_per_wave": [int(units.min()), float(round(units.mean(), 1)), int(units.max())],
            "mean_unit_us": round(float((end - start).sum() / max(units.sum(), 1)), 2),
            "unit_level": summarise_units(unit_rec, int(t0), span)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c3")
    ap.add_argument("--n", type=int, default=8)
    ap.add_argument("--frames", type=int, default=2)
    ap.add_argument("--variant", type=int, default=0)
    ap.add_argument("--dump", default="", help="save per-unit {start, end} ticks (.npz)")
    args = ap.parse_args()
    fd, path = tempfile.mkstemp(suffix=".tl")
    os.close(fd)
    os.environ["RT_TIMELINE_FILE"] = path
    import torch
    cfg = rt.CONFIGS[args.config]
    sp, al = rt.configs.scene_spheres(cfg, rt.SEED)
    r = rt.KernelRenderer(cfg.width, cfg.height, mode="scene", spp=cfg.spp, variant=args.variant)
    r.resize(cfg.width, cfg.height)
    r.setPosition(scene_pose())
    r.set_scene(sp, al, max_depth=cfg.max_depth, leaf_capacity=cfg.leaf_capacity)
    ts = rt.configs.TILE_SIZE
    share = T.tiles_for_rank(cfg.width, cfg.height, 0, args.n, ts)
    slab = torch.zeros(len(share) * ts * ts * 4, dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()
    out = {}
    dumps = {"share_tiles": np.asarray(share, np.uint32)}
    for name, fn in (("full", lambda: r.render()),
                     (f"share_1_of_{args.n}", lambda: r.render_tiles(share, ts, slab.data_ptr()))):
        fn()  # warm-up
        open(path, "wb").close()
        for _ in range(args.frames):
            fn()
        r.synchronize()
        raw = np.fromfile(path, dtype=np.uint64).reshape(args.frames, -1).astype(np.int64)
        unit_end = WAVE_WORDS + (3 << 22)
        out[name] = []
        if args.dump:
            dumps[name] = raw[:, WAVE_WORDS:unit_end].reshape(args.frames, -1, 3)
            dumps[name + "_waves"] = raw[:, :WAVE_WORDS].reshape(args.frames, -1, 4)
        for i in range(args.frames):
            sm = summarise(raw[i, :WAVE_WORDS].reshape(-1, 4), raw[i, WAVE_WORDS:unit_end].reshape(-1, 3))
            ph = raw[i, unit_end:].reshape(-1, 2).sum(0).astype(float)
            sm["phase_ticks_share"] = {"primary": round(ph[0] / max(ph.sum(), 1), 3),
                                       "shadow": round(ph[1] / max(ph.sum(), 1), 3)}
            out[name].append(sm)
        print(name, json.dumps(out[name][-1]), flush=True)
    os.unlink(path)
    if args.dump:
        np.savez_compressed(args.dump, **{k.replace("share_1_of_%d" % args.n, "share"): v
                                          for k, v in dumps.items()})
    r.close()


if __name__ == "__main__":
    main()
