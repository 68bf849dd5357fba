#!/usr/bin/env python3
"""Upper bound on what lane refill could win on the 256-spp sorted rounds
(VERDICT r05 item 3), from the oracle's per-sample walk costs.

    python tools/refill_bound.py --config c5d --pixels 200

For random pixels of a config, each of the pixel's spp samples is traced with
the oracle (nearest hit), and the lit hits cast their shadow ray (any-hit).  A
ray's cost is its walk's node reads plus its sphere-test chunks (two spheres
a chunk), the work a lane's trips do.  Per pixel-wave:

  lockstep (the shipped sorted path, rt_kernels.hip shade_pixel_sorted):
    primary rays 64 at a time in jitter-cell (Morton 8x8) order, each batch
    costing its slowest lane; then the lit samples' shadow rays, 64 at a
    time in that order, the same way;
  refill (ideal): a lane that finishes takes the pixel's next sample at once
    (no set-up cost, no lost coherence): primary makespan of a greedy list
    schedule over 64 lanes, then the shadow rays' the same way, each no less
    than its lanes' total / 64;
  perfect: every lane busy to the end: total / 64 per phase.

  oracle order: lockstep, but the batches formed knowing every ray's cost
    (sorted by it): the most any reordering of the samples could save.

lockstep / refill is the most a refill of finished lanes could save on these
walks (the 1.17-1.24x of C3 in DESIGN 5.1 was the unsorted one-round figure).
"""
from __future__ import annotations

import argparse
import heapq
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def morton_cell(hu: int, hv: int, bits: int = 3) -> int:
    qu, qv = hu >> (32 - bits), hv >> (32 - bits)
    c = 0
    for b in range(bits):
        c |= ((qu >> b) & 1) << (2 * b) | ((qv >> b) & 1) << (2 * b + 1)
    return c


def makespan(costs, lanes=64) -> float:
    """Greedy list schedule in the given order: each job to the lane free first."""
    if not costs:
        return 0.0
    free = [0.0] * min(lanes, len(costs))
    heapq.heapify(free)
    for c in costs:
        t = heapq.heappop(free)
        heapq.heappush(free, t + c)
    return max(free)


def lockstep(costs, lanes=64) -> float:
    return float(sum(max(costs[i:i + lanes]) for i in range(0, len(costs), lanes)))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c5d")
    ap.add_argument("--pixels", type=int, default=200)
    ap.add_argument("--seed", type=int, default=1)
    args = ap.parse_args()
    import oracle
    import raytracingstudy_amd as rt
    from raytracingstudy_amd.camera import scene_pose
    lib = oracle.load()
    c = rt.CONFIGS[args.config]
    sp, al = rt.configs.scene_spheres(c, rt.SEED)
    sc = oracle.Scene(sp, al, max_depth=c.max_depth, leaf_capacity=c.leaf_capacity)
    pose = scene_pose()
    K = oracle.resize_intrinsic(c.width, c.height)
    L = -np.array(rt.configs.LIGHT_DIR, np.float32)
    L = (L / np.float32(np.sqrt((L * L).sum()))).astype(np.float32)
    o = pose.reshape(4, 4)[3, :3].astype(np.float32)
    g = np.random.default_rng(args.seed)
    tot = {"lock_p": 0.0, "lock_s": 0.0, "refill_p": 0.0, "refill_s": 0.0, "perfect_p": 0.0,
           "perfect_s": 0.0, "refill_joint": 0.0, "oracle_order_p": 0.0, "oracle_order_s": 0.0,
           "s_by_sphere": 0.0, "s_by_pcost": 0.0, "s_by_sphere_mod64": 0.0, "s_by_t": 0.0,
           "pixels": 0, "shadow_rays": 0, "samples": 0}
    per_pixel = []
    for _ in range(args.pixels):
        x, y = int(g.integers(0, c.width)), int(g.integers(0, c.height))
        pid = y * c.width + x
        samples = []
        for s in range(c.spp):
            hu = lib.orc_sample_hash(rt.SEED, pid, s, 0)
            hv = lib.orc_sample_hash(rt.SEED, pid, s, 1)
            samples.append((morton_cell(hu, hv), s, hu, hv))
        samples.sort(key=lambda e: (e[0], e[1]))  # stable by sample index within a cell
        pc, sc_cost, joint, keys = [], [], [], []
        for _, s, hu, hv in samples:
            u = x + (hu >> 8) * (1.0 / 16777216.0)
            v = y + (hv >> 8) * (1.0 / 16777216.0)
            d = oracle.get_ray(pose, K, u, v)
            hit, t, idx, cnt = sc.trace(o, d)
            cp = float(cnt[2]) + float(cnt[3]) / 2.0
            pc.append(cp)
            cs = 0.0
            if hit:
                sph = sp[idx].astype(np.float32)
                p = (o + np.float32(t) * d).astype(np.float32)
                n = ((p - sph[:3]) * np.float32(1.0 / sph[3])).astype(np.float32)
                if float((n * L).sum()) > 0.0:
                    so = (p + n * np.float32(1e-5)).astype(np.float32)
                    _, _, _, c2 = sc.trace(so, L, any_hit=True)
                    cs = float(c2[2]) + float(c2[3]) / 2.0
                    sc_cost.append(cs)
                    keys.append((int(idx), cp, float(t)))
            joint.append(cp + cs)
        lp, ls = lockstep(pc), lockstep(sc_cost) if sc_cost else 0.0
        rp, rs = makespan(pc), makespan(sc_cost)
        tot["lock_p"] += lp
        tot["lock_s"] += ls
        tot["refill_p"] += rp
        tot["refill_s"] += rs
        tot["perfect_p"] += sum(pc) / 64.0
        tot["perfect_s"] += sum(sc_cost) / 64.0
        tot["refill_joint"] += makespan(joint)  # primary then its shadow on the same lane
        # any reordering of the batches (lockstep kept): the best is by true cost
        tot["oracle_order_p"] += lockstep(sorted(pc, reverse=True))
        tot["oracle_order_s"] += lockstep(sorted(sc_cost, reverse=True)) if sc_cost else 0.0
        # shadow orders from what the primary walks already know (stable sorts)
        if sc_cost:
            ix = list(range(len(sc_cost)))
            for name, key in (("s_by_sphere", lambda i: keys[i][0]),
                              ("s_by_sphere_mod64", lambda i: keys[i][0] % 64),
                              ("s_by_pcost", lambda i: -keys[i][1]),
                              ("s_by_t", lambda i: keys[i][2])):
                tot[name] += lockstep([sc_cost[i] for i in sorted(ix, key=key)])
        tot["pixels"] += 1
        tot["shadow_rays"] += len(sc_cost)
        tot["samples"] += len(pc)
        if rp + rs > 0:
            per_pixel.append((lp + ls) / (rp + rs))
    lock = tot["lock_p"] + tot["lock_s"]
    out = {
        "config": args.config, "pixels": tot["pixels"], "spp": c.spp,
        "shadow_rays_per_pixel": round(tot["shadow_rays"] / tot["pixels"], 1),
        "cost_per_pixel": {k: round(tot[k] / tot["pixels"], 1)
                           for k in ("lock_p", "lock_s", "refill_p", "refill_s", "perfect_p",
                                     "perfect_s", "refill_joint", "oracle_order_p",
                                     "oracle_order_s", "s_by_sphere", "s_by_sphere_mod64",
                                     "s_by_pcost", "s_by_t")},
        "lockstep_over_oracle_order": round(lock / (tot["oracle_order_p"] + tot["oracle_order_s"]), 3),
        "lockstep_over_refill": round(lock / (tot["refill_p"] + tot["refill_s"]), 3),
        "lockstep_over_refill_joint": round(lock / tot["refill_joint"], 3),
        "lockstep_over_perfect": round(lock / (tot["perfect_p"] + tot["perfect_s"]), 3),
        "lane_use_lockstep": round((tot["perfect_p"] + tot["perfect_s"]) / lock, 3),
        "per_pixel_ratio_p10_p50_p90": [round(float(q), 3) for q in
                                        np.percentile(per_pixel, [10, 50, 90])],
    }
    print(json.dumps(out))


if __name__ == "__main__":
    main()
