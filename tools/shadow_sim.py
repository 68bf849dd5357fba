#!/usr/bin/env python3
"""CPU model of a wave's shadow phase (the oracle's walk as the cost model).

    python tools/shadow_sim.py --config c3 --pixels 400

For random pixels of a config: each of 64 jittered samples is traced with the
oracle (nearest hit), lit hits cast their shadow ray (any-hit), and per ray the
nodes the walk reads stand in for its trips.  Per pixel-wave it reports the
shadow phase's cost as the slowest lane (SIMD lockstep), the lanes' mean, how
many rays are occluded, and how often one sphere occludes them all.  Also the
cost if each lane first tested the occluder its previous sample found
(the previous round of the pixel, or the previous pixel's at one round).
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c3")
    ap.add_argument("--pixels", type=int, default=300)
    ap.add_argument("--seed", type=int, default=1)
    args = ap.parse_args()
    import oracle
    import raytracingstudy_amd as rt
    from raytracingstudy_amd.camera import scene_pose
    oracle.load()
    lib = oracle.load()
    c = rt.CONFIGS[args.config]
    sp, al = rt.configs.scene_spheres(c, rt.SEED)
    sc = oracle.Scene(sp, al, max_depth=c.max_depth)
    pose = scene_pose()
    K = oracle.resize_intrinsic(c.width, c.height)
    L = -np.array(rt.configs.LIGHT_DIR, np.float32)
    L = (L / np.float32(np.sqrt((L * L).sum()))).astype(np.float32)
    o = pose.reshape(4, 4)[3, :3].astype(np.float32)
    g = np.random.default_rng(args.seed)
    spw = min(c.spp, 64)
    rounds = max(1, c.spp // 64)
    res = {"waves": 0, "phases": 0, "lock_cost": 0.0, "mean_cost": 0.0, "rays": 0, "occluded": 0,
           "all_occluded_phases": 0, "one_occluder_phases": 0, "cached_lock_cost": 0.0,
           "primary_lock": 0.0, "primary_mean": 0.0}
    prev_occ = [None] * 64
    for _ in range(args.pixels):
        x, y = int(g.integers(0, c.width)), int(g.integers(0, c.height))
        pid = y * c.width + x
        for r in range(rounds):
            res["waves"] += 1
            costs, occl, occs, cached, pcost = [], [], [], [], []
            for lane in range(spw):
                s = r * spw + lane
                u = x + (lib.orc_sample_hash(rt.SEED, pid, s, 0) >> 8) * (1.0 / 16777216.0)
                v = y + (lib.orc_sample_hash(rt.SEED, pid, s, 1) >> 8) * (1.0 / 16777216.0)
                d = oracle.get_ray(pose, K, u, v)
                hit, t, idx, cnt = sc.trace(o, d)
                pcost.append(int(cnt[2]))
                if not hit:
                    continue
                sph = sp[idx].astype(np.float32)
                p = (o + np.float32(t) * d).astype(np.float32)
                n = ((p - sph[:3]) * np.float32(1.0 / sph[3])).astype(np.float32)
                if float((n * L).sum()) <= 0.0:
                    continue
                so = (p + n * np.float32(1e-5)).astype(np.float32)
                h2, t2, i2, c2 = sc.trace(so, L, any_hit=True)
                costs.append(int(c2[2]))
                occl.append(h2)
                occs.append(i2 if h2 else -1)
                # occluder cache: the sphere that occluded this lane's previous ray
                pc = prev_occ[lane]
                if pc is not None:
                    hit_c = _hits(sp[pc], so, L)
                    cached.append(1 if hit_c else int(c2[2]) + 1)
                else:
                    cached.append(int(c2[2]))
                prev_occ[lane] = i2 if h2 else None
            res["primary_lock"] += max(pcost)
            res["primary_mean"] += float(np.mean(pcost))
            if not costs:
                continue
            res["phases"] += 1
            res["lock_cost"] += max(costs)
            res["mean_cost"] += float(np.mean(costs))
            res["cached_lock_cost"] += max(cached)
            res["rays"] += len(costs)
            res["occluded"] += int(sum(occl))
            if all(occl):
                res["all_occluded_phases"] += 1
                if len(set(occs)) == 1:
                    res["one_occluder_phases"] += 1
    out = {k: (round(v, 1) if isinstance(v, float) else v) for k, v in res.items()}
    ph = max(1, res["phases"])
    out["lanes_per_phase"] = round(res["rays"] / ph, 1)
    out["lock_per_phase"] = round(res["lock_cost"] / ph, 2)
    out["mean_per_phase"] = round(res["mean_cost"] / ph, 2)
    out["cached_lock_per_phase"] = round(res["cached_lock_cost"] / ph, 2)
    out["occluded_share"] = round(res["occluded"] / max(1, res["rays"]), 3)
    out["primary_lock_per_wave"] = round(res["primary_lock"] / res["waves"], 2)
    out["primary_mean_per_wave"] = round(res["primary_mean"] / res["waves"], 2)
    print(args.config, json.dumps(out))


def _hits(s, o, d):
    # isect's discriminant and root test (tmin 0), float32
    s = s.astype(np.float32)
    oc = (o - s[:3]).astype(np.float32)
    b = np.float32((oc * d).sum())
    q = (oc - b * d).astype(np.float32)
    h = np.float32(s[3] * s[3] - (q * q).sum())
    if h < 0:
        return False
    sq = np.float32(np.sqrt(h))
    t = -b - sq
    if not t > 0:
        t = -b + sq
    return bool(t > 0)


if __name__ == "__main__":
    main()
