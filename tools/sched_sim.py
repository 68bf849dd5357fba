#!/usr/bin/env python3
"""List-scheduling what-ifs over a measured per-unit timeline (diagnostic).

    RT_AMD_LIB=abl/librt_timeline.so python tools/timeline.py --config c2 --dump units.npz
    python tools/sched_sim.py units.npz [--frame 1] [--waves 8192]

Takes one frame's measured units {start, end, wave} and replays them on
`waves` identical waves with a greedy list scheduler: in the measured dequeue
order, longest-first (LPT), the heaviest x% first, and with no gap between a
wave's units.  Unit durations are the measured ones, so contention effects of
another order are not modelled: it bounds what reordering could win.
"""
from __future__ import annotations

import argparse
import heapq

import numpy as np


def simulate(dur, order, waves, gap, ramp=1.0):
    h = [(ramp, i) for i in range(waves)]
    heapq.heapify(h)
    end = 0.0
    for k in order:
        t, i = heapq.heappop(h)
        f = t + dur[k]
        end = max(end, f)
        heapq.heappush(h, (f + gap, i))
    return end


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("npz")
    ap.add_argument("--key", default="full")
    ap.add_argument("--frame", type=int, default=1)
    ap.add_argument("--waves", type=int, default=8192)
    args = ap.parse_args()
    u = np.load(args.npz)[args.key][args.frame]
    u = u[u[:, 1] > 0]
    s = (u[:, 0] - u[:, 0].min()) / 100.0  # 10-ns wall-clock ticks -> us
    e = (u[:, 1] - u[:, 0].min()) / 100.0
    w = u[:, 2] & 0xFFFF
    dur = e - s
    o = np.lexsort((s, w))
    same = w[o][1:] == w[o][:-1]
    gaps = (s[o][1:] - e[o][:-1])[same]
    gap = float(np.median(gaps))
    cur = np.argsort(s)
    out = {"units": int(len(dur)), "measured_unit_span_us": round(float(e.max()), 2),
           "dur_us": {"mean": round(float(dur.mean()), 2), "p50": round(float(np.median(dur)), 2),
                      "p99": round(float(np.percentile(dur, 99)), 2), "max": round(float(dur.max()), 2)},
           "gap_us": {"mean": round(float(gaps.mean()), 2), "p50": round(gap, 2)},
           "sim_us": {"measured_order": round(simulate(dur, cur, args.waves, gap), 2),
                      "longest_first": round(simulate(dur, np.argsort(-dur), args.waves, gap), 2),
                      "measured_order_no_gaps": round(simulate(dur, cur, args.waves, 0.0), 2)}}
    for frac in (0.01, 0.03, 0.1):
        k = int(len(dur) * frac)
        top = np.argsort(-dur)[:k]
        rest = cur[~np.isin(cur, top)]
        out["sim_us"][f"heaviest_{int(frac * 100)}pct_first"] = round(
            simulate(dur, np.concatenate([top, rest]), args.waves, gap), 2)
    import json
    print(json.dumps(out))


if __name__ == "__main__":
    main()
