#!/usr/bin/env python3
"""Per-dispatch medians of every counter in tools/pmc_probe.sh outputs.

    python tools/pmc_probe_sum.py gpurun_out/wb_c3_1 gpurun_out/wb_c3_2 ... > summary.json

Each argument is one probe directory; the result maps it to {counter: median
over the scene_kernel_w8 dispatches, "probe": the probe's own JSON line}.
"""
from __future__ import annotations

import csv
import glob
import json
import os
import sys
from collections import defaultdict


def summarise(d: str) -> dict:
    per = defaultdict(lambda: defaultdict(float))
    for path in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(path, newline="") as f:
            for r in csv.DictReader(f):
                if "scene_kernel_w8" not in r.get("Kernel_Name", ""):
                    continue
                per[r["Counter_Name"]][r.get("Dispatch_Id", r.get("Correlation_Id"))] += \
                    float(r["Counter_Value"])
    out = {}
    for k, v in per.items():
        xs = sorted(v.values())
        n = len(xs)
        out[k] = xs[n // 2] if n % 2 else 0.5 * (xs[n // 2 - 1] + xs[n // 2])
        out[k + "@dispatches"] = n
    log = os.path.join(d, "probe.log")
    if os.path.exists(log):
        for line in open(log):
            line = line.strip()
            if line.startswith("{"):
                out["probe"] = json.loads(line)
    return out


def main():
    res = {os.path.basename(os.path.normpath(d)): summarise(d) for d in sys.argv[1:]}
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
