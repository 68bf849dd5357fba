#!/usr/bin/env python3
"""Summarise a tools/ab_libs.sh log: per (config, library) the per-process
kernel medians and their median, plus each library's change against the first.

    python tools/ab_summary.py gpurun_out/r03/mt_ab.log
"""
import collections
import json
import statistics
import sys


def main(path):
    runs = collections.defaultdict(list)
    sigs = collections.defaultdict(set)  # (cfg) -> {(image hash, counters)} over every library
    libs = []
    for line in open(path):
        if line.startswith("#") or not line.strip():
            continue  # the "# cmd: ..." header of tools/ab_libs.sh
        lib, cfg, js = line.split(" ", 2)
        if lib not in libs:
            libs.append(lib)
        for v in json.loads(js).values():
            runs[(cfg, lib)].append(v["ms_median"])
            if "image_sha1" in v:
                sigs[cfg].add((v["image_sha1"], tuple(v.get("counters", ()))))
    for cfg in sorted({c for c, _ in runs}):
        base = statistics.median(runs[(cfg, libs[0])])
        for lib in libs:
            m = statistics.median(runs[(cfg, lib)])
            print(f"{cfg:4s} {lib:10s} {m:8.3f} ms  {100 * (m / base - 1):+5.1f}%  {runs[(cfg, lib)]}")
        if sigs[cfg]:
            print(f"{cfg:4s} images and counters {'IDENTICAL' if len(sigs[cfg]) == 1 else 'DIFFER'} "
                  f"across the libraries ({len(sigs[cfg])} distinct)")


if __name__ == "__main__":
    main(sys.argv[1])
