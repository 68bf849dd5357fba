#!/usr/bin/env python3
"""Register / scratch / occupancy table of every kernel in rt_kernels.hip.

    python tools/resources.py [csrc dir] [extra hipcc flags ...]

Runs the Makefile's `resources` target (hipcc -Rpass-analysis=
kernel-resource-usage) and prints one line per kernel instantiation, the
demangled template arguments kept short.  CPU only: a quick check that an
experiment does not spill or lose occupancy before it goes to the GPU.
"""
from __future__ import annotations

import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    csrc = sys.argv[1] if len(sys.argv) > 1 and sys.argv[1] else os.path.join(ROOT, "raytracingstudy_amd", "csrc")
    extra = " ".join(sys.argv[2:])
    out = subprocess.run(["make", "-s", "-C", csrc, "resources", f"EXTRA_DEVFLAGS={extra}"],
                         capture_output=True, text=True).stderr
    rows, cur = [], None
    for line in out.splitlines():
        m = re.search(r"Function Name: (\S+)", line)
        if m:
            cur = {"name": m.group(1)}
            rows.append(cur)
            continue
        if cur is None:
            continue
        for key, pat in (("sgpr", r"TotalSGPRs: (\d+)"), ("vgpr", r"VGPRs: (\d+)"),
                         ("scratch", r"ScratchSize \[bytes/lane\]: (\d+)"),
                         ("occ", r"Occupancy \[waves/SIMD\]: (\d+)")):
            m = re.search(pat, line)
            if m:
                cur[key] = int(m.group(1))
    names = [r["name"] for r in rows]
    dem = subprocess.run(["c++filt"], input="\n".join(names), capture_output=True,
                         text=True).stdout.splitlines()
    for r, d in zip(rows, dem):
        d = d.replace("rtamd::", "").replace("(rtamd::FrameArgs)", "").replace("(FrameArgs)", "")
        print(f"{d:60s} vgpr {r.get('vgpr', '?'):>3} sgpr {r.get('sgpr', '?'):>3} "
              f"scratch {r.get('scratch', '?'):>3} occ {r.get('occ', '?')}")


if __name__ == "__main__":
    main()
