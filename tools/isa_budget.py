#!/usr/bin/env python3
"""Instruction budget of one kernel from its gfx950 assembly.

    make -C raytracingstudy_amd/csrc asm          # -> raytracingstudy_amd/csrc/rt_kernels.s
    python tools/isa_budget.py [--kernel scene_kernel_w8ILb0ELb0ELb0E] [--asm path]

Splits the kernel's body into basic blocks and counts, per block, the
instructions by issue class:
  valu   v_*                      (vector ALU; v_readlane / v_writelane too)
  salu   s_* scalar ALU           (s_and/s_or/s_xor on exec masks are most of them)
  br     s_branch / s_cbranch_*
  smem   s_load_* / s_buffer_load_*
  vmem   global_/buffer_/flat_ loads (vmem_st: stores, atomics)
  lds    ds_*
  wait   s_waitcnt, s_nop, s_sleep, sched barriers (not issue work)
Prints one line per block with its loop depth and header (from the
compiler's loop comments), then the sum per loop.  With --groups it sums
named block ranges (label:label) so a source region (the leaf chunk, the
exit step) gets one budget line.
"""
from __future__ import annotations

import argparse
import os
import re
import sys
from collections import OrderedDict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CLASSES = ("valu", "salu", "br", "smem", "vmem", "vmem_st", "lds", "wait")


def classify(op: str) -> str | None:
    if op.startswith("v_"):
        return "valu"
    if op.startswith(("global_load", "buffer_load", "flat_load", "scratch_load")):
        return "vmem"
    if op.startswith(("global_store", "buffer_store", "flat_store", "scratch_store", "global_atomic",
                      "buffer_atomic", "flat_atomic")):
        return "vmem_st"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith(("s_load", "s_buffer_load", "s_store", "s_dcache")):
        return "smem"
    if op.startswith(("s_waitcnt", "s_nop", "s_sleep", "s_barrier", "s_setprio", "s_endpgm")):
        return "wait"
    if op.startswith(("s_branch", "s_cbranch")):
        return "br"
    if op.startswith("s_"):
        return "salu"
    return None


def parse(asm_path: str, kernel_sub: str):
    lines = open(asm_path).read().splitlines()
    start = None
    for i, l in enumerate(lines):
        if l.startswith("_Z") and kernel_sub in l and l.split(":")[0].endswith(("E", "v")) and ":" in l:
            if re.match(r"^_Z\S*:", l):
                start = i
                break
    if start is None:
        raise SystemExit(f"kernel matching {kernel_sub!r} not found in {asm_path}")
    blocks = OrderedDict()
    cur = "entry"
    blocks[cur] = {"n": {c: 0 for c in CLASSES}, "depth": 0, "header": "", "ops": []}
    for l in lines[start + 1:]:
        s = l.strip()
        if s.startswith("s_endpgm"):
            blocks[cur]["n"]["wait"] += 1
            break
        m = re.match(r"^(\.LBB\d+_\d+|; %bb\.\d+):?", s)
        if m:
            cur = m.group(1).replace("; ", "")
            depth, header = 0, ""
            dm = re.search(r"Depth=(\d+)", s)
            hm = re.search(r"Header=(BB\d+_\d+)", s)
            if dm:
                depth = int(dm.group(1))
            if hm:
                header = hm.group(1)
            blocks[cur] = {"n": {c: 0 for c in CLASSES}, "depth": depth, "header": header, "ops": []}
            continue
        if not s or s.startswith((";", ".", "//")):
            dm = re.search(r"This (?:Inner )?Loop Header: Depth=(\d+)", s)
            if dm:
                blocks[cur]["depth"] = int(dm.group(1))
                blocks[cur]["header"] = cur.lstrip(".L")
            continue
        op = s.split()[0]
        c = classify(op)
        if c:
            blocks[cur]["n"][c] += 1
            blocks[cur]["ops"].append(op)
    return blocks


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--asm", default=os.path.join(ROOT, "raytracingstudy_amd", "csrc", "rt_kernels.s"))
    ap.add_argument("--kernel", default="scene_kernel_w8ILb0ELb0ELb0E")
    ap.add_argument("--groups", default="",
                    help="name=first:last,... sums of block ranges (inclusive, in layout order)")
    ap.add_argument("--ops", action="store_true", help="also list each block's opcodes")
    args = ap.parse_args()
    blocks = parse(args.asm, args.kernel)
    names = list(blocks)
    print(f"# {args.kernel} in {os.path.relpath(args.asm, ROOT)}: {len(names)} blocks")
    print(f"{'block':14s} {'dep':>3s} {'header':10s} " + " ".join(f"{c:>7s}" for c in CLASSES))
    for b in names:
        n = blocks[b]["n"]
        if not any(n.values()):
            continue
        print(f"{b:14s} {blocks[b]['depth']:3d} {blocks[b]['header']:10s} " +
              " ".join(f"{n[c]:7d}" for c in CLASSES))
        if args.ops:
            print("    " + " ".join(blocks[b]["ops"]))
    if args.groups:
        print("# groups")
        for g in args.groups.split(","):
            name, rng = g.split("=")
            a, z = rng.split(":")
            i0, i1 = names.index(a), names.index(z)
            tot = {c: sum(blocks[b]["n"][c] for b in names[i0:i1 + 1]) for c in CLASSES}
            print(f"{name:24s} " + " ".join(f"{c}={tot[c]}" for c in CLASSES))
    return 0


if __name__ == "__main__":
    sys.exit(main())
