#!/usr/bin/env python3
"""Summarise a tools/profile.sh run into one JSON object (per-launch figures).

    python tools/pmc_traffic.py gpurun_out/prof_<tag> <config> > pmc_summary.json

HBM traffic follows MI355X_MICROARCH.md "HBM": FETCH_SIZE / WRITE_SIZE are in
KiB and come from separate --pmc passes; on gfx950 FETCH_SIZE reports half the
bytes of wide coalesced reads, so the corrected read bytes are 2 x FETCH_SIZE
(the raw sum is reported beside it; the guide notes other access widths are
uncalibrated).  Counters are the median over the scene kernel's dispatches (the timed frames).
"""
from __future__ import annotations

import csv
import glob
import json
import os
import sys
from collections import defaultdict


def _rows(pattern):
    out = []
    for path in sorted(glob.glob(pattern, recursive=True)):
        with open(path, newline="") as f:
            out.extend(csv.DictReader(f))
    return out


def _median(xs):
    xs = sorted(xs)
    n = len(xs)
    return xs[n // 2] if n % 2 else 0.5 * (xs[n // 2 - 1] + xs[n // 2])


def counters(d, kernel_sub="scene_kernel"):
    """Per counter: (median over dispatches, dispatches).  The median, because
    the bench's first dispatch is its stats frame (the work-counting build,
    ~8% more VALU) and every later one is the timed counter-free build."""
    per = defaultdict(lambda: defaultdict(float))
    for r in _rows(os.path.join(d, "**", "*counter_collection.csv")):
        if kernel_sub not in r.get("Kernel_Name", ""):
            continue
        per[r["Counter_Name"]][r.get("Dispatch_Id", r.get("Correlation_Id"))] += float(r["Counter_Value"])
    return {k: (_median(list(v.values())), len(v)) for k, v in per.items() if v}


def kernel_stats(d):
    out = {}
    for r in _rows(os.path.join(d, "**", "*kernel_stats.csv")):
        out[r["Name"]] = {"calls": int(r["Calls"]), "avg_ns": float(r["AverageNs"]),
                          "total_ns": float(r["TotalDurationNs"]), "pct": float(r["Percentage"])}
    return out


def trace_durations(d, kernel_sub="scene_kernel"):
    ds = []
    for r in _rows(os.path.join(d, "**", "*kernel_trace.csv")):
        if kernel_sub in r.get("Kernel_Name", ""):
            ds.append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    return ds


def main():
    root, cfg = sys.argv[1], sys.argv[2]
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from raytracingstudy_amd._lib import kernel_source_id
    # stamp: bench.py takes these counters only while the kernel sources match
    from raytracingstudy_amd.configs import CONFIGS
    # and the octree build parameter the counters were taken at (round 3: a
    # config's leaf capacity changes its work, not its image)
    res = {"config": cfg, "n_gpus": 1, "kernel_source_id": kernel_source_id(),
           "leaf_capacity": CONFIGS[cfg].leaf_capacity}
    ks = kernel_stats(os.path.join(root, "trace"))
    res["kernel_stats"] = ks
    durs = trace_durations(os.path.join(root, "trace"))
    if durs:
        res["scene_kernel_dispatches"] = len(durs)
        res["scene_kernel_avg_ns"] = sum(durs) / len(durs)
        res["scene_kernel_median_ns"] = _median(durs)
    f = counters(os.path.join(root, "fetch")).get("FETCH_SIZE")
    w = counters(os.path.join(root, "write")).get("WRITE_SIZE")
    if f and w:
        res["fetch_size_kib"] = f[0]
        res["write_size_kib"] = w[0]
        res["hbm_bytes_raw"] = (f[0] + w[0]) * 1024.0
        res["hbm_bytes_per_launch"] = (2.0 * f[0] + w[0]) * 1024.0
        res["correction"] = "gfx950: read bytes = 2 x FETCH_SIZE (MI355X_MICROARCH.md HBM); KiB -> B"
    sq = counters(os.path.join(root, "sq"))
    if sq:
        res["sq"] = {k: v[0] for k, v in sq.items()}
        waves = sq.get("SQ_WAVES", (0, 0))[0]
        cyc = sq.get("SQ_WAVE_CYCLES", (0, 0))[0]
        act = sq.get("SQ_ACTIVE_INST_VALU", (0, 0))[0]
        gui = sq.get("GRBM_GUI_ACTIVE", (0, 0))[0]
        if cyc:
            res["valu_active_frac_of_wave_cycles"] = act / cyc
        if gui and durs:
            res["effective_clock_ghz"] = gui / 8.0 / _median(durs)
        if waves:
            res["valu_insts_per_wave"] = sq.get("SQ_INSTS_VALU", (0, 0))[0] / waves
        thr = sq.get("SQ_THREAD_CYCLES_VALU", (0, 0))[0]
        if thr and act:
            # active lanes per VALU instruction cycle (VERDICT r02's lane
            # utilisation: SQ_THREAD_CYCLES_VALU / SQ_ACTIVE_INST_VALU of 64)
            res["valu_lanes_active"] = thr / act
            res["valu_lane_util"] = thr / act / 64.0
        wait = sq.get("SQ_WAIT_ANY", (0, 0))[0]
        if wait and cyc:
            res["wait_any_frac_of_wave_cycles"] = wait / cyc
        if gui and sq.get("SQ_INSTS_SALU"):
            # per CU-cycle (256 CUs, GRBM_GUI_ACTIVE summed over 8 XCDs)
            sc = sq["SQ_INSTS_SALU"][0] + sq.get("SQ_INSTS_BRANCH", (0, 0))[0]
            res["scalar_per_cu_cycle"] = sc / 256.0 / (gui / 8.0)
    vm = counters(os.path.join(root, "vmem"))
    vgui = vm.get("GRBM_GUI_ACTIVE", (0, 0))[0]
    if vm.get("TD_TD_BUSY_sum") and vgui:
        # busy cycles summed over the 256 CUs' TA / TD units, against the
        # CU cycles of the same pass (GRBM_GUI_ACTIVE summed over 8 XCDs)
        cu_cycles = 256.0 * vgui / 8.0
        res["vmem"] = {k: v[0] for k, v in vm.items()}
        res["td_busy_frac"] = vm["TD_TD_BUSY_sum"][0] / cu_cycles
        res["ta_busy_frac"] = vm.get("TA_TA_BUSY_sum", (0, 0))[0] / cu_cycles
        res["td_tc_stall_frac"] = vm.get("TD_TC_STALL_sum", (0, 0))[0] / cu_cycles
    vi = counters(os.path.join(root, "vinst"))
    if vi.get("SQ_INSTS_VMEM_RD"):
        # vector-memory wave-instructions and L1 (TCP) cache accesses per
        # launch (profile pass 6): bench.py prices each read instruction at
        # 64 lanes x 16 B (the TD's per-instruction charge)
        res["vinst"] = {k: v[0] for k, v in vi.items()}
        res["vmem_rd_insts_per_launch"] = vi["SQ_INSTS_VMEM_RD"][0]
        res["vmem_wr_insts_per_launch"] = vi.get("SQ_INSTS_VMEM_WR", (0, 0))[0]
        res["ta_flat_read_wavefronts_per_launch"] = vi.get("TA_FLAT_READ_WAVEFRONTS_sum", (0, 0))[0]
        res["tcp_cache_accesses_per_launch"] = vi.get("TCP_TOTAL_CACHE_ACCESSES_sum", (0, 0))[0]
    cmd = os.path.join(root, "command.txt")
    if os.path.exists(cmd):
        res["command"] = open(cmd).read().strip()
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
