#!/usr/bin/env python3
"""Headline benchmark: Mrays/s (primary + shadow) and ms/frame, 1/2/4/8 GPUs.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config c3]
    torchrun --nproc-per-node N bench.py --gpus N ...     (one process per GPU)
    python bench.py --gpus N                              (N > 1: one process, N GPUs)

A step is one frame of the BASELINE config (default C3: 1920x1080, 64 spp,
100k spheres, depth-7 octree).  `--gpus N` measures N GPUs however it is
launched (launch_mode): under torchrun the world must be N (else exit 2);
without a launcher N > 1 (or --native) drives the N devices from this one
process through the C-ABI's multi-device handle, rt_create_multi, which the
reference's Displayer would call (run_native: RCCL ncclCommInitAll, grouped
send/recv, one unpack); N > visible GPUs exits 2.  N=1 renders the whole
frame.  Under torchrun, N>1 deals 64x64
tiles round-robin over the ranks, each rank renders its tiles
into a packed slab, the slabs are gathered to rank 0 over RCCL and unpacked
into the frame there — the gather is inside the timed step.  The frame is the
same for every N (strong scaling, BASELINE metric "at 1920x1080").  On the
tile path `--inflight F` (default 2) frames are in flight: frame k renders on
stream k mod F with its own renderer (own queue heads and counters), slab and
receive buffer, and its gather (RCCL's stream waits for that render) and
unpack (stream k mod F waits for the gather) overlap frame k+1's render.
Every timed frame is rendered, gathered and unpacked in full inside the
timed region.  N=1 renders whole frames one after another on one stream.

Rank 0 prints ONE JSON line.  Rays are counted by the kernel (primary + shadow
rays actually cast) — the counts equal the CPU oracle's (tests/test_gpu_parity).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

NODE_BYTES = 8     # uint2 node record
PRIM_BYTES = 16    # float4 sphere record per ray-sphere test
PIXEL_BYTES = 4    # RGBA8 framebuffer write
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
# scalar pipeline (SALU + branch instructions) per CU: one per cycle
# (MI355X_MICROARCH.md: 1 scalar unit per CU; measured 0.99 SALU and 1.07
# SALU+branch per CU-cycle by tools/scalar_peak.hip, profiles/r02/scalar_peak.json)
SCALAR_PER_CU_CYCLE = 1.0
L2_PEAK_GBS = 34500.0  # MI355X_MICROARCH.md "L2 (per XCD)": ~34.5 TB/s over the 8 XCDs
# what the TD charges one vector-memory read wave-instruction: 64 lanes x 16 B
# (a dwordx2 or one-lane load costs what a wave-wide dwordx4 does)
VMEM_CHARGE_BYTES = 64 * 16


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    # ~2 s of timed frames at N = 1 (9.3 ms each): long enough for an outside
    # busy probe (rocm-smi) to see the GPU working, and for a stable median
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--config", default="c3")
    ap.add_argument("--cpu-baseline", choices=["auto", "off"], default="auto")
    ap.add_argument("--cpu-seconds", type=float, default=15.0,
                    help="target CPU-baseline sample duration")
    ap.add_argument("--variant", type=int, default=0, help="scene-kernel variant (0 = default)")
    ap.add_argument("--shard", default="",
                    help="R/N: render only rank R's tiles of an N-way split on this one GPU "
                         "(projects the per-GPU kernel time of an N-GPU run; no gather)")
    ap.add_argument("--tiles", action="store_true",
                    help="use the multi-GPU tile path (render_tiles + gather + unpack) even at N=1, "
                         "and check the frame against a whole-frame render")
    ap.add_argument("--backend", default="nccl", choices=("nccl", "gloo"),
                    help="process-group backend for N>1 (nccl = RCCL; gloo only to rehearse "
                         "the multi-rank path on one GPU)")
    ap.add_argument("--inflight", type=int, default=2,
                    help="tile path (N>1, --tiles): frames in flight, each with its own renderer, "
                         "stream, slab and receive buffer, so frame k's gather and unpack overlap "
                         "frame k+1's render (1 = strictly one frame after another)")
    ap.add_argument("--same-device", action="store_true",
                    help="rehearsal: every rank uses cuda:0 (with --backend gloo)")
    ap.add_argument("--secondary", default="c2,c5,c5d",
                    help="N=1 only: also time these configs (a few frames each) and report them "
                         "under `secondary`; '' to skip")
    ap.add_argument("--pmc", default=os.path.join(ROOT, "profiles", "pmc_latest.json"),
                    help="PMC traffic summary written by tools/pmc_traffic.py")
    ap.add_argument("--native", action="store_true",
                    help="drive the N GPUs from this one process through the C-ABI's multi-device "
                         "handle (rt_create_multi: tiles round-robin, RCCL gather, one unpack), the "
                         "path the reference's Displayer calls; the default without a launcher at N > 1")
    ap.add_argument("--transport", default="auto", choices=("auto", "rccl", "peer"),
                    help="--native: slab transport (auto = RCCL for distinct devices)")
    return ap.parse_args(argv)


class stdout_to_stderr:
    """Send file descriptor 1 to stderr for a block: RCCL's version banner and
    gloo's connection messages are printed from C++ on stdout, where the
    bench's one JSON line must be the only output."""

    def __enter__(self):
        sys.stdout.flush()
        self.saved = os.dup(1)
        os.dup2(2, 1)
        return self

    def __exit__(self, *exc):
        sys.stdout.flush()
        os.dup2(self.saved, 1)
        os.close(self.saved)
        return False


def launch_mode(gpus: int, native: bool, env) -> tuple:
    """Which path `--gpus N` measures: ("single" | "torchrun" | "native", None),
    or (None, why) when the launch cannot measure N GPUs as asked.

    * under torchrun (WORLD_SIZE set) the world must be N: one process per GPU,
      the tile path with the RCCL gather (N > 1) or the whole frame (N = 1);
    * without a launcher, N > 1 (or --native) drives N devices from this one
      process through rt_create_multi, as the reference's Displayer would;
    * N = 1 without a launcher renders whole frames on one GPU."""
    if gpus < 1:
        return None, f"--gpus {gpus}: at least 1"
    ws = env.get("WORLD_SIZE")
    if ws is not None:
        if int(ws) != gpus:
            return None, (f"--gpus {gpus} but WORLD_SIZE={ws}: launch torchrun with "
                          f"--nproc-per-node {gpus}, or run without a launcher for the native path")
        if native:
            return None, "--native drives every GPU from one process: run it without torchrun"
        return ("torchrun" if gpus > 1 else "single"), None
    return ("native" if native or gpus > 1 else "single"), None


def cpu_baseline(cfg, K, pose, target_s: float) -> dict:
    """The oracle (scalar C port, OpenMP over rows) on a bounded row sample."""
    import numpy as np

    import oracle
    import raytracingstudy_amd as rt

    sp, al = rt.configs.scene_spheres(cfg, rt.SEED)
    sc = oracle.Scene(sp, al, max_depth=cfg.max_depth, leaf_capacity=cfg.leaf_capacity)
    threads = int(os.environ.get("OMP_NUM_THREADS", "0")) or oracle.max_threads()
    # calibrate on one row, then take every step-th row for ~target_s seconds
    t = time.perf_counter()
    _, _, c = sc.render(cfg.width, cfg.height, pose, K, spp=cfg.spp, rect=(0, cfg.height // 2, cfg.width,
                        cfg.height // 2 + 1), n_threads=1, radiance=False)
    one_row = max(time.perf_counter() - t, 1e-4)
    rows = max(1, min(cfg.height, int(target_s * threads * 0.8 / one_row)))
    step = max(1, cfg.height // rows)
    t = time.perf_counter()
    _, _, c = sc.render(cfg.width, cfg.height, pose, K, spp=cfg.spp, row_step=step, row_phase=step // 2,
                        n_threads=threads, radiance=False)
    el = time.perf_counter() - t
    rays = int(c[0]) + int(c[1])
    n_rows = len(range(step // 2, cfg.height, step))
    # also one core, on 16 evenly spaced rows
    s1 = max(1, cfg.height // 16)
    t = time.perf_counter()
    _, _, c1 = sc.render(cfg.width, cfg.height, pose, K, spp=cfg.spp, row_step=s1, row_phase=s1 // 2,
                         n_threads=1, radiance=False)
    el1 = time.perf_counter() - t
    rays1 = int(c1[0]) + int(c1[1])
    return {"value": round(rays / el / 1e6, 3), "unit": "Mrays/s", "cores": threads, "kind": "port",
            "sample": f"{cfg.name} scene, every {step}th row ({n_rows} rows x {cfg.width} px x "
                      f"{cfg.spp} spp = {int(c[0])} primary + {int(c[1])} shadow rays) in {el:.1f} s",
            "single_core": {"value": round(rays1 / el1 / 1e6, 3), "unit": "Mrays/s", "cores": 1,
                            "sample": f"every {s1}th row ({rays1} rays) in {el1:.2f} s"}}


def load_pmc(path: str, cfg_name: str, world: int, src_id: str, leaf_capacity: int = 8):
    """The committed PMC summary (tools/pmc_traffic.py output) for this config
    and GPU count, or (None, reason) when it is missing, taken on another
    config or octree leaf capacity, or stamped with other kernel sources than
    this build's."""
    try:
        with open(path) as f:
            pm = json.load(f)
    except (OSError, ValueError) as e:
        return None, f"no PMC summary ({e.__class__.__name__})"
    ent = pm if pm.get("config") == cfg_name else pm.get(cfg_name)
    if not isinstance(ent, dict) or ent.get("n_gpus", 1) != world:
        return None, f"PMC summary is not for {cfg_name} on {world} GPU(s)"
    if ent.get("kernel_source_id") != src_id:
        return None, (f"PMC summary stamped {ent.get('kernel_source_id')!r}, kernel sources are "
                      f"{src_id!r}: stale, not used")
    if ent.get("leaf_capacity", 8) != leaf_capacity:
        return None, (f"PMC summary taken at leaf capacity {ent.get('leaf_capacity', 8)}, "
                      f"the config builds {leaf_capacity}: stale, not used")
    return ent, "ok"


# per-launch counts of a PMC summary that scale with the work a launch does
# (a rank's share of the frame); fractions, the clock and lane use do not
PMC_PER_LAUNCH = ("hbm_bytes_per_launch", "valu_insts_per_launch", "vmem_rd_insts_per_launch",
                  "vmem_wr_insts_per_launch", "tcp_cache_accesses_per_launch")


def project_pmc(ent: dict, share: float, note: str) -> dict:
    """The N=1 PMC entry of a config projected onto a launch that does `share`
    of the frame's work (N>1 lines had no PMC roofs).
    Per-launch counts are scaled by the share; busy fractions (TD, TA), the
    clock and lane utilisation are kept as measured at N=1.  The result says
    so in `projected`, which roofline() copies into the line."""
    p = dict(ent)
    for k in PMC_PER_LAUNCH:
        if p.get(k) is not None:
            p[k] = float(p[k]) * share
    if isinstance(p.get("sq"), dict):
        p["sq"] = {k: (float(v) * share if k.startswith("SQ_INSTS") else v) for k, v in p["sq"].items()}
    p["projected"] = note
    return p


def pmc_for_launch(path: str, cfg, world: int, src_id: str, share: float):
    """(PMC entry, note) for a launch doing `share` of `cfg`'s frame on one of
    `world` GPUs: the entry measured at that GPU count if the summary has one,
    else the N=1 entry projected by the share (project_pmc)."""
    ent, note = load_pmc(path, cfg.name, world, src_id, cfg.leaf_capacity)
    if ent is not None and share >= 0.999999:
        return ent, note
    ent1, note1 = load_pmc(path, cfg.name, 1, src_id, cfg.leaf_capacity)
    if ent1 is None:
        return None, note1
    return project_pmc(ent1, share,
                       f"projected from the N=1 counters of {cfg.name} (the whole-frame kernel), per-launch "
                       f"counts scaled by this launch's share of the frame's rays ({share:.4f}); busy "
                       f"fractions, clock and lane use as measured at N=1"), "projected"


def roofline(kern_ms: float, touched_bytes: float, pmc, simds: int, pmc_path: str = "",
             pmc_note: str = "") -> dict:
    """SURVEY 8d D3/D4's roofline of the scene kernel, plus what binds it.

    Headline (`bound`, `achieved`, `peak`, `frac`): the D4 algorithmic bytes
    (node records x 8 B + sphere records x 16 B touched, from the oracle's
    counters which the GPU reproduces, + 4 B per pixel written) per launch
    over the kernel time, against the peak of the level that SERVES them:
    the L2s' aggregate ~34.5 TB/s (MI355X_MICROARCH.md "L2 (per XCD)").  The
    scene is cache-resident, so those bytes never come from HBM:

        frac = D4_bytes / kernel_s / 34.5e12          

    Beside it:
      * hbm_literal: the same bytes against HBM's 8 TB/s, as D3 literally
        prices them.  Above 1, which proves they are not HBM-served;
      * hbm_counter: the HBM bytes the PMC counters saw per launch
        (2 x FETCH_SIZE + WRITE_SIZE, gfx950 correction) over 8 TB/s;
      * binding_unit: the busiest unit by the PMC counters: the texture-data
        (TD) unit that returns vector loads to VGPRs (TD_TD_BUSY per
        CU-cycle; a stalled cycle counts as busy), the VALU issue slots, or
        the CU's one scalar pipe;
      * waste: charged / algorithmic bytes, where a vector-memory read
        wave-instruction (SQ_INSTS_VMEM_RD) is charged 64 lanes x 16 B at the
        TD (a dwordx2 or a one-lane load costs what a dwordx4 does,
        DESIGN.md 5.1 "What the cost is per"); waste_l1 prices the L1's
        64-B cache accesses (TCP_TOTAL_CACHE_ACCESSES) instead.
    `roofs` keeps every roof with its source."""
    secs = kern_ms / 1e3
    roofs = {}
    traffic = None
    src = ""
    clock = None
    if pmc:
        traffic = pmc.get("hbm_bytes_per_launch")
        insts = pmc.get("valu_insts_per_launch", pmc.get("sq", {}).get("SQ_INSTS_VALU"))
        clock = pmc.get("clock_ghz", pmc.get("effective_clock_ghz"))
        src = f"rocprofv3 --pmc ({os.path.relpath(pmc_path, ROOT) if pmc_path else 'PMC summary'}, " \
              f"kernel sources {pmc.get('kernel_source_id')})"
        if insts and clock:
            peak = simds * clock * 1e9 / 2.0
            rate = insts / secs
            roofs["valu_issue"] = {"achieved": round(rate / 1e9, 2), "peak": round(peak / 1e9, 2),
                                   "unit": "G wave-instr/s", "frac": round(rate / peak, 4),
                                   "insts_per_launch": insts, "clock_ghz": round(clock, 4),
                                   "simds": simds, "source": src + ": SQ_INSTS_VALU, GRBM_GUI_ACTIVE"}
        sq = pmc.get("sq", {})
        if sq.get("SQ_INSTS_SALU") and clock:
            # one CU = 4 SIMDs
            sc = sq["SQ_INSTS_SALU"] + sq.get("SQ_INSTS_BRANCH", 0.0)
            peak = simds / 4 * clock * 1e9 * SCALAR_PER_CU_CYCLE
            rate = sc / secs
            roofs["scalar_issue"] = {"achieved": round(rate / 1e9, 2), "peak": round(peak / 1e9, 2),
                                     "unit": "G instr/s", "frac": round(rate / peak, 4),
                                     "salu_per_launch": sq["SQ_INSTS_SALU"],
                                     "branch_per_launch": sq.get("SQ_INSTS_BRANCH"),
                                     "source": src + ": SQ_INSTS_SALU + SQ_INSTS_BRANCH vs 1 per "
                                                     "CU-cycle (tools/scalar_peak.hip)"}
        if pmc.get("td_busy_frac") is not None and clock:
            peak = simds / 4 * clock
            frac = pmc["td_busy_frac"]
            roofs["vmem_return"] = {
                "achieved": round(frac * peak, 2), "peak": round(peak, 2),
                "unit": "G TD-busy CU-cycles/s", "frac": round(frac, 4),
                "ta_busy_frac": round(pmc.get("ta_busy_frac", 0.0), 4),
                "td_tc_stall_frac": round(pmc.get("td_tc_stall_frac", 0.0), 4),
                "source": src + ": TD_TD_BUSY_sum, TA_TA_BUSY_sum, TD_TC_STALL_sum per "
                                "CU-cycle (GRBM_GUI_ACTIVE of the same pass)"}
        if traffic:
            rate = traffic / secs / 1e9
            roofs["hbm"] = {"achieved": round(rate, 3), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                            "frac": round(rate / HBM_PEAK_GBS, 6), "bytes_per_launch": traffic,
                            "source": src + ": 2 x FETCH_SIZE + WRITE_SIZE"}
    l2 = touched_bytes / secs / 1e9
    roofs["l2"] = {"achieved": round(l2, 1), "peak": L2_PEAK_GBS, "unit": "GB/s",
                   "frac": round(l2 / L2_PEAK_GBS, 4), "touched_bytes_per_launch": int(touched_bytes),
                   "source": "SURVEY 8d D4 algorithmic bytes (oracle counters) vs "
                             "MI355X_MICROARCH.md L2 aggregate ~34.5 TB/s; L1/L2-served"}
    top = roofs["l2"]
    out = {"bound": "l2", "achieved": top["achieved"], "peak": top["peak"], "unit": top["unit"],
           "frac": top["frac"], "traffic": traffic,
           "served_by": "L1/L2: the scene is cache-resident (HBM sees the framebuffer and little else)",
           "formula": "frac = D4 bytes per launch / kernel s / 34.5e12 B/s; D4 = nodes_visited x 8 + "
                      "prims_tested x 16 + pixels x 4 (SURVEY 8d D4, DESIGN.md 5.2)",
           "algorithmic_bytes": int(touched_bytes), "kernel_ms": round(kern_ms, 4),
           "hbm_literal": {"achieved": top["achieved"], "peak": HBM_PEAK_GBS, "unit": "GB/s",
                           "frac": round(l2 / HBM_PEAK_GBS, 4), "hbm_served": False,
                           "note": "D4 bytes priced against HBM as SURVEY 8d D3 states it; > 1 "
                                   "because they are served by L1/L2, not HBM"}}
    if "hbm" in roofs:
        h = roofs["hbm"]
        out["hbm_counter"] = {"bytes_per_launch": h["bytes_per_launch"], "achieved": h["achieved"],
                              "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": h["frac"],
                              "source": h["source"]}
    units = {k: roofs[k] for k in ("vmem_return", "valu_issue", "scalar_issue") if k in roofs
             and roofs[k]["frac"] <= 1.0}
    if units:
        b = max(units, key=lambda k: units[k]["frac"])
        names = {"vmem_return": "TD: texture-data unit (vector-memory return to VGPRs)",
                 "valu_issue": "VALU issue", "scalar_issue": "scalar pipe (SALU + branch)"}
        out["binding_unit"] = {"unit": b, "what": names[b], "busy_frac": units[b]["frac"],
                               "others": {k: v["frac"] for k, v in units.items() if k != b}}
        if b == "vmem_return":
            out["binding_unit"]["ta_busy_frac"] = units[b]["ta_busy_frac"]
            out["binding_unit"]["td_tc_stall_frac"] = units[b]["td_tc_stall_frac"]
    if pmc and pmc.get("vmem_rd_insts_per_launch") and touched_bytes:
        rd = float(pmc["vmem_rd_insts_per_launch"])
        charged = rd * VMEM_CHARGE_BYTES
        out["waste"] = round(charged / touched_bytes, 4)
        out["charged_bytes"] = int(charged)
        out["vmem_rd_insts_per_launch"] = int(rd)
        tcp = pmc.get("tcp_cache_accesses_per_launch")
        if tcp:
            out["waste_l1"] = round(tcp * 64.0 / touched_bytes, 4)
        out["waste_source"] = (src + ": SQ_INSTS_VMEM_RD x 64 lanes x 16 B (charged) and "
                               "TCP_TOTAL_CACHE_ACCESSES x 64 B (waste_l1) over the D4 bytes")
    out["roofs"] = roofs
    if not pmc:
        out["pmc"] = pmc_note
    elif pmc.get("projected"):
        out["pmc_projected"] = pmc["projected"]
    return out


def secondary_config(rt, torch, name: str, dev, stream, steps: int = 3, pmc_path: str = "",
                     simds: int = 1024, min_s: float = 0.5, max_frames: int = 400) -> dict:
    """Time another BASELINE config on this GPU: kernel ms (HIP events on the
    launch stream, the median of at least `steps` frames and of as many more
    as fill `min_s` seconds, at most `max_frames`), Mrays/s from the counted
    rays, scene build time, and its roofline when the PMC summary holds this
    config at this build's kernel sources (profiles/pmc_latest.json, key =
    config name)."""
    import numpy as np
    from raytracingstudy_amd.camera import scene_pose

    c = rt.CONFIGS[name]
    sp, al = rt.configs.scene_spheres(c, rt.SEED)
    r2 = rt.KernelRenderer(c.width, c.height, mode="scene", spp=c.spp, device=dev.index)
    try:
        r2.resize(c.width, c.height)
        r2.setPosition(scene_pose())
        info = r2.set_scene(sp, al, max_depth=c.max_depth, leaf_capacity=c.leaf_capacity)
        rebuild = r2.set_scene(sp, al, max_depth=c.max_depth, leaf_capacity=c.leaf_capacity)
        st = r2.render(None, stream.cuda_stream, stats=True)
        rays = st.primary_rays + st.shadow_rays
        ms = []
        while len(ms) < steps or (sum(ms) < 1e3 * min_s and len(ms) < max_frames):
            e0 = torch.cuda.Event(enable_timing=True)
            e1 = torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            r2.render(None, stream.cuda_stream)
            e1.record(stream)
            e1.synchronize()
            ms.append(e0.elapsed_time(e1))
        k = float(np.median(ms))
        alg = (st.nodes_visited * NODE_BYTES + st.prims_tested * PRIM_BYTES +
               c.width * c.height * PIXEL_BYTES)
        pmc, note = (load_pmc(pmc_path, name, 1, rt._lib.kernel_source_id(), c.leaf_capacity)
                     if pmc_path else (None, ""))
        roof = roofline(k, alg, pmc, simds, pmc_path, note)
        roof["time_ms"] = round(k, 4)
        roof["per_ray"] = {"nodes": st.nodes_visited / rays, "prims": st.prims_tested / rays}
        if pmc and pmc.get("valu_lane_util") is not None:
            roof["valu_lane_util"] = round(pmc["valu_lane_util"], 4)
        return {"roofline": roof, "workload": f"{c.width}x{c.height}, {c.spp} spp, {c.n_spheres} {c.scene} spheres, "
                            f"max depth {info['max_depth']}",
                "depth_reached": info["depth_reached"], "cell_table_depth": info["cell_table_depth"],
                "kernel_ms": round(k, 3), "frames": len(ms), "Mrays_s": round(rays / k / 1e3, 1),
                "rays_per_frame": int(rays), "scene_build_ms": round(info["build_ms"], 2),
                "scene_rebuild_ms": round(rebuild["build_ms"], 2),
                "octree_nodes": info["n_nodes"], "prim_refs": info["n_prim_refs"]}
    finally:
        r2.close()


def run_native(args) -> int:
    """`--gpus N` without a launcher: ONE process drives N devices through the
    C-ABI's multi-device handle (rt_create_multi; SURVEY 8e E1 "one process,
    8 devices, ncclCommInitAll"), the path the reference's Displayer calls
    (src/window/displayer.cpp:28,51).  A step is one rt_render
    of the whole frame: every device renders its round-robin 64x64 tiles into
    a slab, the slabs travel to devices[0] (grouped ncclSend / ncclRecv, or
    peer copies) and ONE unpack assembles the frame; two frames are in flight
    inside the handle.  The K timed steps run back to back, bracketed by
    rt_synchronize (every device's streams); ms per step is wall time, with
    HIP events on devices[0]'s output stream beside it."""
    import numpy as np
    import torch

    import raytracingstudy_amd as rt
    from raytracingstudy_amd.camera import scene_pose

    cfg = rt.CONFIGS[args.config]
    if cfg.mode != "scene":
        raise SystemExit("bench runs a scene config (c2..c5)")
    n = args.gpus
    seen = rt.device_count()
    devs = [0] * n if args.same_device else list(range(n))
    if max(devs) >= seen:
        print(f"bench.py: --gpus {n} needs {n} visible GPUs, {seen} visible "
              f"(--same-device rehearses the plan on GPU 0)", file=sys.stderr)
        return 2
    W, H, ts = cfg.width, cfg.height, rt.configs.TILE_SIZE
    sp, al = rt.configs.scene_spheres(cfg, rt.SEED)
    pose = scene_pose()
    kw = dict(mode="scene", spp=cfg.spp, light_dir=rt.configs.LIGHT_DIR, ambient=rt.configs.AMBIENT,
              variant=args.variant)
    with stdout_to_stderr():  # ncclCommInitAll prints RCCL's banner
        r = rt.KernelRenderer(W, H, devices=devs, transport=args.transport, **kw)
    r.resize(W, H)
    r.setPosition(pose)
    info = r.set_scene(sp, al, max_depth=cfg.max_depth, leaf_capacity=cfg.leaf_capacity)
    rebuild = r.set_scene(sp, al, max_depth=cfg.max_depth, leaf_capacity=cfg.leaf_capacity)
    st = r.render(stats=True)  # counters summed over the devices (equal to the oracle's)
    rays_frame = st.primary_rays + st.shadow_rays
    for _ in range(args.warmup):
        r.render()
    r.synchronize()
    dev0 = torch.device("cuda", devs[0])
    out_stream = torch.cuda.ExternalStream(r.stream_ptr(), device=dev0)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(out_stream)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        r.render()
    e1.record(out_stream)
    r.synchronize()
    elapsed = time.perf_counter() - t0
    ev_ms = e0.elapsed_time(e1)
    # outside the timed region: per-device times of single frames (the
    # handle waits after each), the frame against one renderer's whole frame,
    # and devices[0]'s own tiles rendered alone for its counters
    per = []
    try:  # frames record timing events from the first rt_get_multi_timing call on
        r.multi_timing()
    except rt._lib.RtError:
        pass
    for _ in range(5):
        r.render()
        per.append(r.multi_timing())
    mi = r.multi_info()
    img = r.readback()
    r.close()
    ref = rt.KernelRenderer(W, H, device=devs[0], **kw)
    ref.resize(W, H)
    ref.setPosition(pose)
    ref.set_scene(sp, al, max_depth=cfg.max_depth, leaf_capacity=cfg.leaf_capacity)
    ref.render()
    frame_ok = bool(np.array_equal(ref.readback(), img))
    T = -(-W // ts) * -(-H // ts)
    ids0 = [t for t in range(T) if t % n == 0]
    slab = torch.empty(len(ids0) * ts * ts * 4, dtype=torch.uint8, device=dev0)
    s0 = ref.render_tiles(ids0, ts, slab.data_ptr(), stats=True)
    ref.close()
    render_ms = [float(np.median([p["render_ms"][k] for p in per])) for k in range(n)]
    deliver_ms = float(np.median([p["deliver_ms"] for p in per]))
    rays0 = s0.primary_rays + s0.shadow_rays
    alg0 = s0.nodes_visited * NODE_BYTES + s0.prims_tested * PRIM_BYTES + len(ids0) * ts * ts * PIXEL_BYTES
    simds = torch.cuda.get_device_properties(dev0).multi_processor_count * 4
    pmc, note = pmc_for_launch(args.pmc, cfg, n, rt._lib.kernel_source_id(), rays0 / rays_frame)
    roof = roofline(render_ms[0], alg0, pmc, simds, args.pmc, note)
    if pmc and pmc.get("valu_lane_util") is not None:
        roof["valu_lane_util"] = round(pmc["valu_lane_util"], 4)
    roof["time_ms"] = round(render_ms[0], 4)
    roof["time_source"] = ("devices[0]'s render of its tiles, HIP events on its render stream "
                           "(rt_get_multi_timing, median of 5 single frames)")
    roof["per_ray"] = {"nodes": s0.nodes_visited / rays0, "prims": s0.prims_tested / rays0}
    value = rays_frame * args.steps / elapsed / 1e6
    out = {
        "metric": f"Mrays/s (primary+shadow) at {W}x{H}, {cfg.spp} spp, {cfg.n_spheres} spheres",
        "value": round(value, 3),
        "unit": "Mrays/s",
        "n_gpus": n,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 4),
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic (seeded spheres, SURVEY.md 8d)",
        "config": {
            "workload": f"{cfg.name}: {cfg.note}",
            "width": W, "height": H, "spp": cfg.spp, "n_spheres": cfg.n_spheres,
            "octree_depth": info["max_depth"], "octree_nodes": info["n_nodes"],
            "prim_refs": info["n_prim_refs"], "leaf_capacity": cfg.leaf_capacity,
            "parallelism": f"native-tiles{ts}x{n}",
            "launch": "native: one process, rt_create_multi over devices " + str(mi["devices"]),
            "transport": mi["transport"],
            "devices_seen": seen,
            "frames_in_flight": mi["frames_in_flight"],
            "rays_per_frame": int(rays_frame),
            "primary_per_frame": int(st.primary_rays), "shadow_per_frame": int(st.shadow_rays),
            "wall_ms_per_step": round(elapsed / args.steps * 1e3, 4),
            "event_ms_per_step": round(ev_ms / args.steps, 4),
            "device_render_ms": [round(x, 4) for x in render_ms],
            "deliver_ms": round(deliver_ms, 4),
            "tiles_frame_check": frame_ok,
            "scene_build_ms": round(info["build_ms"], 1),
            "scene_rebuild_ms": round(rebuild["build_ms"], 2),
            "scene_upload_ms": round(info["upload_ms"], 1),
        },
        "roofline": roof,
        "cpu_baseline": None,
    }
    if args.same_device:
        out["config"]["note"] = ("rehearsal: every device is GPU 0, so the per-device render times "
                                 "include the other devices' kernels")
    print(json.dumps(out), flush=True)
    return 0 if frame_ok else 1


def main():
    args = parse()
    mode, why = launch_mode(args.gpus, args.native, os.environ)
    if mode is None:
        print(f"bench.py: {why}", file=sys.stderr)
        sys.exit(2)
    if mode == "native":
        sys.exit(run_native(args))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))

    import numpy as np
    import torch
    import torch.distributed as dist

    import raytracingstudy_amd as rt
    from raytracingstudy_amd.camera import scene_pose
    from raytracingstudy_amd.dist import TileFramePipeline, TileSharder

    if args.same_device:
        if args.backend != "gloo":
            raise SystemExit("--same-device is a gloo rehearsal (RCCL needs one GPU per rank)")
        local = 0
    elif local >= torch.cuda.device_count():
        print(f"bench.py: rank {rank} needs GPU {local}, {torch.cuda.device_count()} visible",
              file=sys.stderr)
        sys.exit(2)
    torch.cuda.set_device(local)
    if world > 1:
        with stdout_to_stderr():  # RCCL's banner, gloo's connection messages
            if args.backend == "nccl":
                dist.init_process_group("nccl", device_id=torch.device("cuda", local))
            else:
                dist.init_process_group("gloo")
            dist.barrier()
    cfg = rt.CONFIGS[args.config]
    if cfg.mode != "scene":
        raise SystemExit("bench runs a scene config (c2..c5)")

    sp, al = rt.configs.scene_spheres(cfg, rt.SEED)
    r = rt.KernelRenderer(cfg.width, cfg.height, mode="scene", spp=cfg.spp, device=local,
                          light_dir=rt.configs.LIGHT_DIR, ambient=rt.configs.AMBIENT,
                          variant=args.variant)
    r.resize(cfg.width, cfg.height)
    pose = scene_pose()
    r.setPosition(pose)
    info = r.set_scene(sp, al, max_depth=cfg.max_depth, leaf_capacity=cfg.leaf_capacity)
    # the same scene again: a rebuild into the buffers the first build sized
    # (the per-frame cost of a dynamic scene; the first build also allocates)
    rebuild = r.set_scene(sp, al, max_depth=cfg.max_depth, leaf_capacity=cfg.leaf_capacity)
    _, K = r.camera()

    dev = torch.device("cuda", local)
    tiled = world > 1 or args.tiles or bool(args.shard)
    F = max(1, args.inflight) if tiled else 1
    # frames in flight: one renderer per frame slot (the queue heads and
    # counters are per renderer; the scene is built again, seeded the same)
    rs = [r]
    for _ in range(F - 1):
        r2 = rt.KernelRenderer(cfg.width, cfg.height, mode="scene", spp=cfg.spp, device=local,
                               light_dir=rt.configs.LIGHT_DIR, ambient=rt.configs.AMBIENT,
                               variant=args.variant)
        r2.resize(cfg.width, cfg.height)
        r2.setPosition(pose)
        r2.set_scene(sp, al, max_depth=cfg.max_depth, leaf_capacity=cfg.leaf_capacity)
        rs.append(r2)
    # a real (non-null) stream: the kernels, the HIP events and RCCL all run on it
    if F == 1:
        streams = [torch.cuda.Stream(dev)]
    else:
        # each frame slot on its renderer's own stream: streams made one after
        # another sit on different hardware queues, so the slots' kernels
        # overlap (two streams from torch's pool can share a queue and then
        # run one after the other, tools/stream_probe.py)
        streams = [torch.cuda.ExternalStream(rr.stream_ptr(), device=dev) for rr in rs]
    stream = streams[0]
    torch.cuda.set_stream(stream)
    sptr = stream.cuda_stream
    assert sptr, "need a non-null HIP stream handle"
    W, H, ts = cfg.width, cfg.height, rt.configs.TILE_SIZE
    frames = [torch.empty(W * H * 4, dtype=torch.uint8, device=dev) for _ in range(F)]
    frame = frames[0]
    if tiled:
        # tests/test_tiles_dist.py drives the same TileSharder with gloo on CPU
        if args.shard:
            sr, sn = (int(v) for v in args.shard.split("/"))
            sharder = TileSharder(W, H, sr, sn, ts)
            sharder.world = 1  # local projection: no gather, this GPU renders rank sr's tiles
            sharder.rank = 0
        else:
            sharder = TileSharder(W, H, rank, world, ts)
        my_ids = sharder.ids
        slabs = [sharder.new_slab(torch, device=dev) for _ in range(F)]
        packed = slabs[0]

    events = []     # [render start, render end] per timed frame
    gu_events = []  # [render end, step end (gather + unpack enqueued)] per timed frame (tile path)
    recording = [False]

    def on_render(k, phase):
        if not recording[0]:
            return
        if phase == 0:
            events.append([torch.cuda.Event(enable_timing=True), None])
            events[-1][0].record(streams[k])
        elif phase == 1:
            events[-1][1] = torch.cuda.Event(enable_timing=True)
            events[-1][1].record(streams[k])
        else:
            e = torch.cuda.Event(enable_timing=True)
            e.record(streams[k])
            gu_events.append([events[-1][1], e])

    if not tiled:
        def step(i: int, record: bool):
            k = i % F
            recording[0] = record
            with torch.cuda.stream(streams[k]):
                on_render(k, 0)
                rs[k].render(frames[k].data_ptr(), streams[k].cuda_stream)
                on_render(k, 1)
    else:
        # render -> async gather -> work.wait() -> fused unpack, F frames in
        # flight: raytracingstudy_amd.dist.TileFramePipeline, the same step
        # tests/test_tiles_dist.py drives with gloo on CPU
        pipe = TileFramePipeline(
            sharder, slabs,
            render=lambda k, slab: rs[k].render_tiles(my_ids, ts, slab.data_ptr(),
                                                      streams[k].cuda_stream),
            unpack=lambda k, buf, ids: rs[k].unpack_tiles(buf.data_ptr(), ids, ts,
                                                          frames[k].data_ptr(),
                                                          streams[k].cuda_stream),
            stream=lambda k: torch.cuda.stream(streams[k]),  # the collective waits for it
            gather=not args.shard, on_render=on_render)

        def step(i: int, record: bool):
            recording[0] = record
            pipe.step(i)

    # counted rays of one frame on this rank (deterministic; equal to the oracle's)
    if not tiled:
        st = r.render(frame.data_ptr(), sptr, stats=True)
    else:
        st = r.render_tiles(my_ids, ts, packed.data_ptr(), sptr, stats=True)
    cnt = torch.tensor([st.primary_rays, st.shadow_rays, st.nodes_visited, st.prims_tested],
                       dtype=torch.float64, device=dev)

    with stdout_to_stderr():  # a collective's first use may print too
        for i in range(args.warmup):
            step(i, False)
        torch.cuda.synchronize(dev)
        if world > 1:
            dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for i in range(args.steps):
        step(i, True)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    elapsed = time.perf_counter() - t0

    kern_ms = float(np.mean([a.elapsed_time(b) for a, b in events])) if events else float("nan")
    tile_report = None
    if tiled and not args.shard:
        # VERDICT r03 item 4, outside the timed region: per-rank render and
        # gather+unpack spans of the timed frames, this rank's tiles rendered
        # alone (one frame at a time), rank 0's whole frame alone
        gu_ms = float(np.mean([a.elapsed_time(b) for a, b in gu_events])) if gu_events else 0.0

        def alone(fn, n=5):
            ts_ = []
            for _ in range(n):
                e0 = torch.cuda.Event(enable_timing=True)
                e1 = torch.cuda.Event(enable_timing=True)
                e0.record(stream)
                fn()
                e1.record(stream)
                e1.synchronize()
                ts_.append(e0.elapsed_time(e1))
            return float(np.median(ts_))

        if world > 1:
            dist.barrier()
        share_ms = alone(lambda: r.render_tiles(my_ids, ts, packed.data_ptr(), sptr))
        if world > 1:
            dist.barrier()
        whole_ms = None
        if rank == 0:
            wbuf = torch.empty_like(frame)
            whole_ms = alone(lambda: r.render(wbuf.data_ptr(), sptr))
        from raytracingstudy_amd.dist import rank_timing_report
        tile_report = rank_timing_report(kern_ms, gu_ms, share_ms, whole_ms)
    red_dev = dev if args.backend == "nccl" else torch.device("cpu")
    el_t = torch.tensor([elapsed], dtype=torch.float64, device=red_dev)
    tot = cnt.clone().to(red_dev)
    if world > 1:
        dist.all_reduce(el_t, op=dist.ReduceOp.MAX)
        dist.all_reduce(tot, op=dist.ReduceOp.SUM)
    elapsed = float(el_t.item())
    rays_frame = float(tot[0].item() + tot[1].item())

    if rank == 0:
        value = rays_frame * args.steps / elapsed / 1e6
        # roofline of the dominant kernel on this rank: algorithmic bytes per launch
        pix = (W * H) if not tiled else len(my_ids) * ts * ts
        alg_bytes = float(cnt[2].item()) * NODE_BYTES + float(cnt[3].item()) * PRIM_BYTES + pix * PIXEL_BYTES
        simds = torch.cuda.get_device_properties(dev).multi_processor_count * 4
        src_id = rt._lib.kernel_source_id()
        if not tiled:
            pmc, pmc_note = load_pmc(args.pmc, cfg.name, world, src_id, cfg.leaf_capacity)
        elif args.shard:
            pmc, pmc_note = None, "--shard projection: no PMC roofs"
        else:
            # the tile path: this rank's launch does its share of the frame's
            # rays; the N=1 counters projected onto it
            share = float(cnt[0].item() + cnt[1].item()) / rays_frame
            pmc, pmc_note = pmc_for_launch(args.pmc, cfg, world, src_id, share)
        # frames in flight overlap, so one frame's event span is not its share
        # of the GPU: price a frame per step of wall time instead
        roof_ms = kern_ms if F == 1 else elapsed / args.steps * 1e3
        roof = roofline(roof_ms, alg_bytes, pmc, simds, args.pmc, pmc_note)
        if pmc and pmc.get("valu_lane_util") is not None:
            roof["valu_lane_util"] = round(pmc["valu_lane_util"], 4)
        roof["time_ms"] = round(roof_ms, 4)
        roof["time_source"] = ("kernel HIP events on the launch stream" if F == 1 else
                               f"wall time per step ({F} frames in flight)")
        roof["per_ray"] = {"nodes": float(cnt[2].item()) / float(cnt[0].item() + cnt[1].item()),
                           "prims": float(cnt[3].item()) / float(cnt[0].item() + cnt[1].item())}
        out = {
            "metric": f"Mrays/s (primary+shadow) at {W}x{H}, {cfg.spp} spp, {cfg.n_spheres} spheres",
            "value": round(value, 3),
            "unit": "Mrays/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic (seeded spheres, SURVEY.md 8d)",
            "config": {
                "workload": f"{cfg.name}: {cfg.note}",
                "width": W, "height": H, "spp": cfg.spp, "n_spheres": cfg.n_spheres,
                "octree_depth": info["max_depth"], "octree_nodes": info["n_nodes"],
                "prim_refs": info["n_prim_refs"], "leaf_capacity": cfg.leaf_capacity,
                "parallelism": f"tiles{ts}x{world}" if tiled else "single",
                "frames_in_flight": F,
                "rays_per_frame": int(rays_frame),
                "primary_per_frame": int(tot[0].item()), "shadow_per_frame": int(tot[1].item()),
                # with frames in flight a frame's event span overlaps the
                # other slots' kernels: it is reported as a span, not a kernel time
                "kernel_ms": round(kern_ms, 4) if F == 1 else None,
                "render_span_ms": round(kern_ms, 4),
                "wall_ms_per_step": round(elapsed / args.steps * 1e3, 4),
                "scene_build_ms": round(info["build_ms"], 1),
                "scene_rebuild_ms": round(rebuild["build_ms"], 2),
                "scene_upload_ms": round(info["upload_ms"], 1),
            },
            "roofline": roof,
            "cpu_baseline": None,
        }
        if args.shard:
            out["config"]["shard"] = args.shard
            out["metric"] += f" [projection: rank {args.shard} tiles only]"
        if tiled and not args.shard:
            # the gathered frame must equal a whole-frame render, byte for byte
            whole = torch.empty_like(frame)
            r.render(whole.data_ptr(), sptr)
            torch.cuda.synchronize(dev)
            used = frames[:min(F, args.warmup + args.steps)]  # slots that received a frame
            out["config"]["tiles_frame_check"] = all(bool(torch.equal(whole, f)) for f in used)
            if tile_report is not None:
                if args.same_device:
                    tile_report["note"] = ("rehearsal: every rank on one GPU, so the per-rank times "
                                           "include the other ranks' kernels")
                out["config"]["tile_path"] = tile_report
        if world == 1 and not args.shard and args.secondary:
            out["secondary"] = {}
            for name in [c for c in args.secondary.split(",") if c and c != cfg.name]:
                try:
                    out["secondary"][name] = secondary_config(rt, torch, name, dev, stream,
                                                              pmc_path=args.pmc, simds=simds)
                except Exception as e:  # reported, never fatal for the headline
                    out["secondary"][name] = {"error": repr(e)}
        if world == 1 and args.cpu_baseline == "auto":
            try:
                out["cpu_baseline"] = cpu_baseline(cfg, K, pose, args.cpu_seconds)
            except Exception as e:  # reported, never fatal for the GPU number
                out["cpu_baseline"] = {"error": repr(e)}
        print(json.dumps(out), flush=True)
    for rr in rs:
        rr.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
