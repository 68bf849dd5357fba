"""bench.py's `--gpus N` contract (CPU): N GPUs are
measured whichever way the bench is launched, a launch that cannot measure N
GPUs exits non-zero, and an N>1 line carries PMC roofs projected from the
N=1 counters."""
import json
import os
import subprocess
import sys

import pytest

import bench
import raytracingstudy_amd as rt
from raytracingstudy_amd._lib import kernel_source_id

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PMC = os.path.join(ROOT, "profiles", "pmc_latest.json")


def test_launch_mode_table():
    lm = bench.launch_mode
    assert lm(1, False, {}) == ("single", None)
    assert lm(8, False, {}) == ("native", None)          # no launcher, N > 1: one process
    assert lm(1, True, {}) == ("native", None)           # forced native at N = 1
    assert lm(8, False, {"WORLD_SIZE": "8"}) == ("torchrun", None)
    assert lm(1, False, {"WORLD_SIZE": "1"}) == ("single", None)
    mode, why = lm(8, False, {"WORLD_SIZE": "4"})
    assert mode is None and "WORLD_SIZE=4" in why
    mode, why = lm(2, True, {"WORLD_SIZE": "2"})
    assert mode is None and "without torchrun" in why
    assert lm(0, False, {})[0] is None


def _run_bench(args, env_extra):
    env = dict(os.environ)
    env.update(env_extra)
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, env=env,
                          capture_output=True, text=True, timeout=240)


def test_world_size_mismatch_exits_nonzero():
    """--gpus 4 under a world of 2: exit 2 before anything touches a GPU."""
    p = _run_bench(["--gpus", "4"], {"WORLD_SIZE": "2", "RANK": "0", "LOCAL_RANK": "0"})
    assert p.returncode == 2, p.stderr
    assert "WORLD_SIZE=2" in p.stderr and not p.stdout.strip()


def test_more_gpus_than_visible_exits_nonzero():
    """--gpus N without a launcher takes the native path, which refuses N >
    visible devices (this container sees none)."""
    n = rt.device_count() + 3
    env_clean = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(n),
                        "--config", "c2", "--steps", "1", "--warmup", "0"],
                       env=env_clean, capture_output=True, text=True, timeout=240)
    assert p.returncode == 2, (p.returncode, p.stderr[-2000:])
    assert "visible" in p.stderr and not p.stdout.strip()


def _c3_pmc():
    with open(PMC) as f:
        return json.load(f)["c3"]


def test_projected_pmc_scales_counts_and_keeps_fractions():
    ent = _c3_pmc()
    p = bench.project_pmc(ent, 0.125, "note")
    assert p["projected"] == "note"
    for k in bench.PMC_PER_LAUNCH:
        if ent.get(k) is not None:
            assert p[k] == pytest.approx(ent[k] * 0.125)
    assert p["sq"]["SQ_INSTS_VALU"] == pytest.approx(ent["sq"]["SQ_INSTS_VALU"] * 0.125)
    assert p["sq"].get("GRBM_GUI_ACTIVE") == ent["sq"].get("GRBM_GUI_ACTIVE")
    for k in ("td_busy_frac", "ta_busy_frac", "valu_lane_util", "effective_clock_ghz"):
        assert p.get(k) == ent.get(k)
    assert ent.get("projected") is None  # the source entry is untouched


def test_n_gt_1_line_carries_projected_binding_unit_and_waste():
    """a rank's launch of 1/2 of the C3 frame (the gloo
    world-2 rehearsal's shape) prices its own bytes over its own time and
    names the binding unit and the waste from the projected counters."""
    cfg = rt.CONFIGS["c3"]
    pmc, note = bench.pmc_for_launch(PMC, cfg, 2, kernel_source_id(), 0.5)
    assert pmc is not None and note == "projected", note
    ent = _c3_pmc()
    kern_ms = ent["scene_kernel_avg_ns"] / 1e6 / 2  # half the frame in half the time
    touched = 191.32e9 / 2
    r = bench.roofline(kern_ms, touched, pmc, 1024)
    assert "projected from the N=1 counters of c3" in r["pmc_projected"]
    assert r["binding_unit"]["unit"] in ("vmem_return", "valu_issue", "scalar_issue")
    full = bench.roofline(kern_ms * 2, touched * 2, ent, 1024)
    # half the work in half the time: the same waste, unit and fraction as N = 1
    assert r["waste"] == pytest.approx(full["waste"], rel=1e-6)
    assert r["binding_unit"]["unit"] == full["binding_unit"]["unit"]
    assert r["frac"] == pytest.approx(full["frac"], rel=1e-6)
    # at N = 1 with the whole frame the measured entry itself is used
    same, why = bench.pmc_for_launch(PMC, cfg, 1, kernel_source_id(), 1.0)
    assert why == "ok" and "projected" not in same
