"""bench.py's roofline block (CPU): every roof comes from measured data, a
fraction above 1 is never reported, and algorithmic (cache-served) bytes are
never priced against HBM."""
import json
import os

import pytest

import bench
from raytracingstudy_amd._lib import kernel_source_id
import raytracingstudy_amd as rt

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PMC = os.path.join(ROOT, "profiles", "pmc_latest.json")
SIMDS = 1024  # 256 CUs x 4 SIMDs


def _pmc(cfg="c3"):
    """One config's entry of the committed summary ({config name: entry})."""
    with open(PMC) as f:
        return json.load(f)[cfg]


def test_valu_issue_is_the_bound_when_hbm_traffic_is_tiny():
    pmc = _pmc()
    kern_ms = pmc["scene_kernel_avg_ns"] / 1e6
    # C3 touches ~182 GB of node/sphere records per launch:
    # more than HBM could move in that time, so it must not be an HBM fraction
    touched = 182.19e9
    r = bench.roofline(kern_ms, touched, pmc, SIMDS)
    assert r["frac"] is not None and 0 < r["frac"] <= 1.0
    assert r["traffic"] / touched < 0.01
    # an issue roof (scalar pipe or VALU) or the vector-memory return path
    # binds, never HBM
    assert r["bound"] in ("scalar_issue", "valu_issue", "vmem_return")
    v = r["roofs"]["valu_issue"]
    insts = pmc["sq"]["SQ_INSTS_VALU"]
    peak = SIMDS * pmc["effective_clock_ghz"] / 2.0  # G wave-instructions / s
    assert v["frac"] == pytest.approx(insts / (kern_ms / 1e3) / 1e9 / peak, rel=1e-3)
    assert all(x["frac"] <= 1.0 for k, x in r["roofs"].items() if k == r["bound"])


def test_vmem_return_roof_from_td_busy():
    pmc = dict(_pmc(), td_busy_frac=0.9, ta_busy_frac=0.8, td_tc_stall_frac=0.1)
    r = bench.roofline(pmc["scene_kernel_avg_ns"] / 1e6, 182.19e9, pmc, SIMDS)
    v = r["roofs"]["vmem_return"]
    assert v["frac"] == pytest.approx(0.9)
    assert v["peak"] == pytest.approx(SIMDS / 4 * pmc["effective_clock_ghz"], rel=1e-3)
    assert v["achieved"] == pytest.approx(0.9 * v["peak"], rel=1e-3)
    assert v["ta_busy_frac"] == pytest.approx(0.8) and v["td_tc_stall_frac"] == pytest.approx(0.1)
    valid = {k: x["frac"] for k, x in r["roofs"].items() if x["frac"] <= 1.0}
    assert r["bound"] == max(valid, key=valid.get)
    # a summary without the TA/TD pass has no such roof
    q = {k: x for k, x in _pmc().items() if k not in ("td_busy_frac", "ta_busy_frac", "td_tc_stall_frac")}
    assert "vmem_return" not in bench.roofline(q["scene_kernel_avg_ns"] / 1e6, 1e9, q, SIMDS)["roofs"]


def test_over_unity_roofs_are_never_chosen():
    pmc = dict(_pmc())
    pmc["sq"] = dict(pmc["sq"], SQ_INSTS_VALU=pmc["sq"]["SQ_INSTS_VALU"] * 5)  # impossible rate
    r = bench.roofline(pmc["scene_kernel_avg_ns"] / 1e6, 1e9, pmc, SIMDS)
    assert r["roofs"]["valu_issue"]["frac"] > 1.0
    assert r["bound"] != "valu_issue" and (r["frac"] is None or r["frac"] <= 1.0)


def test_without_pmc_only_the_cache_roof_remains():
    r = bench.roofline(12.0, 182.19e9, None, SIMDS, pmc_note="stale")
    assert r["bound"] == "l2" and r["frac"] <= 1.0 and r["traffic"] is None
    assert r["pmc"] == "stale" and "hbm" not in r["roofs"]


def test_stale_pmc_summary_is_refused(tmp_path):
    pmc = dict(_pmc(), kernel_source_id="0000000000000000")
    p = tmp_path / "pmc.json"
    p.write_text(json.dumps(pmc))
    ent, why = bench.load_pmc(str(p), pmc["config"], 1, kernel_source_id())
    assert ent is None and "stale" in why
    pmc["kernel_source_id"] = kernel_source_id()
    p.write_text(json.dumps(pmc))
    ent, why = bench.load_pmc(str(p), pmc["config"], 1, kernel_source_id(),
                              pmc.get("leaf_capacity", 8))
    assert ent is not None and why == "ok"
    assert bench.load_pmc(str(p), "c5", 1, kernel_source_id())[0] is None
    # counters taken on a tree of another leaf capacity are another workload
    ent, why = bench.load_pmc(str(p), pmc["config"], 1, kernel_source_id(),
                              pmc.get("leaf_capacity", 8) + 4)
    assert ent is None and "leaf capacity" in why


def test_summary_holds_c3_and_c5_with_lane_counters():
    """the lane-utilisation counters on HEAD's kernel, for C3 and C5."""
    for cfg in ("c3", "c5"):
        ent, why = bench.load_pmc(PMC, cfg, 1, kernel_source_id(), rt.CONFIGS[cfg].leaf_capacity)
        assert ent is not None, why
        sq = ent["sq"]
        assert ent["valu_lane_util"] == pytest.approx(
            sq["SQ_THREAD_CYCLES_VALU"] / sq["SQ_ACTIVE_INST_VALU"] / 64.0)
        assert 0.0 < ent["valu_lane_util"] <= 1.0


def test_scalar_issue_roof_when_counted():
    pmc = dict(_pmc())
    sq = dict(pmc["sq"], SQ_INSTS_SALU=4.81e9, SQ_INSTS_BRANCH=1.13e9)
    pmc["sq"] = sq
    kern_ms = 11.65
    r = bench.roofline(kern_ms, 182e9, pmc, SIMDS)
    s = r["roofs"]["scalar_issue"]
    peak = SIMDS / 4 * pmc["effective_clock_ghz"]  # G instr/s
    assert s["frac"] == pytest.approx((4.81 + 1.13) / (kern_ms / 1e3) / peak, rel=1e-3)
    # the binding roof is the largest valid fraction
    valid = {k: v["frac"] for k, v in r["roofs"].items() if v["frac"] <= 1}
    assert r["bound"] == max(valid, key=valid.get)
