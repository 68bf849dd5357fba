"""bench.py's roofline block (CPU): the headline is SURVEY 8d D4's algorithmic
bytes over the peak of the level that serves them (the L2 aggregate), the
literal HBM pricing and the counter HBM fraction ride beside it, the busiest
unit is named separately, and every figure comes from measured data."""
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


def test_headline_is_d4_bytes_over_the_l2_peak():
    """frac is recomputable by one division."""
    pmc = _pmc()
    kern_ms = pmc["scene_kernel_avg_ns"] / 1e6
    # C3 touches ~191 GB of node/sphere records per launch:
    # more than HBM could move in that time
    touched = 191.32e9
    r = bench.roofline(kern_ms, touched, pmc, SIMDS)
    assert r["bound"] == "l2" and r["peak"] == bench.L2_PEAK_GBS and r["unit"] == "GB/s"
    assert r["frac"] == pytest.approx(touched / (kern_ms / 1e3) / 34.5e12, rel=1e-3)
    assert r["achieved"] == pytest.approx(touched / (kern_ms / 1e3) / 1e9, rel=1e-3)
    # the literal D3 pricing against HBM is reported, above 1 and marked not HBM-served
    h = r["hbm_literal"]
    assert h["frac"] == pytest.approx(touched / (kern_ms / 1e3) / 8e12, rel=1e-3)
    assert h["frac"] > 1.0 and h["hbm_served"] is False
    # the counters' HBM bytes are a tiny fraction of peak
    assert r["traffic"] / touched < 0.01
    assert r["hbm_counter"]["frac"] == pytest.approx(r["traffic"] / (kern_ms / 1e3) / 8e12, rel=1e-3)
    # the busiest unit is reported separately, never as the roofline
    assert r["binding_unit"]["unit"] in ("scalar_issue", "valu_issue", "vmem_return")
    assert 0 < r["binding_unit"]["busy_frac"] <= 1.0
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
    units = {k: r["roofs"][k]["frac"] for k in ("vmem_return", "valu_issue", "scalar_issue")
             if k in r["roofs"] and r["roofs"][k]["frac"] <= 1.0}
    assert r["binding_unit"]["unit"] == max(units, key=units.get)
    # a summary without the TA/TD pass has no such roof
    q = {k: x for k, x in _pmc().items() if k not in ("td_busy_frac", "ta_busy_frac", "td_tc_stall_frac")}
    assert "vmem_return" not in bench.roofline(q["scene_kernel_avg_ns"] / 1e6, 1e9, q, SIMDS)["roofs"]


def test_over_unity_units_are_never_named_binding():
    pmc = dict(_pmc())
    pmc["sq"] = dict(pmc["sq"], SQ_INSTS_VALU=pmc["sq"]["SQ_INSTS_VALU"] * 5)  # impossible rate
    r = bench.roofline(pmc["scene_kernel_avg_ns"] / 1e6, 1e9, pmc, SIMDS)
    assert r["roofs"]["valu_issue"]["frac"] > 1.0
    assert r["binding_unit"]["unit"] != "valu_issue" and r["bound"] == "l2"


def test_waste_is_charged_over_algorithmic_bytes():
    """the vector-memory instructions per launch (profile
    pass 6) priced at 64 lanes x 16 B, over the D4 bytes."""
    pmc = dict(_pmc(), vmem_rd_insts_per_launch=272e6, tcp_cache_accesses_per_launch=4.19e9)
    r = bench.roofline(pmc["scene_kernel_avg_ns"] / 1e6, 191.32e9, pmc, SIMDS)
    assert r["charged_bytes"] == int(272e6 * 1024)
    assert r["waste"] == pytest.approx(272e6 * 1024 / 191.32e9, rel=1e-3)
    assert r["waste_l1"] == pytest.approx(4.19e9 * 64 / 191.32e9, rel=1e-3)
    q = {k: v for k, v in _pmc().items() if k != "vmem_rd_insts_per_launch"}
    assert "waste" not in bench.roofline(8.6, 191e9, q, SIMDS)


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
    # the binding unit is the busiest valid one
    units = {k: r["roofs"][k]["frac"] for k in ("vmem_return", "valu_issue", "scalar_issue")
             if k in r["roofs"] and r["roofs"][k]["frac"] <= 1}
    assert r["binding_unit"]["unit"] == max(units, key=units.get)
