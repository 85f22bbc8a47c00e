"""bench.py's roofline object on CPU: the committed profiles (profiles/sq_*.json, valu_mix_*.json, valu_ceiling.json,
pmc_traffic_*.json) priced the way the bench line prices them, with the round-3 render times. Every fraction of a
binding resource must stay <= 1: a kernel cannot beat the ceiling it is priced against."""
import argparse
import json
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def _args(config, kernel):
    return argparse.Namespace(steps=1, config=config, kernel=kernel, bvh="midpoint", pmc_json=None)


def _counters(**kw):
    c = dict(sphere_tests=0, node_pops=0, interior_visits=0, triangle_tests=0, hits=0, draw_fetches=0, pixels=0)
    c.update(kw)
    return c


def _profile(name):
    return json.load(open(os.path.join(ROOT, "profiles", name)))


def test_valu_ceiling_classes_and_mix_ceiling():
    ceil = _profile("valu_ceiling.json")
    rates = ceil["class_gwave_instr_per_s"]
    assert ceil["spec_gwave_instr_per_s"] == pytest.approx(bench.VALU_PEAK_GINSTR)
    for cfg in ("c2", "ref", "c3"):
        mix = _profile(f"valu_mix_{cfg}.json")["class_fraction"]
        assert set(mix) <= set(rates)
        assert sum(mix.values()) == pytest.approx(1.0, abs=1e-3)
        m = bench._valu_mix_ceiling(cfg)
        # a weighted harmonic mean of the class rates lies between the slowest and the fastest class used
        used = [rates[c] for c, f in mix.items() if f > 0]
        assert min(used) <= m <= max(used)


@pytest.mark.parametrize("config,render_ms", [("c2", 0.3701), ("ref", 1.259)])
def test_valu_roofline_fractions_at_most_one(config, render_ms):
    sq = _profile(f"sq_{config}.json")
    assert sq["bound"] == "valu_issue"
    r = bench.roofline(_args(config, sq["kernel"]), _counters(pixels=1920 * 1080), render_ms * 1e-3, render_ms * 1e-3)
    assert r["bound"] == "valu_issue" and r["unit"] == "G wave64 VALU instructions/s"
    assert r["peak"] == pytest.approx(1228.8)
    assert 0 < r["frac"] <= 1.0
    assert 0 < r["measured_frac"] <= 1.0
    assert r["measured_ceiling"] < r["peak"]
    # the achieved rate is the committed VALU count over the render time
    valu = sq["counters_per_launch"]["SQ_INSTS_VALU"]
    assert r["achieved"] == pytest.approx(valu / (render_ms * 1e-3) / 1e9, rel=1e-3)
    assert r["traffic"] is not None and 0 < r["hbm_measured_frac"] < 1.0


def test_memory_latency_roofline_c3():
    sq = _profile("sq_c3.json")
    assert sq["bound"] == "memory_latency"
    # one c3 frame's exact counts (round 3): 8.57 M segments, 453 M interior visits, 105 M triangle tests
    tot = _counters(interior_visits=453249769, triangle_tests=104965350, node_pops=915070762, pixels=1920 * 1080)
    r = bench.roofline(_args("c3", sq["kernel"]), tot, 4.97e-3, 4.97e-3)
    assert r["bound"] == "memory_latency"
    assert 0 < r["frac"] <= 1.0
    assert r["not_a_roofline"]["note"].startswith("cache-served")


def test_c4_profiles_priced_per_frame():
    # c4 (3840x2160, 16 spp, 4 bounces): 2 pipelines x 65 trace launches per frame -- 5 segments for sample 0 and 4 for
    # each later sample, whose primary segment reuses sample 0's record; the PMC traffic is whole-frame
    sq = _profile("sq_c4.json")
    assert sq["bound"] == "memory_latency" and sq["launches_per_frame"] == 2 * (5 + 15 * 4)
    assert sq["counters_per_launch"]["SQ_WAVES"] > 0
    r = bench.roofline(_args("c4", sq["kernel"]), _counters(pixels=3840 * 2160), 0.2612, 0.2612)
    assert r["traffic"] == _profile("pmc_traffic_c4.json")["hbm_bytes_per_frame"]
    assert 0 < r["hbm_measured_frac"] < 1.0


def test_memory_latency_roofline_takes_out_reused_primary_visits():
    # with samples > 1 the render traces each pixel's primary ray once; the reference's counts (COUNT build) include
    # the other samples' primary traversals, which bench.py passes as reused_primary_lines and prices out
    sq = _profile("sq_c4.json")
    tot = _counters(interior_visits=30_000_000_000, triangle_tests=5_000_000_000, pixels=3840 * 2160)
    full = bench.roofline(_args("c4", sq["kernel"]), dict(tot), 0.2121, 0.2121)
    tot["reused_primary_lines"] = 8_000_000_000
    r = bench.roofline(_args("c4", sq["kernel"]), tot, 0.2121, 0.2121)
    assert r["reused_primary_lines_per_frame"] == 8_000_000_000
    assert r["achieved"] == pytest.approx(full["achieved"] * (35 - 8) / 35, rel=1e-3)
    assert 0 < r["frac"] < full["frac"] <= 1.0
    # the algorithmic (reference-work) bytes are not reduced: they price the reference's traversal
    assert (r["not_a_roofline"]["algorithmic_bytes_per_render"] ==
            full["not_a_roofline"]["algorithmic_bytes_per_render"])


@pytest.mark.parametrize("config,kernel,render_ms", [("c2", 0, 0.3701), ("ref", 0, 1.259), ("c3", 2, 4.97),
                                                     ("c4", 2, 212.1)])
def test_every_frac_in_the_roofline_head_is_physical(config, kernel, render_ms):
    """every `frac` at the top level of the roofline object is a fraction of a physical ceiling
    (<= 1); the SURVEY 8(d) bytes, which exceed the HBM peak on these cache-resident scenes, live under
    not_a_roofline only."""
    tot = _counters(interior_visits=453249769, triangle_tests=104965350, node_pops=915070762, sphere_tests=10 ** 9,
                    hits=10 ** 7, draw_fetches=10 ** 7, pixels=1920 * 1080)
    r = bench.roofline(_args(config, kernel), tot, render_ms * 1e-3, render_ms * 1e-3)
    fracs = {k: v for k, v in r.items() if k.endswith("frac") and v is not None}
    assert fracs and all(0 < v <= 1.0 for v in fracs.values()), fracs
    assert not any(k.startswith("algorithmic") for k in r)
    assert r["not_a_roofline"]["algorithmic_gbs"] > 0


@pytest.mark.parametrize("config,kernel,frame_ms,block_ms", [("c2", 0, 0.07, 0.052), ("c3", 2, 0.75, 0.70)])
def test_multi_gpu_roofline_prices_the_frame_against_every_device(config, kernel, frame_ms, block_ms):
    """An 8-GPU line renders one frame over 8 devices: its whole-frame work over the slowest block's time is priced
    against 8 x each per-GPU ceiling, so every frac stays <= 1 and equals the one-GPU frac of the same per-GPU rate.
    A rehearsal (4 ranks on one GPU) is priced against that one GPU over the frame time."""
    tot = _counters(interior_visits=453249769, triangle_tests=104965350, node_pops=915070762, sphere_tests=10 ** 9,
                    hits=10 ** 7, draw_fetches=10 ** 7, pixels=1920 * 1080)
    r8 = bench.roofline(_args(config, kernel), dict(tot), block_ms * 1e-3, frame_ms * 1e-3, devices=8, ranks=8)
    r1 = bench.roofline(_args(config, kernel), dict(tot), 8 * block_ms * 1e-3, 8 * frame_ms * 1e-3)
    assert r8["devices"] == 8 and "devices" not in r1
    assert r8["peak"] == pytest.approx(8 * r1["peak"], rel=1e-3)
    assert r8["frac"] == pytest.approx(r1["frac"], rel=2e-3)
    fracs = {k: v for k, v in r8.items() if k.endswith("frac") and v is not None}
    assert fracs and all(0 < v <= 1.0 for v in fracs.values()), fracs
    reh = bench.roofline(_args(config, kernel), dict(tot), 0.2e-3, 8 * frame_ms * 1e-3, devices=1, ranks=4)
    whole = bench.roofline(_args(config, kernel), dict(tot), 8 * frame_ms * 1e-3, 8 * frame_ms * 1e-3)
    assert reh["frac"] == pytest.approx(whole["frac"], rel=2e-3) and "devices" not in reh
