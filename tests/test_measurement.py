"""The bench line's launch basis: consecutive trace launches overlap on two streams, so the roofline
divides by the union of the timed launches' spans per launch, from the library's HIP events (hg_counters.trace_busy_ms,
read through bench.launch_seconds) and from rocprofv3's kernel trace (tools/summarize_profile.interval_union)."""
import importlib.util
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]


def _load(name, path):
    spec = importlib.util.spec_from_file_location(name, path)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


@pytest.fixture(scope="module")
def summ():
    return _load("summarize_profile", ROOT / "tools" / "summarize_profile.py")


@pytest.fixture(scope="module")
def bench():
    sys.path.insert(0, str(ROOT))
    return _load("bench_mod", ROOT / "bench.py")


def test_interval_union(summ):
    u = summ.interval_union
    assert u([]) == 0
    assert u([(0, 10)]) == 10
    assert u([(0, 10), (20, 30)]) == 20  # disjoint
    assert u([(0, 10), (5, 15)]) == 15  # overlapping neighbours (two trace streams)
    assert u([(5, 15), (0, 10), (12, 14)]) == 15  # unsorted, nested
    assert u([(0, 10), (10, 20)]) == 20  # touching
    # steady pipeline: launches of 48 starting every 38 units -> the union per launch tends to the period
    spans = [(38 * k, 38 * k + 48) for k in range(100)]
    assert u(spans) / len(spans) == pytest.approx(38.1)


def test_launch_seconds(bench):
    busy, span = bench.launch_seconds({"trace_busy_ms": 387.0, "trace_ms": 485.0, "trace_launches": 10})
    assert busy == pytest.approx(0.0387) and span == pytest.approx(0.0485)
    # a library without the union counter falls back to the span mean
    busy, span = bench.launch_seconds({"trace_ms": 485.0, "trace_launches": 10})
    assert busy == pytest.approx(0.0485) == span


def test_roofline_prices_the_binding_unit(bench, monkeypatch):
    """roofline.bound is the vector-memory data path when the committed profile has the VMEM instruction counts: frac
    = (SQ_INSTS_VMEM_RD + _WR) per launch / launch time / (256 CUs x 2.4 GHz / 20 cycles); VALU is the secondary
    object.  Without those counts the line falls back to the VALU issue rate."""
    monkeypatch.setattr(bench, "library_sha256", lambda: "x")
    pmc = {"valu_insts_per_launch": 26.92e9, "vmem_insts_per_launch": 0.66e9, "vmem_rd_insts_per_launch": 0.657e9,
           "vmem_wr_insts_per_launch": 0.003e9, "vmem_unit_busy": {"td_busy": 0.956, "td_stalled_on_l1": 0.51},
           "valu_lane_util": 0.51, "library_sha256": "x"}
    r = bench.roofline_of(pmc, 0.0384, 625e9, "hg_trace_stream_kernel")
    assert r["bound"] == "vmem" and r["unit"] == "Ginst/s"
    assert r["peak"] == pytest.approx(256 * 2.4 / 20)
    assert r["achieved"] == pytest.approx(0.66e9 / 0.0384 / 1e9)
    assert r["frac"] == pytest.approx(r["achieved"] / r["peak"])
    assert r["vmem"]["td_busy"] == 0.956 and r["valu"]["frac"] == pytest.approx(26.92 / 0.0384 / 1228.8)
    assert r["counters_library_matches"] is True
    del pmc["vmem_insts_per_launch"]
    r = bench.roofline_of(pmc, 0.0384, 625e9, "hg_trace_stream_kernel")
    assert r["bound"] == "valu" and r["frac"] == pytest.approx(26.92 / 0.0384 / 1228.8)


def test_committed_bench_line_keeps_the_contract():
    """The round's committed bench line (profiles/r06f_bench.json, the shipped library on the GPU box) carries the
    driver's contract keys, the roofline priced on the vector-memory unit from the committed profile of the same
    library, the cpu_baseline, and the second numbers beside the headline (framed, per_frame, fast_bvh)."""
    import json

    line = json.loads((ROOT / "profiles" / "r06f_bench.json").read_text().strip().splitlines()[-1])
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
              "vs_baseline", "dtype", "data", "config", "roofline", "cpu_baseline"):
        assert k in line, k
    assert line["unit"] == "Mpaths/s" and line["n_gpus"] == 1 and line["higher_is_better"] is True
    assert line["config"]["workload"].startswith("C3") and line["config"]["frames_per_step"] == 64
    r = line["roofline"]
    assert r["bound"] == "vmem" and r["counters_library_matches"] is True
    assert r["counters_from"] == "profiles/r06f_C3_summary.json" and (ROOT / r["counters_from"]).exists()
    assert r["frac"] == pytest.approx(r["achieved"] / r["peak"]) and 0.3 < r["frac"] < 1.0
    cpu = line["cpu_baseline"]
    assert cpu["kind"] == "port" and cpu["cores"] >= 1 and cpu["value"] > 0
    assert line["counting_replay_bit_identical"] is True
    ident = line["per_frame"]["bit_identical_to_batched"]
    assert {"coalesce_1", "coalesce_32"} <= set(ident) and all(ident.values()), ident
    # the operating points as the line's last key, inside the driver's 8-KB tail
    assert list(line)[-1] == "summary"
    tail = (ROOT / "profiles" / "r06f_bench.json").read_text()[-8192:]
    assert '"strict": {"value"' in tail and '"one_behind"' in tail
    sm = line["summary"]
    assert sm["per_frame"]["strict"]["frac_of_batched"] > 0.85
    assert sm["per_frame"]["display_r11g11b10f"]["one_behind"] > 0.7
    fast = line["fast_bvh"]
    assert fast["value"] > line["value"] and fast["pixels_differing_from_headline_image"] < 1e-3
    fr = fast["roofline"]
    assert fr["bound"] == "vmem" and fr["counters_library_matches"] is True
    assert fr["counters_from"] == "profiles/r06f_sah_C3_summary.json" and (ROOT / fr["counters_from"]).exists()
