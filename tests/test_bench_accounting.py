"""CPU tests of bench.py's roofline accounting (no GPU): the algorithmic bytes each stage is priced
at follow the path the waves took (LDS level 1, grid-wide counting or radix grouping, text staged by
the first walk, no run contraction), every stage gets a roofline, and the dominant one is the stage
with the most device time."""
import os
import sys

import pytest

sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
import bench  # noqa: E402

STAGES = ["classify", "runs", "sortb", "count", "scan", "place", "link", "walk1", "rank", "walk2",
          "expand", "digest", "doctree", "text"]


class _Batch:
    docs = 4


def _stats(ns, launches, runs, text, waves=1):
    return [{"stage_ns": {k: ns.get(k, 0.0) for k in STAGES},
             "stage_launches": {k: launches.get(k, 0) for k in STAGES},
             "runs": runs, "text_bytes": text, "waves": waves}]


def test_lds_path_prices_the_headline_stages():
    items = 1_000_000
    st = _stats({"classify": 1e5, "runs": 9e4, "doctree": 8e4, "digest": 1e4},
                {"classify": 1, "runs": 6, "doctree": 1, "digest": 2}, runs=30_000, text=250_000)
    rf = bench.roofline_fields(st, _Batch(), items, 1e-3, pmc=False)
    slots = items + _Batch.docs
    want = 3.3828125 * slots + 8.0 * 30_000 + 1.0 * 250_000
    assert rf["rooflines"]["classify"]["alg_bytes_per_launch"] == pytest.approx(want)
    assert rf["roofline"]["kernel"] == "k_classify"  # the most device time
    # k_doctree stages the text from the tile segments: k_runs moves no text (stile_text 2), and
    # with stile_text 0 it copies every tile's text to sbytes
    assert rf["rooflines"]["runs"]["alg_bytes_per_launch"] == pytest.approx(1.125 * slots + 38.0 * 30_000)
    rf0 = bench.roofline_fields(st, _Batch(), items, 1e-3, pmc=False, stile_text=0)
    assert rf0["rooflines"]["runs"]["alg_bytes_per_launch"] == pytest.approx(
        1.125 * slots + 38.0 * 30_000 + 2.0 * 250_000)
    assert set(rf["rooflines"]) == {"classify", "runs", "doctree", "digest"}
    assert all(r["traffic"] is None for r in rf["rooflines"].values())  # (pmc=False)


def test_radix_passes_priced_per_pass():
    items, runs = 1_000_000, 900_000
    npass, npass_b = 3, 1
    st = _stats({"classify": 1e5, "runs": 1e5, "count": 1e4, "place": 3e5, "link": 5e4,
                 "sortb": 1e5, "walk1": 2e5, "rank": 1e4, "walk2": 1e5, "expand": 5e4,
                 "digest": 1e4},
                {"classify": 1, "runs": 6, "count": 1, "scan": 1, "place": npass, "link": 2,
                 "sortb": npass_b + 2, "walk1": 1, "rank": 4, "walk2": 2, "expand": 1,
                 "digest": 2}, runs=runs, text=100_000)
    rf = bench.roofline_fields(st, _Batch(), items, 1e-3, pmc=False)
    r = rf["rooflines"]
    assert r["place"]["alg_bytes_per_launch"] == pytest.approx((28.0 + 32.0 * (npass - 1)) * runs)
    assert r["sortb"]["alg_bytes_per_launch"] == pytest.approx((16.0 * npass_b + 12 + 32) * runs)
    assert r["link"]["alg_bytes_per_launch"] == pytest.approx(28.0 * runs)
    # waves without contraction (runs > half the slots): classify reads no parents
    slots = items + _Batch.docs
    assert r["classify"]["alg_bytes_per_launch"] == pytest.approx(3.3828125 * slots + 100_000)
    # (the global level 1 reads the text from sbytes: k_runs copies it)
    assert r["runs"]["alg_bytes_per_launch"] == pytest.approx(1.125 * slots + 32.0 * runs + 2.0 * 100_000)
    assert rf["roofline"]["kernel"] == "place"


def test_text_mode_prices_the_staged_walk():
    items, runs, text = 1_000_000, 950_000, 400_000
    st = _stats({"classify": 1e5, "runs": 1e5, "count": 1e4, "place": 3e5, "link": 5e4,
                 "sortb": 1e5, "walk1": 2e5, "rank": 1e4, "walk2": 3e4, "digest": 1e4},
                {"classify": 1, "runs": 6, "count": 1, "scan": 1, "place": 3, "link": 2,
                 "sortb": 3, "walk1": 1, "rank": 4, "walk2": 4, "digest": 2},
                runs=runs, text=text)
    rf = bench.roofline_fields(st, _Batch(), items, 1e-3, pmc=False)
    r = rf["rooflines"]
    assert r["walk1"]["alg_bytes_per_launch"] == pytest.approx(32.0 * runs + 1.0 * text)
    assert r["walk2"]["alg_bytes_per_launch"] == pytest.approx(0.5 * runs + 2.0 * text)
    assert r["sortb"]["alg_bytes_per_launch"] == pytest.approx((16.0 + 12 + 32 + 17) * runs)
    assert rf["batched_merge"]["frac"] > 0


def test_text_scatter_mode_prices_the_text_kernel():
    """text_scatter 1: k_doctree stops at the run offsets (no text in or out of it), and the text
    stage (k_tscatter) is priced at its own in/out: the tiles' prefixes, per run its weight prefix
    and place, the tiles' text in and the documents out."""
    items, runs, text = 1_000_000, 30_000, 250_000
    st = _stats({"classify": 1e5, "runs": 9e4, "doctree": 6e4, "text": 3e4, "digest": 1e4},
                {"classify": 1, "runs": 6, "doctree": 1, "text": 1, "digest": 2}, runs=runs,
                text=text)
    rf = bench.roofline_fields(st, _Batch(), items, 1e-3, pmc=False)
    slots = items + _Batch.docs
    assert rf["rooflines"]["doctree"]["alg_bytes_per_launch"] == pytest.approx(20.0 * runs)
    assert rf["rooflines"]["text"]["alg_bytes_per_launch"] == pytest.approx(
        8.0 / 4096 * slots + 8.0 * runs + 2.0 * text)
    assert rf["rooflines"]["text"]["kernel"] == "k_tscatter"
    assert set(rf["rooflines"]) == {"classify", "runs", "doctree", "text", "digest"}

