"""The whole-frame goldens of the BASELINE frames (tools/make_goldens.py --frames: the
reference's own render of C3, the headline and C4, scene.cpp:31-64) are self-consistent, and the
host frame finish (rt_tonemap_u8, scene.cpp:54-64) turns their float rows into the
reference's 8-bit rows.  CPU only; the GPU comparison is tests/test_gpu_configs.py
test_whole_frame_matches_reference."""
import json
import os

import numpy as np
import pytest

import rtref

FRAMES = json.load(open(os.path.join(rtref.GOLD, "golden_meta.json"))).get("frames", {})


@pytest.mark.parametrize("config", ["c3", "headline", "c4"])
def test_frame_golden_is_consistent(rt, config):
    f = FRAMES[config]
    W, H, S = f["width"], f["height"], f["spp"]
    g = rtref.golden(f["file"])
    assert g["row_fnv1a"].shape == (H,)
    rows = g["rows"]
    assert np.array_equal(rtref.row_hash(g["row_sums"]), g["row_fnv1a"][rows])
    assert int(g["counters"][0]) == f["sums"]["rays"]
    if "row_u8" in g:
        assert np.array_equal(rt.tonemap(g["row_sums"], S), g["row_u8"])


def test_bench_knows_the_reference_frame():
    import importlib.util
    import sys
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(rtref.ROOT, "bench.py"))
    b = importlib.util.module_from_spec(spec)
    argv = sys.argv
    try:
        spec.loader.exec_module(b)
    finally:
        sys.argv = argv
    f = FRAMES["headline"]
    assert b.reference_frame_sha1("sponza", 1920, 1080, 256) == f["frame_u8_sha1"]
    assert b.reference_frame_sha1("sponza", 1920, 1080, 1024) == FRAMES["c4"]["frame_u8_sha1"]
    assert b.reference_frame_sha1("sponza", 1920, 1080, 64) is None


def test_c5_row_golden_is_consistent():
    """The C5 full-row golden (tools/make_goldens.py --c5rows): 8 rows of each rank's shard of
    the 8-way split (rows with (row / 8) % 8 == rank), the full rows' hashes equal their
    entries, and the per-row counters add up to the reference's totals for those pixels."""
    c = json.load(open(os.path.join(rtref.GOLD, "golden_meta.json")))["configs"]["c5_rows"]
    g = rtref.golden(c["file"])
    rows = g["rows"].astype(np.int64)
    per = c["rows_per_rank"]
    assert len(rows) == c["world"] * per == len(np.unique(rows))
    for rank in range(c["world"]):
        assert all((int(r) // 8) % c["world"] == rank for r in rows[rank * per:(rank + 1) * per])
    assert np.array_equal(g["full_rows"], rows[::per])
    assert np.array_equal(rtref.row_hash(g["full_row_sums"]), g["row_fnv1a"][::per])
    tot = g["row_counters"].sum(axis=0)
    p = c["pixels"]
    assert [int(x) for x in tot] == [p["rays"], p["aabb"], p["tri"], p["light_queries"], p["light_aabb"], p["light_tri"]]
    assert p["pixels"] == len(rows) * c["width"]
