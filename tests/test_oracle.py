"""The oracle (oracle/rt_oracle.cpp, the CPU restatement used as the checker) pinned against the
reference's own outputs (tests/golden, written by oracle/ref_harness built from the reference
sources): per-pixel sums and traversal counters, ray-level closest hits and light pdfs, and
rows of BASELINE.json's C2 frame (cornell 512x512x64)."""
import numpy as np
import pytest

import rtref

CASES = [("cornell", 33, 17, 3), ("cornell", 64, 64, 8), ("cornell_blob", 48, 48, 4),
         ("practice6_1", 256, 256, 4), ("sponza_mini", 64, 36, 4)]


@pytest.mark.parametrize("name,w,h,s", CASES)
def test_oracle_sums_match_reference(rt, oracle, name, w, h, s):
    g = rtref.golden(f"{name}_sums_{w}x{h}x{s}.rtd")
    out, cnt, _ = oracle.render(rtref.ref_arrays(rt, name, w, h, s), s)
    assert np.array_equal(rtref.bits(out), rtref.bits(g["sums"].reshape(-1, 3)))
    assert list(cnt) == list(g["counters"])


@pytest.mark.parametrize("name", ["cornell", "cornell_blob", "practice6_1", "sponza_mini"])
def test_oracle_rays_match_reference(rt, oracle, name):
    g = rtref.golden(f"{name}_rays.rtd")
    out_f, out_i = oracle.rays(rtref.ref_arrays(rt, name, 64, 64, 1), g["origin"], g["direction"])
    hit = g["hit"].astype(bool)
    assert np.array_equal(out_i[:, 0].astype(bool), hit)
    assert np.array_equal(out_i[hit, 1], g["object_id"][hit])
    assert np.array_equal(rtref.bits(out_f[hit, 0]), rtref.bits(g["t"][hit]))
    assert np.array_equal(rtref.bits(out_f[hit, 1:3]), rtref.bits(g["uv"][hit]))
    assert np.array_equal(rtref.bits(out_f[:, 3]), rtref.bits(g["light_pdf"]))
    assert np.array_equal(out_i[:, 2], g["n_aabb"].astype(np.int64))
    assert np.array_equal(out_i[:, 3], g["n_tri"].astype(np.int64))
    assert np.array_equal(out_i[:, 4], g["n_light_aabb"].astype(np.int64))
    assert np.array_equal(out_i[:, 5], g["n_light_tri"].astype(np.int64))


def test_oracle_c2_rows_match_reference(rt, oracle):
    """BASELINE.json configs[1] (cornell 512x512x64): the 8 full rows kept in the golden,
    bit-exact, and their per-row FNV-1a hashes."""
    g = rtref.golden("cornell_512x512x64_rowhash.rtd")
    arrays = rtref.ref_arrays(rt, "cornell", 512, 512, 64)
    for k, row in enumerate(g["rows"]):
        out, _, _ = oracle.render(arrays, 64, int(row) * 512, int(row + 1) * 512)
        assert np.array_equal(rtref.bits(out), rtref.bits(g["row_sums"][k]))
        assert rtref.row_hash(out.reshape(1, 512, 3))[0] == g["row_fnv1a"][row]
