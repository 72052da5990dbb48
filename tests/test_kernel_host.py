"""The GPU kernel source, compiled for the host (tests/native/kernel_host.cpp), against the
reference's own per-pixel sums and counters (tests/golden, made by oracle/ref_harness).

Three schedules of the same per-pixel arithmetic are checked bit-exactly:
  * render_pixel      (rt_path.h: the reference's recursion order, closest_hit by stack),
  * wavefront         (rt_wavefront.h slot functions, kernel 4: closest_hit_wf with the
                       sibling-pair fetch and 8-byte frames),
  * lane-resident     (rt_mega.h, kernel 0, the default: several waves of 64 lanes sharing
                       the pixel queue, batched shading, any pixel order).
"""
import ctypes
import os
import subprocess

import numpy as np
import pytest

import rtref

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "tests", "native", "kernel_host.cpp")
CASES = [("cornell", 33, 17, 3), ("cornell", 64, 64, 8), ("cornell_blob", 48, 48, 4),
         ("practice6_1", 256, 256, 4), ("sponza_mini", 64, 36, 4)]


def _build_kh(tmp_path_factory, *defines):
    out = str(tmp_path_factory.mktemp("kh") / "libkh.so")
    subprocess.run(["g++", "-O2", "-fno-tree-vectorize", "-fno-tree-slp-vectorize", "-ffp-contract=off", "-fopenmp",
                    "-std=c++17", "-shared", "-fPIC", *defines, SRC, "-o", out], check=True)
    lib = ctypes.CDLL(out)
    V, I, L = ctypes.c_void_p, ctypes.c_int, ctypes.c_int64
    lib.kh_render.argtypes = [V, I, L, L, V, V]
    lib.kh_render.restype = None
    lib.kh_render_wf.argtypes = [V, I, I, I, I, V, V, V]
    lib.kh_render_wf.restype = I
    lib.kh_render_mega.argtypes = [V, I, I, I, I, I, I, V, V, V]
    lib.kh_render_mega.restype = I
    lib.kh_render_mega_lsplit.argtypes = [V, I, I, I, I, I, I, V, V]
    lib.kh_render_mega_lsplit.restype = I
    lib.kh_box_pair_check.argtypes = [ctypes.c_int64, ctypes.c_uint32]
    lib.kh_box_pair_check.restype = ctypes.c_int64
    lib.kh_decode_check.argtypes = []
    lib.kh_decode_check.restype = ctypes.c_int64
    lib.kh_div_magic_check.argtypes = [ctypes.c_uint32, ctypes.c_uint32]
    lib.kh_div_magic_check.restype = ctypes.c_int64
    return lib


@pytest.fixture(scope="module")
def kh(tmp_path_factory):
    return _build_kh(tmp_path_factory)


def _golden(name, w, h, s):
    g = rtref.golden(f"{name}_sums_{w}x{h}x{s}.rtd")
    return g["sums"].reshape(h * w, 3), g["counters"]


def _view(rt, name, w, h, s):
    return rt.make_view(rtref.ref_arrays(rt, name, w, h, s))


@pytest.mark.parametrize("name,w,h,s", CASES)
def test_pixel_schedule_matches_reference(rt, kh, name, w, h, s):
    want, cnt_want = _golden(name, w, h, s)
    v, keep = _view(rt, name, w, h, s)
    out = np.zeros((h * w, 3), np.float32)
    cnt = np.zeros(6, np.uint64)
    kh.kh_render(ctypes.addressof(v), s, 0, w * h, out.ctypes.data, cnt.ctypes.data)
    assert np.array_equal(rtref.bits(out), rtref.bits(want))
    assert list(cnt) == list(cnt_want)


@pytest.mark.parametrize("name,w,h,s", CASES)
def test_wavefront_matches_reference(rt, kh, name, w, h, s):
    want, cnt_want = _golden(name, w, h, s)
    v, keep = _view(rt, name, w, h, s)
    out = np.zeros((h * w, 3), np.float32)
    cnt = np.zeros(7, np.uint64)
    it = np.zeros(1, np.int64)
    assert kh.kh_render_wf(ctypes.addressof(v), s, 0, 1, 8, out.ctypes.data, cnt.ctypes.data, it.ctypes.data) == 0
    assert np.array_equal(rtref.bits(out), rtref.bits(want))
    assert list(cnt[:6]) == list(cnt_want)
    assert it[0] <= s * int(v.ray_depth) + 1


@pytest.mark.parametrize("world", [2, 3])
def test_wavefront_shards_reassemble(rt, kh, world):
    name, w, h, s = "cornell", 33, 17, 3
    want, _ = _golden(name, w, h, s)
    v, keep = _view(rt, name, w, h, s)
    frame = np.zeros((h, w, 3), np.float32)
    for rank in range(world):
        rows = [r for r in range(h) if (r // 4) % world == rank]
        out = np.zeros((len(rows) * w, 3), np.float32)
        cnt = np.zeros(7, np.uint64)
        assert kh.kh_render_wf(ctypes.addressof(v), s, rank, world, 4, out.ctypes.data, cnt.ctypes.data, None) == 0
        frame[rows] = out.reshape(len(rows), w, 3)
    assert np.array_equal(rtref.bits(frame.reshape(-1, 3)), rtref.bits(want))


def test_scene_sampler_matches_reference(rt, kh):
    """SceneDistribution::sample / ::pdf (random.cpp:194-218) of the kernel source against the
    reference on 2000 random shading frames, including the number of RNG draws consumed."""
    g = rtref.golden("cornell_samplers.rtd")
    v, keep = _view(rt, "cornell", 64, 64, 1)
    n = len(g["seed"])
    frame = np.ascontiguousarray(g["frame"], np.float32)
    seed = np.ascontiguousarray(g["seed"], np.uint32)
    d = np.zeros((n, 3), np.float32)
    pdf = np.zeros(n, np.float32)
    nxt = np.zeros(n, np.uint32)
    kh.kh_samplers.argtypes = [ctypes.c_void_p, ctypes.c_int64] + [ctypes.c_void_p] * 5
    kh.kh_samplers(ctypes.addressof(v), n, frame.ctypes.data, seed.ctypes.data, d.ctypes.data, pdf.ctypes.data,
                   nxt.ctypes.data)
    assert np.array_equal(rtref.bits(d), rtref.bits(g["dir"]))
    assert np.array_equal(rtref.bits(pdf), rtref.bits(g["pdf"]))
    assert np.array_equal(nxt, g["next"])


def test_rng_sequences_match_reference(kh):
    """minstd_rand0 engine, uniform_real_distribution(-1, 1) and the polar normal_distribution
    (random.cpp:12-46, libstdc++ random.tcc) for five seeds."""
    g = rtref.golden("cornell_samplers.rtd")
    kh.kh_rng.argtypes = [ctypes.c_uint32, ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p]
    for row, seed in enumerate([1, 2, 12345, 2147483646, 65536]):
        u = np.zeros(8, np.uint32)
        f = np.zeros(8, np.float32)
        kh.kh_rng(seed, 0, 8, f.ctypes.data, u.ctypes.data)
        assert np.array_equal(u, g["raw_engine"][row])
        kh.kh_rng(seed, 1, 8, f.ctypes.data, u.ctypes.data)
        assert np.array_equal(rtref.bits(f), rtref.bits(g["raw_uniform"][row]))
        kh.kh_rng(seed, 2, 8, f.ctypes.data, u.ctypes.data)
        assert np.array_equal(rtref.bits(f), rtref.bits(g["raw_normal"][row]))


@pytest.mark.parametrize("name,w,h,s,waves,shade_min", [("cornell_blob", 48, 48, 4, 2, 32), ("sponza_mini", 64, 36, 4, 3, 1),
                                                        ("cornell", 33, 17, 3, 1, 64)])
def test_lane_resident_emulation(rt, kh, name, w, h, s, waves, shade_min):
    """Kernel 4 (rt_mega.h): lanes own whole pixels, traversal steps per iteration, batched
    shading; bit-exact sums and counters."""
    want, cnt_want = _golden(name, w, h, s)
    v, keep = _view(rt, name, w, h, s)
    out = np.zeros((h * w, 3), np.float32)
    cnt = np.zeros(7, np.uint64)
    assert kh.kh_render_mega(ctypes.addressof(v), s, 0, 1, 8, waves, shade_min, None, out.ctypes.data,
                             cnt.ctypes.data) == 0
    assert np.array_equal(rtref.bits(out), rtref.bits(want))
    assert list(cnt[:6]) == list(cnt_want)


@pytest.mark.parametrize("name,w,h,s,waves,world", [("cornell_blob", 48, 48, 4, 2, 1), ("sponza_mini", 64, 36, 4, 3, 1),
                                                    ("cornell", 33, 17, 3, 1, 1), ("practice6_1", 256, 256, 4, 40, 1),
                                                    ("sponza_mini", 64, 36, 4, 40, 1), ("sponza_mini", 64, 36, 4, 2, 3)])
def test_lane_resident_runahead_emulation(rt, kh, name, w, h, s, waves, world):
    """Speculative sample runahead (rt_mega.h spec_*): once the pixel queue is empty a wave's
    idle lanes run later samples of its unfinished pixels from predicted start states, and
    only results whose start state is proven are added.  Bit-exact sums, with the tail
    reached late (few waves) and at once (more lanes than pixels), and on row-block shards."""
    want, _ = _golden(name, w, h, s)
    want = want.reshape(h, w, 3)
    v, keep = _view(rt, name, w, h, s)
    kh.kh_render_mega_spec.argtypes = kh.kh_render_mega.argtypes
    kh.kh_render_mega_spec.restype = ctypes.c_int
    for rank in range(world):
        rows = rt.shard_rows(h, rank, world, 8)
        out = np.zeros((len(rows) * w, 3), np.float32)
        cnt = np.zeros(7, np.uint64)
        assert kh.kh_render_mega_spec(ctypes.addressof(v), s, rank, world, 8, waves, 48, None, out.ctypes.data,
                                      cnt.ctypes.data) == 0
        assert np.array_equal(rtref.bits(out), rtref.bits(want[rows].reshape(-1, 3)))


@pytest.mark.parametrize("name,w,h,s,waves", [("sponza_mini", 32, 18, 48, 4), ("cornell_blob", 24, 24, 64, 6)])
def test_lane_resident_runahead_long_chains(rt, kh, name, w, h, s, waves):
    """Runahead over long sample chains (48-64 spp, many confirmations and invalidations per
    pixel) against the plain per-pixel schedule (rt_path.h render_pixel, pinned to the
    reference by test_pixel_schedule_matches_reference)."""
    v, keep = _view(rt, name, w, h, s)
    want = np.zeros((h * w, 3), np.float32)
    kh.kh_render(ctypes.addressof(v), s, 0, w * h, want.ctypes.data, np.zeros(6, np.uint64).ctypes.data)
    kh.kh_render_mega_spec.argtypes = kh.kh_render_mega.argtypes
    kh.kh_render_mega_spec.restype = ctypes.c_int
    kh.kh_spec_stats.argtypes = [ctypes.c_void_p]
    out = np.zeros((h * w, 3), np.float32)
    stats = np.zeros(5, np.uint64)
    kh.kh_spec_stats(stats.ctypes.data)
    assert kh.kh_render_mega_spec(ctypes.addressof(v), s, 0, 1, 8, waves, 48, None, out.ctypes.data,
                                  np.zeros(7, np.uint64).ctypes.data) == 0
    kh.kh_spec_stats(stats.ctypes.data)
    print(f"management passes {stats[0]}, frontier jobs {stats[1]}, runahead jobs {stats[2]}, added {stats[3]}, "
          f"invalidations {stats[4]}")
    assert stats[1] > 0 and stats[2] > 0 and stats[3] > stats[1]   # some runahead jobs were added
    assert np.array_equal(rtref.bits(out), rtref.bits(want))


@pytest.mark.parametrize("prio", [0, 1])
def test_runahead_priority_orders(rt, tmp_path_factory, prio):
    """The order in which records take idle lanes (rt_mega.h RT_SPEC_PRIO: record order, or
    fewest samples added first through the wave sort wave_order, the default) over long chains
    and a short frame with more lanes than pixels: the plain per-pixel schedule's bits either way."""
    lib = _build_kh(tmp_path_factory, f"-DRT_SPEC_PRIO={prio}")
    lib.kh_render_mega_spec.argtypes = lib.kh_render_mega.argtypes
    lib.kh_render_mega_spec.restype = ctypes.c_int
    for name, w, h, s, waves in [("sponza_mini", 32, 18, 48, 4), ("cornell_blob", 24, 24, 64, 6),
                                 ("practice6_1", 40, 30, 12, 40)]:
        v, keep = _view(rt, name, w, h, s)
        want = np.zeros((h * w, 3), np.float32)
        lib.kh_render(ctypes.addressof(v), s, 0, w * h, want.ctypes.data, np.zeros(6, np.uint64).ctypes.data)
        out = np.zeros((h * w, 3), np.float32)
        assert lib.kh_render_mega_spec(ctypes.addressof(v), s, 0, 1, 8, waves, 48, None, out.ctypes.data,
                                       np.zeros(7, np.uint64).ctypes.data) == 0
        assert np.array_equal(rtref.bits(out), rtref.bits(want)), name


@pytest.mark.parametrize("name,w,h,s,waves", [("cornell_blob", 48, 48, 4, 2), ("sponza_mini", 64, 36, 4, 3)])
def test_lane_resident_any_pixel_order(rt, kh, name, w, h, s, waves):
    """The ordered render (rt_device.hip launch_order: queue item p renders pixel order[p])
    gives the same bits for any permutation: reversed, and a seeded shuffle."""
    want, cnt_want = _golden(name, w, h, s)
    v, keep = _view(rt, name, w, h, s)
    rng = np.random.default_rng(5)
    for order in (np.arange(w * h, dtype=np.int32)[::-1].copy(), rng.permutation(w * h).astype(np.int32)):
        out = np.zeros((h * w, 3), np.float32)
        cnt = np.zeros(7, np.uint64)
        assert kh.kh_render_mega(ctypes.addressof(v), s, 0, 1, 8, waves, 48, order.ctypes.data, out.ctypes.data,
                                 cnt.ctypes.data) == 0
        assert np.array_equal(rtref.bits(out), rtref.bits(want))
        assert list(cnt[:6]) == list(cnt_want)


@pytest.mark.parametrize("name,w,h,s,waves,shade_min", [("practice6_1", 256, 256, 4, 6, 48), ("sponza_mini", 64, 36, 4, 3, 1),
                                                        ("cornell", 33, 17, 3, 1, 64)])
def test_lane_resident_light_split_emulation(rt, kh, name, w, h, s, waves, shade_min):
    """Light-split kernel (rt_mega.h light_step / mega_shade_split): the
    light pdf's light-BVH walk as a lane state between shade_pre and shade_post; bit-exact
    sums and reference counters (practice6_1: 1,152 emissive triangles)."""
    want, cnt_want = _golden(name, w, h, s)
    v, keep = _view(rt, name, w, h, s)
    out = np.zeros((h * w, 3), np.float32)
    cnt = np.zeros(7, np.uint64)
    assert kh.kh_render_mega_lsplit(ctypes.addressof(v), s, 0, 1, 8, waves, shade_min, out.ctypes.data,
                                    cnt.ctypes.data) == 0
    assert np.array_equal(rtref.bits(out), rtref.bits(want))
    assert list(cnt[:6]) == list(cnt_want)


@pytest.mark.parametrize("leaf_n", [1, 3, 4])
def test_lane_resident_leaf_triangles(rt, tmp_path_factory, leaf_n):
    """RT_LEAF_N (default 2, covered by the tests above): 1, 3 or 4 triangles of a leaf per
    traversal step through the shared load registers; bit-exact sums and reference counters."""
    kh_n = _build_kh(tmp_path_factory, f"-DRT_LEAF_N={leaf_n}")
    for name, w, h, s, waves, shade_min in [("cornell_blob", 48, 48, 4, 2, 32), ("sponza_mini", 64, 36, 4, 3, 1)]:
        want, cnt_want = _golden(name, w, h, s)
        v, keep = _view(rt, name, w, h, s)
        out = np.zeros((h * w, 3), np.float32)
        cnt = np.zeros(7, np.uint64)
        assert kh_n.kh_render_mega(ctypes.addressof(v), s, 0, 1, 8, waves, shade_min, None, out.ctypes.data,
                                   cnt.ctypes.data) == 0
        assert np.array_equal(rtref.bits(out), rtref.bits(want))
        assert list(cnt[:6]) == list(cnt_want)


def test_box_pair_matches_single_box_test(kh):
    """box_pair_hit (the traversal's pair test) agrees with box_hit_pt (AABB::intersect,
    primitive.cpp:146-208, restated op for op) on 4 M random cases rich in special values:
    signed zeros, infinities, NaN, flat and inverted boxes, planes through the origin."""
    assert kh.kh_box_pair_check(4_000_000, 7) == 0


@pytest.mark.parametrize("name,w,h", [("cornell", 64, 64), ("cornell_blob", 48, 48), ("practice6_1", 64, 64),
                                      ("sponza_mini", 64, 36)])
def test_runahead_state_prediction(rt, kh, name, w, h):
    """The speculative runahead's prediction (rt_path.h rng_skip_sample): the RNG state a
    sample ends in is a function of its start state and its path's vertex count alone, so
    skipping the draws of v vertices reproduces it exactly.  Checked on every sample of 256
    pixels at 64 spp (parity RNG convention); the runahead itself still compares states
    before it uses a speculative result (rt_mega.h spec_manage)."""
    v, keep = _view(rt, name, w, h, 64)
    rng = np.random.default_rng(5)
    pix = np.ascontiguousarray(rng.choice(w * h, 256, replace=False), np.int64)
    stats = np.zeros(3, np.uint64)
    kh.kh_skip_check.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int64, ctypes.c_void_p, ctypes.c_void_p]
    kh.kh_skip_check(ctypes.addressof(v), 64, len(pix), pix.ctypes.data, stats.ctypes.data)
    assert stats[0] == 256 * 64
    assert stats[1] == 0, f"{stats[1]} of {stats[0]} sample end states differ from the prediction"
    assert stats[2] > 0


@pytest.mark.parametrize("per_wave", [7, 24, 64])
def test_runahead_with_spare_lanes(rt, kh, per_wave):
    """The runahead's management pass when a wave has idle lanes from its first iteration
    (the harness's static allotment of `per_wave` pixels per wave, no queue: DESIGN.md §7
    study): same bits as the per-pixel schedule, and fewer main-loop rounds than without
    runahead."""
    name, w, h, s = "sponza_mini", 48, 27, 6
    v, keep = rt.make_view(rtref.ref_arrays(rt, name, w, h, s))
    want = np.zeros((h * w, 3), np.float32)
    kh.kh_render(ctypes.addressof(v), s, 0, w * h, want.ctypes.data, np.zeros(6, np.uint64).ctypes.data)
    kh.kh_render_mega_spec.argtypes = kh.kh_render_mega.argtypes
    kh.kh_render_mega_spec.restype = ctypes.c_int
    kh.kh_set_static_per_wave.argtypes = [ctypes.c_int]
    kh.kh_rounds.restype = ctypes.c_uint64
    waves = (w * h + per_wave - 1) // per_wave
    rounds = []
    try:
        kh.kh_set_static_per_wave(per_wave)
        for fn in (kh.kh_render_mega, kh.kh_render_mega_spec):
            out = np.zeros((h * w, 3), np.float32)
            assert fn(ctypes.addressof(v), s, 0, 1, 8, waves, 48, None, out.ctypes.data,
                      np.zeros(7, np.uint64).ctypes.data) == 0
            assert np.array_equal(rtref.bits(out), rtref.bits(want))
            rounds.append(kh.kh_rounds())
    finally:
        kh.kh_set_static_per_wave(0)
    assert rounds[1] < rounds[0]


@pytest.mark.parametrize("spread", [1, 0])
@pytest.mark.parametrize("name,w,h,s,waves,spec_waves,below,pct", [
    ("sponza_mini", 48, 27, 6, 6, 4, 48, 100), ("sponza_mini", 48, 27, 6, 6, 3, 32, 60),
    ("cornell_blob", 40, 40, 8, 8, 8, 56, 100), ("practice6_1", 40, 30, 6, 5, 2, 40, 50)])
def test_handoff_matches_per_pixel(rt, kh, name, w, h, s, waves, spec_waves, below, pct, spread):
    """Hand-off (rt_device.hip RT_HANDOFF): the plain lane-resident kernel parks the pixels of
    its sparse tail waves at a sample boundary (rt_mega.h park_pixel: pixel, next sample, RNG
    state, sum so far, by lane slot), and the runahead kernel resumes them (static allotment of
    `pct` percent, the rest claimed in the tail), in park-list slot order or (`spread`,
    RT_HANDOFF_SPREAD) through the map that deals the pixels with the most work left one per
    wave.  Same bits as the per-pixel schedule, and pixels were parked."""
    kh.kh_set_handoff_spread.argtypes = [ctypes.c_int]
    kh.kh_set_handoff_spread(spread)
    v, keep = rt.make_view(rtref.ref_arrays(rt, name, w, h, s))
    want = np.zeros((h * w, 3), np.float32)
    kh.kh_render(ctypes.addressof(v), s, 0, w * h, want.ctypes.data, np.zeros(6, np.uint64).ctypes.data)
    kh.kh_render_mega_handoff.argtypes = [ctypes.c_void_p] + [ctypes.c_int] * 9 + [ctypes.c_void_p] * 4
    kh.kh_render_mega_handoff.restype = ctypes.c_int
    out = np.zeros((h * w, 3), np.float32)
    parked = np.zeros(1, np.uint64)
    assert kh.kh_render_mega_handoff(ctypes.addressof(v), s, 0, 1, 8, waves, spec_waves, 48, below, pct, None,
                                     out.ctypes.data, np.zeros(7, np.uint64).ctypes.data, parked.ctypes.data) == 0
    kh.kh_set_handoff_spread(1)
    assert np.array_equal(rtref.bits(out), rtref.bits(want))
    assert parked[0] > 0


def test_lane_resident_translucent_materials(rt, kh):
    """Materials with alpha != 1 (the reference multiplies the bounce by material.alpha,
    scene.cpp:151; every fixture is opaque): the lane-resident kernel stores alpha only for
    such vertices (rt_path.h LaneRec), with and without runahead, against the per-pixel
    schedule on the same arrays."""
    name, w, h, s = "sponza_mini", 48, 27, 6
    a = rtref.ref_arrays(rt, name, w, h, s)
    a["mesh_f"] = a["mesh_f"].copy()
    a["mesh_f"][::2, 8] = np.float32(0.37)
    a["mesh_f"][1::4, 8] = np.float32(1.0000001)
    v, keep = rt.make_view(a)
    want = np.zeros((h * w, 3), np.float32)
    kh.kh_render(ctypes.addressof(v), s, 0, w * h, want.ctypes.data, np.zeros(6, np.uint64).ctypes.data)
    kh.kh_render_mega_spec.argtypes = kh.kh_render_mega.argtypes
    kh.kh_render_mega_spec.restype = ctypes.c_int
    for fn in (kh.kh_render_mega, kh.kh_render_mega_spec):
        out = np.zeros((h * w, 3), np.float32)
        assert fn(ctypes.addressof(v), s, 0, 1, 8, 3, 48, None, out.ctypes.data, np.zeros(7, np.uint64).ctypes.data) == 0
        assert np.array_equal(rtref.bits(out), rtref.bits(want))
    assert not np.array_equal(want, 0)


def test_runahead_without_lights(rt, kh):
    """A scene without emissive triangles (SceneDistribution::sample then picks between
    cosine and VNDF only, random.cpp:196-199): the runahead's state prediction and the
    runahead schedule against the per-pixel schedule."""
    name, w, h, s = "cornell_blob", 40, 40, 24
    a = rtref.ref_arrays(rt, name, w, h, s)
    a["light"] = np.zeros((0, 16), np.float32)
    a["light_node"] = np.zeros((0, 8), np.float32)
    v, keep = rt.make_view(a)
    assert v.n_lights == 0
    stats = np.zeros(3, np.uint64)
    pix = np.arange(w * h, dtype=np.int64)
    kh.kh_skip_check.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int64, ctypes.c_void_p, ctypes.c_void_p]
    kh.kh_skip_check(ctypes.addressof(v), s, len(pix), pix.ctypes.data, stats.ctypes.data)
    assert stats[0] == w * h * s and stats[1] == 0 and stats[2] > 0
    want = np.zeros((h * w, 3), np.float32)
    kh.kh_render(ctypes.addressof(v), s, 0, w * h, want.ctypes.data, np.zeros(6, np.uint64).ctypes.data)
    kh.kh_render_mega_spec.argtypes = kh.kh_render_mega.argtypes
    kh.kh_render_mega_spec.restype = ctypes.c_int
    out = np.zeros((h * w, 3), np.float32)
    assert kh.kh_render_mega_spec(ctypes.addressof(v), s, 0, 1, 8, 5, 48, None, out.ctypes.data,
                                  np.zeros(7, np.uint64).ctypes.data) == 0
    assert np.array_equal(rtref.bits(out), rtref.bits(want))


def test_linear_texel_decode_and_rng_word(kh):
    """rt_path.h unorm8 (b times the float nearest 1/255, one fma correction) equals the
    division (float)b / 255.f the reference's linear texel decode does (primitive.h:172-215)
    for every byte; the lane-resident kernel's packed RNG word (minstd state and normal-cache
    flag in one LDS word) round-trips.  The device runs the same checks
    (rt_device_selfcheck 1, tests/test_gpu_parity.py)."""
    assert kh.kh_decode_check() == 0


@pytest.mark.parametrize("d", [1, 2, 3, 7, 8, 33, 64, 255, 256, 1000, 1023, 1024, 1025, 1920, 3840, 7680,
                               65535, 65536, 99991, (1 << 30) - 1, 1 << 30, (1 << 30) + 1, (1 << 31) - 1])
def test_div_magic_matches_division(kh, d):
    """The kernels' pixel -> (column, shard row) divisions (rt_wavefront.h div_magic: multiply
    and shift with host-made constants) equal integer division for every n < 2^31 they can see:
    all small n, the top 2^20, every multiple of d and its predecessor, and 2^20 seeded draws."""
    assert kh.kh_div_magic_check(d, 1 << 20) == 0
