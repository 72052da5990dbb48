"""GPU parity: the HIP kernels (through the C ABI) against the reference's own outputs.

Bar: bit-exact float32 per-pixel sums (the path is integer-seeded and fully IEEE, so any
difference is a bug), identical AABB / triangle test counts (same traversal order), and
identical results across kernels and pixel partitions.
"""
import os

import numpy as np
import pytest

import rtref

pytestmark = pytest.mark.gpu

CASES = [("cornell", 64, 64, 8), ("cornell", 33, 17, 3), ("cornell_blob", 48, 48, 4),
         ("sponza_mini", 64, 36, 4), ("practice6_1", 256, 256, 4)]


@pytest.fixture(scope="module")
def gpu(rt):
    # torch first: it must initialise the HIP runtime it shares with librt_hw_amd.so
    # (torch cannot initialise after the library has)
    import torch
    if torch.cuda.is_available():
        torch.zeros(1, device="cuda")
    if rt.device_count() < 1:
        pytest.fail("no HIP device visible: the GPU tests must run on the MI355X box")
    return rt


def _sums(scene, spp, **kw):
    out, st = scene.render_sums(spp, **kw)
    return out.reshape(-1, 3), st


@pytest.mark.parametrize("kernel,order", [(0, "heavy"), (0, "natural"), (0, "auto"), (4, "auto")])
@pytest.mark.parametrize("name,w,h,s", CASES)
def test_sums_match_reference(gpu, name, w, h, s, kernel, order):
    """Both schedules (lane-resident with its in-frame heaviest-first order, in row-major
    order, or as the spp threshold picks; wavefront) against the reference's sums and
    traversal counters."""
    scene = gpu.Scene.from_view(rtref.ref_arrays(gpu, name, w, h, s))
    out, st = _sums(scene, s, count=True, kernel=kernel, natural_order=order == "natural",
                    heavy_order=order == "heavy")
    g = rtref.golden(f"{name}_sums_{w}x{h}x{s}.rtd")
    ref = g["sums"].reshape(-1, 3)
    bad = (rtref.bits(out) != rtref.bits(ref)).any(1)
    assert bad.sum() == 0, f"{bad.sum()} pixels differ, max |d| {np.abs(out - ref).max()}"
    c = g["counters"]
    assert [st["rays"], st["aabb_tests"], st["tri_tests"], st["light_queries"], st["light_aabb_tests"],
            st["light_tri_tests"]] == [int(x) for x in c]


def test_many_pixels_per_lane_vs_oracle(gpu, oracle):
    """The lane-resident kernel where every lane runs several pixels (a 1920x1080 frame: 2.07 M
    pixels for at most 327 k lane slots), 16-sample chains, translucent materials: both pixel
    orders give the same frame, and sampled pixels equal the CPU oracle."""
    name, W, H, S = "sponza_mini", 1920, 1080, 16
    a = rtref.ref_arrays(gpu, name, W, H, S)
    a["mesh_f"] = a["mesh_f"].copy()
    a["mesh_f"][::3, 8] = np.float32(0.5)
    scene = gpu.Scene.from_view(a)
    lane, st0 = scene.render_sums(S, runahead=False, heavy_order=True)
    lane_n, _ = scene.render_sums(S, runahead=False, natural_order=True)
    assert st0["schedule"] == gpu.SCHED_LANE
    assert np.array_equal(rtref.bits(lane), rtref.bits(lane_n))
    # the hand-off (the tail's parked pixels resumed by the runahead kernel), both orders
    for kw in (dict(heavy_order=True), dict(natural_order=True)):
        ho, sth = scene.render_sums(S, **kw)
        assert sth["schedule"] == gpu.SCHED_LANE | gpu.SCHED_RUNAHEAD
        assert np.array_equal(rtref.bits(ho), rtref.bits(lane)), kw
    rng = np.random.default_rng(5)
    for p in rng.choice(W * H, 10, replace=False):
        ref, _, _ = oracle.render(a, S, int(p), int(p) + 1, threads=1)
        assert np.array_equal(rtref.bits(lane.reshape(-1, 3)[p]), rtref.bits(ref[0])), f"pixel {p}"


@pytest.mark.parametrize("name,w,h,s", CASES)
def test_loader_path_matches_reference(gpu, name, w, h, s):
    """Own glTF loader + BVH builder (rt_scene_load_gltf) -> GPU: same bits as the reference
    binary end to end, rotated meshes (cornell_blob, practice6_1) included."""
    scene = gpu.Scene.load(rtref.scene_path(name), w, h, s)
    out, st = _sums(scene, s, count=True)
    g = rtref.golden(f"{name}_sums_{w}x{h}x{s}.rtd")
    ref = g["sums"].reshape(-1, 3)
    bad = (rtref.bits(out) != rtref.bits(ref)).any(1)
    assert bad.sum() == 0, f"{bad.sum()} pixels differ, L-inf of the mean {np.abs(out - ref).max() / s}"
    assert st["rays"] == int(g["counters"][0]) and st["aabb_tests"] == int(g["counters"][1])


@pytest.mark.parametrize("name,w,h,s", CASES)
def test_runahead_matches_reference(gpu, name, w, h, s):
    """Speculative sample runahead (default for non-counting parity renders; rt_mega.h
    spec_manage): the whole frame and its 8 row-block shards (more lanes than pixels, so
    every wave is in its tail from its first claim) against the reference's sums, and the
    same frame with the runahead off."""
    scene = gpu.Scene.from_view(rtref.ref_arrays(gpu, name, w, h, s))
    ref = rtref.golden(f"{name}_sums_{w}x{h}x{s}.rtd")["sums"].reshape(h, w, 3)
    full, _ = scene.render_sums(s, heavy_order=True)
    assert np.array_equal(rtref.bits(full), rtref.bits(ref))
    off, _ = scene.render_sums(s, runahead=False)
    assert np.array_equal(rtref.bits(off), rtref.bits(ref))
    frame = np.zeros_like(full)
    for rank in range(8):
        rows = gpu.shard_rows(h, rank, 8, 8)
        if len(rows):
            frame[rows] = scene.render_sums(s, rank=rank, world=8, heavy_order=rank % 2 == 0)[0]
    assert np.array_equal(rtref.bits(frame), rtref.bits(ref))


@pytest.mark.parametrize("spp", [1, 2, 5])
def test_runahead_short_chains_vs_oracle(gpu, oracle, spp):
    """Runahead with chains shorter than its window (1, 2 and 5 samples per pixel), whole
    frame and 8-way shards, against the CPU oracle."""
    w, h = 33, 17
    scene = gpu.Scene.load(rtref.scene_path("cornell_blob"), w, h, spp)
    ref, _, _ = oracle.render(scene.view(), spp)
    ref = ref.reshape(h, w, 3)
    full, _ = scene.render_sums(spp)
    assert np.array_equal(rtref.bits(full), rtref.bits(ref))
    for rank in range(8):
        rows = gpu.shard_rows(h, rank, 8, 8)
        if len(rows):
            part, _ = scene.render_sums(spp, rank=rank, world=8)
            assert np.array_equal(rtref.bits(part), rtref.bits(ref[rows]))


def test_runahead_long_chains_vs_oracle(gpu, oracle):
    """Runahead over 128-sample chains (many confirmations and invalidations per pixel) on
    sponza_mini: runahead on = off, and sampled pixels = the CPU oracle."""
    w, h, s = 64, 36, 128
    scene = gpu.Scene.load(rtref.scene_path("sponza_mini"), w, h, s)
    on, _ = scene.render_sums(s, rank=1, world=2)
    off, _ = scene.render_sums(s, rank=1, world=2, runahead=False)
    assert np.array_equal(rtref.bits(on), rtref.bits(off))
    rows = gpu.shard_rows(h, 1, 2, 8)
    arrays = scene.view()
    rng = np.random.default_rng(13)
    for k in rng.choice(len(rows) * w, 12, replace=False):
        p = int(rows[k // w]) * w + int(k % w)
        ref, _, _ = oracle.render(arrays, s, p, p + 1, threads=1)
        assert np.array_equal(rtref.bits(on[k // w, k % w]), rtref.bits(ref[0])), f"pixel {p}"


def test_translucent_materials_vs_oracle(gpu, oracle):
    """Materials with alpha != 1 (scene.cpp:151; every fixture is opaque): the lane-resident
    kernel stores alpha only for such vertices (rt_path.h LaneRec).  Both kernels, with and
    without runahead, against the CPU oracle on the same arrays."""
    name, w, h, s = "sponza_mini", 48, 27, 6
    a = rtref.ref_arrays(gpu, name, w, h, s)
    a["mesh_f"] = a["mesh_f"].copy()
    a["mesh_f"][::2, 8] = np.float32(0.37)
    a["mesh_f"][1::4, 8] = np.float32(1.0000001)
    scene = gpu.Scene.from_view(a)
    ref, _, _ = oracle.render(a, s)
    for kw in ({}, {"runahead": False}, {"kernel": 4}, {"count": True}):
        out, _ = _sums(scene, s, **kw)
        assert np.array_equal(rtref.bits(out), rtref.bits(ref)), kw


def test_scene_without_lights_vs_oracle(gpu, oracle):
    """No emissive triangles (SceneDistribution picks between cosine and VNDF only,
    random.cpp:196-199; the pdf has no light term): both kernels, with and without runahead,
    against the CPU oracle."""
    name, w, h, s = "cornell_blob", 40, 40, 12
    a = rtref.ref_arrays(gpu, name, w, h, s)
    a["light"] = np.zeros((0, 16), np.float32)
    a["light_node"] = np.zeros((0, 8), np.float32)
    scene = gpu.Scene.from_view(a)
    ref, _, _ = oracle.render(a, s)
    for kw in ({}, {"runahead": False}, {"kernel": 4}):
        out, _ = _sums(scene, s, **kw)
        assert np.array_equal(rtref.bits(out), rtref.bits(ref)), kw


@pytest.mark.parametrize("name", ["cornell", "cornell_blob", "practice6_1", "sponza_mini"])
def test_rays_match_reference(gpu, name):
    g = rtref.golden(f"{name}_rays.rtd")
    scene = gpu.Scene.from_view(rtref.ref_arrays(gpu, name, 64, 64, 1))
    f, i = scene.intersect_rays(g["origin"], g["direction"])
    assert np.array_equal(i[:, 0], g["hit"])
    assert np.array_equal(i[:, 1], g["object_id"])
    assert np.array_equal(rtref.bits(f[:, 0]), rtref.bits(g["t"]))
    assert np.array_equal(rtref.bits(f[:, 1:3]), rtref.bits(g["uv"]))
    assert np.array_equal(i[:, 2], g["n_aabb"].astype(np.int64))
    assert np.array_equal(i[:, 3], g["n_tri"].astype(np.int64))
    assert np.array_equal(rtref.bits(f[:, 3]), rtref.bits(g["light_pdf"]))
    assert np.array_equal(i[:, 4], g["n_light_aabb"].astype(np.int64))
    assert np.array_equal(i[:, 5], g["n_light_tri"].astype(np.int64))


@pytest.mark.parametrize("kernel", [0, 4])
@pytest.mark.parametrize("world", [2, 3, 8])
def test_partition_invariance(gpu, world, kernel):
    """Row-block shards (the multi-GPU partition) reassemble to the single-shard frame."""
    w, h, s = 40, 70, 2
    scene = gpu.Scene.load(rtref.scene_path("sponza_mini"), w, h, s)
    full, _ = scene.render_sums(s, kernel=kernel)
    frame = np.zeros_like(full)
    for rank in range(world):
        rows = gpu.shard_rows(h, rank, world, 8)
        part, _ = scene.render_sums(s, rank=rank, world=world, row_block=8, kernel=kernel)
        frame[rows] = part
    assert np.array_equal(rtref.bits(frame), rtref.bits(full))


def test_cornell_c2_full_size_rowhash(gpu):
    """BASELINE configs[1] (cornell 512x512x64) at full size: per-row checksums + 8 full rows."""
    g = rtref.golden("cornell_512x512x64_rowhash.rtd")
    scene = gpu.Scene.load(rtref.scene_path("cornell"), 512, 512, 64)
    out, st = scene.render_sums(64, count=True)
    assert np.array_equal(rtref.row_hash(out), g["row_fnv1a"])
    assert np.array_equal(rtref.bits(out[g["rows"]]), rtref.bits(g["row_sums"]))
    assert st["rays"] == int(g["counters"][0])


def test_sponza_full_frame_pixels_vs_oracle(gpu, oracle):
    """Full-size sponza proxy (BASELINE headline scene): a seeded sample of pixels of the
    1920x1080 frame, GPU vs the CPU oracle on the very same flattened scene."""
    scenes = rtref.scenes_module()
    import tempfile, os
    d = os.path.join(tempfile.gettempdir(), "rt_scenes")
    path = scenes.ensure_scene("sponza", d)
    W, H, S = 1920, 1080, 2
    scene = gpu.Scene.load(path, W, H, S)
    out, _ = scene.render_sums(S)
    out = out.reshape(-1, 3)
    arrays = scene.view()
    rng = np.random.default_rng(7)
    for p in rng.choice(W * H, 48, replace=False):
        ref, _, _ = oracle.render(arrays, S, int(p), int(p) + 1, threads=1)
        assert np.array_equal(rtref.bits(out[p]), rtref.bits(ref[0])), f"pixel {p}"


def test_pixel_order_does_not_change_the_frame(gpu):
    """The heaviest-first order from an in-frame counting pre-pass (rt_device.hip
    launch_order; the default from 128 spp, RT_FLAG_HEAVY_ORDER below) and row-major order
    (RT_FLAG_NATURAL_ORDER) give the same bits and counters, at several shard sizes (fewer
    and more pixels than lanes)."""
    name, w, h, s = "sponza_mini", 64, 36, 4
    scene = gpu.Scene.from_view(rtref.ref_arrays(gpu, name, w, h, s))
    g = rtref.golden(f"{name}_sums_{w}x{h}x{s}.rtd")
    a, sa = _sums(scene, s, count=True, heavy_order=True)
    b, sb = _sums(scene, s, count=True, natural_order=True)
    assert np.array_equal(rtref.bits(a), rtref.bits(g["sums"].reshape(-1, 3)))
    assert np.array_equal(rtref.bits(a), rtref.bits(b))
    assert sa["rays"] == sb["rays"] == int(g["counters"][0])
    big = gpu.Scene.load(rtref.scene_path("sponza_mini"), 640, 360, 2)
    x, _ = big.render_sums(2, heavy_order=True)
    y, _ = big.render_sums(2, natural_order=True)
    assert np.array_equal(rtref.bits(x), rtref.bits(y))
    with pytest.raises(gpu.RtError):   # the two order flags exclude each other
        big.render_sums(2, heavy_order=True, natural_order=True)


def test_render_multi_matches_single_device(gpu):
    """rt_render_multi (one host thread per device, row-block shards, frame assembled on the
    host) on every visible device and on one: the single-call frame, bit for bit."""
    name, w, h, s = "sponza_mini", 64, 36, 4
    scene = gpu.Scene.load(rtref.scene_path(name), w, h, s)
    ref = rtref.golden(f"{name}_sums_{w}x{h}x{s}.rtd")["sums"].reshape(h, w, 3)
    for n in (1, 0):
        frame, st = scene.render_multi(s, n_devices=n, count=True)
        assert np.array_equal(rtref.bits(frame), rtref.bits(ref))
        assert st["devices"] == (n or gpu.device_count())
        assert st["rays"] == int(rtref.golden(f"{name}_sums_{w}x{h}x{s}.rtd")["counters"][0])


@pytest.mark.parametrize("n_shards", [1, 3, 8])
@pytest.mark.parametrize("name,w,h,s", [("sponza_mini", 64, 36, 4), ("cornell", 33, 17, 3)])
def test_render_frame_device_gather(gpu, n_shards, name, w, h, s):
    """rt_render_frame with every shard on device 0 (the pool's boxes have one GPU): each shard
    rendered and finished to 8 bits on the device, copied device-to-device into the root's
    staging buffer and placed in frame order there.  Float frame = the reference's sums and
    8-bit frame = the reference's finished PPM, bit for bit, at 1, 3 and 8 shards (the row
    scatter of a 3- and an 8-way split; 33 pixels = 99-byte rows take the byte path, and
    17 rows of 4-row blocks leave shards 5-7 empty).  The n > 1 device case (xGMI peer copies
    between MI355X) runs the same code with other device ids; it is not exercised on one GPU."""
    scene = gpu.Scene.load(rtref.scene_path(name), w, h, s)
    ref = rtref.golden(f"{name}_sums_{w}x{h}x{s}.rtd")["sums"].reshape(h, w, 3)
    ppm = open(os.path.join(rtref.GOLD, f"{name}_{w}x{h}x{s}.ppm"), "rb").read()
    rgb, sums, st = scene.render_frame(s, devices=[0] * n_shards, row_block=4)
    assert np.array_equal(rtref.bits(sums), rtref.bits(ref))
    assert rgb.tobytes() == ppm[len(b"P6\n%d %d\n255\n" % (w, h)):]
    assert st["devices"] == 1 and st["pixels"] == w * h and st["gather_ms"] > 0
    rgb2, none, _ = scene.render_frame(s, devices=[0] * n_shards, row_block=4, sums=False)
    assert none is None and np.array_equal(rgb2, rgb)


def test_render_frame_distinct_devices(gpu):
    """rt_render_frame with shards on distinct devices (per-device worker threads, peer access,
    hipMemcpyPeerAsync into the root's staging buffer, the root's event waits): the frame equals
    the reference's.  Runs only where more than one GPU is visible (this pool's boxes have one:
    skipped there, so the peer path stays unmeasured until a multi-GPU run of the suite)."""
    n = gpu.device_count()
    if n < 2:
        pytest.skip("one visible GPU: the peer-copy path needs two or more")
    name, w, h, s = "sponza_mini", 64, 36, 4
    scene = gpu.Scene.load(rtref.scene_path(name), w, h, s)
    ref = rtref.golden(f"{name}_sums_{w}x{h}x{s}.rtd")["sums"].reshape(h, w, 3)
    ppm = open(os.path.join(rtref.GOLD, f"{name}_{w}x{h}x{s}.ppm"), "rb").read()
    for devices in ([k % n for k in range(8)], [n - 1 - (k % n) for k in range(5)]):
        rgb, sums, st = scene.render_frame(s, devices=devices, row_block=4)
        assert np.array_equal(rtref.bits(sums), rtref.bits(ref))
        assert rgb.tobytes() == ppm[len(b"P6\n%d %d\n255\n" % (w, h)):]
        assert st["devices"] == len(set(devices))


def test_concurrent_scenes_on_one_device(gpu):
    """Two scene copies rendering at once on one device, each on its own stream with no wait
    between the launches (include/rt_hw.h: only one render per (scene, device) may be in
    flight; separate scenes share no device state): every frame equals the reference's."""
    import torch
    name, w, h, s = "sponza_mini", 64, 36, 4
    ref = rtref.golden(f"{name}_sums_{w}x{h}x{s}.rtd")["sums"].reshape(-1)
    scenes = [gpu.Scene.load(rtref.scene_path(name), w, h, s) for _ in range(2)]
    for sc in scenes:
        sc.upload(0)
    streams = [torch.cuda.Stream() for _ in range(2)]
    outs = [torch.full((h * w * 3,), float("nan"), dtype=torch.float32, device="cuda") for _ in range(6)]
    torch.cuda.synchronize()
    for i, o in enumerate(outs):
        scenes[i % 2].render_device(o.data_ptr(), streams[i % 2].cuda_stream, spp=s, natural_order=(i % 3 == 2))
    torch.cuda.synchronize()
    for o in outs:
        assert np.array_equal(rtref.bits(o.cpu().numpy()), rtref.bits(ref))


def test_device_finish_matches_reference(gpu):
    """rt_tonemap_u8_device (scene.cpp:54-64 on the GPU) against the reference's own 8-bit
    finish of the golden sums (NaN, inf, negative, saturating values included) and against
    the host rt_tonemap_u8 on a wide random range."""
    import torch
    g = rtref.golden("finish_37x23x16.rtd")
    spp = int(g["spp"][0])
    want = open(rtref.os.path.join(rtref.GOLD, "finish_37x23x16.ppm"), "rb").read()[len(b"P6\n37 23\n255\n"):]
    d_sum = torch.from_numpy(np.array(g["sums"], np.float32, copy=True)).cuda()
    d_rgb = torch.zeros(d_sum.numel(), dtype=torch.uint8, device="cuda")
    gpu.tonemap_device(d_sum.data_ptr(), 37, 23, spp, d_rgb.data_ptr())
    torch.cuda.synchronize()
    assert d_rgb.cpu().numpy().tobytes() == want
    rng = np.random.default_rng(7)
    sums = (rng.standard_normal((300, 200, 3)) * np.exp(rng.uniform(-20, 8, (300, 200, 3)))).astype(np.float32)
    sums.reshape(-1)[::997] = np.nan
    sums.reshape(-1)[::991] = np.inf
    host = gpu.tonemap(sums, 16)
    d_sum = torch.from_numpy(sums).cuda()
    d_rgb = torch.zeros(sums.size, dtype=torch.uint8, device="cuda")
    gpu.tonemap_device(d_sum.data_ptr(), 200, 300, 16, d_rgb.data_ptr())
    torch.cuda.synchronize()
    assert np.array_equal(d_rgb.cpu().numpy().reshape(300, 200, 3), host)


def test_fast_reciprocal_is_exact(gpu):
    """The traversal's 1/det (rt_wavefront.h rcp_ieee: v_rcp_f32 + one fma correction) equals
    the IEEE division for every float with a normal reciprocal (2^32 values on the device)."""
    assert gpu.device_selfcheck(0) == 0


def test_texel_decode_and_rng_word_are_exact(gpu):
    """The computed linear texel decode (rt_path.h unorm8) equals (float)b / 255.f for every
    byte, and the packed LDS RNG word round-trips for every minstd state and both cache flags,
    on the device (rt_device_selfcheck 1)."""
    assert gpu.device_selfcheck(1) == 0


def test_coop_leaf_step_ties_and_nan(gpu):
    """The cooperative leaf step (rt_wavefront.h trav_step_coop: four helper lanes per leaf
    lane, DPP quad min with the triangle index as tie-break, NaN t as no hit) against the
    per-lane in-order strict-< loop (bvh.cpp:226-232 over primitive.cpp:17-57) on 2^16
    synthetic leaves of 1-7 triangles full of exact duplicates (equal t, u, v), coplanar
    triangles (equal t), NaN and infinite vertices, with one round per step and with every
    leaf lane served per step, 8 and 16 leaf records (rt_device_selfcheck 2)."""
    assert gpu.device_selfcheck(2) == 0


def test_schedule_reported(gpu):
    """rt_stats.schedule names the kernel that rendered: the plain lane-resident kernel for a
    frame of more pixels than lanes (or a counting render), the runahead kernel for its 8-way
    shards, fast mode, the light-split kernel and the wavefront launches."""
    scene = gpu.Scene.load(rtref.scene_path("sponza_mini"), 64, 36, 4)
    big = gpu.Scene.load(rtref.scene_path("sponza_mini"), 1280, 720, 1)
    # (the plain kernel, its tail handed off to the runahead kernel: rt_device.hip hand-off)
    assert big.render_sums(1)[1]["schedule"] == gpu.SCHED_LANE | gpu.SCHED_RUNAHEAD
    assert big.render_sums(1, runahead=False)[1]["schedule"] == gpu.SCHED_LANE
    assert scene.render_sums(4, count=True)[1]["schedule"] == gpu.SCHED_LANE
    assert scene.render_sums(4, rank=1, world=8)[1]["schedule"] == gpu.SCHED_RUNAHEAD
    assert scene.render_sums(4, runahead=False)[1]["schedule"] == gpu.SCHED_LANE
    assert scene.render_sums(4, fast=True)[1]["schedule"] == gpu.SCHED_FAST
    assert scene.render_sums(4, light_split=True)[1]["schedule"] == gpu.SCHED_LIGHT_SPLIT
    assert scene.render_sums(4, kernel=4)[1]["schedule"] == gpu.SCHED_WAVEFRONT
    _, _, st = scene.render_frame(4, devices=[0] * 8, sums=False)
    assert st["schedule"] == gpu.SCHED_RUNAHEAD


@pytest.mark.parametrize("name,w,h,s", CASES)
def test_light_split_kernel(gpu, name, w, h, s):
    """Light-split kernel (rt_mega.h light_step; RT_FLAG_LIGHT_SPLIT, off by
    default): bit-exact sums and counters, practice6_1's 1,152 emissive triangles included."""
    scene = gpu.Scene.from_view(rtref.ref_arrays(gpu, name, w, h, s))
    out, st = _sums(scene, s, count=True, light_split=True)
    g = rtref.golden(f"{name}_sums_{w}x{h}x{s}.rtd")
    assert np.array_equal(rtref.bits(out), rtref.bits(g["sums"].reshape(-1, 3)))
    assert [st["rays"], st["aabb_tests"], st["tri_tests"], st["light_queries"], st["light_aabb_tests"],
            st["light_tri_tests"]] == [int(x) for x in g["counters"]]


@pytest.mark.parametrize("name,W,H", [("sponza_dragon_mini", 96, 54), ("sponza_dragon", 3840, 2160)])
def test_sponza_dragon_c5_pixels_vs_oracle(gpu, oracle, name, W, H):
    """BASELINE.json configs[4] (C5: dragon-100k proxy + sponza proxy, 3840x2160): a seeded
    sample of pixels, GPU vs the CPU oracle on the very same flattened scene (2 spp)."""
    scenes = rtref.scenes_module()
    import tempfile, os
    path = scenes.ensure_scene(name, os.path.join(tempfile.gettempdir(), "rt_scenes"))
    S = 2
    scene = gpu.Scene.load(path, W, H, S)
    out, st = scene.render_sums(S, count=True)
    out = out.reshape(-1, 3)
    assert st["rays"] >= W * H * S
    arrays = scene.view()
    rng = np.random.default_rng(11)
    pix = rng.choice(W * H, 40, replace=False) if W * H > 10000 else np.arange(W * H)
    for p in pix:
        ref, _, _ = oracle.render(arrays, S, int(p), int(p) + 1, threads=1)
        assert np.array_equal(rtref.bits(out[p]), rtref.bits(ref[0])), f"pixel {p}"


def test_idle_lanes_after_another_kernel(gpu):
    """A lane-resident launch with fewer pixels than lanes right after a wavefront launch: the
    lanes that never get a pixel start with the previous kernel's register contents, and the
    shading pass packs their phase and stack depth with their state (rt_device.hip
    RT_PACK_TRAV), so the kernel sets both at its start.  Counting and plain renders of the
    33x17 frame (561 pixels, 768 lanes) after the wavefront kernel on 64x64 must be the
    reference's sums (round 5: this sequence faulted before the fix)."""
    big = gpu.Scene.from_view(rtref.ref_arrays(gpu, "cornell", 64, 64, 8))
    _sums(big, 8, count=True, kernel=4)
    small = gpu.Scene.from_view(rtref.ref_arrays(gpu, "cornell", 33, 17, 3))
    ref = rtref.golden("cornell_sums_33x17x3.rtd")["sums"].reshape(-1, 3)
    for kw in [dict(count=True, heavy_order=True), dict(count=True, natural_order=True), dict(runahead=False)]:
        _sums(big, 8, count=True, kernel=4)
        out, _ = _sums(small, 3, **kw)
        assert (rtref.bits(out) == rtref.bits(ref)).all(), kw


def test_pack_masks_poisoned_lanes(gpu):
    """The shading pass's packing (rt_device.hip RT_PACK_TRAV) is guarded two ways: the fields
    are masked, and the index-checked debug build checks phase < 4, state < 8, sp <= kStack
    before every pack (RT_CHECK 14).  With every lane's phase and stack depth poisoned out of
    range at the kernel's start (rt_debug_set_poison: the leftovers behind round 5's fault),
    the lanes that never get a pixel (33x17 = 561 pixels, 768 lanes) carry them into every
    shading pass: the counting render must still be the reference's sums, and the check must
    report them.  Debug build only (RT_LIB=raytracing-hw_amd/debug/librt_hw_amd.so)."""
    if not gpu.is_debug_build():
        pytest.skip("needs the index-checked debug build (make -C raytracing-hw_amd debug)")
    small = gpu.Scene.from_view(rtref.ref_arrays(gpu, "cornell", 33, 17, 3))
    ref = rtref.golden("cornell_sums_33x17x3.rtd")["sums"].reshape(-1, 3)
    gpu.debug_raise = False
    try:
        gpu.debug_take()
        gpu.debug_set_poison(1)
        out, st = _sums(small, 3, count=True, natural_order=True)
        word = gpu.debug_take()
    finally:
        gpu.debug_set_poison(0)
        gpu.debug_raise = True
    assert st["schedule"] == gpu.SCHED_LANE
    assert (rtref.bits(out) == rtref.bits(ref)).all()
    assert word >> 56 == 14, hex(word)
    out, _ = _sums(small, 3, count=True, natural_order=True)   # unpoisoned: no check fires (raises otherwise)
    assert (rtref.bits(out) == rtref.bits(ref)).all()
