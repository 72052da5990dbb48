"""BASELINE.json configs at their full size and full spp on the GPU, bit-exact against the
reference (tests/golden/<config>_*_pixels_*.rtd: seeded pixels rendered by the reference's own
sources, oracle/ref_harness `pixels`, per-pixel RNG convention of SURVEY.md §8c).

  C3        sponza proxy 1024x1024x256, whole frame on one GPU
  headline  sponza proxy 1920x1080x256, whole frame on one GPU
  C4        sponza proxy 1920x1080x1024, each of the 8 row-block shards of the 8-GPU split
  C5        dragon-100k + sponza proxy 3840x2160x4096, every rank's shard of the 8-GPU split:
            64 FULL rows (8 per rank) against the reference's render of them, 256 seeded pixels
            of rank 0 and 64 of each of ranks 1-7
  whole frames: C3, the headline and C4, every row of the float
            frame (per-row FNV-1a hashes of the reference's own full render,
            tools/make_goldens.py --frames), 8 full rows, the frame counters, and the sha1 of
            the reference's finished 8-bit frame; rendered on one GPU (the plain kernel) and as
            the 4- and 8-way splits (the runahead kernel), reassembled

These are the frames whose per-pixel sample chains (256 to 4096 sequential samples, RNG
state and pixel sum held in LDS between uses: rt_mega.h) the small parity cases cannot reach.
The scene files are regenerated here and checked against the sha256 the goldens were made
from, so generator drift cannot pass as a render difference.
"""
import json
import os
import tempfile

import numpy as np
import pytest

import rtref

pytestmark = pytest.mark.gpu
_META = json.load(open(os.path.join(rtref.GOLD, "golden_meta.json")))
META = _META["configs"]
FRAMES = _META.get("frames", {})
SCENE_DIR = os.path.join(tempfile.gettempdir(), "rt_scenes")


@pytest.fixture(scope="module")
def gpu(rt):
    import torch   # initialises the HIP runtime librt_hw_amd.so shares (see test_gpu_parity.py)
    if torch.cuda.is_available():
        torch.zeros(1, device="cuda")
    if rt.device_count() < 1:
        pytest.fail("no HIP device visible: the GPU tests must run on the MI355X box")
    return rt


_scenes = {}


def _scene(gpu, name, W, H, S):
    if name not in _scenes:
        path = rtref.scenes_module().ensure_scene(name, SCENE_DIR)
        assert rtref.scene_sha256(SCENE_DIR, name) == META[name]["scene_sha256"], "scene generator drifted"
        _scenes[name] = path
    return gpu.Scene.load(_scenes[name], W, H, S)


def _check(out_rows, rows, W, g, world, rank, row_block=8):
    """out_rows: the shard's (n_rows, W, 3) sums; g: golden (index, sums); checks the golden
    pixels that fall in this shard; returns how many were checked."""
    idx = g["index"].astype(np.int64)
    want = g["sums"].reshape(-1, 3)
    row_of = {int(r): k for k, r in enumerate(rows)}
    n = 0
    for p, ref in zip(idx, want):
        j, i = int(p // W), int(p % W)
        if (j // row_block) % world != rank:
            continue
        got = out_rows[row_of[j], i]
        assert np.array_equal(rtref.bits(got), rtref.bits(ref)), f"pixel ({i}, {j}): {got} vs {ref}"
        n += 1
    return n


@pytest.mark.parametrize("config", ["c3", "headline"])
def test_full_frame_pixels_match_reference(gpu, config):
    c = META[config]
    W, H, S = c["width"], c["height"], c["spp"]
    scene = _scene(gpu, c["scene"], W, H, S)
    out, st = scene.render_sums(S)
    assert st["samples"] == W * H * S
    g = rtref.golden(c["file"])
    assert _check(out, np.arange(H), W, g, 1, 0) == len(g["index"])


def test_c4_every_shard_matches_reference(gpu):
    c = META["c4"]
    W, H, S, world = c["width"], c["height"], c["spp"], c["world"]
    scene = _scene(gpu, c["scene"], W, H, S)
    g = rtref.golden(c["file"])
    checked = 0
    for rank in range(world):
        out, _ = scene.render_sums(S, rank=rank, world=world)
        checked += _check(out, gpu.shard_rows(H, rank, world), W, g, world, rank)
    assert checked == len(g["index"])


_c5 = {}


def _c5_shard(gpu, rank):
    """Rank `rank`'s shard of C5's 8-way split at 4096 spp (rendered once per module: three
    tests read it)."""
    c = META["c5"]
    W, H, S, world = c["width"], c["height"], c["spp"], c["world"]
    if rank not in _c5:
        scene = _scene(gpu, c["scene"], W, H, S)
        out, st = scene.render_sums(S, rank=rank, world=world)
        assert st["samples"] == out.shape[0] * W * S
        _c5[rank] = out
    return _c5[rank]


def test_c5_shard_matches_reference(gpu):
    c = META["c5"]
    W, H, world = c["width"], c["height"], c["world"]
    out = _c5_shard(gpu, 0)
    g = rtref.golden(c["file"])
    assert _check(out, gpu.shard_rows(H, 0, world), W, g, world, 0) == len(g["index"])


def test_c5_fast_mode_full_spp(gpu, oracle):
    """Fast mode at C5's 4096 spp on rank 0's shard: at most 128 work units per pixel (32
    samples each here), 64-bit work queue; no RT_ERR_LIMIT, and sampled pixels bit-exact
    against the oracle's restatement with the same chunking."""
    c = META["c5"]
    W, H, S, world = c["width"], c["height"], c["spp"], c["world"]
    scene = _scene(gpu, c["scene"], W, H, S)
    out, st = scene.render_sums(S, rank=0, world=world, fast=True, fast_chunk=2)
    chunk = max(2, -(-S // 128))
    assert chunk == 32
    rows = gpu.shard_rows(H, 0, world)
    arrays = scene.view()
    rng = np.random.default_rng(3)
    for k in rng.choice(len(rows) * W, 6, replace=False):
        p = int(rows[k // W]) * W + int(k % W)
        ref, _ = oracle.render_fast(arrays, S, chunk, p, p + 1, threads=1)
        assert np.array_equal(rtref.bits(out[k // W, k % W]), rtref.bits(ref[0])), f"pixel {p}"


def test_c5_ranks_1_to_7_match_reference(gpu):
    """64 seeded pixels of each of ranks 1-7 of C5's 8-way split at 4096 spp (rank 0 above)."""
    c = META["c5_ranks"]
    W, H, world = c["width"], c["height"], c["world"]
    g = rtref.golden(c["file"])
    checked = 0
    for rank in c["ranks"]:
        checked += _check(_c5_shard(gpu, rank), gpu.shard_rows(H, rank, world), W, g, world, rank)
    assert checked == len(g["index"]) == 64 * len(c["ranks"])


def test_c5_full_rows_every_rank_match_reference(gpu):
    """64 FULL rows of C5 (dragon + sponza 3840x2160 at 4096 spp), 8 seeded rows of every
    rank's shard of the 8-way split, rendered by the reference here (tools/make_goldens.py
    --c5rows: 245,760 pixels, 3,911 s on 6 threads; scene.cpp:31-52): every row's FNV-1a hash
    of its float sums, and one row per rank bit for bit."""
    c = META["c5_rows"]
    W, H, world = c["width"], c["height"], c["world"]
    g = rtref.golden(c["file"])
    rows = g["rows"].astype(np.int64)
    assert len(rows) == world * c["rows_per_rank"]
    got = np.zeros((len(rows), W, 3), np.float32)
    for rank in range(world):
        mine = gpu.shard_rows(H, rank, world)
        pos = {int(r): k for k, r in enumerate(mine)}
        out = _c5_shard(gpu, rank)
        for i, r in enumerate(rows):
            if int(r) in pos:
                got[i] = out[pos[int(r)]]
    bad = np.nonzero(rtref.row_hash(got) != g["row_fnv1a"])[0]
    assert len(bad) == 0, f"{len(bad)} of {len(rows)} rows differ, first rows {rows[bad[:8]]}"
    for r, want in zip(g["full_rows"], g["full_row_sums"]):
        i = int(np.nonzero(rows == r)[0][0])
        assert np.array_equal(rtref.bits(got[i]), rtref.bits(want)), f"row {r}"


@pytest.mark.parametrize("world", [4, 8])
@pytest.mark.parametrize("config", sorted(FRAMES))
def test_split_frame_runahead_matches_reference(gpu, config, world):
    """The whole BASELINE frame as the shards of the 4- and 8-way split, each rendered by the
    runahead kernel (rt_mega.h spec_manage: one and two pixels per lane), reassembled and
    compared row by row with the reference's own render of the frame (every row's FNV-1a
    hash, 8 full rows; scene.cpp:31-64).  The 8-way split also goes through rt_render_frame
    (each shard finished to 8 bits on the device and gathered there), whose 8-bit frame must
    be the reference's PPM body (canvas.h:76-89)."""
    import hashlib
    f = FRAMES[config]
    W, H, S = f["width"], f["height"], f["spp"]
    scene = _scene(gpu, f["scene"], W, H, S)
    frame = np.full((H, W, 3), np.nan, np.float32)
    for rank in range(world):
        rows = gpu.shard_rows(H, rank, world)
        part, st = scene.render_sums(S, rank=rank, world=world)
        assert st["schedule"] == gpu.SCHED_RUNAHEAD, f"rank {rank}: schedule {st['schedule']}"
        frame[rows] = part
    g = rtref.golden(f["file"])
    bad = np.nonzero(rtref.row_hash(frame) != g["row_fnv1a"])[0]
    assert len(bad) == 0, f"{len(bad)} of {H} rows differ, first {bad[:8]}"
    assert np.array_equal(rtref.bits(frame[g["rows"]]), rtref.bits(g["row_sums"]))
    if world == 8:
        rgb, _, st = scene.render_frame(S, n_shards=8, devices=[0] * 8, sums=False)
        assert st["schedule"] == gpu.SCHED_RUNAHEAD
        assert hashlib.sha1(rgb.tobytes()).hexdigest() == f["frame_u8_sha1"]


@pytest.mark.parametrize("config", sorted(FRAMES))
def test_whole_frame_matches_reference(gpu, config):
    """The whole BASELINE frame against the reference's own render of it (scene.cpp:31-64):
    every row's FNV-1a hash of the float sums, 8 full rows bit for bit, and the sha1 of the
    8-bit frame finished on the device (rt_finish_kernel) against the reference's PPM body.
    C3 also counts (rays, AABB and triangle tests, light queries against the reference's)."""
    import hashlib
    f = FRAMES[config]
    W, H, S = f["width"], f["height"], f["spp"]
    assert f["scene_sha256"] == META[f["scene"]]["scene_sha256"]
    scene = _scene(gpu, f["scene"], W, H, S)
    count = config == "c3"
    out, st = scene.render_sums(S, count=count)
    g = rtref.golden(f["file"])
    bad = np.nonzero(rtref.row_hash(out) != g["row_fnv1a"])[0]
    assert len(bad) == 0, f"{len(bad)} of {H} rows differ, first {bad[:8]}"
    assert np.array_equal(rtref.bits(out[g["rows"]]), rtref.bits(g["row_sums"]))
    if count:
        ref = f["sums"]
        assert (st["rays"], st["aabb_tests"], st["tri_tests"], st["light_queries"], st["light_tri_tests"]) == \
            (ref["rays"], ref["aabb"], ref["tri"], ref["light_queries"], ref["light_tri"])
    rgb, _, _ = scene.render_frame(S, n_shards=1, devices=[0], sums=False)
    assert hashlib.sha1(rgb.tobytes()).hexdigest() == f["frame_u8_sha1"]
