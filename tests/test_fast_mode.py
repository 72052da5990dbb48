"""Fast mode (include/rt_hw.h RT_FLAG_FAST): per-(pixel, sample) Philox-seeded
streams, samples run as independent work units.  Not the reference's RNG convention, so the
bar is: (1) the oracle's restatement of fast mode is pinned by Random123's Philox known-answer
vectors and by its sample-for-sample construction from the parity integrator (whose sums the
reference goldens pin); (2) the GPU's fast mode is bit-exact against that restatement;
(3) fast mode agrees with the reference's image statistically."""
import numpy as np
import pytest

import rtref

# Random123 kat_vectors, philox4x32 10 rounds: (ctr, key, out)
PHILOX_KAT = [
    ([0, 0, 0, 0], [0, 0], [0x6627e8d5, 0xe169c58d, 0xbc57ac4c, 0x9b00dbd8]),
    ([0xffffffff] * 4, [0xffffffff] * 2, [0x408f276d, 0x41c83b0e, 0xa20bc7c6, 0x6d5451fd]),
    ([0x243f6a88, 0x85a308d3, 0x13198a2e, 0x03707344], [0xa4093822, 0x299f31d0],
     [0xd16cfe09, 0x94fdcceb, 0x5001e420, 0x24126ea1]),
]


@pytest.fixture(scope="module")
def gpu(rt):
    import torch   # initialises the HIP runtime librt_hw_amd.so shares (see test_gpu_parity.py)
    if torch.cuda.is_available():
        torch.zeros(1, device="cuda")
    if rt.device_count() < 1:
        pytest.fail("no HIP device visible: the GPU tests must run on the MI355X box")
    return rt


@pytest.mark.parametrize("ctr,key,out", PHILOX_KAT)
def test_oracle_philox_known_answers(oracle, ctr, key, out):
    assert [int(x) for x in oracle.philox(ctr, key)] == out


def test_oracle_fast_chunk_invariance(rt, oracle):
    """chunk 1 and chunk = spp add the same samples in the same order: identical bits; a
    ragged chunk (3 of 8) regroups the additions only."""
    arrays = rtref.ref_arrays(rt, "cornell", 33, 17, 8)
    a, _ = oracle.render_fast(arrays, 8, 1)
    b, _ = oracle.render_fast(arrays, 8, 8)
    c, _ = oracle.render_fast(arrays, 8, 3)
    assert np.array_equal(rtref.bits(a), rtref.bits(b))
    assert np.allclose(a, c, rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("name,w,h,s", [("cornell", 64, 64, 8), ("sponza_mini", 64, 36, 4)])
def test_oracle_fast_matches_reference_statistically(rt, oracle, name, w, h, s):
    """Fast mode's frame against the reference's own frame (golden sums): per-channel frame
    means agree within 4 standard errors of the per-pixel difference."""
    ref = rtref.golden(f"{name}_sums_{w}x{h}x{s}.rtd")["sums"].reshape(-1, 3).astype(np.float64) / s
    fast, _ = oracle.render_fast(rtref.ref_arrays(rt, name, w, h, s), s, 2)
    fast = fast.astype(np.float64) / s
    assert np.isfinite(fast).all()
    d = fast - ref
    se = d.std(0) / np.sqrt(len(d))
    assert (np.abs(d.mean(0)) <= 4 * se + 1e-6).all(), (d.mean(0), se)
    # not the parity stream: most pixels differ
    assert (rtref.bits(fast.astype(np.float32)) != rtref.bits(ref.astype(np.float32))).any(1).mean() > 0.5


FAST_CASES = [("cornell", 64, 64, 8, 3), ("cornell", 33, 17, 5, 1), ("sponza_mini", 64, 36, 4, 2),
              ("practice6_1", 96, 96, 4, 4)]


@pytest.mark.gpu
@pytest.mark.parametrize("name,w,h,s,chunk", FAST_CASES)
def test_gpu_fast_matches_oracle(gpu, oracle, name, w, h, s, chunk):
    arrays = rtref.ref_arrays(gpu, name, w, h, s)
    scene = gpu.Scene.from_view(arrays)
    out, st = scene.render_sums(s, fast=True, fast_chunk=chunk, count=True)
    ref, _ = oracle.render_fast(arrays, s, chunk)
    bad = (rtref.bits(out.reshape(-1, 3)) != rtref.bits(ref)).any(1)
    assert bad.sum() == 0, f"{bad.sum()} pixels differ, max |d| {np.abs(out.reshape(-1, 3) - ref).max()}"
    assert st["samples"] == w * h * s and st["rays"] >= w * h * s


@pytest.mark.gpu
@pytest.mark.parametrize("world", [2, 3])
def test_gpu_fast_partition_invariance(gpu, world):
    arrays = rtref.ref_arrays(gpu, "sponza_mini", 64, 36, 4)
    scene = gpu.Scene.from_view(arrays)
    full, _ = scene.render_sums(4, fast=True, fast_chunk=2)
    for r in range(world):
        rows = gpu.shard_rows(36, r, world, 8)
        part, _ = scene.render_sums(4, rank=r, world=world, fast=True, fast_chunk=2)
        assert np.array_equal(rtref.bits(part), rtref.bits(full[rows]))


@pytest.mark.gpu
def test_gpu_fast_rejects_other_kernels(gpu):
    scene = gpu.Scene.from_view(rtref.ref_arrays(gpu, "cornell", 16, 16, 2))
    with pytest.raises(gpu.RtError, match="kernel 0"):
        scene.render_sums(2, fast=True, kernel=4)
