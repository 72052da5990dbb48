"""The C5 proxy scene (BASELINE.json configs[4]: dragon-100k + sponza): generator, loader
and oracle on CPU.  The GPU side is test_gpu_parity.py::test_sponza_dragon_c5_pixels_vs_oracle."""
import os

import numpy as np

import rtref


def test_dragon_100k_proxy():
    scenes = rtref.scenes_module()
    src = np.load(scenes.DRAGON_FIXTURE)
    assert src.shape == (9992, 3, 3)   # the reference's practice5_dragon_10k.txt triangles
    t = scenes.dragon_100k()
    assert t.shape == (100001, 3, 3) and np.isfinite(t).all()
    # subdivision keeps the surface: same bounding box, same total area
    assert np.allclose(t.reshape(-1, 3).min(0), src.reshape(-1, 3).min(0))
    area = lambda a: 0.5 * np.linalg.norm(np.cross(a[:, 1] - a[:, 0], a[:, 2] - a[:, 0]), axis=1).sum()
    assert abs(area(t.astype(np.float64)) / area(src.astype(np.float64)) - 1) < 1e-5


def test_sponza_dragon_mini_loads_and_renders(rt, oracle, tmp_path):
    scenes = rtref.scenes_module()
    path = scenes.ensure_scene("sponza_dragon_mini", str(tmp_path))
    base = rt.Scene.load(scenes.ensure_scene("sponza_mini", str(tmp_path)), 32, 18, 1)
    scene = rt.Scene.load(path, 32, 18, 1)
    v = scene.view()
    assert v["tri"].shape[0] == base.view()["tri"].shape[0] + 100001
    out, cnt, _ = oracle.render(v, 1, 0, 32 * 18, threads=2)
    assert np.isfinite(out).all() and int(cnt[0]) >= 32 * 18
