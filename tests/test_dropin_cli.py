"""The drop-in CLIs end to end on the GPU, against the reference's own final images
(tests/golden/<scene>_<W>x<H>x<S>.ppm: the reference's sums finished and written by its own
aces_tonemap / pow / normal_to_ch8bit / Canvas::write_to, oracle/ref_harness `sums ... ppm`).

  rt_solution    this build's host (glTF loader, BVH build) -> librt_hw_amd.so on every visible
                 GPU (rt_render_multi) -> frame finish -> PPM: the `run.sh in.gltf W H spp out.ppm`
                 surface (main.cpp:22-60)
  render_mi355x  the reference's own parse_scene_gltf and main flow, Scene::render replaced by the
                 binding of integration/render_mi355x.cpp (built from the reference's objects in
                 this container; skipped where it was not built)
Both must write the reference's PPM byte for byte, with 1 device and with RT_GPUS unset (all).
"""
import os
import subprocess

import pytest

import rtref

pytestmark = pytest.mark.gpu
CASES = [("cornell", 33, 17, 3), ("practice6_1", 256, 256, 4), ("sponza_mini", 64, 36, 4)]
SOLUTION = os.path.join(rtref.ROOT, "raytracing-hw_amd", "rt_solution")
BINDING = os.path.join(rtref.ROOT, "oracle", "_ref", "render_mi355x")


def _run(exe, name, w, h, s, out, gpus):
    env = dict(os.environ)
    env.pop("RT_GPUS", None)
    if gpus:
        env["RT_GPUS"] = str(gpus)
    r = subprocess.run([exe, rtref.scene_path(name), str(w), str(h), str(s), out], env=env, capture_output=True,
                       text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    assert "Frame drawn into" in r.stdout
    return open(out, "rb").read()


@pytest.mark.parametrize("gpus", [1, 0])
@pytest.mark.parametrize("name,w,h,s", CASES)
def test_rt_solution_writes_reference_ppm(tmp_path, name, w, h, s, gpus):
    want = open(os.path.join(rtref.GOLD, f"{name}_{w}x{h}x{s}.ppm"), "rb").read()
    assert _run(SOLUTION, name, w, h, s, str(tmp_path / "out.ppm"), gpus) == want


@pytest.mark.parametrize("name,w,h,s", CASES)
def test_reference_binding_writes_reference_ppm(tmp_path, name, w, h, s):
    if not os.path.exists(BINDING):
        pytest.skip("integration binary not built (needs the reference build: make -C oracle integration)")
    want = open(os.path.join(rtref.GOLD, f"{name}_{w}x{h}x{s}.ppm"), "rb").read()
    assert _run(BINDING, name, w, h, s, str(tmp_path / "out.ppm"), 0) == want
