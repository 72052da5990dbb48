"""The reference-side binding (integration/render_mi355x.cpp) on the host.

render_mi355x is the reference's own main flow (parse_scene_gltf from the reference's objects)
with Scene::render swapped for this library.  `--view` runs the reference's parser, the
binding's flattening of the parsed Scene, rt_scene_from_view and rt_scene_get_view, and dumps
the arrays the kernels would read; they must equal, bit for bit, the reference's post-BVH
scene (tests/golden/*_dump.rtd, ref_harness `dump`) and this build's own loader.  The binary
links the reference's objects, so it exists only where the reference was built (this
container; oracle/Makefile `integration`)."""
import os
import subprocess

import numpy as np
import pytest

import rtref

EXE = os.path.join(rtref.ROOT, "oracle", "_ref", "render_mi355x")
KEYS = ["tri", "tri_attr", "tri_tan", "node", "light", "light_node", "mesh_f", "mesh_tex", "mesh_normal_transform"]


def _raw(a):
    return np.ascontiguousarray(a).view(np.uint8)


@pytest.fixture(scope="module")
def exe():
    if not os.path.exists(EXE):
        pytest.skip("reference build absent (make -C oracle integration needs /root/reference)")
    return EXE


@pytest.mark.parametrize("name", ["cornell", "cornell_blob", "practice6_1", "sponza_mini"])
def test_binding_view_matches_reference_dump(rt, exe, tmp_path, name):
    out = str(tmp_path / "view.rtd")
    subprocess.run([exe, "--view", rtref.scene_path(name), "64", "64", out], check=True, capture_output=True)
    v = rtref.rtdump.load(out)
    ref = rtref.ref_arrays(rt, name, 64, 64, 1)
    mine = rt.Scene.load(rtref.scene_path(name), 64, 64, 1).view()
    for k in KEYS:
        assert np.array_equal(_raw(v[k]), _raw(ref[k])), k
        assert np.array_equal(_raw(v[k]), _raw(mine[k])), k
    cam = v["camera"]
    assert np.array_equal(rtref.bits(cam[:3]), rtref.bits(mine["cam_pos"]))
    assert np.array_equal(rtref.bits(cam[3:12]), rtref.bits(np.asarray(mine["cam_axes"]).reshape(-1)))
    assert np.array_equal(rtref.bits(cam[12:16]), rtref.bits(np.concatenate([mine["cam_fov"], mine["tan_half_fov"]])))
    assert cam[16] == mine["max_distance"] == 100.0   # the glTF camera's zfar (scene_parser.cpp:119-120)
    meta = v["meta"]
    assert list(meta[:4]) == [64, 64, 1, int(mine["ray_depth"])]
    assert np.array_equal(v["texels"], mine["texels"])
    assert np.array_equal(v["tex_info"], mine["tex_info"])


def test_binding_usage_error(exe):
    r = subprocess.run([exe], capture_output=True, text=True)
    assert r.returncode != 0
