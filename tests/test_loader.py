"""Host scene path: glTF loader, BVH build, light list, textures — against the reference's own
parsed and BVH-built scene (tests/golden/*_dump.rtd, written by oracle/ref_harness `dump`).

cornell and sponza_mini are bit-exact (triangles, attributes, tangents, BVH nodes, light BVH,
materials, normal transforms, decoded texels).  cornell_blob and practice6_1 have rotated
meshes: the reference's scene_parser.o, built by GCC 11 at -O3, lets the SLP vectorizer drop
float roundings in those transforms, so their vertices differ from the source
semantics by a few ulp and the SAH build then splits differently; for them the test checks
the triangle set within a relative 1e-5, and the render parity tests use the reference's
own arrays through rt_scene_from_view.
"""
import numpy as np
import pytest

import rtref

EXACT = ["cornell", "sponza_mini"]
ROTATED = ["cornell_blob", "practice6_1"]
KEYS = ["tri", "tri_attr", "tri_tan", "node", "light", "light_node", "mesh_f", "mesh_tex", "mesh_normal_transform"]


def _mine(rt, name):
    return rt.Scene.load(rtref.scene_path(name), 64, 64, 1).view()


@pytest.mark.parametrize("name", EXACT)
def test_loader_bit_exact(rt, name):
    mine = _mine(rt, name)
    ref = rtref.ref_arrays(rt, name, 64, 64, 1)
    for k in KEYS:
        a, b = np.ascontiguousarray(mine[k]), np.ascontiguousarray(ref[k])
        assert a.shape == b.shape, k
        assert np.array_equal(a.view(np.uint8), b.view(np.uint8)), k
    d = rtref.golden(f"{name}_dump.rtd")
    assert int(mine["ray_depth"]) == int(d["ray_depth"][0])


@pytest.mark.parametrize("name", EXACT + ROTATED)
def test_camera_matches_reference(rt, name):
    mine = _mine(rt, name)
    cam = rtref.golden(f"{name}_dump.rtd")["camera"]
    assert np.array_equal(rtref.bits(mine["cam_pos"]), rtref.bits(cam[:3]))
    assert np.array_equal(rtref.bits(np.asarray(mine["cam_axes"]).reshape(-1)), rtref.bits(cam[3:12]))
    assert np.array_equal(rtref.bits(mine["cam_fov"]), rtref.bits(cam[12:14]))


@pytest.mark.parametrize("name", ROTATED)
def test_loader_rotated_within_tolerance(rt, name):
    mine = _mine(rt, name)
    d = rtref.golden(f"{name}_dump.rtd")
    n = len(d["obj_mesh_id"])
    assert mine["tri"].shape[0] == n
    ref_v0 = d["obj_position"].reshape(n, 9)[:, :3].astype(np.float64)
    my_v0 = np.asarray(mine["tri"])[:, :3].astype(np.float64)
    ref_id = d["obj_mesh_id"].astype(np.int64)
    my_id = np.asarray(mine["tri_attr"])[:, 15].view(np.int32).astype(np.int64)

    def order(v, ids):
        key = np.round(v * 1e3).astype(np.int64)
        return np.lexsort((key[:, 2], key[:, 1], key[:, 0], ids))

    a, b = my_v0[order(my_v0, my_id)], ref_v0[order(ref_v0, ref_id)]
    scale = np.maximum(np.abs(b), 1.0)
    assert np.max(np.abs(a - b) / scale) < 1e-5
    # materials and the light list do not depend on the transforms
    for k in ["light", "mesh_f", "mesh_tex", "mesh_normal_transform"]:
        ref = rtref.ref_arrays(rt, name, 64, 64, 1)
        assert np.array_equal(np.ascontiguousarray(mine[k]).view(np.uint8), np.ascontiguousarray(ref[k]).view(np.uint8)), k


def test_texels_match_reference(rt):
    name = "sponza_mini"
    mine = _mine(rt, name)
    d = rtref.golden(f"{name}_dump.rtd")
    info = np.asarray(mine["tex_info"])
    tex = np.asarray(mine["texels"])
    assert len(info) == len(d["tex_fnv1a"])
    for (off, w, h, ch), (rw, rh, rch), want in zip(info, d["tex_dim"], d["tex_fnv1a"]):
        assert (w, h) == (rw, rh)
        # texels are stored RGBA8 from texel `off`; the reference keeps `channels` bytes per texel
        px = tex[4 * int(off):4 * (int(off) + int(w) * int(h))].reshape(-1, 4)[:, :int(rch)]
        hsh = 1469598103934665603
        for byte in px.reshape(-1).tobytes():
            hsh = ((hsh ^ byte) * 1099511628211) & 0xFFFFFFFFFFFFFFFF
        assert hsh == int(want)


def test_scene_generator_deterministic(tmp_path):
    sc = rtref.scenes_module()
    a = sc.SCENES["cornell_blob"](str(tmp_path / "a"))
    b = sc.SCENES["cornell_blob"](str(tmp_path / "b"))
    import filecmp
    import os
    for f in sorted(os.listdir(os.path.dirname(a))):
        assert filecmp.cmp(os.path.join(os.path.dirname(a), f), os.path.join(os.path.dirname(b), f), shallow=False), f


def test_loader_errors(rt, tmp_path):
    with pytest.raises(rt.RtError):
        rt.Scene.load(str(tmp_path / "missing.gltf"), 8, 8, 1)
    bad = tmp_path / "bad.gltf"
    bad.write_text("{ not json")
    with pytest.raises(rt.RtError):
        rt.Scene.load(str(bad), 8, 8, 1)
