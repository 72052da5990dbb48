"""The drop-in boundary (include/rt_hw.h, librt_hw_amd.so) on the host: every declared entry
point is exported, argument / error behaviour, the pixel-row partition, and the frame finish
(tonemap + 8-bit + PPM) against the reference's own output (tests/golden/finish_*, written by
oracle/ref_harness `finish` through the reference's aces_tonemap / pow / normal_to_ch8bit /
Canvas::write_to).  No GPU is touched: render calls must fail loudly without one."""
import ctypes
import os
import re
import subprocess

import numpy as np
import pytest

import rtref

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "rt_hw.h")


def declared_functions():
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"^\s*[A-Za-z_][\w\s\*]*?\b(rt_\w+)\s*\(", text, flags=re.M)))


def test_header_declares_the_boundary():
    names = declared_functions()
    for must in ["rt_scene_load_gltf", "rt_scene_from_view", "rt_render", "rt_render_device", "rt_intersect_rays",
                 "rt_tonemap_u8", "rt_write_ppm", "rt_shard_rows", "rt_last_error", "rt_abi_version",
                 "rt_render_multi", "rt_render_frame"]:
        assert must in names


def test_library_exports_every_declared_symbol(rt):
    lib = ctypes.CDLL(rt.LIB_PATH)
    missing = [n for n in declared_functions() if not hasattr(lib, n)]
    assert not missing, missing
    assert set(rt.ABI) == set(declared_functions())


def test_abi_version(rt):
    assert rt.lib().rt_abi_version() == rt.ABI_VERSION == 6
    assert ctypes.sizeof(rt.RtParams) == 36
    assert ctypes.sizeof(rt.RtStats) == 9 * 8 + 3 * 8 + 3 * 8 + 3 * 8 + 8   # ABI 5: + schedule


@pytest.mark.parametrize("height,world,rb", [(1080, 1, 8), (1080, 2, 8), (1080, 3, 8), (1080, 8, 8), (17, 3, 4),
                                            (7, 8, 8), (33, 5, 1)])
def test_shard_rows_partition(rt, height, world, rb):
    lib = rt.lib()
    seen = []
    for rank in range(world):
        n = lib.rt_shard_rows(height, rank, world, rb, None)
        rows = (ctypes.c_int32 * max(n, 1))()
        assert lib.rt_shard_rows(height, rank, world, rb, rows) == n
        got = list(rows)[:n]
        assert got == sorted(got)
        assert got == [r for r in range(height) if (r // rb) % world == rank]
        assert got == list(rt.shard_rows(height, rank, world, rb))
        seen += got
    assert sorted(seen) == list(range(height))


def test_shard_rows_rejects_bad_arguments(rt):
    lib = rt.lib()
    assert lib.rt_shard_rows(10, 0, 0, 8, None) < 0
    assert lib.rt_shard_rows(10, 2, 2, 8, None) < 0
    assert lib.rt_shard_rows(10, -1, 2, 8, None) < 0
    assert lib.rt_shard_rows(-1, 0, 1, 8, None) < 0


def test_frame_finish_matches_reference(rt, tmp_path):
    g = rtref.golden("finish_37x23x16.rtd")
    spp = int(g["spp"][0])
    rgb = rt.tonemap(g["sums"], spp)
    want = open(os.path.join(rtref.GOLD, "finish_37x23x16.ppm"), "rb").read()
    header = b"P6\n37 23\n255\n"
    assert want.startswith(header)
    assert rgb.tobytes() == want[len(header):]
    out = tmp_path / "frame.ppm"
    rt.write_ppm(str(out), rgb)
    assert out.read_bytes() == want


def test_errors_are_reported(rt, tmp_path):
    with pytest.raises(rt.RtError) as e:
        rt.Scene.load(str(tmp_path / "nope.gltf"), 4, 4, 1)
    assert str(e.value)
    assert rt.lib().rt_last_error()
    s = rt.Scene.load(rtref.scene_path("cornell"), 8, 8, 1)
    lib = rt.lib()
    p = rt.RtParams(1, 0, 1, 8, 0, 0, 0, 0, 0)
    assert lib.rt_render(s.handle, ctypes.byref(p), None, None) == -1   # RT_ERR_ARG
    out = np.zeros(8 * 8 * 3, np.float32)
    assert lib.rt_render_multi(s.handle, ctypes.byref(p), 1, None, None) == -1   # RT_ERR_ARG
    assert lib.rt_render_frame(s.handle, ctypes.byref(p), 1, None, None, None, None) == -1   # no output
    dev = (ctypes.c_int32 * 2)(0, 0)   # a devices array needs n_shards (its length)
    assert lib.rt_render_frame(s.handle, ctypes.byref(p), 0, dev, None, out.ctypes.data_as(rt._c_f), None) == -1
    assert b"n_shards" in lib.rt_last_error()
    if rt.device_count() == 0:   # no GPU: every render entry fails loudly (no CPU fallback)
        assert lib.rt_render(s.handle, ctypes.byref(p), out.ctypes.data_as(rt._c_f), None) == -4   # RT_ERR_DEVICE
        assert lib.rt_render_multi(s.handle, ctypes.byref(p), 0, out.ctypes.data_as(rt._c_f), None) == -4
        assert lib.rt_render_frame(s.handle, ctypes.byref(p), 2, None, None, out.ctypes.data_as(rt._c_f), None) == -4
    assert lib.rt_tonemap_u8(None, 4, 4, 1, None) == -1


def test_unknown_flags_rejected(rt):
    """Flag bits outside RT_FLAG_ALL fail with RT_ERR_ARG on every render entry, before any
    device work (a caller built against ABI 5 passing RT_FLAG_POOL = 64 gets an error, not the
    default schedule)."""
    s = rt.Scene.load(rtref.scene_path("cornell"), 8, 8, 1)
    lib = rt.lib()
    out = np.zeros(8 * 8 * 3, np.float32)
    rgb = np.zeros(8 * 8 * 3, np.uint8)
    for bad in (64, 1 << 20, -1):
        p = rt.RtParams(1, 0, 1, 8, 0, 0, bad, 0, 0)
        assert lib.rt_render(s.handle, ctypes.byref(p), out.ctypes.data_as(rt._c_f), None) == -1
        assert b"unknown flag" in lib.rt_last_error()
        assert lib.rt_render_device(s.handle, ctypes.byref(p), ctypes.c_void_p(1), None, None) == -1
        assert lib.rt_render_multi(s.handle, ctypes.byref(p), 1, out.ctypes.data_as(rt._c_f), None) == -1
        assert lib.rt_render_frame(s.handle, ctypes.byref(p), 1, None, rgb.ctypes.data_as(rt._c_b), None, None) == -1
        assert b"unknown flag" in lib.rt_last_error()


def test_scene_from_view_validates(rt):
    a = rtref.ref_arrays(rt, "cornell", 16, 16, 1)
    s = rt.Scene.from_view(a)
    v = s.view()
    for k in ["tri", "node", "light", "mesh_f"]:
        assert np.array_equal(np.ascontiguousarray(v[k]).view(np.uint8), np.ascontiguousarray(a[k]).view(np.uint8))
    bad = dict(a)
    bad["node"] = a["node"].copy()
    bad["node"][0, 6] = np.uint32(10 ** 6).view(np.float32)   # child index out of range
    with pytest.raises(rt.RtError):
        rt.Scene.from_view(bad)


def test_render_without_gpu_fails_loudly(rt):
    if rt.device_count() > 0:
        pytest.skip("GPU present: the render path is covered by the gpu tests")
    s = rt.Scene.load(rtref.scene_path("cornell"), 8, 8, 1)
    with pytest.raises(rt.RtError):
        s.render_sums(1)
    assert rt.device_count() == 0


def test_cli_usage_error():
    exe = os.path.join(ROOT, "raytracing-hw_amd", "rt_solution")
    if not os.path.exists(exe):
        subprocess.run(["make", "-C", os.path.join(ROOT, "raytracing-hw_amd"), "-s"], check=True)
    r = subprocess.run([exe], capture_output=True, text=True)
    assert r.returncode != 0
    assert "Invalid arguments" in r.stderr
