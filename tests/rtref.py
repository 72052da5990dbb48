"""Test helpers: package import, the CPU oracle (oracle/liboracle.so), golden fixtures.

The oracle is test infrastructure (oracle/rt_oracle.cpp); it is only ever used here as
the checker.  Goldens under tests/golden/ were produced by the reference itself
(tools/make_goldens.py, oracle/ref_harness.cpp).
"""
import ctypes
import importlib.util
import os
import subprocess
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
GOLD = os.path.join(HERE, "golden")
PKG_DIR = os.path.join(ROOT, "raytracing-hw_amd")
sys.path.insert(0, HERE)
import rtdump  # noqa: E402

_pkg = None


def _make(directory, target=None):
    cmd = ["make", "-s", "-j8", "-C", directory] + ([target] if target else [])
    subprocess.run(cmd, check=True)


def package():
    """Import raytracing-hw_amd (hyphenated dir) as `raytracing_hw_amd`, building it if needed."""
    global _pkg
    if _pkg is None:
        if not os.path.exists(os.path.join(PKG_DIR, "librt_hw_amd.so")):
            _make(PKG_DIR)
        if "raytracing_hw_amd" in sys.modules:
            _pkg = sys.modules["raytracing_hw_amd"]
        else:
            spec = importlib.util.spec_from_file_location("raytracing_hw_amd", os.path.join(PKG_DIR, "__init__.py"),
                                                          submodule_search_locations=[PKG_DIR])
            _pkg = importlib.util.module_from_spec(spec)
            sys.modules["raytracing_hw_amd"] = _pkg
            spec.loader.exec_module(_pkg)
    return _pkg


def scenes_module():
    spec = importlib.util.spec_from_file_location("rt_scenes", os.path.join(PKG_DIR, "scenes.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


def scene_sha256(directory, scene):
    """sha256 over a generated scene's files (name + bytes, sorted by name): the value
    tools/make_goldens.py records for the BASELINE-config goldens."""
    import hashlib
    h = hashlib.sha256()
    files = sorted(f for f in os.listdir(directory) if f == scene + ".gltf" or f.startswith(scene + "_tex")
                   or f == scene + ".bin")
    for f in files:
        h.update(f.encode())
        with open(os.path.join(directory, f), "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()


def golden(name):
    return rtdump.load(os.path.join(GOLD, name))


def scene_path(name):
    return os.path.join(GOLD, "scenes", name, name + ".gltf")


def _f(u):
    return np.asarray(u, np.uint32).view(np.float32)


def ref_arrays(rt, name, width, height, spp, dump=None, path=None):
    """Flattened arrays of the reference's own parsed + BVH-built scene (golden dump, or
    `dump` as loaded by rtdump), completed with this build's camera constants and decoded
    texels (pinned equal to the reference's by test_loader).  path: the scene's .gltf when it
    is not a committed fixture."""
    mine = rt.Scene.load(path or scene_path(name), width, height, spp).view()
    d = golden(f"{name}_dump.rtd") if dump is None else dump
    n = len(d["obj_mesh_id"])
    a = dict(mine)
    a["tri"] = np.concatenate([d["obj_position"].reshape(n, 9), d["obj_geo_normal"]], 1).astype(np.float32)
    tc = d.get("obj_texcoord", np.zeros((n, 3, 2), np.float32)).reshape(n, 6)
    a["tri_attr"] = np.concatenate([d["obj_normal"].reshape(n, 9), tc,
                                    d["obj_mesh_id"].astype(np.int32).view(np.float32)[:, None]], 1)
    a["tri_tan"] = d.get("obj_tangent", np.zeros((n, 3, 4), np.float32)).reshape(n, 12).astype(np.float32)

    def nodes(box, meta):
        meta = meta.astype(np.int64)
        leaf = meta[:, 4] > 0
        A = np.where(leaf, meta[:, 3], meta[:, 0]).astype(np.uint32)
        B = np.where(leaf, 3 | (meta[:, 4] << 2), meta[:, 2]).astype(np.uint32)
        return np.concatenate([box, _f(A)[:, None], _f(B)[:, None]], 1).astype(np.float32)

    a["node"] = nodes(d["node_aabb"], d["node_meta"])
    nl = len(d["light_mesh_id"])
    a["light"] = np.zeros((nl, 16), np.float32)
    if nl:
        a["light"][:, :9] = d["light_position"].reshape(nl, 9)
        a["light"][:, 9:12] = d["light_geo_normal"]
        a["light"][:, 12] = d["light_area"]
        a["light_node"] = nodes(d["lnode_aabb"], d["lnode_meta"])
    else:
        a["light_node"] = np.zeros((0, 8), np.float32)
    mf = d["mesh_f"]  # ior, alpha, base.xyz, emission.xyz, metallic, roughness2
    a["mesh_f"] = np.zeros((len(mf), 12), np.float32)
    a["mesh_f"][:, 0:3] = mf[:, 2:5]
    a["mesh_f"][:, 3:6] = mf[:, 5:8]
    a["mesh_f"][:, 6] = mf[:, 8]
    a["mesh_f"][:, 7] = mf[:, 9]
    a["mesh_f"][:, 8] = mf[:, 1]
    a["mesh_f"][:, 9] = mf[:, 0]
    a["mesh_tex"] = d["mesh_tex"].astype(np.int32)
    a["mesh_normal_transform"] = d["mesh_normal_transform"].astype(np.float64)
    cam = d["camera"]
    assert np.array_equal(cam[:3].view(np.uint32), mine["cam_pos"].view(np.uint32))
    return a


class Oracle:
    """ctypes front of oracle/liboracle.so (the CPU restatement)."""

    def __init__(self):
        path = os.path.join(ROOT, "oracle", "liboracle.so")
        if not os.path.exists(path):
            _make(os.path.join(ROOT, "oracle"), "oracle")
        self.lib = ctypes.CDLL(path)
        V = ctypes.c_void_p
        self.lib.rt_oracle_render.restype = ctypes.c_double
        self.lib.rt_oracle_render.argtypes = [V, ctypes.c_int, ctypes.c_int64, ctypes.c_int64, ctypes.c_int, V, V]
        self.lib.rt_oracle_render_fast.restype = ctypes.c_double
        self.lib.rt_oracle_render_fast.argtypes = [V, ctypes.c_int, ctypes.c_int, ctypes.c_int64, ctypes.c_int64,
                                                   ctypes.c_int, V]
        self.lib.rt_oracle_philox.restype = None
        self.lib.rt_oracle_philox.argtypes = [V, V, V]
        self.lib.rt_oracle_rays.restype = None
        self.lib.rt_oracle_rays.argtypes = [V, ctypes.c_int64, V, V, V, V]

    def render(self, arrays, spp, p0=0, p1=None, threads=0):
        rt = package()
        v, keep = rt.make_view(arrays)
        W, H = int(arrays["width"]), int(arrays["height"])
        p1 = W * H if p1 is None else p1
        out = np.zeros((p1 - p0, 3), np.float32)
        cnt = np.zeros(6, np.uint64)
        secs = self.lib.rt_oracle_render(ctypes.addressof(v), spp, p0, p1, threads, out.ctypes.data, cnt.ctypes.data)
        del keep
        return out, cnt, secs

    def render_fast(self, arrays, spp, chunk, p0=0, p1=None, threads=0):
        """Fast mode (RT_FLAG_FAST) restated: per-sample Philox seeds, chunk partials."""
        rt = package()
        v, keep = rt.make_view(arrays)
        W, H = int(arrays["width"]), int(arrays["height"])
        p1 = W * H if p1 is None else p1
        out = np.zeros((p1 - p0, 3), np.float32)
        secs = self.lib.rt_oracle_render_fast(ctypes.addressof(v), spp, chunk, p0, p1, threads, out.ctypes.data)
        del keep
        return out, secs

    def philox(self, ctr, key):
        c = np.ascontiguousarray(ctr, np.uint32)
        k = np.ascontiguousarray(key, np.uint32)
        o = np.zeros(4, np.uint32)
        self.lib.rt_oracle_philox(c.ctypes.data, k.ctypes.data, o.ctypes.data)
        return o

    def rays(self, arrays, org, dirs):
        rt = package()
        v, keep = rt.make_view(arrays)
        org = np.ascontiguousarray(org, np.float32)
        dirs = np.ascontiguousarray(dirs, np.float32)
        n = len(org)
        out_f = np.zeros((n, 4), np.float32)
        out_i = np.zeros((n, 6), np.int64)
        self.lib.rt_oracle_rays(ctypes.addressof(v), n, org.ctypes.data, dirs.ctypes.data, out_f.ctypes.data,
                                out_i.ctypes.data)
        del keep
        return out_f, out_i


def bits(a):
    return np.ascontiguousarray(a, np.float32).view(np.uint32)


def row_hash(sums):
    h = np.full(sums.shape[0], 1469598103934665603, np.uint64)
    b = np.ascontiguousarray(sums).view(np.uint8).reshape(sums.shape[0], -1)
    with np.errstate(over="ignore"):
        for k in range(b.shape[1]):
            h = (h ^ b[:, k].astype(np.uint64)) * np.uint64(1099511628211)
    return h
