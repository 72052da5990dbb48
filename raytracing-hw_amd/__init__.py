"""raytracing-hw_amd — MI355X-native path-tracing core behind the reference's render seam.

Python host mirror of the reference's hot-path interface (Korinin38/raytracing-hw):

    parse_scene_gltf(path, width, height, samples) -> Scene   # src/io/scene_parser.cpp:25
    Scene.render()                                          # src/core/scene.cpp:17-65
    Scene.draw_into(filename)                               # src/core/scene.cpp:67 / canvas.h:76-89

plus the float-level entry points the tests and the benchmark use
(`Scene.render_sums`, `Scene.render_device`).  Everything runs through the C ABI of
``librt_hw_amd.so`` (include/rt_hw.h); there is no CPU fallback — if the library or a
GPU is missing the calls raise.
"""
from __future__ import annotations

import ctypes
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
# RT_LIB may point at the index-checked debug build (make -C raytracing-hw_amd debug)
LIB_PATH = os.environ.get("RT_LIB") or os.path.join(_HERE, "librt_hw_amd.so")
REPO_ROOT = os.path.dirname(_HERE)

_c_f = ctypes.POINTER(ctypes.c_float)
_c_i = ctypes.POINTER(ctypes.c_int32)
_c_u = ctypes.POINTER(ctypes.c_uint32)
_c_d = ctypes.POINTER(ctypes.c_double)
_c_b = ctypes.POINTER(ctypes.c_uint8)


class RtSceneView(ctypes.Structure):
    _fields_ = [
        ("width", ctypes.c_int32), ("height", ctypes.c_int32), ("samples", ctypes.c_int32), ("ray_depth", ctypes.c_int32),
        ("max_distance", ctypes.c_float), ("cam_pos", ctypes.c_float * 3), ("cam_axes", ctypes.c_float * 9),
        ("cam_fov", ctypes.c_float * 2), ("tan_half_fov", ctypes.c_float * 2),
        ("n_tris", ctypes.c_uint32), ("tri", _c_f), ("tri_attr", _c_f), ("tri_tan", _c_f),
        ("n_nodes", ctypes.c_uint32), ("node", _c_f), ("bvh_depth", ctypes.c_uint32),
        ("n_lights", ctypes.c_uint32), ("light", _c_f), ("n_light_nodes", ctypes.c_uint32), ("light_node", _c_f),
        ("light_bvh_depth", ctypes.c_uint32),
        ("n_meshes", ctypes.c_uint32), ("mesh_f", _c_f), ("mesh_tex", _c_i), ("mesh_normal_transform", _c_d),
        ("n_textures", ctypes.c_uint32), ("tex_info", _c_u), ("texels", _c_b), ("n_texel_bytes", ctypes.c_uint64),
    ]


ABI_VERSION = 6          # include/rt_hw.h RT_ABI_VERSION
KERNEL_LANE = 0          # RT_KERNEL_LANE: lane-resident persistent kernel (default)
KERNEL_WAVEFRONT = 4     # RT_KERNEL_WAVEFRONT: init / extend / shade launches
FLAG_KERNEL_TIMES = 1    # RT_FLAG_KERNEL_TIMES
FLAG_FAST = 2            # RT_FLAG_FAST: per-(pixel, sample) Philox-seeded streams, not bit-identical to the reference
FLAG_LIGHT_SPLIT = 4     # RT_FLAG_LIGHT_SPLIT: light-pdf walk as its own traversal state (same bits)
FLAG_NATURAL_ORDER = 8   # RT_FLAG_NATURAL_ORDER: row-major pixel order instead of the in-frame heaviest-first order
FLAG_NO_RUNAHEAD = 16    # RT_FLAG_NO_RUNAHEAD: no speculative sample runahead in the waves' tails (same bits)
FLAG_HEAVY_ORDER = 32    # RT_FLAG_HEAVY_ORDER: the heaviest-first order below 128 spp too (same bits)
# RtStats.schedule bits (include/rt_hw.h RT_SCHED_*): the kernels that rendered
SCHED_LANE, SCHED_RUNAHEAD, SCHED_FAST, SCHED_LIGHT_SPLIT, SCHED_WAVEFRONT = 1, 2, 4, 8, 16


class RtParams(ctypes.Structure):
    _fields_ = [("spp", ctypes.c_int32), ("rank", ctypes.c_int32), ("world", ctypes.c_int32),
                ("row_block", ctypes.c_int32), ("count", ctypes.c_int32), ("kernel", ctypes.c_int32),
                ("flags", ctypes.c_int32), ("fast_chunk", ctypes.c_int32), ("device", ctypes.c_int32)]


class RtStats(ctypes.Structure):
    _fields_ = [("pixels", ctypes.c_uint64), ("samples", ctypes.c_uint64), ("rays", ctypes.c_uint64),
                ("aabb_tests", ctypes.c_uint64), ("tri_tests", ctypes.c_uint64), ("light_queries", ctypes.c_uint64),
                ("light_aabb_tests", ctypes.c_uint64), ("light_tri_tests", ctypes.c_uint64), ("shading_hits", ctypes.c_uint64),
                ("render_ms", ctypes.c_double), ("extend_ms", ctypes.c_double), ("shade_ms", ctypes.c_double),
                ("extend_launches", ctypes.c_uint64), ("shade_launches", ctypes.c_uint64), ("extend_rays", ctypes.c_uint64),
                ("order_ms", ctypes.c_double), ("gather_ms", ctypes.c_double), ("devices", ctypes.c_uint64),
                ("schedule", ctypes.c_uint64)]

    def as_dict(self):
        return {k: getattr(self, k) for k, _ in self._fields_}


# every symbol include/rt_hw.h declares, with its ctypes signature
ABI = {
    "rt_scene_load_gltf": (ctypes.c_int, [ctypes.c_char_p, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32,
                                          ctypes.POINTER(ctypes.c_void_p)]),
    "rt_scene_from_view": (ctypes.c_int, [ctypes.POINTER(RtSceneView), ctypes.POINTER(ctypes.c_void_p)]),
    "rt_scene_get_view": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(RtSceneView)]),
    "rt_scene_free": (None, [ctypes.c_void_p]),
    "rt_scene_upload": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int32]),
    "rt_shard_rows": (ctypes.c_int64, [ctypes.c_int32, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32, _c_i]),
    "rt_render": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(RtParams), _c_f, ctypes.POINTER(RtStats)]),
    "rt_render_device": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(RtParams), ctypes.c_void_p, ctypes.c_void_p,
                                        ctypes.POINTER(RtStats)]),
    "rt_render_multi": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(RtParams), ctypes.c_int32, _c_f,
                                       ctypes.POINTER(RtStats)]),
    "rt_render_frame": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(RtParams), ctypes.c_int32, _c_i, _c_b, _c_f,
                                       ctypes.POINTER(RtStats)]),
    "rt_intersect_rays": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int64, _c_f, _c_f, _c_f,
                                         ctypes.POINTER(ctypes.c_int64)]),
    "rt_tonemap_u8": (ctypes.c_int, [_c_f, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32, _c_b]),
    "rt_tonemap_u8_device": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32,
                                            ctypes.c_void_p, ctypes.c_void_p]),
    "rt_write_ppm": (ctypes.c_int, [ctypes.c_char_p, _c_b, ctypes.c_int32, ctypes.c_int32]),
    "rt_last_error": (ctypes.c_char_p, []),
    "rt_abi_version": (ctypes.c_int32, []),
    "rt_device_count": (ctypes.c_int32, []),
    "rt_device_synchronize": (ctypes.c_int, []),
    "rt_device_selfcheck": (ctypes.c_int, [ctypes.c_int32, ctypes.POINTER(ctypes.c_uint64)]),
}

_lib_handle = None
# debug builds (make -C raytracing-hw_amd debug, RT_LIB=.../debug/librt_hw_amd.so) export
# rt_debug_take: every render then raises on a recorded device check (rt_path.h RT_CHECK)
# unless debug_raise is cleared (tests that provoke one)
debug_raise = True


def lib():
    """Load librt_hw_amd.so (built in-tree by `make -C raytracing-hw_amd`); raise if absent."""
    global _lib_handle
    if _lib_handle is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f"{LIB_PATH} missing: build it with `make -C raytracing-hw_amd` "
                               "(there is no CPU fallback for the render path)")
        h = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in ABI.items():
            fn = getattr(h, name)
            fn.restype = res
            fn.argtypes = args
        if hasattr(h, "rt_debug_take"):
            h.rt_debug_take.restype = ctypes.c_int
            h.rt_debug_take.argtypes = [ctypes.POINTER(ctypes.c_uint64)]
            h.rt_debug_set_poison.restype = ctypes.c_int
            h.rt_debug_set_poison.argtypes = [ctypes.c_int]
        _lib_handle = h
    return _lib_handle


def is_debug_build():
    return hasattr(lib(), "rt_debug_take")


def debug_take():
    """Debug builds: the first device check violation since the last call (code << 56 | value),
    0 = none; None on a release build."""
    if not is_debug_build():
        return None
    w = ctypes.c_uint64(0)
    _check(lib().rt_debug_take(ctypes.byref(w)))
    return int(w.value)


def debug_set_poison(on):
    """Debug builds: poison every lane's traversal phase and stack depth at the lane-resident
    kernel's start (the packing test)."""
    _check(lib().rt_debug_set_poison(int(on)))


def _after_render():
    if debug_raise and _lib_handle is not None and hasattr(_lib_handle, "rt_debug_take"):
        w = debug_take()
        if w:
            raise RtError(f"device check {w >> 56} failed (value {w & ((1 << 56) - 1):#x})")


class RtError(RuntimeError):
    pass


def _check(rc):
    if rc != 0:
        raise RtError(lib().rt_last_error().decode())


def shard_rows(height, rank=0, world=1, row_block=8):
    n = lib().rt_shard_rows(height, rank, world, row_block, None)
    if n < 0:
        raise RtError(lib().rt_last_error().decode())
    rows = np.zeros(max(n, 1), np.int32)
    lib().rt_shard_rows(height, rank, world, row_block, rows.ctypes.data_as(_c_i))
    return rows[:n]


def _arr(ptr, n, dtype):
    if n == 0:
        return np.zeros(0, dtype)
    return np.ctypeslib.as_array(ptr, shape=(n,)).astype(dtype, copy=True)


class Scene:
    """Flattened scene (reference `Scene`, src/core/scene.h:14-38) owned by librt_hw_amd."""

    def __init__(self, handle, width, height, samples):
        self._h = ctypes.c_void_p(handle)
        self.width, self.height, self.samples = width, height, samples
        self.canvas = None

    @classmethod
    def load(cls, path, width, height, samples):
        h = ctypes.c_void_p()
        _check(lib().rt_scene_load_gltf(os.fsencode(path), width, height, samples, ctypes.byref(h)))
        return cls(h.value, width, height, samples)

    @classmethod
    def from_view(cls, arrays):
        """Scene from flattened arrays (dict as returned by view()); see rt_scene_from_view."""
        v, keep = make_view(arrays)
        h = ctypes.c_void_p()
        _check(lib().rt_scene_from_view(ctypes.byref(v), ctypes.byref(h)))
        del keep
        return cls(h.value, int(arrays["width"]), int(arrays["height"]), int(arrays["samples"]))

    def intersect_rays(self, org, dirs):
        """Closest hit + light pdf per ray: returns (f32 n x 4 [t,u,v,light_pdf], i64 n x 6)."""
        org = np.ascontiguousarray(org, np.float32).reshape(-1, 3)
        dirs = np.ascontiguousarray(dirs, np.float32).reshape(-1, 3)
        n = org.shape[0]
        out_f = np.zeros((n, 4), np.float32)
        out_i = np.zeros((n, 6), np.int64)
        _check(lib().rt_intersect_rays(self._h, n, org.ctypes.data_as(_c_f), dirs.ctypes.data_as(_c_f),
                                       out_f.ctypes.data_as(_c_f), out_i.ctypes.data_as(ctypes.POINTER(ctypes.c_int64))))
        _after_render()
        return out_f, out_i

    def __del__(self):
        h = getattr(self, "_h", None)
        if h is not None and h.value and _lib_handle is not None:
            _lib_handle.rt_scene_free(h)
            self._h = None

    def view(self):
        """Copies of the flattened arrays (the HBM layout, include/rt_hw.h rt_scene_view)."""
        v = RtSceneView()
        _check(lib().rt_scene_get_view(self._h, ctypes.byref(v)))
        out = {k: getattr(v, k) for k in ("width", "height", "samples", "ray_depth", "max_distance", "bvh_depth",
                                          "light_bvh_depth")}
        out["cam_pos"] = np.array(v.cam_pos[:], np.float32)
        out["cam_axes"] = np.array(v.cam_axes[:], np.float32).reshape(3, 3)
        out["cam_fov"] = np.array(v.cam_fov[:], np.float32)
        out["tan_half_fov"] = np.array(v.tan_half_fov[:], np.float32)
        out["tri"] = _arr(v.tri, 12 * v.n_tris, np.float32).reshape(-1, 12)
        out["tri_attr"] = _arr(v.tri_attr, 16 * v.n_tris, np.float32).reshape(-1, 16)
        out["tri_tan"] = _arr(v.tri_tan, 12 * v.n_tris, np.float32).reshape(-1, 12)
        out["node"] = _arr(v.node, 8 * v.n_nodes, np.float32).reshape(-1, 8)
        out["light"] = _arr(v.light, 16 * v.n_lights, np.float32).reshape(-1, 16)
        out["light_node"] = _arr(v.light_node, 8 * v.n_light_nodes, np.float32).reshape(-1, 8)
        out["mesh_f"] = _arr(v.mesh_f, 12 * v.n_meshes, np.float32).reshape(-1, 12)
        out["mesh_tex"] = _arr(v.mesh_tex, 4 * v.n_meshes, np.int32).reshape(-1, 4)
        out["mesh_normal_transform"] = _arr(v.mesh_normal_transform, 16 * v.n_meshes, np.float64).reshape(-1, 16)
        out["tex_info"] = _arr(v.tex_info, 4 * v.n_textures, np.uint32).reshape(-1, 4)
        out["texels"] = _arr(v.texels, int(v.n_texel_bytes), np.uint8)
        return out

    @property
    def handle(self):
        return self._h

    def upload(self, device=0):
        _check(lib().rt_scene_upload(self._h, device))

    def _params(self, spp, rank, world, row_block, count, kernel, kernel_times=False, fast=False, fast_chunk=0,
                device=0, light_split=False, natural_order=False, runahead=True, heavy_order=False):
        flags = ((FLAG_KERNEL_TIMES if kernel_times else 0) | (FLAG_FAST if fast else 0) |
                 (FLAG_LIGHT_SPLIT if light_split else 0) | (FLAG_NATURAL_ORDER if natural_order else 0) |
                 (0 if runahead else FLAG_NO_RUNAHEAD) | (FLAG_HEAVY_ORDER if heavy_order else 0))
        return RtParams(spp or 0, rank, world, row_block, int(count), kernel, flags, fast_chunk, device)

    def render_sums(self, spp=None, rank=0, world=1, row_block=8, count=False, kernel=0, device=0, fast=False,
                    fast_chunk=0, light_split=False, natural_order=False, runahead=True, heavy_order=False):
        """Per-pixel float RGB sums of the owned rows (sample_canvas, scene.cpp:20,42).
        fast=True: fast mode (RT_FLAG_FAST, work units of fast_chunk samples): statistically
        equivalent to the reference, not bit-identical.  light_split / natural_order /
        heavy_order / runahead=False: other schedules of the same bits (RT_FLAG_LIGHT_SPLIT,
        RT_FLAG_NATURAL_ORDER, RT_FLAG_HEAVY_ORDER, RT_FLAG_NO_RUNAHEAD)."""
        rows = shard_rows(self.height, rank, world, row_block)
        out = np.zeros((len(rows), self.width, 3), np.float32)
        st = RtStats()
        p = self._params(spp, rank, world, row_block, count, kernel, fast=fast, fast_chunk=fast_chunk, device=device,
                         light_split=light_split, natural_order=natural_order, runahead=runahead,
                         heavy_order=heavy_order)
        _check(lib().rt_render(self._h, ctypes.byref(p), out.ctypes.data_as(_c_f), ctypes.byref(st)))
        _after_render()
        return out, st.as_dict()

    def render_multi(self, spp=None, n_devices=0, row_block=8, count=False, kernel=0, fast=False, fast_chunk=0):
        """The whole frame over devices 0..n_devices-1 (0 = all visible; rt_render_multi):
        one host thread per device, each rendering its row-block shard; (H, W, 3) sums."""
        out = np.zeros((self.height, self.width, 3), np.float32)
        st = RtStats()
        p = self._params(spp, 0, 1, row_block, count, kernel, fast=fast, fast_chunk=fast_chunk)
        _check(lib().rt_render_multi(self._h, ctypes.byref(p), n_devices, out.ctypes.data_as(_c_f), ctypes.byref(st)))
        _after_render()
        return out, st.as_dict()

    def render_frame(self, spp=None, n_shards=0, devices=None, row_block=8, sums=True, rgb=True, kernel=0,
                     fast=False, fast_chunk=0, runahead=True):
        """The whole frame as shards 0..n_shards-1 (0 = one per visible device), shard r on
        device devices[r] (None: device r; rt_render_frame): each shard is finished to 8 bits
        on its device and gathered device-to-device onto devices[0].  Returns (rgb (H, W, 3)
        uint8 or None, sums (H, W, 3) float32 or None, stats)."""
        out_rgb = np.zeros((self.height, self.width, 3), np.uint8) if rgb else None
        out_sum = np.zeros((self.height, self.width, 3), np.float32) if sums else None
        dev = None
        if devices is not None:
            dev = np.ascontiguousarray(devices, np.int32)
            if n_shards and len(dev) != n_shards:
                raise ValueError("devices must name one device per shard")
            n_shards = len(dev)
        st = RtStats()
        p = self._params(spp, 0, 1, row_block, False, kernel, fast=fast, fast_chunk=fast_chunk, runahead=runahead)
        _check(lib().rt_render_frame(self._h, ctypes.byref(p), n_shards,
                                     dev.ctypes.data_as(_c_i) if dev is not None else None,
                                     out_rgb.ctypes.data_as(_c_b) if rgb else None,
                                     out_sum.ctypes.data_as(_c_f) if sums else None, ctypes.byref(st)))
        _after_render()
        return out_rgb, out_sum, st.as_dict()

    def render_device(self, d_out_ptr, stream_ptr=None, spp=None, rank=0, world=1, row_block=8, count=False,
                      kernel=0, stats=False, kernel_times=False, fast=False, fast_chunk=0, device=0,
                      light_split=False, natural_order=False, runahead=True, heavy_order=False):
        """Launch into device memory (e.g. a torch tensor's data_ptr()) on a HIP stream, on
        `device` (upload(device) first).  kernel_times: per-launch HIP-event timing of the
        wavefront kernels (needs stats).  fast: fast mode (RT_FLAG_FAST), see render_sums."""
        p = self._params(spp, rank, world, row_block, count, kernel, kernel_times, fast, fast_chunk, device,
                         light_split, natural_order, runahead, heavy_order)
        st = RtStats() if stats else None
        _check(lib().rt_render_device(self._h, ctypes.byref(p), ctypes.c_void_p(d_out_ptr),
                                      ctypes.c_void_p(stream_ptr or 0), ctypes.byref(st) if st else None))
        _after_render()
        return st.as_dict() if st else None

    def render(self):
        """Scene::render (scene.cpp:17-65): sample loop on the GPU, then the 8-bit frame finish."""
        sums, _ = self.render_sums(self.samples)
        self.canvas = tonemap(sums, self.samples)
        return self.canvas

    def draw_into(self, filename):
        if self.canvas is None:
            raise RtError("render() first")
        write_ppm(filename, self.canvas)


def make_view(a):
    """Build an RtSceneView over numpy arrays (dict layout of Scene.view()); returns (view, keepalive)."""
    keep = {}

    def ptr(name, dtype, ctype):
        arr = np.ascontiguousarray(a[name], dtype).reshape(-1)
        if arr.size == 0:
            arr = np.zeros(1, dtype)
        keep[name] = arr
        return arr.ctypes.data_as(ctype)

    v = RtSceneView()
    v.width, v.height, v.samples, v.ray_depth = int(a["width"]), int(a["height"]), int(a["samples"]), int(a["ray_depth"])
    v.max_distance = float(a["max_distance"])
    v.cam_pos[:] = [float(x) for x in np.asarray(a["cam_pos"], np.float32)]
    v.cam_axes[:] = [float(x) for x in np.asarray(a["cam_axes"], np.float32).reshape(-1)]
    v.cam_fov[:] = [float(x) for x in np.asarray(a["cam_fov"], np.float32)]
    v.tan_half_fov[:] = [float(x) for x in np.asarray(a["tan_half_fov"], np.float32)]
    v.n_tris = len(a["tri"])
    v.tri, v.tri_attr, v.tri_tan = ptr("tri", np.float32, _c_f), ptr("tri_attr", np.float32, _c_f), ptr("tri_tan", np.float32, _c_f)
    v.n_nodes, v.node = len(a["node"]), ptr("node", np.float32, _c_f)
    v.bvh_depth = int(a.get("bvh_depth", 0))
    v.n_lights, v.light = len(a["light"]), ptr("light", np.float32, _c_f)
    v.n_light_nodes, v.light_node = len(a["light_node"]), ptr("light_node", np.float32, _c_f)
    v.light_bvh_depth = int(a.get("light_bvh_depth", 0))
    v.n_meshes = len(a["mesh_f"])
    v.mesh_f, v.mesh_tex = ptr("mesh_f", np.float32, _c_f), ptr("mesh_tex", np.int32, _c_i)
    v.mesh_normal_transform = ptr("mesh_normal_transform", np.float64, _c_d)
    v.n_textures, v.tex_info = len(a["tex_info"]), ptr("tex_info", np.uint32, _c_u)
    v.texels, v.n_texel_bytes = ptr("texels", np.uint8, _c_b), int(np.asarray(a["texels"]).size)
    return v, keep


def parse_scene_gltf(path, width, height, samples):
    return Scene.load(path, width, height, samples)


def tonemap(sums, spp):
    sums = np.ascontiguousarray(sums, np.float32)
    h, w = sums.shape[0], sums.shape[1]
    rgb = np.zeros((h, w, 3), np.uint8)
    _check(lib().rt_tonemap_u8(sums.ctypes.data_as(_c_f), w, h, spp, rgb.ctypes.data_as(_c_b)))
    return rgb


def tonemap_device(d_sum_ptr, width, height, spp, d_rgb_ptr, stream_ptr=None):
    """rt_tonemap_u8_device: the frame finish on the GPU (device pointers, e.g. torch tensors)."""
    _check(lib().rt_tonemap_u8_device(ctypes.c_void_p(d_sum_ptr), width, height, spp, ctypes.c_void_p(d_rgb_ptr),
                                      ctypes.c_void_p(stream_ptr or 0)))


def write_ppm(filename, rgb):
    rgb = np.ascontiguousarray(rgb, np.uint8)
    _check(lib().rt_write_ppm(os.fsencode(filename), rgb.ctypes.data_as(_c_b), rgb.shape[1], rgb.shape[0]))


def device_count():
    return int(lib().rt_device_count())


def device_selfcheck(which=0):
    """rt_device_selfcheck: mismatches of the kernels' hardware-dependent exact arithmetic
    (0: the fast reciprocal over every float with a normal reciprocal; 1: the computed linear
    texel decode over every byte and the packed LDS RNG word over every minstd state)."""
    n = ctypes.c_uint64(0)
    _check(lib().rt_device_selfcheck(which, ctypes.byref(n)))
    return int(n.value)
