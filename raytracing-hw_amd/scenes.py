"""Deterministic glTF scene-fixture synthesizer.

Every example scene shipped with the reference points at a ``.bin`` buffer that is
not in the tree (``examples/*.gltf`` → ``practice*.bin`` / ``untitled.bin``, see
SURVEY.md §0.3), so neither the reference nor this build can load any of them as
shipped.  This module writes NEW self-contained ``.gltf + .bin (+ .ppm textures)``
files whose scene parameters (camera TRS, node TRS, materials, light) are the numbers
from the reference's example JSON, and whose meshes are procedural stand-ins sized to
the reference's accessor budgets:

* ``cornell``         — examples/practice7_1.gltf: 6 planes + 2 boxes (36 tris, exact
                         geometry from the accessor min/max).
* ``cornell_blob``    — cornell + a displaced UV sphere (10,000 tris) in place of the
                         reference's dragon (practice7_3.gltf / practice5_dragon_10k.txt).
* ``practice6_1``     — examples/practice6_1.gltf: plane, torus 48x12 (1,152 emissive
                         tris), cube, Suzanne stand-in (15,744 tris ellipsoid).
* ``sponza``          — examples/sponza/sponza.gltf proxy: 25 textured + normal-mapped
                         material primitives with the reference's per-primitive triangle
                         budgets (262,267 tris) placed inside each primitive's accessor
                         AABB as floor / colonnades / block rings, the reference camera,
                         and the 2-triangle emissive plane (strength 100).
                         Textures are procedural RGBA8 written as binary PPM (P6), which
                         stb_image (reference) and this build's loader both decode.
* ``sponza_mini``     — the same generator with budgets /32 and 16x16 textures (parity tests).

The textures are read by the reference through tinygltf/stb_image with ``req_comp=4``
(thirdparty/tinygltf/tiny_gltf.h:2609), i.e. RGBA8 with alpha 255 for P6 input.

Pure numpy; everything is seeded so two runs produce byte-identical files.
"""
from __future__ import annotations

import json
import math
import os

import numpy as np

F32 = np.float32

# --------------------------------------------------------------------------------------
# generic glTF writer
# --------------------------------------------------------------------------------------


class GltfBuilder:
    def __init__(self):
        self.bin = bytearray()
        self.buffer_views = []
        self.accessors = []
        self.meshes = []
        self.nodes = []
        self.materials = []
        self.cameras = []
        self.images = []
        self.textures = []
        self.extensions_used = set()

    def _view(self, data: bytes) -> int:
        while len(self.bin) % 4:
            self.bin.append(0)
        off = len(self.bin)
        self.bin += data
        self.buffer_views.append({"buffer": 0, "byteOffset": off, "byteLength": len(data)})
        return len(self.buffer_views) - 1

    def accessor(self, arr: np.ndarray, kind: str, minmax: bool = False) -> int:
        if arr.dtype == np.float32:
            ctype = 5126
        elif arr.dtype == np.uint16:
            ctype = 5123
        elif arr.dtype == np.uint32:
            ctype = 5125
        else:
            raise TypeError(arr.dtype)
        arr = np.ascontiguousarray(arr)
        view = self._view(arr.tobytes())
        acc = {"bufferView": view, "componentType": ctype, "count": int(arr.shape[0]), "type": kind}
        if minmax:
            acc["min"] = [float(v) for v in arr.min(axis=0)]
            acc["max"] = [float(v) for v in arr.max(axis=0)]
        self.accessors.append(acc)
        return len(self.accessors) - 1

    def primitive(self, pos, nrm, idx, material, uv=None, tan=None) -> dict:
        attrs = {"POSITION": self.accessor(pos.astype(F32), "VEC3", True),
                 "NORMAL": self.accessor(nrm.astype(F32), "VEC3")}
        if tan is not None:
            attrs["TANGENT"] = self.accessor(tan.astype(F32), "VEC4")
        if uv is not None:
            attrs["TEXCOORD_0"] = self.accessor(uv.astype(F32), "VEC2")
        idx = np.asarray(idx)
        itype = np.uint16 if pos.shape[0] <= 65535 else np.uint32
        prim = {"attributes": attrs, "indices": self.accessor(idx.astype(itype).reshape(-1), "SCALAR")}
        if material is not None:
            prim["material"] = material
        return prim

    def mesh(self, name: str, prims) -> int:
        self.meshes.append({"name": name, "primitives": list(prims)})
        return len(self.meshes) - 1

    def write(self, directory: str, name: str) -> str:
        os.makedirs(directory, exist_ok=True)
        bin_name = name + ".bin"
        with open(os.path.join(directory, bin_name), "wb") as f:
            f.write(bytes(self.bin))
        doc = {
            "asset": {"generator": "raytracing-hw_amd scenes.py", "version": "2.0"},
            "scene": 0,
            "scenes": [{"name": "Scene", "nodes": list(range(len(self.nodes)))}],
            "nodes": self.nodes,
            "cameras": self.cameras,
            "materials": self.materials,
            "meshes": self.meshes,
            "accessors": self.accessors,
            "bufferViews": self.buffer_views,
            "buffers": [{"byteLength": len(self.bin), "uri": bin_name}],
        }
        if self.extensions_used:
            doc["extensionsUsed"] = sorted(self.extensions_used)
        if self.images:
            doc["images"] = self.images
            doc["textures"] = self.textures
            doc["samplers"] = [{"magFilter": 9729, "minFilter": 9987}]
        path = os.path.join(directory, name + ".gltf")
        with open(path, "w") as f:
            json.dump(doc, f, indent=1)
        return path


def write_ppm(path: str, rgb: np.ndarray) -> None:
    h, w, _ = rgb.shape
    with open(path, "wb") as f:
        f.write(b"P6\n%d %d\n255\n" % (w, h))
        f.write(np.ascontiguousarray(rgb, dtype=np.uint8).tobytes())


# --------------------------------------------------------------------------------------
# mesh primitives
# --------------------------------------------------------------------------------------


def plane_mesh():
    """Blender-style unit plane (examples/*.gltf accessor min/max [-1,0,-1]..[1,0,1])."""
    pos = np.array([[-1, 0, 1], [1, 0, 1], [-1, 0, -1], [1, 0, -1]], F32)
    nrm = np.tile(np.array([[0, 1, 0]], F32), (4, 1))
    uv = np.array([[0, 1], [1, 1], [0, 0], [1, 0]], F32)
    tan = np.tile(np.array([[1, 0, 0, 1]], F32), (4, 1))
    idx = np.array([0, 1, 3, 0, 3, 2], np.uint32)
    return pos, nrm, uv, tan, idx


_FACES = [  # (normal axis, sign, u axis, v axis)
    (0, +1, 2, 1), (0, -1, 2, 1), (1, +1, 0, 2), (1, -1, 0, 2), (2, +1, 0, 1), (2, -1, 0, 1)]


def box_mesh(lo, hi, g: int = 1, uv_scale: float = 1.0):
    """Axis-aligned box spanning [lo, hi], each face tessellated g x g quads (12 g^2 tris)."""
    lo = np.asarray(lo, np.float64)
    hi = np.asarray(hi, np.float64)
    P, N, U, T, I = [], [], [], [], []
    base = 0
    t = np.linspace(0.0, 1.0, g + 1)
    for ax, sgn, ua, va in _FACES:
        a, b = np.meshgrid(t, t, indexing="xy")
        p = np.zeros((g + 1, g + 1, 3))
        p[..., ax] = hi[ax] if sgn > 0 else lo[ax]
        p[..., ua] = lo[ua] + a * (hi[ua] - lo[ua])
        p[..., va] = lo[va] + b * (hi[va] - lo[va])
        n = np.zeros(3)
        n[ax] = sgn
        tg = np.zeros(4)
        tg[ua] = 1.0
        tg[3] = 1.0
        uvs = np.stack([p[..., ua] * uv_scale, p[..., va] * uv_scale], -1)
        P.append(p.reshape(-1, 3))
        N.append(np.tile(n, ((g + 1) ** 2, 1)))
        T.append(np.tile(tg, ((g + 1) ** 2, 1)))
        U.append(uvs.reshape(-1, 2))
        for j in range(g):
            for i in range(g):
                v00 = base + j * (g + 1) + i
                v10, v01, v11 = v00 + 1, v00 + g + 1, v00 + g + 2
                if sgn > 0:
                    I += [v00, v10, v11, v00, v11, v01]
                else:
                    I += [v00, v11, v10, v00, v01, v11]
        base += (g + 1) ** 2
    return (np.concatenate(P).astype(F32), np.concatenate(N).astype(F32), np.concatenate(U).astype(F32),
            np.concatenate(T).astype(F32), np.array(I, np.uint32))


def grid_mesh(lo, hi, nx: int, nz: int, y: float, uv_scale: float = 1.0, extra_tri: bool = False):
    """Horizontal grid at height y over [lo.x,hi.x]x[lo.z,hi.z]: 2*nx*nz (+1) triangles."""
    xs = np.linspace(lo[0], hi[0], nx + 1)
    zs = np.linspace(lo[2], hi[2], nz + 1)
    X, Z = np.meshgrid(xs, zs, indexing="xy")
    pos = np.stack([X, np.full_like(X, y), Z], -1).reshape(-1, 3)
    nrm = np.tile([0.0, 1.0, 0.0], (pos.shape[0], 1))
    tan = np.tile([1.0, 0.0, 0.0, 1.0], (pos.shape[0], 1))
    uv = np.stack([pos[:, 0] * uv_scale, pos[:, 2] * uv_scale], -1)
    I = []
    for j in range(nz):
        for i in range(nx):
            v00 = j * (nx + 1) + i
            v10, v01, v11 = v00 + 1, v00 + nx + 1, v00 + nx + 2
            I += [v00, v01, v11, v00, v11, v10]
    if extra_tri:
        I += [0, nx + 1, 1]
    return pos.astype(F32), nrm.astype(F32), uv.astype(F32), tan.astype(F32), np.array(I, np.uint32)


def cylinder_mesh(center, radius, y0, y1, nseg: int, nring: int, uv_scale: float = 1.0):
    """Open vertical cylinder (column shaft): 2*nseg*nring triangles, smooth normals."""
    ang = np.linspace(0.0, 2 * math.pi, nseg + 1)
    hs = np.linspace(y0, y1, nring + 1)
    A, H = np.meshgrid(ang, hs, indexing="xy")
    cx, cz = center
    pos = np.stack([cx + radius * np.cos(A), H, cz + radius * np.sin(A)], -1).reshape(-1, 3)
    nrm = np.stack([np.cos(A), np.zeros_like(A), np.sin(A)], -1).reshape(-1, 3)
    tan = np.stack([-np.sin(A), np.zeros_like(A), np.cos(A), np.ones_like(A)], -1).reshape(-1, 4)
    uv = np.stack([A / (2 * math.pi) * 4.0, H * uv_scale], -1).reshape(-1, 2)
    I = []
    for j in range(nring):
        for i in range(nseg):
            v00 = j * (nseg + 1) + i
            v10, v01, v11 = v00 + 1, v00 + nseg + 1, v00 + nseg + 2
            I += [v00, v01, v11, v00, v11, v10]
    return pos.astype(F32), nrm.astype(F32), uv.astype(F32), tan.astype(F32), np.array(I, np.uint32)


def uv_sphere(center, radii, nlon: int, nlat: int, displace=None):
    """UV sphere / ellipsoid with 2*nlon*(nlat-1) triangles (pole fans + quad bands)."""
    P, N = [], []
    for j in range(nlat + 1):
        th = math.pi * j / nlat
        for i in range(nlon + 1):
            ph = 2 * math.pi * i / nlon
            d = np.array([math.sin(th) * math.cos(ph), math.cos(th), math.sin(th) * math.sin(ph)])
            r = 1.0 if displace is None else displace(th, ph)
            P.append(np.asarray(center) + r * np.asarray(radii) * d)
            N.append(d)
    I = []
    for j in range(nlat):
        for i in range(nlon):
            v00 = j * (nlon + 1) + i
            v10, v01, v11 = v00 + 1, v00 + nlon + 1, v00 + nlon + 2
            if j != 0:
                I += [v00, v10, v11]
            if j != nlat - 1:
                I += [v00, v11, v01]
    pos = np.array(P, F32)
    nrm = np.array(N, F32)
    return pos, nrm, np.array(I, np.uint32)


def torus_mesh(R: float, r: float, nmaj: int, nmin: int):
    P, N, UV = [], [], []
    for j in range(nmaj + 1):
        a = 2 * math.pi * j / nmaj
        for i in range(nmin + 1):
            b = 2 * math.pi * i / nmin
            n = np.array([math.cos(a) * math.cos(b), math.sin(b), math.sin(a) * math.cos(b)])
            c = np.array([R * math.cos(a), 0.0, R * math.sin(a)])
            P.append(c + r * n)
            N.append(n)
            UV.append([j / nmaj, i / nmin])
    I = []
    for j in range(nmaj):
        for i in range(nmin):
            v00 = j * (nmin + 1) + i
            v10, v01, v11 = v00 + 1, v00 + nmin + 1, v00 + nmin + 2
            I += [v00, v10, v11, v00, v11, v01]
    return np.array(P, F32), np.array(N, F32), np.array(UV, F32), np.array(I, np.uint32)


# --------------------------------------------------------------------------------------
# scene parameters taken (as numbers) from the reference's example JSON
# --------------------------------------------------------------------------------------

_EMISSIVE = "KHR_materials_emissive_strength"

# examples/practice7_1.gltf: nodes / materials / camera
CORNELL_NODES = [
    {"camera": 0, "name": "Camera", "translation": [0, 0, 6]},
    {"mesh": 0, "name": "Plane", "scale": [2, 2, 2], "translation": [0, -2, 0]},
    {"mesh": 1, "name": "Plane.001", "scale": [2, 2, 2], "translation": [0, 2, 0]},
    {"mesh": 2, "name": "Plane.002", "rotation": [0.7071068286895752, 0, 0, 0.7071068286895752],
     "scale": [2, 2, 2], "translation": [0, 0, -2]},
    {"mesh": 3, "name": "Plane.003", "rotation": [0.5, 0.5, -0.5, 0.5], "scale": [2, 2, 2], "translation": [2, 0, 0]},
    {"mesh": 4, "name": "Plane.004", "rotation": [0.5, 0.5, -0.5, 0.5], "scale": [2, 2, 2], "translation": [-2, 0, 0]},
    {"mesh": 5, "name": "Plane.005", "translation": [0, 1.9805891513824463, 0]},
    {"mesh": 6, "name": "Cube", "rotation": [0, 0.2583293914794922, 0, 0.9660568833351135],
     "scale": [0.5, 1, 0.5], "translation": [-0.7352063655853271, -1, -0.6174172163009644]},
    {"mesh": 7, "name": "Cube.001", "rotation": [0, -0.17631350457668304, 0, 0.9843340516090393],
     "scale": [0.5, 0.5, 0.5], "translation": [0.9308327436447144, -1.5, 0]},
]
CORNELL_MATERIALS = [
    {"doubleSided": True, "name": "Wall", "pbrMetallicRoughness": {
        "baseColorFactor": [0.800000011920929, 0.800000011920929, 0.800000011920929, 1], "metallicFactor": 0}},
    {"doubleSided": True, "name": "Blue wall", "pbrMetallicRoughness": {
        "baseColorFactor": [0.20000000298023224, 0.20000000298023224, 0.800000011920929, 1], "roughnessFactor": 0}},
    {"doubleSided": True, "name": "Red wall", "pbrMetallicRoughness": {
        "baseColorFactor": [0.800000011920929, 0.20000000298023224, 0.20000000298023224, 1], "roughnessFactor": 0}},
    {"doubleSided": True, "emissiveFactor": [1, 1, 1], "extensions": {_EMISSIVE: {"emissiveStrength": 5}},
     "name": "Light", "pbrMetallicRoughness": {"baseColorFactor": [0, 0, 0, 1], "metallicFactor": 0, "roughnessFactor": 0}},
    {"doubleSided": True, "name": "Cube", "pbrMetallicRoughness": {
        "baseColorFactor": [0.800000011920929, 0.800000011920929, 0.800000011920929, 1], "metallicFactor": 0}},
]
CORNELL_CAMERA = {"name": "Camera", "type": "perspective", "perspective": {
    "aspectRatio": 1, "yfov": 0.9272952079772949, "zfar": 100, "znear": 0.10000000149011612}}
# (mesh index -> material) and the two cube accessor extents (accessors 19 and 23)
CORNELL_PLANE_MATERIALS = [0, 0, 0, 1, 2, 3]
CORNELL_CUBES = [([-1, -1, -1], [1, 0.5, 1]), ([-1, -1, -1], [1, 1, 1])]


def _cornell_base(b: GltfBuilder):
    b.extensions_used.add(_EMISSIVE)
    b.nodes = [dict(n) for n in CORNELL_NODES]
    b.materials = [dict(m) for m in CORNELL_MATERIALS]
    b.cameras = [CORNELL_CAMERA]
    pos, nrm, uv, _, idx = plane_mesh()
    for k, mat in enumerate(CORNELL_PLANE_MATERIALS):
        b.mesh(f"Plane.{k:03d}", [b.primitive(pos, nrm, idx, mat, uv=uv)])
    for k, (lo, hi) in enumerate(CORNELL_CUBES):
        p, n, u, _, i = box_mesh(lo, hi, 1)
        b.mesh(f"Cube.{k + 2:03d}", [b.primitive(p, n, i, 4, uv=u)])


def make_cornell(directory: str) -> str:
    b = GltfBuilder()
    _cornell_base(b)
    return b.write(directory, "cornell")


def make_cornell_blob(directory: str, nlon: int = 100, nlat: int = 51) -> str:
    """Cornell box + displaced sphere (2*nlon*(nlat-1) = 10,000 tris by default)."""
    b = GltfBuilder()
    _cornell_base(b)

    def disp(th, ph):
        return 1.0 + 0.18 * math.sin(5 * th) * math.cos(3 * ph) + 0.07 * math.sin(11 * ph + 2 * th)

    pos, nrm, idx = uv_sphere([0.0, 0.0, 0.0], [1.0, 1.0, 1.0], nlon, nlat, disp)
    mat = len(b.materials)
    b.materials.append({"doubleSided": True, "name": "Blob", "pbrMetallicRoughness": {
        "baseColorFactor": [0.8, 0.6, 0.2, 1], "metallicFactor": 0.5, "roughnessFactor": 0.4}})
    m = b.mesh("blob", [b.primitive(pos, nrm, idx, mat)])
    # the reference's dragon node (practice7_3.gltf) places its mesh at these TRS values
    b.nodes.append({"mesh": m, "name": "blob", "rotation": [0, 0.2, 0, 0.9797958971132712],
                    "scale": [0.8, 0.8, 0.8], "translation": [0.1, -1.1, 0.3]})
    return b.write(directory, "cornell_blob")


# examples/practice6_1.gltf
P61_NODES = [
    {"camera": 0, "name": "Camera", "rotation": [-0.20997299253940582, 0.3857799470424652, 0.09062844514846802, 0.8937962055206299],
     "translation": [7.358891487121582, 4.958309173583984, 6.925790786743164]},
    {"mesh": 0, "name": "Plane", "scale": [3, 3, 3]},
    {"mesh": 1, "name": "Torus", "translation": [0, 0.2639119327068329, 0]},
    {"mesh": 2, "name": "Cube", "rotation": [0, -0.1469700187444687, 0, 0.9891409277915955],
     "scale": [0.7720770239830017, 0.37140536308288574, 0.37140533328056335],
     "translation": [1.5750142335891724, 0.317305326461792, -1.5621356964111328]},
    {"mesh": 3, "name": "Suzanne", "rotation": [0.09827060997486115, 0.48264047503471375, 0.029198922216892242, 0.8697980046272278],
     "scale": [0.6423652172088623, 0.6423652172088623, 0.6423652172088623],
     "translation": [-1.8808989524841309, 0.871877908706665, -1.0177081823349]},
]
P61_MATERIALS = [
    {"doubleSided": True, "name": "Material.001", "pbrMetallicRoughness": {
        "baseColorFactor": [0.800000011920929, 0.800000011920929, 0.800000011920929, 1], "metallicFactor": 0, "roughnessFactor": 0}},
    {"doubleSided": True, "emissiveFactor": [1, 1, 1], "extensions": {_EMISSIVE: {"emissiveStrength": 10}},
     "name": "Material.002", "pbrMetallicRoughness": {"baseColorFactor": [0, 0, 0, 1], "metallicFactor": 0, "roughnessFactor": 0.5}},
    {"doubleSided": True, "name": "Material.003", "pbrMetallicRoughness": {
        "baseColorFactor": [0.08583559095859528, 0.16039040684700012, 0.8000000715255737, 1], "metallicFactor": 0, "roughnessFactor": 0.5}},
    {"doubleSided": True, "name": "Material.006", "pbrMetallicRoughness": {
        "baseColorFactor": [0.8000000715255737, 0.12973719835281372, 0.044038381427526474, 1], "roughnessFactor": 0}},
]
P61_CAMERA = {"name": "Camera", "type": "perspective", "perspective": {
    "aspectRatio": 1.3333333333333333, "yfov": 0.5274237051253257, "zfar": 100, "znear": 0.10000000149011612}}
SUZANNE_AABB = ([-1.3281859159469604, -0.971822202205658, -0.7782661318778992],
                [1.3281859159469604, 0.9392362236976624, 0.8224415183067322])


def make_practice6_1(directory: str) -> str:
    b = GltfBuilder()
    b.extensions_used.add(_EMISSIVE)
    b.nodes = [dict(n) for n in P61_NODES]
    b.materials = [dict(m) for m in P61_MATERIALS]
    b.cameras = [P61_CAMERA]
    pos, nrm, uv, _, idx = plane_mesh()
    b.mesh("Plane", [b.primitive(pos, nrm, idx, 0, uv=uv)])
    p, n, u, i = torus_mesh(1.0, 0.0625, 48, 12)            # 1,152 tris, bounds +-1.0625
    b.mesh("Torus", [b.primitive(p, n, i, 1, uv=u)])
    p, n, u, _, i = box_mesh([-1, -1, -1], [1, 1, 1], 1)     # 12 tris
    b.mesh("Cube.001", [b.primitive(p, n, i, 2, uv=u)])
    lo, hi = np.array(SUZANNE_AABB[0]), np.array(SUZANNE_AABB[1])
    p, n, i = uv_sphere((lo + hi) / 2, (hi - lo) / 2, 96, 83)  # 15,744 tris
    b.mesh("Suzanne", [b.primitive(p, n, i, 3)])
    return b.write(directory, "practice6_1")


# examples/sponza/sponza.gltf: (material, reference vertex count, triangle budget, accessor min, max)
SPONZA_PRIMS = [
    (0, 24162, 31436, [-680.2642211914062, -28.04960060119629, -341.1361999511719], [551.2263793945312, 225.1020965576172, 266.4422912597656]),
    (1, 3932, 3472, [-992.9603881835938, 42.31909942626953, -261.83648681640625], [861.8858032226562, 73.12359619140625, 187.85159301757812]),
    (2, 9848, 17688, [-990.7388916015625, -4.030700206756592, -251.64309692382812], [859.2954711914062, 56.199501037597656, 179.31080627441406]),
    (3, 2259, 4086, [-1428.27490234375, 40.818599700927734, -163.38650512695312], [1299.8668212890625, 758.5531005859375, 88.62689971923828]),
    (4, 1855, 796, [-1866.98291015625, -126.44249725341797, -1139.030517578125], [1746.69287109375, 1347.19580078125, 1039.711181640625]),
    (5, 16361, 10168, [-1052.875732421875, 211.39549255371094, -318.1059875488281], [921.9354858398438, 1275.01123046875, 245.81419372558594]),
    (6, 6037, 5876, [-1429.452392578125, 215.80360412597656, -645.1483154296875], [1302.20166015625, 1263.927978515625, 574.9027099609375]),
    (7, 3844, 2816, [-1057.22021484375, -2.460700035095215, -316.86920166015625], [925.6038208007812, 220.99710083007812, 246.61489868164062]),
    (8, 40, 21, [-1432.224365234375, -2.506200075149536, -645.4310302734375], [1302.220947265625, 415.5303039550781, 574.1851806640625]),
    (9, 16735, 7088, [-1430.30517578125, 182.6522979736328, -646.9678955078125], [1303.27197265625, 695.3228149414062, 575.7255249023438]),
    (10, 1823, 880, [-509.68328857421875, -2.2155001163482666, -651.5385131835938], [1315.5244140625, 716.8505859375, 605.0136108398438]),
    (11, 25540, 23208, [-1037.651611328125, 506.6332092285156, -309.70550537109375], [907.4069213867188, 699.61181640625, 234.77340698242188]),
    (12, 46, 18, [-119.40730285644531, 256.7309875488281, 568.6583862304688], [-8.262900352478027, 348.1973876953125, 575.5051879882812]),
    (13, 12436, 16496, [-958.6978149414062, 274.9595947265625, -289.70361328125], [830.2938842773438, 886.1389770507812, 209.11500549316406]),
    (14, 12906, 16512, [-783.794189453125, 339.4429931640625, -324.5262145996094], [651.9561767578125, 520.5938720703125, 252.28579711914062]),
    (15, 12929, 16512, [-786.898681640625, 339.4429931640625, -324.5262145996094], [648.8516845703125, 520.5938720703125, 252.28570556640625]),
    (16, 8615, 11008, [-418.2926025390625, 339.4429931640625, -324.5262145996094], [283.3501892089844, 520.5938720703125, 252.2855987548828]),
    (17, 7739, 14336, [-577.6201782226562, -0.30889999866485596, -295.25439453125], [820.1740112304688, 283.6809997558594, 213.4824981689453]),
    (18, 10248, 18944, [-946.2379150390625, -0.30889999866485596, -295.25439453125], [820.1740112304688, 283.6809997558594, 213.4824981689453]),
    (19, 7739, 14336, [-946.2379150390625, -0.30889999866485596, -289.25689697265625], [448.0338134765625, 283.6809997558594, 213.4824981689453]),
    (20, 92, 32, [-644.93310546875, 133.72129821777344, -221.48719787597656], [513.3607788085938, 214.3549041748047, 145.12840270996094]),
    (21, 11828, 19828, [-654.1837768554688, 98.67289733886719, -246.83450317382812], [522.611572265625, 216.9512939453125, 170.47579956054688]),
    (22, 5390, 9184, [-1276.67333984375, -0.6934000253677368, -523.4995727539062], [1194.1705322265625, 133.0167999267578, 478.2618103027344]),
    (23, 1732, 3042, [-1427.434326171875, 79.90480041503906, -114.69149780273438], [1299.0263671875, 264.7611999511719, 42.85340118408203]),
    (24, 12440, 14484, [-1920.9459228515625, 1280.513427734375, -1182.80712890625], [1799.9080810546875, 1429.4332275390625, 1105.426025390625]),
]
# textures[i].source of sponza.gltf (73 textures over 69 images)
SPONZA_TEXTURE_SOURCES = [0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16, 17, 18, 19, 20, 21, 22, 23, 24, 25,
                          26, 27, 28, 29, 30, 31, 32, 33, 34, 35, 36, 37, 38, 39, 40, 41, 42, 43, 44, 42, 45, 46, 42, 47,
                          48, 49, 50, 51, 49, 52, 53, 49, 54, 55, 56, 57, 58, 59, 60, 61, 62, 63, 64, 65, 66, 67, 68]
SPONZA_NODES = [
    {"mesh": 0, "name": "Mesh_0", "scale": [0.00800000037997961, 0.00800000037997961, 0.00800000037997961]},
    {"camera": 0, "name": "Camera", "rotation": [-0.013672934845089912, 0.789801299571991, 0.007879254408180714, 0.6131597757339478],
     "translation": [9.900933265686035, 0.9098806381225586, -1.275167465209961]},
    {"mesh": 1, "name": "Plane", "scale": [14.854633331298828, 5.98621129989624, 9.352560043334961],
     "translation": [-0.3724990487098694, 15.377957344055176, 0]},
]
SPONZA_CAMERA = {"name": "Camera.001", "type": "perspective", "perspective": {
    "aspectRatio": 1.7777777777777777, "yfov": 0.769618570804596, "zfar": 100, "znear": 0.10000000149011612}}
SPONZA_BASE = 0.5879999995231628


def _sponza_materials():
    """sponza.gltf materials: 0..11 use textures 3m..3m+2, 12 base colour only, 13..24 use 3m-2..3m."""
    mats = []
    for m in range(25):
        pbr = {"baseColorFactor": [SPONZA_BASE] * 3 + [1]}
        if m == 12:   # Material_2: base colour texture only, metallicFactor 0
            pbr.update({"baseColorTexture": {"index": 36}, "metallicFactor": 0})
            mats.append({"name": "Material_2", "pbrMetallicRoughness": pbr})
            continue
        base = 3 * m if m < 12 else 3 * m - 2
        pbr.update({"baseColorTexture": {"index": base + 1}, "metallicRoughnessTexture": {"index": base + 2}})
        mats.append({"name": f"Material_{m}", "normalTexture": {"index": base}, "pbrMetallicRoughness": pbr})
    mats.append({"doubleSided": True, "emissiveFactor": [1, 1, 1], "extensions": {_EMISSIVE: {"emissiveStrength": 100.0}},
                 "name": "Material.001", "pbrMetallicRoughness": {"baseColorFactor": [0, 0, 0, 1],
                                                                  "metallicFactor": 0, "roughnessFactor": 0.5}})
    return mats


def _texture_roles(mats):
    roles = {}
    for m in mats:
        pbr = m.get("pbrMetallicRoughness", {})
        for key, role in (("normalTexture", "normal"),):
            if key in m:
                roles.setdefault(SPONZA_TEXTURE_SOURCES[m[key]["index"]], role)
        if "baseColorTexture" in pbr:
            roles.setdefault(SPONZA_TEXTURE_SOURCES[pbr["baseColorTexture"]["index"]], "base")
        if "metallicRoughnessTexture" in pbr:
            roles.setdefault(SPONZA_TEXTURE_SOURCES[pbr["metallicRoughnessTexture"]["index"]], "mr")
    return roles


def _procedural_texture(img: int, role: str, size: int) -> np.ndarray:
    rng = np.random.default_rng(20261015 + img)
    y, x = np.mgrid[0:size, 0:size].astype(np.float32) / np.float32(size)
    f1, f2 = rng.uniform(2.0, 9.0, 2)
    p1, p2 = rng.uniform(0.0, 6.283, 2)
    wave = 0.5 + 0.25 * np.sin(2 * np.pi * f1 * x + p1) * np.cos(2 * np.pi * f2 * y + p2)
    noise = rng.random((size, size), dtype=np.float32)
    if role == "normal":
        nx = 128 + 50 * np.sin(2 * np.pi * f1 * x + p1) + 20 * (noise - 0.5)
        ny = 128 + 50 * np.cos(2 * np.pi * f2 * y + p2) + 20 * (rng.random((size, size), dtype=np.float32) - 0.5)
        nz = np.full_like(nx, 235.0)
        rgb = np.stack([nx, ny, nz], -1)
    elif role == "mr":
        rough = 40 + 215 * (0.5 * wave + 0.5 * noise)
        metal = 255 * noise ** 4
        rgb = np.stack([np.zeros_like(rough), rough, metal], -1)
    else:
        tint = rng.uniform(0.5, 1.0, 3)
        lum = 255 * (0.55 * wave + 0.45 * noise)
        rgb = np.stack([lum * tint[0], lum * tint[1], lum * tint[2]], -1)
    return np.clip(np.rint(rgb), 0, 255).astype(np.uint8)


class _PrimAccum:
    def __init__(self):
        self.P, self.N, self.U, self.T, self.I = [], [], [], [], []
        self.nv = 0

    def add(self, pos, nrm, uv, tan, idx):
        self.P.append(pos)
        self.N.append(nrm)
        self.U.append(uv)
        self.T.append(tan)
        self.I.append(idx.astype(np.int64) + self.nv)
        self.nv += pos.shape[0]

    def ntris(self):
        return sum(i.shape[0] for i in self.I) // 3

    def arrays(self):
        return (np.concatenate(self.P), np.concatenate(self.N), np.concatenate(self.U),
                np.concatenate(self.T), np.concatenate(self.I))


def _fill_remainder(acc: _PrimAccum, lo, hi, rem: int, uv_scale: float):
    """Spend the leftover triangle budget on a thin horizontal grid strip along z=lo edge."""
    if rem <= 0:
        return
    quads = rem // 2
    y = lo[1] + 0.02 * (hi[1] - lo[1])
    if quads == 0:
        p = np.array([[lo[0], y, lo[2]], [lo[0], y, lo[2] + 1.0], [lo[0] + 1.0, y, lo[2]]], F32)
        n = np.tile(np.array([[0, 1, 0]], F32), (3, 1))
        u = (p[:, [0, 2]] * uv_scale).astype(F32)
        t = np.tile(np.array([[1, 0, 0, 1]], F32), (3, 1))
        acc.add(p, n, u, t, np.array([0, 1, 2]))
        return
    zl = lo[2] + 0.05 * (hi[2] - lo[2])
    acc.add(*grid_mesh([lo[0], y, lo[2]], [hi[0], y, zl], quads, 1, y, uv_scale, extra_tri=bool(rem % 2)))


def _sponza_primitive(mat: int, budget: int, lo, hi, rng) -> tuple:
    lo = np.asarray(lo, np.float64)
    hi = np.asarray(hi, np.float64)
    ext = hi - lo
    acc = _PrimAccum()
    uvs = 1.0 / 150.0
    if budget < 12:
        _fill_remainder(acc, lo, hi, budget, uvs)
        return acc.arrays()
    if mat == 22:                                   # floor: one grid over the accessor x-z extent
        nx = max(1, int(math.sqrt(budget / 2 * ext[0] / ext[2])))
        nz = max(1, budget // (2 * nx))
        acc.add(*grid_mesh(lo, hi, nx, nz, lo[1], uvs))
    elif mat in (17, 18, 19):                       # colonnades: two rows of column shafts
        ncol = 8 if mat != 18 else 10
        nseg = 24 if budget >= 4 * 24 * ncol else 6
        ncol = max(1, min(ncol, budget // (4 * nseg)))
        per = budget // (2 * ncol)
        nring = max(1, per // (2 * nseg))
        r = 0.045 * ext[2]
        for row, z in enumerate((lo[2] + 1.2 * r, hi[2] - 1.2 * r)):
            for k in range(ncol):
                x = lo[0] + (k + 0.5) * ext[0] / ncol + rng.uniform(-0.1, 0.1) * ext[0] / ncol
                acc.add(*cylinder_mesh((x, z), r * rng.uniform(0.8, 1.0), lo[1], hi[1], nseg, nring, uvs))
    else:                                           # ring of tessellated blocks around the perimeter
        nblk = int(np.clip(budget // 700, 1, 48))
        g = max(1, int(math.sqrt(budget / (12.0 * nblk))))
        nblk = max(1, budget // (12 * g * g))
        thick = 0.06 * min(ext[0], ext[2]) + 1e-3
        perim = 2 * (ext[0] + ext[2])
        for k in range(nblk):
            s = (k + rng.uniform(0.2, 0.8)) / nblk * perim
            if s < ext[0]:
                cx, cz = lo[0] + s, lo[2] + thick
            elif s < ext[0] + ext[2]:
                cx, cz = hi[0] - thick, lo[2] + (s - ext[0])
            elif s < 2 * ext[0] + ext[2]:
                cx, cz = hi[0] - (s - ext[0] - ext[2]), hi[2] - thick
            else:
                cx, cz = lo[0] + thick, hi[2] - (s - 2 * ext[0] - ext[2])
            half = np.array([rng.uniform(0.4, 1.0) * min(perim / nblk / 2, 4 * thick), 0.0, thick])
            y0 = lo[1] + rng.uniform(0.0, 0.3) * ext[1]
            y1 = hi[1] - rng.uniform(0.0, 0.3) * ext[1]
            if mat == 24:        # roof ring: thin slabs at the top of the accessor range
                y0, y1 = lo[1], lo[1] + 0.3 * ext[1]
            bl = [np.clip(cx - half[0], lo[0], hi[0]), y0, np.clip(cz - half[2], lo[2], hi[2])]
            bh = [np.clip(cx + half[0], lo[0], hi[0]), max(y1, y0 + 1.0), np.clip(cz + half[2], lo[2], hi[2])]
            acc.add(*box_mesh(bl, bh, g, uvs))
    _fill_remainder(acc, lo, hi, budget - acc.ntris(), uvs)
    assert acc.ntris() == budget, (mat, acc.ntris(), budget)
    return acc.arrays()


DRAGON_FIXTURE = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests", "golden",
                              "dragon10k_tris.npy")


def dragon_100k() -> np.ndarray:
    """C5's dragon proxy: the 9,992 triangles of the reference's
    practice5_dragon_10k.txt (tests/golden/dragon10k_tris.npy, tools/make_dragon_fixture.py),
    1->4 midpoint subdivision, then the first 20,011 of those again: 100,001 triangles,
    (n, 3, 3) float32, in the fixture's coordinates."""
    def split(t):
        a, b, c = t[:, 0], t[:, 1], t[:, 2]
        ab, bc, ca = (a + b) * 0.5, (b + c) * 0.5, (c + a) * 0.5
        return np.stack([np.stack([a, ab, ca], 1), np.stack([ab, b, bc], 1), np.stack([ca, bc, c], 1),
                         np.stack([ab, bc, ca], 1)], 1).reshape(-1, 3, 3)
    t = split(np.load(DRAGON_FIXTURE).astype(np.float64))
    k = 20011
    return np.concatenate([split(t[:k]), t[k:]]).astype(np.float32)


def _dragon_in_sponza(b: "GltfBuilder") -> None:
    """The dragon on the sponza proxy's floor, 5 m in front of its camera (scale 0.25,
    flat normals, one untextured metallic material)."""
    t = dragon_100k().astype(np.float64)
    lo = t.reshape(-1, 3).min(0)
    t = (t - np.array([0.0, lo[1], 0.0])) * 0.25 + np.array([5.0, 0.0, -0.6])
    n = np.cross(t[:, 1] - t[:, 0], t[:, 2] - t[:, 0])
    n /= np.maximum(np.linalg.norm(n, axis=1, keepdims=True), 1e-30)
    pos = t.reshape(-1, 3)
    nrm = np.repeat(n, 3, axis=0)
    idx = np.arange(pos.shape[0])
    mat = len(b.materials)
    b.materials.append({"name": "Dragon", "pbrMetallicRoughness": {
        "baseColorFactor": [0.72, 0.52, 0.3, 1], "metallicFactor": 0.6, "roughnessFactor": 0.35}})
    mesh = b.mesh("Dragon", [b.primitive(pos, nrm, idx, mat)])
    b.nodes.append({"mesh": mesh, "name": "Dragon"})


def make_sponza(directory: str, tri_scale: float = 1.0, tex_size: int = 1024, name: str = "sponza",
                dragon: bool = False) -> str:
    b = GltfBuilder()
    b.extensions_used.add(_EMISSIVE)
    b.nodes = [dict(n) for n in SPONZA_NODES]
    b.cameras = [SPONZA_CAMERA]
    b.materials = _sponza_materials()
    prims = []
    for mat, _nv, ntri, lo, hi in SPONZA_PRIMS:
        budget = max(2, int(round(ntri * tri_scale))) if tri_scale != 1.0 else ntri
        rng = np.random.default_rng(20261015 + mat)
        pos, nrm, uv, tan, idx = _sponza_primitive(mat, budget, lo, hi, rng)
        prims.append(b.primitive(pos, nrm, idx, mat, uv=uv, tan=tan))
    b.mesh("Mesh_0", prims)
    pos, nrm, uv, tan, idx = plane_mesh()
    b.mesh("Plane", [b.primitive(pos, nrm, idx, 25, uv=uv, tan=tan)])
    roles = _texture_roles(b.materials)
    os.makedirs(directory, exist_ok=True)
    for img in range(69):
        fname = f"{name}_tex{img:02d}.ppm"
        b.images.append({"name": f"tex{img:02d}", "uri": fname})
        path = os.path.join(directory, fname)
        write_ppm(path, _procedural_texture(img, roles.get(img, "base"), tex_size))
    b.textures = [{"sampler": 0, "source": s} for s in SPONZA_TEXTURE_SOURCES]
    if dragon:
        _dragon_in_sponza(b)
    return b.write(directory, name)


SCENES = {
    "cornell": lambda d: make_cornell(d),
    "cornell_blob": lambda d: make_cornell_blob(d),
    "practice6_1": lambda d: make_practice6_1(d),
    "sponza_mini": lambda d: make_sponza(d, tri_scale=1.0 / 32, tex_size=16, name="sponza_mini"),
    "sponza": lambda d: make_sponza(d),
    # BASELINE.json configs[4] (C5): dragon-100k proxy + sponza proxy
    "sponza_dragon": lambda d: make_sponza(d, dragon=True, name="sponza_dragon"),
    "sponza_dragon_mini": lambda d: make_sponza(d, tri_scale=1.0 / 32, tex_size=16, name="sponza_dragon_mini",
                                                dragon=True),
}


def ensure_scene(name: str, directory: str) -> str:
    """Generate scene `name` into `directory` unless it is already there; return the .gltf path."""
    path = os.path.join(directory, name + ".gltf")
    if not os.path.exists(path):
        SCENES[name](directory)
    return path


if __name__ == "__main__":
    import sys
    out = sys.argv[1] if len(sys.argv) > 1 else "/tmp/rt_scenes"
    for n in (sys.argv[2:] or ["cornell", "cornell_blob", "practice6_1", "sponza_mini"]):
        print(SCENES[n](out))
