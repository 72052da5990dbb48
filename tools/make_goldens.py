#!/usr/bin/env python3
"""Generate the committed golden fixtures under tests/golden/ from the REFERENCE ITSELF.

Runs only in the build container (needs /root/reference and oracle/_ref built by
`make -C oracle ref`).  Every expected value below is produced by the reference's own
compiled sources (oracle/ref_harness.cpp linked against /root/reference/src objects);
nothing here is computed by this build's code.

    python tools/make_goldens.py            # all fixtures
Outputs (tests/golden/):
    scenes/<name>/...                 the synthesized input scenes (raytracing-hw_amd/scenes.py)
    <name>_dump.rtd                   reference post-BVH scene arrays (ref_harness dump)
    <name>_sums_<W>x<H>x<S>.rtd       per-pixel float sums, per-pixel RNG reset (ref_harness sums)
    <name>_<W>x<H>x<S>.ppm            the reference's finished 8-bit frame of those sums
    shipped_<name>_<W>x<H>x<S>.ppm    the UNMODIFIED reference binary (oracle/_ref/solution: its
                                      own OpenMP loop, shared normal cache, random_device seed
                                      for pixel 0) -- statistical comparison only
    <name>_rays.rtd                   closest-hit / light-pdf known answers (ref_harness rays)
    cornell_samplers.rtd              SceneDistribution sample/pdf + RNG sequences
    cornell_512x512x64_rowhash.rtd    BASELINE configs[1] full-size frame as per-row hashes
    <scene>_pixels_<W>x<H>x<S>[_w<N>].rtd
                                      BASELINE configs C3-C5 and the headline at full size and
                                      full spp: seeded pixels of the frame (of each rank's
                                      shard for C4, of rank 0's for C5), reference sums +
                                      per-pixel test counts (ref_harness pixels)
    golden_meta.json "configs"        sha256 of the generated scene files (pins the generator)
                                      and of the reference's post-BVH arrays of the large
                                      scenes in this build's layout (pins the loader)

    python tools/make_goldens.py --configs   # only the BASELINE-config fixtures
"""
import hashlib
import importlib.util
import json
import os
import shutil
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLD = os.path.join(ROOT, "tests", "golden")
HARNESS = os.path.join(ROOT, "oracle", "_ref", "ref_harness")
sys.path.insert(0, os.path.join(ROOT, "tests"))
import rtdump  # noqa: E402
import rtref  # noqa: E402,F401  (tests/rtref.py: reference arrays in this build's layout)

spec = importlib.util.spec_from_file_location("rt_scenes", os.path.join(ROOT, "raytracing-hw_amd", "scenes.py"))
scenes = importlib.util.module_from_spec(spec)
spec.loader.exec_module(scenes)

SCENES = ["cornell", "cornell_blob", "practice6_1", "sponza_mini"]
SUMS = {  # scene -> (W, H, spp) list
    "cornell": [(64, 64, 8), (33, 17, 3)],
    "cornell_blob": [(48, 48, 4)],
    "practice6_1": [(256, 256, 4)],          # BASELINE.json configs[0] (C1), full size
    "sponza_mini": [(64, 36, 4)],
}
RAYS = {"cornell": 3000, "cornell_blob": 2000, "practice6_1": 1500, "sponza_mini": 2000}


def harness(*args):
    out = subprocess.run([HARNESS, *map(str, args)], check=True, capture_output=True, text=True).stdout
    return json.loads(out.strip().splitlines()[-1])


def compact_dump(src, dst):
    """Keep only the fields the tests read (drops all-zero tangent / texcoord blocks)."""
    d = rtdump.load(src)
    keep = {}
    for k, v in d.items():
        if k.endswith("_aabb") and k.startswith(("obj_", "light_")):
            continue  # per-primitive boxes are re-derived, not needed
        if (k.endswith("tangent") or k.endswith("texcoord")) and not np.any(v):
            continue
        keep[k] = v
    rtdump.save(dst, keep)


def row_hash(sums):
    """FNV-1a 64 of each row's float32 bit patterns (a checksum of checksums)."""
    h = np.full(sums.shape[0], 1469598103934665603, np.uint64)
    b = np.ascontiguousarray(sums).view(np.uint8).reshape(sums.shape[0], -1)
    with np.errstate(over="ignore"):
        for k in range(b.shape[1]):
            h = (h ^ b[:, k].astype(np.uint64)) * np.uint64(1099511628211)
    return h


def finish_golden(meta):
    """Frame finish (tonemap + 8-bit + PPM) of the reference on synthetic sums."""
    ppm = os.path.join(GOLD, "finish_37x23x16.ppm")
    meta["finish"] = harness("finish", os.path.join(GOLD, "finish_37x23x16.rtd"), ppm, 37, 23, 16)


# BASELINE.json configs at their full size and spp: (name, scene, W, H, spp, world, pixels per shard)
CONFIGS = [
    ("c3", "sponza", 1024, 1024, 256, 1, 1024),
    ("headline", "sponza", 1920, 1080, 256, 1, 1024),
    ("c4", "sponza", 1920, 1080, 1024, 8, 128),     # every rank of the 8-way split
    ("c5", "sponza_dragon", 3840, 2160, 4096, 8, 256),   # rank 0's shard of the 8-way split
]
SCENE_DIR = "/tmp/rt_scenes"


def scene_sha256(scene):
    """sha256 over the generated scene's files (name + bytes, sorted by name)."""
    h = hashlib.sha256()
    files = sorted(f for f in os.listdir(SCENE_DIR) if f == scene + ".gltf" or f.startswith(scene + "_tex")
                   or f == scene + ".bin")
    for f in files:
        h.update(f.encode())
        with open(os.path.join(SCENE_DIR, f), "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()


def layout_sha256(arrays):
    """sha256 per flattened array (this build's rt_scene_view layout)."""
    keys = ["tri", "tri_attr", "tri_tan", "node", "light", "light_node", "mesh_f", "mesh_tex", "mesh_normal_transform"]
    return {k: hashlib.sha256(np.ascontiguousarray(arrays[k]).tobytes()).hexdigest() for k in keys}


def shard_pixels(W, H, world, rank, n, seed, row_block=8):
    rows = np.array([r for r in range(H) if (r // row_block) % world == rank])
    rng = np.random.default_rng(seed)
    pick = rng.choice(len(rows) * W, n, replace=False)
    pick.sort()
    return (rows[pick // W] * W + pick % W).astype(np.int64)


def config_goldens(meta):
    import rtref
    rt = rtref.package()
    meta.setdefault("configs", {})
    for scene in sorted({c[1] for c in CONFIGS}):
        path = scenes.ensure_scene(scene, SCENE_DIR)
        raw = os.path.join("/tmp", f"{scene}_dump_full.rtd")
        harness("dump", path, 64, 64, raw)
        ref = rtref.ref_arrays(rt, scene, 64, 64, 1, dump=rtdump.load(raw), path=path)
        meta["configs"][scene] = {"scene_sha256": scene_sha256(scene), "ref_layout_sha256": layout_sha256(ref)}
    for name, scene, W, H, S, world, n in CONFIGS:
        path = os.path.join(SCENE_DIR, scene + ".gltf")
        ranks = range(world) if name == "c4" else [0]
        idx = np.concatenate([shard_pixels(W, H, world, r, n, 1000 + r) for r in ranks])
        lst = f"/tmp/{name}_idx.i64"
        idx.tofile(lst)
        out = os.path.join(GOLD, f"{name}_{scene}_pixels_{W}x{H}x{S}" + (f"_w{world}" if world > 1 else "") + ".rtd")
        meta["configs"][name] = {"scene": scene, "width": W, "height": H, "spp": S, "world": world,
                                 "file": os.path.basename(out), "pixels": harness("pixels", path, W, H, S, lst, out)}
        print(name, meta["configs"][name]["pixels"], flush=True)


FRAMES = [("c3", "sponza", 1024, 1024, 256), ("headline", "sponza", 1920, 1080, 256),
          ("c4", "sponza", 1920, 1080, 1024)]   # C4 whole frame: about 1.8 h on 8 threads here
C5_RANKS_PIXELS = 64     # pixels per rank for the every-rank C5 golden


def frame_goldens(meta, save, threads=8):
    """Whole BASELINE frames rendered by the reference (ref_harness sums, scene.cpp:31-64):
    per-row FNV-1a hashes of every row's float sums, 8 full rows, the frame's counters and the
    sha1 of the reference's finished 8-bit frame (the body of its PPM, canvas.h:76-89)."""
    meta.setdefault("frames", {})
    for name, scene, W, H, S in FRAMES:
        out = os.path.join(GOLD, f"{name}_{scene}_rowhash_{W}x{H}x{S}.rtd")
        if os.path.exists(out) and name in meta["frames"]:
            continue
        path = scenes.ensure_scene(scene, SCENE_DIR)
        full, ppm = f"/tmp/{name}_{scene}_{W}x{H}x{S}.rtd", f"/tmp/{name}_{scene}_{W}x{H}x{S}.ppm"
        info = harness("sums", path, W, H, S, full, threads, ppm)
        d = rtdump.load(full)
        s = d["sums"]
        rows = np.arange(0, H, H // 8).astype(np.int32)
        body = open(ppm, "rb").read()
        header = b"P6\n%d %d\n255\n" % (W, H)
        assert body.startswith(header)
        u8 = np.frombuffer(body[len(header):], np.uint8).reshape(H, W, 3)
        rtdump.save(out, {"row_fnv1a": row_hash(s), "rows": rows, "row_sums": s[rows], "row_u8": u8[rows],
                          "counters": d["counters"]})
        meta["frames"][name] = {"scene": scene, "width": W, "height": H, "spp": S, "file": os.path.basename(out),
                                "frame_u8_sha1": hashlib.sha1(body[len(header):]).hexdigest(),
                                "ppm_sha1": hashlib.sha1(body).hexdigest(), "sums": info,
                                "scene_sha256": scene_sha256(scene)}
        print(name, meta["frames"][name], flush=True)
        save(meta)
    # C5: seeded pixels of every rank's shard of the 8-way split (rank 0 has its own 256-pixel file)
    name, scene, W, H, S, world, _ = CONFIGS[3]
    out = os.path.join(GOLD, f"{name}_{scene}_pixels_{W}x{H}x{S}_w{world}_ranks1to7.rtd")
    if not (os.path.exists(out) and "c5_ranks" in meta.get("configs", {})):
        path = scenes.ensure_scene(scene, SCENE_DIR)
        idx = np.concatenate([shard_pixels(W, H, world, r, C5_RANKS_PIXELS, 2000 + r) for r in range(1, world)])
        lst = f"/tmp/{name}_ranks_idx.i64"
        idx.tofile(lst)
        meta.setdefault("configs", {})["c5_ranks"] = {
            "scene": scene, "width": W, "height": H, "spp": S, "world": world, "ranks": list(range(1, world)),
            "pixels_per_rank": C5_RANKS_PIXELS, "file": os.path.basename(out),
            "pixels": harness("pixels", path, W, H, S, lst, out, threads)}
        print("c5_ranks", meta["configs"]["c5_ranks"], flush=True)


C5_ROWS_PER_RANK = 8      # full rows per rank for the C5 row golden (64 rows, 245,760 pixels)


def c5_row_goldens(meta, save, threads=6):
    """C5 (dragon + sponza 3840x2160x4096, the 8-way split) as FULL ROWS: 8 seeded rows of every
    rank's shard, every pixel of them rendered by the reference at 4096 spp (ref_harness pixels,
    scene.cpp:31-52).  Kept compact: every row's FNV-1a hash of its float sums, one full row per
    rank, and per-row totals of the reference's test counters (rays, AABB, triangle, light)."""
    name, scene, W, H, S, world, _ = CONFIGS[3]
    out = os.path.join(GOLD, f"{name}_{scene}_rows_{W}x{H}x{S}_w{world}.rtd")
    if os.path.exists(out) and "c5_rows" in meta.get("configs", {}):
        return
    path = scenes.ensure_scene(scene, SCENE_DIR)
    rows = []
    for r in range(world):
        mine = np.array([j for j in range(H) if (j // 8) % world == r])
        pick = np.sort(np.random.default_rng(3000 + r).choice(mine, C5_ROWS_PER_RANK, replace=False))
        rows.extend(int(j) for j in pick)
    rows = np.array(rows, np.int64)
    idx = (rows[:, None] * W + np.arange(W)[None, :]).reshape(-1).astype(np.int64)
    lst = f"/tmp/{name}_rows_idx.i64"
    idx.tofile(lst)
    raw = f"/tmp/{name}_{scene}_rows_{W}x{H}x{S}_full.rtd"
    info = harness("pixels", path, W, H, S, lst, raw, threads)
    d = rtdump.load(raw)
    assert np.array_equal(d["index"], idx)
    sums = d["sums"].reshape(len(rows), W, 3).astype(np.float32)
    pc = d["pixel_counters"].reshape(len(rows), W, 6).astype(np.uint64).sum(axis=1)
    full = np.arange(0, len(rows), C5_ROWS_PER_RANK)          # the first picked row of each rank
    rtdump.save(out, {"rows": rows.astype(np.int32), "row_fnv1a": row_hash(sums), "full_rows": rows[full].astype(np.int32),
                      "full_row_sums": sums[full], "row_counters": pc})
    meta.setdefault("configs", {})["c5_rows"] = {
        "scene": scene, "width": W, "height": H, "spp": S, "world": world, "rows_per_rank": C5_ROWS_PER_RANK,
        "file": os.path.basename(out), "pixels": info}
    print("c5_rows", meta["configs"]["c5_rows"], flush=True)
    save(meta)


SHIPPED = [("cornell", 128, 128, 256), ("sponza_mini", 128, 72, 256)]


def shipped_goldens(meta):
    """Frames of the shipped reference binary itself (not bit-reproducible: see above)."""
    solution = os.path.join(ROOT, "oracle", "_ref", "solution")
    meta.setdefault("shipped", {})
    for name, w, h, s in SHIPPED:
        gltf = os.path.join(GOLD, "scenes", name, name + ".gltf")
        out = os.path.join(GOLD, f"shipped_{name}_{w}x{h}x{s}.ppm")
        r = subprocess.run([solution, gltf, str(w), str(h), str(s), out], check=True, capture_output=True, text=True)
        meta["shipped"][f"{name}_{w}x{h}x{s}"] = {"cmd": f"oracle/_ref/solution {name}.gltf {w} {h} {s}",
                                                   "log": r.stdout.strip().splitlines()[-2:]}


def main():
    if "--shipped" in sys.argv:
        path = os.path.join(GOLD, "golden_meta.json")
        meta = json.load(open(path))
        shipped_goldens(meta)
        with open(path, "w") as f:
            json.dump(meta, f, indent=1, sort_keys=True)
        return
    if "--frames" in sys.argv or "--c5rows" in sys.argv:
        path = os.path.join(GOLD, "golden_meta.json")
        meta = json.load(open(path))
        def save(m):
            with open(path, "w") as f:
                json.dump(m, f, indent=1, sort_keys=True)
        if "--c5rows" in sys.argv:
            c5_row_goldens(meta, save)
        else:
            frame_goldens(meta, save)
        save(meta)
        return
    if "--configs" in sys.argv:
        path = os.path.join(GOLD, "golden_meta.json")
        meta = json.load(open(path))
        config_goldens(meta)
        with open(path, "w") as f:
            json.dump(meta, f, indent=1, sort_keys=True)
        return
    if not os.path.exists(HARNESS):
        sys.exit("build the reference harness first: make -C oracle ref")
    os.makedirs(GOLD, exist_ok=True)
    if "--finish-only" in sys.argv:
        path = os.path.join(GOLD, "golden_meta.json")
        meta = json.load(open(path))
        finish_golden(meta)
        with open(path, "w") as f:
            json.dump(meta, f, indent=1, sort_keys=True)
        return
    meta = {}
    finish_golden(meta)
    for name in SCENES:
        sdir = os.path.join(GOLD, "scenes", name)
        if os.path.isdir(sdir):
            shutil.rmtree(sdir)
        gltf = scenes.SCENES[name](sdir)
        raw = os.path.join("/tmp", f"{name}_dump_full.rtd")
        meta[name] = {"dump": harness("dump", gltf, 64, 64, raw)}
        compact_dump(raw, os.path.join(GOLD, f"{name}_dump.rtd"))
        for (w, h, s) in SUMS[name]:
            out = os.path.join(GOLD, f"{name}_sums_{w}x{h}x{s}.rtd")
            ppm = os.path.join(GOLD, f"{name}_{w}x{h}x{s}.ppm")   # the reference's finished frame
            meta[name][f"sums_{w}x{h}x{s}"] = harness("sums", gltf, w, h, s, out, 8, ppm)
        meta[name]["rays"] = harness("rays", gltf, 64, 64, RAYS[name], os.path.join(GOLD, f"{name}_rays.rtd"))
    cornell = os.path.join(GOLD, "scenes", "cornell", "cornell.gltf")
    meta["cornell"]["samplers"] = harness("samplers", cornell, 64, 64, 2000, os.path.join(GOLD, "cornell_samplers.rtd"))
    # BASELINE.json configs[1] (C2): cornell 512x512x64 -- kept as per-row hashes + 8 full rows
    full = "/tmp/cornell_512x512x64.rtd"
    meta["cornell"]["sums_512x512x64"] = harness("sums", cornell, 512, 512, 64, full, 8)
    s = rtdump.load(full)["sums"]
    rows = np.arange(0, 512, 64)
    rtdump.save(os.path.join(GOLD, "cornell_512x512x64_rowhash.rtd"),
                {"row_fnv1a": row_hash(s), "rows": rows.astype(np.int32), "row_sums": s[rows],
                 "counters": rtdump.load(full)["counters"]})
    config_goldens(meta)
    shipped_goldens(meta)
    with open(os.path.join(GOLD, "golden_meta.json"), "w") as f:
        json.dump(meta, f, indent=1, sort_keys=True)
    print(json.dumps(meta, indent=1)[:2000])


if __name__ == "__main__":
    main()
