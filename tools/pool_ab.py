#!/usr/bin/env python3
"""A/B of the lane-resident kernel's two schedules on one GPU: the plain lane-per-path kernel
and the path pool (rt_pool.h, RT_FLAG_POOL), same frame, same bits.

    python tools/pool_ab.py [--spp 256] [--steps 2] [--worlds 1,2] [--libs a.so,b.so]

Prints one JSON line per (library, world, schedule): rank 0's shard time (HIP events around the
render, pre-pass included) and the frame digest, which must not depend on the schedule."""
import argparse
import ctypes
import hashlib
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scene", default="sponza")
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--spp", type=int, default=256)
    ap.add_argument("--steps", type=int, default=2)
    ap.add_argument("--worlds", default="1")
    ap.add_argument("--modes", default="lane,pool")
    ap.add_argument("--libs", default="", help="comma-separated librt_hw_amd.so variants (default: the in-tree one)")
    args = ap.parse_args()
    torch.zeros(1, device="cuda")
    libs = [x for x in args.libs.split(",") if x] or [None]
    scenes = bench.load_scenes_module()
    path = scenes.ensure_scene(args.scene, os.environ.get("RT_SCENE_DIR", "/tmp/rt_scenes"))
    W, H, S = args.width, args.height, args.spp
    for lib in libs:
        if lib:
            os.environ["RT_LIB"] = lib
        for m in [k for k in list(sys.modules) if k.startswith("raytracing_hw_amd")]:
            del sys.modules[m]
        import importlib.util
        pkg = os.path.join(ROOT, "raytracing-hw_amd")
        spec = importlib.util.spec_from_file_location("raytracing_hw_amd", os.path.join(pkg, "__init__.py"),
                                                      submodule_search_locations=[pkg])
        rt = importlib.util.module_from_spec(spec)
        sys.modules["raytracing_hw_amd"] = rt
        spec.loader.exec_module(rt)
        rt._lib_handle = None
        scene = rt.Scene.load(path, W, H, S)
        scene.upload(0)
        stream = torch.cuda.current_stream().cuda_stream
        for world in [int(x) for x in args.worlds.split(",")]:
            rows = len(rt.shard_rows(H, 0, world))
            out = torch.zeros(rows * W * 3, dtype=torch.float32, device="cuda")
            for mode in args.modes.split(","):
                # pool: the path pool wherever it is chosen (runahead off, which would take shards of
                # <= 2 pixels per lane); lane: the default (runahead where it applies); lane_norun
                kw = dict(pool=mode == "pool", runahead=mode == "lane")
                st = scene.render_device(out.data_ptr(), stream, spp=S, rank=0, world=world, stats=True, **kw)
                ms = []
                for _ in range(args.steps):
                    st = scene.render_device(out.data_ptr(), stream, spp=S, rank=0, world=world, stats=True, **kw)
                    ms.append(st["render_ms"])
                torch.cuda.synchronize()
                digest = hashlib.sha1(out.cpu().numpy().tobytes()).hexdigest()[:16]
                print(json.dumps({"lib": lib or "in-tree", "world": world, "mode": mode, "schedule": st["schedule"],
                                  "ms": [round(x, 2) for x in ms], "best_ms": round(min(ms), 2),
                                  "order_ms": round(st["order_ms"], 2), "digest": digest}), flush=True)


if __name__ == "__main__":
    main()
