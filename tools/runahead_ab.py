#!/usr/bin/env python3
"""Speculative sample runahead A/B (RT_FLAG_NO_RUNAHEAD): the 1-GPU frame and every shard of
an N-way split (the slowest shard is the N-GPU frame time), runahead on and off, same build.

    python tools/runahead_ab.py [--world 8] [--spp 256]
"""
import argparse
import json
import os
import sys

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
    ap.add_argument("--worlds", default="8", help="comma-separated N of the N-way splits to time")
    ap.add_argument("--steps", type=int, default=2)
    ap.add_argument("--off", type=int, default=1, help="also time with the runahead off")
    ap.add_argument("--max-ranks", type=int, default=0, help="time only the first ranks of each split (0 = all)")
    ap.add_argument("--full", type=int, default=1, help="also time the whole frame on one GPU")
    ap.add_argument("--row-block", type=int, default=8, help="rows per interleaved block of the split")
    ap.add_argument("--rank-stride", type=int, default=1, help="time every k-th rank only")
    args = ap.parse_args()
    rt = bench.import_pkg()
    path = bench.load_scenes_module().ensure_scene(args.scene, os.environ.get("RT_SCENE_DIR", "/tmp/rt_scenes"))
    W, H, S = args.width, args.height, args.spp
    scene = rt.Scene.load(path, W, H, S)
    scene.upload(0)
    rtdist = __import__("importlib").import_module("raytracing_hw_amd.dist")
    stream = torch.cuda.current_stream().cuda_stream
    res = {"lib": os.environ.get("RT_LIB", "default"), "scene": args.scene, "frame": [W, H, S]}

    def t(world, rank, steps, on):
        out = torch.zeros(rtdist.max_shard_rows(H, world, args.row_block) * W * 3, dtype=torch.float32, device="cuda")
        ms = [scene.render_device(out.data_ptr(), stream, spp=S, rank=rank, world=world, row_block=args.row_block,
                                  stats=True, runahead=on)["render_ms"] for _ in range(steps)]
        return min(ms)

    worlds = [int(x) for x in args.worlds.split(",")]
    if args.full:
        t(1, 0, 1, True)   # warm
    else:
        t(worlds[0], 0, 1, True)
    for on in ([True, False] if args.off else [True]):
        tag = "on" if on else "off"
        if args.full:
            res[f"full_ms_{tag}"] = round(t(1, 0, args.steps, on), 1)
        for world in worlds:
            sh = [t(world, r, 1, on) for r in range(0, min(world, args.max_ranks or world), args.rank_stride)]
            res[f"shard{world}_ms_{tag}"] = [round(x, 1) for x in sh]
            res[f"shard{world}_max_ms_{tag}"] = round(max(sh), 1)
            if args.full:
                res[f"speedup{world}_{tag}"] = round(res[f"full_ms_{tag}"] / max(sh), 3)
        print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
