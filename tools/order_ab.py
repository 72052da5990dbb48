#!/usr/bin/env python3
"""A/B of pixel-order builds (RT_LIB=...): the 1-GPU frame in the default (pre-pass) order and
in row-major order, and every shard of an N-way split (the max is the N-GPU frame time).

    RT_LIB=raytracing-hw_amd/v1/librt_hw_amd.so python tools/order_ab.py [--world 8]
"""
import argparse
import json
import os
import sys
import time

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
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--steps", type=int, default=2)
    ap.add_argument("--natural", type=int, default=1)
    ap.add_argument("--shard-steps", type=int, default=1)
    ap.add_argument("--row-block", type=int, default=8, help="rows per interleave block of the N-way split")
    ap.add_argument("--full", type=int, default=1, help="0: skip the 1-GPU frame (shards only)")
    args = ap.parse_args()
    rt = bench.import_pkg()
    path = bench.load_scenes_module().ensure_scene(args.scene, os.environ.get("RT_SCENE_DIR", "/tmp/rt_scenes"))
    W, H, S = args.width, args.height, args.spp
    scene = rt.Scene.load(path, W, H, S)
    scene.upload(0)
    rtdist = __import__("importlib").import_module("raytracing_hw_amd.dist")
    stream = torch.cuda.current_stream().cuda_stream
    res = {"lib": os.environ.get("RT_LIB", "default"), "row_block": args.row_block}

    import hashlib
    shard_hash = hashlib.sha1()

    def t(world, rank, steps, natural):
        rb = args.row_block if world > 1 else 8
        out = torch.zeros(rtdist.max_shard_rows(H, world, rb) * W * 3, dtype=torch.float32, device="cuda")
        ms, order = [], []
        for _ in range(steps):
            st = scene.render_device(out.data_ptr(), stream, spp=S, rank=rank, world=world, row_block=rb, stats=True,
                                     natural_order=natural)
            ms.append(st["render_ms"])
            order.append(st["order_ms"])
        if world > 1 and not natural:
            shard_hash.update(out.cpu().numpy().tobytes())
        return min(ms), min(order)

    t(1, 0, 1, False)   # warm
    if args.full:
        res["full_ms"], res["full_order_ms"] = t(1, 0, args.steps, False)
        full = torch.zeros(H * W * 3, dtype=torch.float32, device="cuda")
        scene.render_device(full.data_ptr(), stream, spp=S, rank=0, world=1)
        torch.cuda.synchronize()
        res["full_sha1"] = __import__("hashlib").sha1(full.cpu().numpy().tobytes()).hexdigest()[:16]
    if args.natural:
        res["full_natural_ms"], _ = t(1, 0, args.steps, True)
    sh = [t(args.world, r, args.shard_steps, False)[0] for r in range(args.world)]
    res[f"shard{args.world}_ms"] = [round(x, 1) for x in sh]
    res[f"shard{args.world}_max_ms"] = max(sh)
    res[f"shard{args.world}_sha1"] = shard_hash.hexdigest()[:16]   # the shards' float sums (same bits across builds)
    if args.natural:
        shn = [t(args.world, r, 1, True)[0] for r in range(args.world)]
        res[f"shard{args.world}_natural_max_ms"] = max(shn)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
