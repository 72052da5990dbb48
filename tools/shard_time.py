#!/usr/bin/env python3
"""Per-GPU time of one pixel-row shard, for estimating strong scaling on one GPU.

    python tools/shard_time.py [--spp 256] [--worlds 1,2,4,8]

For each world size N this renders rank 0's shard of an N-way split (rows with
(row / 8) % N == 0: exactly the work one GPU does when bench.py runs on N GPUs) and prints
its kernel time and rays.  The N-GPU frame time is about the slowest rank's time plus the
all-gather; rows are interleaved in 8-row blocks, so the ranks are close.  This is a
diagnostic: bench.py --gpus N on N GPUs is the measurement.
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
    ap.add_argument("--worlds", default="1,2,4,8")
    ap.add_argument("--steps", type=int, default=2)
    ap.add_argument("--kernels", default="0")
    ap.add_argument("--chunks", default="0", help="0 = parity mode; k > 0 = fast mode (RT_FLAG_FAST) with k-sample units")
    args = ap.parse_args()
    rt = bench.import_pkg()
    scenes = bench.load_scenes_module()
    scene_dir = os.environ.get("RT_SCENE_DIR", "/tmp/rt_scenes")
    path = scenes.ensure_scene(args.scene, scene_dir)
    W, H, S = args.width, args.height, args.spp
    scene = rt.Scene.load(path, W, H, S)
    scene.upload(0)
    rtdist = __import__("importlib").import_module("raytracing_hw_amd.dist")
    stream = torch.cuda.current_stream().cuda_stream
    base = None
    modes = [(k, c) for k in [int(x) for x in args.kernels.split(",")] for c in [int(x) for x in args.chunks.split(",")]]
    for kernel, chunk in modes:
        base = None
        kw = dict(fast=chunk > 0, fast_chunk=max(chunk, 0))
        for world in [int(x) for x in args.worlds.split(",")]:
            rows = rtdist.max_shard_rows(H, world)
            out = torch.zeros(rows * W * 3, dtype=torch.float32, device="cuda")
            st = scene.render_device(out.data_ptr(), stream, spp=S, rank=0, world=world, count=True, stats=True,
                                     kernel=kernel, **kw)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(args.steps):
                scene.render_device(out.data_ptr(), stream, spp=S, rank=0, world=world, stats=True, kernel=kernel, **kw)
            torch.cuda.synchronize()
            ms = (time.perf_counter() - t0) / args.steps * 1e3
            base = base or ms
            print(json.dumps({"kernel": kernel, "fast_chunk": chunk, "world": world, "rank0_ms": round(ms, 2), "rank0_rays": st["rays"],
                              "rank0_mrays_s": round(st["rays"] / ms / 1e3, 1),
                              "est_speedup_vs_1": round(base / ms, 2)}), flush=True)


if __name__ == "__main__":
    main()
