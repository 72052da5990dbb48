#!/usr/bin/env python3
"""Frames in flight: K frames (or K copies of one shard of an N-way split) rendered one after
another on one stream, against the same K launched round-robin over F independent scene
copies and streams with no wait between them (frame i+1's blocks fill the CUs that frame i's
tail leaves idle).  Same bits per frame; prints wall ms per frame for both.

    python tools/overlap_ab.py [--worlds 1,8] [--frames 4] [--inflight 2]
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
    ap.add_argument("--worlds", default="1,8")
    ap.add_argument("--frames", type=int, default=4)
    ap.add_argument("--inflight", type=int, default=2)
    args = ap.parse_args()
    rt = bench.import_pkg()
    path = bench.load_scenes_module().ensure_scene(args.scene, os.environ.get("RT_SCENE_DIR", "/tmp/rt_scenes"))
    W, H, S = args.width, args.height, args.spp
    F = args.inflight
    scenes = [rt.Scene.load(path, W, H, S) for _ in range(F)]
    for s in scenes:
        s.upload(0)
    rtdist = __import__("importlib").import_module("raytracing_hw_amd.dist")
    streams = [torch.cuda.Stream() for _ in range(F)]
    for world in [int(x) for x in args.worlds.split(",")]:
        n = rtdist.max_shard_rows(H, world) * W * 3
        outs = [torch.zeros(n, dtype=torch.float32, device="cuda") for _ in range(F)]
        torch.cuda.synchronize()   # (the zero fills run on torch's stream, the renders on their own)
        for f in range(F):   # warm every copy (workspace allocation)
            scenes[f].render_device(outs[f].data_ptr(), streams[f].cuda_stream, spp=S, rank=0, world=world)
        torch.cuda.synchronize()
        ref = outs[0].clone()

        def run(k_inflight):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for i in range(args.frames):
                f = i % k_inflight
                scenes[f].render_device(outs[f].data_ptr(), streams[f].cuda_stream, spp=S, rank=0, world=world)
            torch.cuda.synchronize()
            return (time.perf_counter() - t0) * 1e3 / args.frames

        seq = run(1)
        ovl = run(F)
        same = all(torch.equal(o, ref) for o in outs)
        print(json.dumps({"world": world, "frames": args.frames, "inflight": F, "seq_ms_per_frame": round(seq, 1),
                          "overlap_ms_per_frame": round(ovl, 1), "gain": round(seq / ovl, 3), "bits_equal": same}),
              flush=True)


if __name__ == "__main__":
    main()
