#!/usr/bin/env python3
"""Offline study of the runahead's vertex-count prediction (rt_mega.h).

Traces every sample of the heaviest pixels of the headline frame on the host (the kernel
source compiled for the CPU, tests/native/kernel_host.cpp kh_v_trace) and reports, per
predictor of a sample's vertex count v, how often the prediction is right and how long the
runs of consecutive hits are (a runahead window only pays while its links hold):

    python tools/runahead_predict.py [--pixels 128] [--spp 256]
"""
import argparse
import ctypes
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))


def build_kh(out):
    subprocess.run(["g++", "-O2", "-fno-tree-vectorize", "-fno-tree-slp-vectorize", "-ffp-contract=off", "-fopenmp",
                    "-std=c++17", "-shared", "-fPIC", os.path.join(ROOT, "tests", "native", "kernel_host.cpp"),
                    "-o", out], check=True)
    lib = ctypes.CDLL(out)
    V, L = ctypes.c_void_p, ctypes.c_int64
    lib.kh_v_trace.argtypes = [V, ctypes.c_int, L, V, V, V]
    lib.kh_v_trace.restype = None
    return lib


def trace(lib, view, pix, spp):
    pix = np.ascontiguousarray(pix, np.int64)
    nv = np.zeros((len(pix), spp), np.uint8)
    cost = np.zeros((len(pix), spp), np.uint32)
    lib.kh_v_trace(ctypes.addressof(view), spp, len(pix), pix.ctypes.data, nv.ctypes.data, cost.ctypes.data)
    return nv, cost


def predictors(depth):
    def always_depth(hist):
        return [depth]

    def last(hist):
        return [hist[-1]] if hist else [depth]

    def mode(hist):
        if not hist:
            return [depth]
        return [int(np.bincount(hist, minlength=depth + 1).argmax())]

    def top(k):
        def f(hist):
            c = np.bincount(hist, minlength=depth + 1) if hist else np.zeros(depth + 1)
            c = c.astype(float)
            c[depth] += 0.5   # ties toward depth
            return list(np.argsort(-c)[:k])
        f.__name__ = f"top{k}"
        return f

    def majority(hist):
        # a Boyer-Moore majority vote with a saturating 3-bit count, starting from ray_depth
        c, k = depth, 0
        for v in hist:
            if k == 0:
                c, k = v, 1
            elif v == c:
                k = min(k + 1, 7)
            else:
                k -= 1
        return [c]

    def nibble(prior):
        # the per-record vote built and measured in round 6: a 4-bit count
        # per vertex count, all halved when one would pass 15, ray_depth's count starting at
        # `prior`; the largest count wins, ties to the larger v
        def f(hist):
            n = [0] * (depth + 1)
            n[depth] = prior
            for v in hist:
                if n[v] == 15:
                    n = [x >> 1 for x in n]
                n[v] += 1
            best = depth
            for v in range(depth, -1, -1):
                if n[v] > n[best]:
                    best = v
            return [best]
        f.__name__ = f"vote_prior{prior}"
        return f

    return [always_depth, last, mode, majority, nibble(0), nibble(1), nibble(2), nibble(3), top(2), top(3), top(4)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--pixels", type=int, default=128)
    ap.add_argument("--spp", type=int, default=256)
    ap.add_argument("--scene-dir", default="/tmp/rt_scenes")
    ap.add_argument("--select", default="heavy", choices=["heavy", "random"],
                    help="the heaviest pixels (the 8-way drain's chains) or a uniform sample of the frame")
    args = ap.parse_args()
    import importlib.util
    spec = importlib.util.spec_from_file_location("rt", os.path.join(ROOT, "raytracing-hw_amd", "__init__.py"),
                                                  submodule_search_locations=[os.path.join(ROOT, "raytracing-hw_amd")])
    rt = importlib.util.module_from_spec(spec)
    sys.modules["raytracing_hw_amd"] = rt
    spec.loader.exec_module(rt)
    sspec = importlib.util.spec_from_file_location("rt_scenes", os.path.join(ROOT, "raytracing-hw_amd", "scenes.py"))
    scenes = importlib.util.module_from_spec(sspec)
    sspec.loader.exec_module(scenes)
    path = scenes.ensure_scene("sponza", args.scene_dir)
    W, H = 1920, 1080
    sc = rt.Scene.load(path, W, H, args.spp)
    view, _keep = rt.make_view(sc.view())
    depth = 6
    lib = build_kh("/tmp/libkh_predict.so")
    # coarse cost map: every 12th pixel at 4 spp, heaviest first
    ys, xs = np.mgrid[0:H:12, 0:W:12]
    cand = (ys * W + xs).ravel()
    _, c4 = trace(lib, view, cand, 4)
    if args.select == "heavy":
        heavy = cand[np.argsort(-c4.sum(1).astype(np.int64))[: args.pixels]]
    else:
        heavy = np.random.default_rng(1).choice(cand, args.pixels, replace=False)
    nv, cost = trace(lib, view, heavy, args.spp)
    hist_v = np.bincount(nv.ravel(), minlength=depth + 1)
    print(f"v histogram ({args.select} pixels):", (hist_v / hist_v.sum()).round(3).tolist())
    w = cost.astype(np.float64)
    print("cost share by v:", [round(float(w[nv == k].sum() / w.sum()), 3) for k in range(depth + 1)])
    for pred in predictors(depth):
        hits = np.zeros_like(nv, bool)
        for q in range(nv.shape[0]):
            hist = []
            for s in range(nv.shape[1]):
                hits[q, s] = nv[q, s] in pred(hist)
                hist.append(int(nv[q, s]))
        # mean run of consecutive hits starting at a sample (capped at 8): window payoff
        runs = []
        for q in range(nv.shape[0]):
            h = hits[q]
            for s in range(0, nv.shape[1] - 8):
                r = 0
                while r < 8 and h[s + r]:
                    r += 1
                runs.append(r)
        print(f"{pred.__name__:>13}: hit {hits.mean():.3f}  mean run {np.mean(runs):.2f}")


if __name__ == "__main__":
    main()
