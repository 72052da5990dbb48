#!/usr/bin/env python3
"""Headline benchmark: Mrays/s + frame time, sponza proxy 1920x1080x256spp (BASELINE.json).

    python bench.py [--gpus N --steps K --warmup W]            (N>1: launched by torch.distributed.run)

A step = one full frame of the workload: every pixel of the 1920x1080 frame traced at
256 spp, depth 6, split into interleaved 8-row blocks over the N ranks (one MI355X each),
finished to the 8-bit frame on each GPU (rt_tonemap_u8_device, scene.cpp:54-64) and
all-gathered over RCCL (6.2 MB).  Rank 0 prints one JSON line.

value    = scene closest-hit queries (rays, counted in-kernel during warmup; the count is
           deterministic per frame) of all ranks x K / max-over-ranks wall time of the K steps.
           Every frame is rendered from scratch: the heaviest-first pixel order comes from a
           counting pre-pass inside the same call (rt_device.hip launch_order), inside the
           timed region; nothing measured in one frame is reused by the next.
cold_ms_per_step = the very first frame after the scene upload (one-time workspace
           allocation and code-object load included), max over ranks.
natural_order = the same frame in row-major pixel order (RT_FLAG_NATURAL_ORDER, no pre-pass).
roofline = rank 0's render kernel.  Default (kernel 0, lane-resident rt_mega_kernel): the
           frame is one launch (the runahead kernel: 4- and 8-way shards) or one launch pair
           (the plain kernel, then the runahead kernel resuming its parked tail: the hand-off),
           so achieved = the algorithmic bytes of the whole path (24 B per AABB
           test + 36 B per triangle test, scene and light BVH, + 156 B per shaded hit) / the
           render's duration (HIP events on the launch stream around the launch or the pair;
           the counters of a pair are added).
           With --kernel 4 (wavefront) it is the extend kernel alone: 24 B per AABB test +
           36 B per triangle test + 44 B of ray/hit I/O per ray, per launch / its average
           duration.  Peak: 8 TB/s HBM3E.  `traffic` is the HBM-side bytes per launch from
           the committed rocprofv3 PMC passes of this command: FETCH_SIZE x the calibrated
           factor of this kernel's load shapes + WRITE_SIZE.  The factor comes from
           tools/fetch_calib.hip (profiles/<CALIB_PREFIX>_fetch_calib.csv: FETCH_SIZE against
           the 128-B lines filled, per shape: 64-B node pairs, 48-B triangle quads, 4-B texel
           gathers), weighted by the shapes' shares of the algorithmic bytes; `traffic_range`
           spans the shapes' factors, `traffic_undoubled` is FETCH_SIZE as counted (+ WRITE_SIZE),
           `traffic_frac` = traffic / launch time / peak.
cpu_baseline: the reference itself (oracle/_ref/ref_render, built from /root/reference's
           sources) timing its Scene::render loop on the host cores this process may use
           (min(nproc, cgroup CPU quota) threads; `cores` says how many) over a bounded sample
           of the same frame (every 8th row, 16 spp); a counting build of the same sources
           counts its rays.  Falls back to the build's CPU restatement (oracle/) when _ref is
           absent.
roofline.bound follows the committed counters: "latency/issue" when the HBM-side traffic
           is under half the algorithmic model's or below the VALU issue utilisation
           (roofline.issue: VALU instructions per SIMD-cycle from the SQ passes against the
           SIMD-32 ceiling of 0.5, lane utilisation, SALU share, wait share), else "hbm";
           "unmeasured" when no PMC pass of the command is committed.  --gpus N reads rank 0's
           shard passes (profiles/<SHARD_PROFILE_PREFIX>_shard_*_w<N>.csv, tools/pmc_shard.sh)
           for the kernel that rendered it (the runahead instantiation at 4 and 8 ways).
ranks:    --gpus N: every rank's render kernel time, pre-pass time, schedule, rays and
           algorithmic roofline fraction (all-gathered), and the slowest rank: the N-GPU step is
           as slow as it.
frame_matches_reference: the 8-bit frame's sha1 against the reference's own finished frame of
           the same workload (tests/golden/golden_meta.json "frames"), computed after the timed
           region.
"""
import argparse
import hashlib
import json
import os
import subprocess
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
HBM_PEAK_GBS = 8000.0      # MI355X HBM3E spec (MI355X_MICROARCH.md)
B_AABB, B_TRI, B_SHADE = 24, 36, 156
B_RAY_IO = 24 + 4 + 16     # wf_extend per ray: ray (6 floats) + queue slot in, hit (t, u, v, prim) out
PROFILE_PREFIX = "r06"   # profiles/<prefix>_{fetch,write,sq1,sq2}_1080p256.csv of the default command
# profiles/<prefix>_shard_{fetch,write,sq1,sq2}_w<N>.csv: rank 0's shard of the N-way split
# (tools/pmc_shard.sh), the counters of an --gpus N line
SHARD_PROFILE_PREFIX = "r06"
# profiles/<prefix>_fetch_calib.csv: FETCH_SIZE per filled 128-B line for each load shape
# (tools/fetch_calib.sh)
CALIB_PREFIX = "r06"
# rocprofv3 names of the two parity instantiations of the default kernel: the plain one (one
# GPU) and the runahead one (shards of at most 2 pixels per lane: the 4- and 8-way splits)
KERNEL_PLAIN = "void rt_mega_kernel<false, false, false, false>"
KERNEL_SPEC = "void rt_mega_kernel<false, false, false, true>"


def pmc_file(prefix, kind, world):
    """The committed PMC summary of pass `kind` for this world size."""
    return f"{prefix}_{kind}_1080p256.csv" if world == 1 else f"{prefix}_shard_{kind}_w{world}.csv"


def import_pkg():
    import importlib.util
    pkg = os.path.join(ROOT, "raytracing-hw_amd")
    if "raytracing_hw_amd" in sys.modules:
        return sys.modules["raytracing_hw_amd"]
    spec = importlib.util.spec_from_file_location("raytracing_hw_amd", os.path.join(pkg, "__init__.py"),
                                                  submodule_search_locations=[pkg])
    mod = importlib.util.module_from_spec(spec)
    sys.modules["raytracing_hw_amd"] = mod
    spec.loader.exec_module(mod)
    return mod


def load_scenes_module():
    import importlib.util
    spec = importlib.util.spec_from_file_location("rt_scenes", os.path.join(ROOT, "raytracing-hw_amd", "scenes.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


def cpu_quota():
    """CPUs this process may use: the cgroup v2 quota (cpu.max), else None."""
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        return None if q == "max" else float(q) / float(per)
    except Exception:  # noqa: BLE001
        return None


def cpu_baseline(scene_path, width, height, spp, rows, stride, threads):
    """Time the reference's CPU path on a bounded sample (`rows` rows, every `stride`-th, `spp` spp).

    The reference (oracle/_ref, built from /root/reference's sources by oracle/Makefile):
    ref_render runs the sample loop of Scene::render (scene.cpp:31-44) and is timed;
    ref_harness (same sources, counting wraps) counts the rays of the same sample."""
    ref_dir = os.path.join(ROOT, "oracle", "_ref")
    timer, counter = os.path.join(ref_dir, "ref_render"), os.path.join(ref_dir, "ref_harness")
    env = dict(os.environ, OMP_NUM_THREADS=str(threads))
    sample = f"{rows} rows (every {stride}th) x {width} of the {width}x{height} frame at {spp} spp"
    args = ["time", scene_path, str(width), str(height), str(spp), str(rows), str(stride)]
    if os.path.exists(timer) and os.path.exists(counter):
        try:
            def run(exe):
                out = subprocess.run([exe, *args], env=env, capture_output=True, text=True, timeout=600,
                                     check=True).stdout
                return json.loads(out.strip().splitlines()[-1])
            t = run(timer)
            c = run(counter)
            return {"value": c["rays"] / t["seconds"] / 1e6, "unit": "Mrays/s", "cores": threads, "kind": "reference",
                    "sample": sample + " (reference Scene::render sample loop; rays counted by a second, counting "
                                       "build of the same sources)",
                    "seconds": t["seconds"], "rays": c["rays"]}
        except Exception as e:  # noqa: BLE001
            print(f"[bench] reference CPU baseline failed: {e}", file=sys.stderr)
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import rtref
    rt = import_pkg()
    s = rt.Scene.load(scene_path, width, height, spp)
    _, cnt, secs = rtref.Oracle().render(s.view(), spp, 0, width * rows, threads)   # (first rows)
    return {"value": float(cnt[0]) / secs / 1e6, "unit": "Mrays/s", "cores": threads, "kind": "port",
            "sample": sample + " (oracle/rt_oracle.cpp restatement)", "seconds": secs}


def pmc_mean(path, counter, kname, duration=False):
    """Mean per dispatch of `counter` for the launch of kernel `kname` (its full template list,
    KERNEL_PLAIN or KERNEL_SPEC) in a rocprofv3 --stats PMC summary (None when absent); with
    duration=True, that pass's average dispatch duration in seconds instead.  `kname` may be a
    tuple of kernels launched once per frame each (the hand-off: the plain kernel, then the
    runahead kernel): their means (or durations) are added."""
    import csv
    if not os.path.exists(path):
        return None
    if isinstance(kname, tuple):
        vals = [pmc_mean(path, counter, k, duration) for k in kname]
        return None if any(v is None for v in vals) else sum(vals)
    for row in csv.reader(open(path)):
        if row and row[0].startswith(kname + "(") and row[1] == counter:
            return float(row[5]) * 1e-9 if duration else float(row[4])
    return None


SIMDS = 256 * 4            # MI355X: 256 CUs x 4 SIMD-32
NOMINAL_CLOCK_HZ = 2.4e9   # used only when no GRBM_GUI_ACTIVE pass is committed


# VALU issue ceiling of one SIMD: a wave64 VALU instruction occupies a SIMD-32 for 2 cycles
# (MI355X_MICROARCH.md, "Wave scheduling" and the constants row "v_fma_f32 (wave64) 2 cyc
# (SIMD-32)"), so at most 0.5 wave-instructions issue per SIMD per cycle.
VALU_ISSUE_CEILING = 0.5


def pmc_issue(prefix, kname, world=1):
    """Issue-side picture of the launch from the committed SQ passes (tools/profile.sh,
    tools/pmc_shard.sh): VALU wave-instructions per SIMD per cycle over the pass's own dispatch
    duration and its share of VALU_ISSUE_CEILING, the VALU lane utilisation and the wait share."""
    sq1, sq2 = pmc_file(prefix, "sq1", world), pmc_file(prefix, "sq2", world)
    valu = pmc_mean(sq2, "SQ_INSTS_VALU", kname)
    salu = pmc_mean(sq2, "SQ_INSTS_SALU", kname)
    tcv = pmc_mean(sq1, "SQ_THREAD_CYCLES_VALU", kname)
    aiv = pmc_mean(sq1, "SQ_ACTIVE_INST_VALU", kname)
    wait = pmc_mean(sq1, "SQ_WAIT_ANY", kname)
    wcyc = pmc_mean(sq1, "SQ_WAVE_CYCLES", kname)
    grbm = pmc_mean(sq1, "GRBM_GUI_ACTIVE", kname)
    avg_s = pmc_mean(sq2, "SQ_INSTS_VALU", kname, duration=True)
    if valu is None or not avg_s:
        return None
    clock = grbm / 8.0 / avg_s if grbm else NOMINAL_CLOCK_HZ
    per_simd_cycle = valu / (SIMDS * avg_s * clock)
    return {"valu_inst_per_simd_cycle": round(per_simd_cycle, 4),
            "issue_frac_of_simd32_peak": round(per_simd_cycle / VALU_ISSUE_CEILING, 4),
            "issue_ceiling": "0.5 wave64 VALU instructions per SIMD-32 per cycle (MI355X_MICROARCH.md, Wave scheduling)",
            "lane_util": None if not (tcv and aiv) else round(tcv / (aiv * 64.0), 4),
            "salu_per_valu": None if salu is None else round(salu / valu, 4),
            "wait_any_frac": None if not (wait and wcyc) else round(wait / wcyc, 4),
            "clock_hz": round(clock / 1e6, 1) * 1e6,
            "clock_source": "GRBM_GUI_ACTIVE / 8 / launch time" if grbm else "nominal 2.4 GHz (no GRBM pass)",
            "source": os.path.relpath(sq2, ROOT) + " + " + os.path.relpath(sq1, ROOT)}


def reference_frame_sha1(scene, W, H, S):
    """sha1 of the reference's own finished 8-bit frame of this workload, if one is committed
    (tests/golden/golden_meta.json "frames", tools/make_goldens.py --frames)."""
    try:
        meta = json.load(open(os.path.join(ROOT, "tests", "golden", "golden_meta.json")))
    except Exception:  # noqa: BLE001
        return None
    for f in meta.get("frames", {}).values():
        if (f["scene"], f["width"], f["height"], f["spp"]) == (scene, W, H, S):
            return f["frame_u8_sha1"]
    return None


def fetch_calibration(shares):
    """FETCH_SIZE -> HBM bytes factor for the render kernel's loads: the committed calibration
    (tools/fetch_calib.sh: per shape, lines x 128 B / FETCH_SIZE bytes on a 2 GiB buffer)
    weighted by `shares` (the kernel's algorithmic bytes per shape: node pairs, triangles,
    texels), and the shapes' min / max factors.  Without a committed calibration: the guide's
    streaming factor 2 (uncalibrated for these shapes)."""
    import csv
    path = os.path.join(ROOT, "profiles", f"{CALIB_PREFIX}_fetch_calib.csv")
    fac = {}
    if os.path.exists(path):
        for row in csv.DictReader(open(path)):
            if row["hbm_per_fetch"] not in ("", "None"):
                fac[row["kernel"]] = float(row["hbm_per_fetch"])
    shapes = ["calib_pair", "calib_tri", "calib_texel"]
    if not all(k in fac for k in shapes):
        return 2.0, 2.0, 2.0, "uncalibrated: x2 (MI355X_MICROARCH.md streaming-read factor)"
    tot = sum(shares) or 1.0
    f = sum(fac[k] * w for k, w in zip(shapes, shares)) / tot
    vals = [fac[k] for k in shapes]
    return f, min(vals), max(vals), os.path.relpath(path, ROOT)


def pmc_traffic(fetch_csv, write_csv, kname, shares):
    """HBM-side bytes per launch of kernel `kname` from rocprofv3 PMC summaries
    (tools/profile.sh, tools/pmc_shard.sh: separate --pmc passes of the same workload):
    FETCH_SIZE x the calibrated factor (fetch_calibration) plus WRITE_SIZE, both KiB per
    dispatch.  Returns (bytes, low, high, FETCH_SIZE + WRITE_SIZE as counted, calibration)."""
    f, w = pmc_mean(fetch_csv, "FETCH_SIZE", kname), pmc_mean(write_csv, "WRITE_SIZE", kname)
    if f is None or w is None:
        return None
    fac, lo, hi, src = fetch_calibration(shares)
    fb, wb = f * 1024.0, w * 1024.0
    return fac * fb + wb, lo * fb + wb, hi * fb + wb, fb + wb, {"factor": round(fac, 4), "min": lo, "max": hi,
                                                                "source": src}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--scene", default="sponza")
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--spp", type=int, default=256)
    ap.add_argument("--kernel", type=int, default=0, choices=[0, 4], help="0 lane-resident (default), 4 wavefront")
    ap.add_argument("--row-block", type=int, default=8)
    ap.add_argument("--cpu-rows", type=int, default=135, help="rows of the frame in the CPU baseline sample")
    ap.add_argument("--cpu-stride", type=int, default=8, help="CPU baseline sample: every n-th row")
    ap.add_argument("--cpu-spp", type=int, default=16)
    ap.add_argument("--cpu-threads", type=int, default=0, help="CPU baseline threads (0 = min(nproc, cgroup quota))")
    ap.add_argument("--natural-steps", type=int, default=1,
                    help="timed frames in row-major pixel order (no pre-pass), reported beside the headline")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--fast-steps", type=int, default=2,
                    help="timed frames of fast mode (RT_FLAG_FAST, reported beside the headline; 0 = skip)")
    ap.add_argument("--fast-chunk", type=int, default=2, help="fast mode: samples per work unit")
    ap.add_argument("--traffic-from", default="auto",
                    help="PMC summaries for roofline.traffic: a path prefix P (P_fetch*.csv / P_write*.csv from "
                         "tools/profile.sh of this same command), 'auto' (the committed profiles/ pair when the "
                         "workload is the default one) or 'none'")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        print(f"[bench] --gpus {args.gpus} but WORLD_SIZE={world}; using WORLD_SIZE", file=sys.stderr)
    # RT_BENCH_SHARE_GPU=1: rehearsal of the N-rank logic on a one-GPU box (every rank on
    # device 0, gloo collectives on host copies); its timings mean nothing
    share = os.environ.get("RT_BENCH_SHARE_GPU") == "1"
    dev = 0 if share else local
    torch.cuda.set_device(dev)
    if world > 1:
        if share:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))

    def barrier():
        if world > 1:
            dist.barrier()

    def all_reduce(t, op):
        if world == 1:
            return
        if share:
            c = t.cpu()
            dist.all_reduce(c, op=op)
            t.copy_(c)
        else:
            dist.all_reduce(t, op=op)

    rt = import_pkg()
    scene_dir = os.environ.get("RT_SCENE_DIR", "/tmp/rt_scenes")
    scenes = load_scenes_module()
    if rank == 0:
        path = scenes.ensure_scene(args.scene, scene_dir)
    barrier()
    path = os.path.join(scene_dir, args.scene + ".gltf")
    W, H, S = args.width, args.height, args.spp
    t0 = time.time()
    scene = rt.Scene.load(path, W, H, S)
    scene.upload(dev)
    load_s = time.time() - t0
    n_tris = scene.view()["tri"].shape[0]

    import importlib
    rtdist = importlib.import_module("raytracing_hw_amd.dist")
    max_rows = rtdist.max_shard_rows(H, world, args.row_block)
    out = torch.zeros(max_rows * W * 3, dtype=torch.float32, device="cuda")
    rgb = torch.zeros(max_rows * W * 3, dtype=torch.uint8, device="cuda")
    frame = torch.empty((H, W, 3), dtype=torch.uint8, device="cuda")
    stream = torch.cuda.current_stream().cuda_stream

    def step(count=False, fast=False, natural=False):
        # render the shard, finish it to 8 bits on the GPU (scene.cpp:54-64), gather the frame
        st = scene.render_device(out.data_ptr(), stream, spp=S, rank=rank, world=world, row_block=args.row_block,
                                 count=count, kernel=args.kernel, stats=True, kernel_times=not count, fast=fast,
                                 fast_chunk=args.fast_chunk, device=dev, natural_order=natural)
        rt.tonemap_device(out.data_ptr(), W, max_rows, S, rgb.data_ptr(), stream)
        if share and world > 1:
            frame.copy_(rtdist.gather_frame(rgb.cpu(), H, W, rank, world, args.row_block))
        else:
            rtdist.gather_frame(rgb, H, W, rank, world, args.row_block, out=frame)   # RCCL all-gather (N > 1)
        return st

    def timed(n, **kw):
        """n frames between barriers + synchronize; returns (max-over-ranks seconds, stats)."""
        sts = []
        barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(n):
            sts.append(step(**kw))
        torch.cuda.synchronize()
        barrier()
        t = torch.tensor([time.perf_counter() - t0], dtype=torch.float64, device="cuda")
        all_reduce(t, dist.ReduceOp.MAX)
        return float(t.item()), sts

    # the very first frame of this scene on this device: nothing from an earlier render
    cold_s, _ = timed(1)
    # warmup; the first one counts rays / tests (deterministic per frame, so valid for every step)
    counts = None
    for w in range(max(args.warmup, 1)):
        st = step(count=(w == 0))
        if w == 0:
            counts = st
    torch.cuda.synchronize()

    kernel_ms, ext_ms, ext_n, ext_rays, order_ms, sched = [], [], [], [], [], 0
    barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        st = step()
        kernel_ms.append(st["render_ms"])
        order_ms.append(st["order_ms"])
        ext_ms.append(st["extend_ms"])
        ext_n.append(st["extend_launches"])
        ext_rays.append(st["extend_rays"])
        sched |= st["schedule"]
    torch.cuda.synchronize()
    barrier()
    elapsed = time.perf_counter() - t0
    # digest of the gathered 8-bit frame (outside the timed region): the parity path is
    # bit-exact whatever the sharding, so this must agree across --gpus 1/2/4/8 runs
    digest = hashlib.sha1(frame.cpu().numpy().tobytes()).hexdigest()[:16] if rank == 0 else None

    natural_s = None
    if args.natural_steps > 0 and args.kernel == 0:
        natural_s, _ = timed(args.natural_steps, natural=True)

    # fast mode (RT_FLAG_FAST): same frame, per-(pixel, sample) Philox streams, samples as
    # independent work units; its own ray count (other random paths), same timing protocol
    fast_line = None
    if args.fast_steps > 0 and args.kernel == 0:
        fc = step(count=True, fast=True)
        torch.cuda.synchronize()
        barrier()
        torch.cuda.synchronize()
        tf = time.perf_counter()
        fast_ms = []
        for _ in range(args.fast_steps):
            fast_ms.append(step(fast=True)["render_ms"])
        torch.cuda.synchronize()
        barrier()
        t_fast = torch.tensor([time.perf_counter() - tf], dtype=torch.float64, device="cuda")
        r_fast = torch.tensor([float(fc["rays"])], dtype=torch.float64, device="cuda")
        all_reduce(t_fast, dist.ReduceOp.MAX)
        all_reduce(r_fast, dist.ReduceOp.SUM)
        fe, frays = float(t_fast.item()), float(r_fast.item())
        fast_line = {"value": round(frays * args.fast_steps / fe / 1e6, 3), "unit": "Mrays/s",
                     "ms_per_step": round(fe / args.fast_steps * 1e3, 3), "steps": args.fast_steps,
                     "chunk": args.fast_chunk, "rays_per_frame": int(frays),
                     "kernel_ms": round(float(np.mean(fast_ms)), 3),
                     "note": "RT_FLAG_FAST: Philox4x32-10 seed per (pixel, sample), work units of `chunk` samples; "
                             "statistically equivalent to the reference, NOT bit-identical (not the headline)"}

    def all_gather_rows(vals):
        """Every rank's `vals` (a list of floats), in rank order."""
        if world == 1:
            return [list(vals)]
        t = torch.tensor(vals, dtype=torch.float64, device="cuda")
        if share:
            t = t.cpu()
        outs = [torch.zeros_like(t) for _ in range(world)]
        dist.all_gather(outs, t)
        return [o.tolist() for o in outs]

    # every rank's own render: kernel time, pre-pass, schedule, rays, algorithmic bytes
    my_bytes = (B_AABB * (counts["aabb_tests"] + counts["light_aabb_tests"])
                + B_TRI * (counts["tri_tests"] + counts["light_tri_tests"]) + B_SHADE * counts["shading_hits"])
    per_rank = all_gather_rows([float(np.mean(kernel_ms)), float(np.max(kernel_ms)), float(np.mean(order_ms)),
                                float(sched), float(counts["rays"]), float(my_bytes)])

    keys = ["rays", "aabb_tests", "tri_tests", "light_queries", "light_aabb_tests", "light_tri_tests", "shading_hits"]
    local_counts = torch.tensor([counts[k] for k in keys], dtype=torch.float64, device="cuda")
    t = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
    all_reduce(local_counts, dist.ReduceOp.SUM)
    all_reduce(t, dist.ReduceOp.MAX)
    total = dict(zip(keys, local_counts.tolist()))
    elapsed = float(t.item())

    if rank == 0:
        rays_per_frame = total["rays"]
        value = rays_per_frame * args.steps / elapsed / 1e6
        # rank 0's own kernel: algorithmic bytes per launch / average launch time
        c0 = counts
        # whole path: every BVH node / triangle record + shading fetch per frame
        bytes_frame = (B_AABB * (c0["aabb_tests"] + c0["light_aabb_tests"]) + B_TRI * (c0["tri_tests"] + c0["light_tri_tests"])
                       + B_SHADE * c0["shading_hits"])
        frame_s = float(np.mean(kernel_ms)) / 1e3
        if args.kernel == 4 and sum(ext_n) > 0:
            # dominant kernel = wf_extend: scene-BVH node pairs + triangles + per-ray SoA in/out
            ext_bytes = B_AABB * c0["aabb_tests"] + B_TRI * c0["tri_tests"] + B_RAY_IO * ext_rays[0]
            launches = float(np.mean(ext_n))
            bytes_launch = ext_bytes / launches
            avg_s = float(np.sum(ext_ms)) / float(np.sum(ext_n)) / 1e3
            kname = "wf_extend_kernel"
        else:
            # one launch (or the hand-off's pair) renders the frame (rank 0's shard): the whole-path
            # model over the render time
            bytes_launch, avg_s, launches = bytes_frame, frame_s, 1.0
            # the plain kernel, the runahead kernel (the 4- and 8-way shards), or both once per
            # frame (the hand-off: the plain kernel's tail resumed by the runahead kernel)
            kname = ((KERNEL_PLAIN, KERNEL_SPEC) if sched & rt.SCHED_LANE else KERNEL_SPEC) \
                if sched & rt.SCHED_RUNAHEAD else KERNEL_PLAIN
        achieved = bytes_launch / avg_s / 1e9
        traffic, traffic_u, traffic_src, issue, traffic_rng, calib = None, None, None, None, None, None
        # the kernel's algorithmic bytes per load shape (node pairs, triangles, texels + shading)
        shares = [B_AABB * (c0["aabb_tests"] + c0["light_aabb_tests"]), B_TRI * (c0["tri_tests"] + c0["light_tri_tests"]),
                  B_SHADE * c0["shading_hits"]]
        if args.traffic_from != "none":
            prefix = args.traffic_from
            default_cfg = (args.scene, W, H, S, args.kernel) == ("sponza", 1920, 1080, 256, 0)
            if prefix == "auto":
                prefix = os.path.join(ROOT, "profiles", PROFILE_PREFIX if world == 1 else SHARD_PROFILE_PREFIX) \
                    if default_cfg else None
            if prefix:
                fc, wc = pmc_file(prefix, "fetch", world), pmc_file(prefix, "write", world)
                if os.path.exists(fc) and os.path.exists(wc):
                    t = pmc_traffic(fc, wc, kname, shares)
                    if t is not None:
                        traffic, traffic_u = t[0] / launches, t[3] / launches
                        traffic_rng = [int(t[1] / launches), int(t[2] / launches)]
                        calib = t[4]
                        traffic_src = os.path.relpath(fc, ROOT) + " + " + os.path.relpath(wc, ROOT)
                issue = pmc_issue(prefix, kname, world)
        frac = achieved / HBM_PEAK_GBS
        traffic_frac = None if traffic is None else traffic / avg_s / 1e9 / HBM_PEAK_GBS
        # the label follows the counters: HBM-bound only when the measured
        # HBM-side traffic is at least half of what the algorithmic model asks for and the
        # memory side is busier than the issue side (VALU issue rate / VALU_ISSUE_CEILING)
        issue_share = None if issue is None else issue["issue_frac_of_simd32_peak"]
        if traffic_frac is None:
            bound = "unmeasured (no PMC pass committed for this command)"
        elif traffic_frac < 0.5 * frac or (issue_share is not None and issue_share > traffic_frac):
            bound = "latency/issue"
        else:
            bound = "hbm"
        ref_sha = reference_frame_sha1(args.scene, W, H, S)
        line = {
            "metric": "Mrays/sec + frame time, Sponza 1920x1080x256spp at 1/2/4/8 MI355X",
            "value": round(value, 3),
            "unit": "Mrays/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 3),
            "cold_ms_per_step": round(cold_s * 1e3, 3),
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic: procedural sponza proxy (reference camera/materials/light, accessor-budget geometry, "
                    "procedural RGBA8 textures; SURVEY.md App. C)",
            "config": {"workload": f"{args.scene} proxy {W}x{H}x{S}spp depth 6, one frame per step",
                       "scene": args.scene, "width": W, "height": H, "spp": S, "triangles": int(n_tris),
                       "kernel": {0: "lane-resident", 4: "wavefront"}[args.kernel],
                       "parallelism": f"pixel-rows x{world}",
                       "pixel_order": ("heaviest-first from a counting pre-pass inside each timed frame" if S >= 128
                                       else "row-major (below 128 spp the library skips the pre-pass)")
                                      if args.kernel == 0 else "row-major",
                       "order_ms": round(float(np.mean(order_ms)), 3),
                       "rays_per_frame": int(rays_per_frame), "samples_per_frame": W * H * S,
                       "msamples_per_s": round(W * H * S * args.steps / elapsed / 1e6, 3),
                       "scene_load_s": round(load_s, 3), "frame_sha1": digest,
                       "reference_frame_sha1": None if ref_sha is None else ref_sha[:16],
                       "frame_matches_reference": None if ref_sha is None else digest == ref_sha[:16]},
            "roofline": {"bound": bound, "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(frac, 4),
                         "traffic": None if traffic is None else int(traffic),
                         "traffic_range": traffic_rng,
                         "traffic_undoubled": None if traffic_u is None else int(traffic_u),
                         "fetch_calibration": calib,
                         "traffic_frac": None if traffic_frac is None else round(traffic_frac, 4),
                         "issue": issue,
                         "traffic_source": traffic_src,
                         "kernel": " + ".join(kname) if isinstance(kname, tuple) else kname,
                         "bytes_per_launch": int(bytes_launch), "avg_launch_ms": round(avg_s * 1e3, 4),
                         "launches_per_frame": launches,
                         "path_frame_bytes": int(bytes_frame), "path_frame_ms": round(frame_s * 1e3, 3),
                         "path_achieved": round(bytes_frame / frame_s / 1e9, 1)},
            "cpu_baseline": None,
            "natural_order": None if natural_s is None else {
                "ms_per_step": round(natural_s / args.natural_steps * 1e3, 3), "steps": args.natural_steps,
                "value": round(rays_per_frame * args.natural_steps / natural_s / 1e6, 3), "unit": "Mrays/s",
                "note": "RT_FLAG_NATURAL_ORDER: row-major pixel order, no pre-pass (same bits; the default "
                        "below 128 spp)"},
            "fast_mode": fast_line,
        }
        sched_names = {rt.SCHED_LANE: "lane-resident", rt.SCHED_RUNAHEAD: "runahead", rt.SCHED_FAST: "fast",
                       rt.SCHED_LIGHT_SPLIT: "light-split", rt.SCHED_WAVEFRONT: "wavefront"}
        ranks = []
        for r, (kms, kmax, oms, sc, rays_r, bytes_r) in enumerate(per_rank):
            ranks.append({"rank": r, "render_ms": round(kms, 3), "render_ms_max": round(kmax, 3),
                          "order_ms": round(oms, 3),
                          "schedule": "+".join(v for b, v in sched_names.items() if int(sc) & b) or None,
                          "rays": int(rays_r), "roofline_frac": round(bytes_r / (kms / 1e3) / 1e9 / HBM_PEAK_GBS, 4)})
        slow = max(ranks, key=lambda x: x["render_ms"])
        line["ranks"] = ranks
        line["slowest_rank"] = {"rank": slow["rank"], "render_ms": slow["render_ms"],
                                "spread_ms": round(slow["render_ms"] - min(x["render_ms"] for x in ranks), 3),
                                "gather_and_host_ms": round(elapsed / args.steps * 1e3 - slow["render_ms"], 3)}
        if world == 1 and not args.no_cpu_baseline:
            # the host cores this process may use: min(nproc, cgroup quota); --cpu-threads overrides
            quota = cpu_quota()
            usable = os.cpu_count() or 1
            if quota:
                usable = max(1, min(usable, int(quota)))
            threads = args.cpu_threads or usable
            cb = cpu_baseline(path, W, H, args.cpu_spp, min(args.cpu_rows, H), args.cpu_stride, threads)
            cb["nproc"] = os.cpu_count()
            cb["cgroup_cpu_quota"] = quota
            line["cpu_baseline"] = cb
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
