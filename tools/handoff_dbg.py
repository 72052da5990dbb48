#!/usr/bin/env python3
"""Hand-off diagnostics (debug build, RT_LIB=...): one 1-GPU headline frame, then the first
recorded device check (rt_debug_take), printed."""
import os, sys, time
import torch
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
rt = bench.import_pkg()
rt.debug_raise = False
path = bench.load_scenes_module().ensure_scene("sponza", "/tmp/rt_scenes")
spp = int(sys.argv[1]) if len(sys.argv) > 1 else 256
scene = rt.Scene.load(path, 1920, 1080, spp)
scene.upload(0)
out = torch.zeros(1920 * 1080 * 3, dtype=torch.float32, device="cuda")
for k in range(2):
    t = time.time()
    st = scene.render_device(out.data_ptr(), torch.cuda.current_stream().cuda_stream, spp=spp, stats=True)
    torch.cuda.synchronize()
    w = rt.debug_take()
    print(f"frame {k}: {st['render_ms']:.1f} ms schedule {st['schedule']} debug word {w:#x} code {w >> 56}", flush=True)
