#!/usr/bin/env python3
"""Do consecutive frames on two streams overlap on the device?  Renders rank 0 of
an N-way screen split (the per-GPU work at N GPUs) alternating two streams; run it
under `rocprofv3 --kernel-trace` and read the kernels' start/end stamps.
Usage: python tools/overlap_probe.py [--nranks 8] [--quad 0] [--frames 16]"""
import argparse
import ctypes
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from cpp_volume_rendering_amd import _native as N  # noqa: E402
from cpp_volume_rendering_amd import datasets as D  # noqa: E402
from cpp_volume_rendering_amd import screen_tiles as T  # noqa: E402
from cpp_volume_rendering_amd.renderer import Camera, Device, build_tf_rgbt, make_frame  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--nranks", type=int, default=8)
ap.add_argument("--quad", type=int, default=0)
ap.add_argument("--frames", type=int, default=16)
ap.add_argument("--order", type=int, default=1)
ap.add_argument("--streams", default="1,2,3,4")
ap.add_argument("--quads", default="")
a = ap.parse_args()
W = 1024
dev = Device(0)
dev.set_volume(D.marschner_lobb_u8(512), D.voxel_scale(512))
dev.set_transfer_function(build_tf_rgbt(D.BONSAI_TF_RGB, D.BONSAI_TF_ALPHA))
L = N.lib()
L.cvr_set_option(dev.handle, b"quad", a.quad)
L.cvr_set_option(dev.handle, b"tile_order", a.order)
frame = make_frame(Camera(**D.INITIAL_STATE_CAMERA), W, W, 32, 0, a.nranks) if a.nranks > 1 \
    else make_frame(Camera(**D.INITIAL_STATE_CAMERA), W, W)
npx = (T.tiles_for_rank(W, W, 32, 0, a.nranks) * 1024) if a.nranks > 1 else W * W
p = N.Rc1passParams()
p.step = 0.5
quads = [int(q) for q in a.quads.split(",")] if a.quads else [a.quad]
pool = [torch.cuda.Stream() for _ in range(8)]
for q in quads:
    L.cvr_set_option(dev.handle, b"quad", q)
    for ns in [int(x) for x in a.streams.split(",")]:
        st = pool[:ns]
        bufs = [torch.zeros((npx, 4), dtype=torch.float16, device="cuda") for _ in range(ns)]
        outs = [N.Output(b.data_ptr(), None, None, 1, 1) for b in bufs]
        best = 1e9
        for rep in range(3):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for i in range(a.frames):
                dev.set_stream(st[i % ns].cuda_stream)
                N.check(L.cvr_render_rc1pass(dev.handle, ctypes.byref(frame), ctypes.byref(p),
                                             ctypes.byref(outs[i % ns])), "render", dev.handle)
            torch.cuda.synchronize()
            best = min(best, (time.perf_counter() - t0) / a.frames * 1e3)
        print(f"nranks {a.nranks} quad {q} streams {ns}: {best:.4f} ms/frame", flush=True)
