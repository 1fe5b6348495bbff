#!/usr/bin/env python3
"""Per-rank cost of the screen-tile split, measured on ONE GPU.

At N GPUs every rank renders the packed tiles of one rank of the split
(cvr_frame.rank/nranks).  This renders exactly that work on one device for
rank 0 and rank N-1, for several quad (sample-parallel) shares, and reports
the kernel time (library HIP events), the back-to-back frame time (wall clock
over many frames, launch overhead included) and the host time of one render
call.  Images are checked bit-equal across variants.
Usage: python tools/split_probe.py [--ranks 1,2,4,8] [--quads 0,25,100]"""
import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from cpp_volume_rendering_amd import _native as N  # noqa: E402
from cpp_volume_rendering_amd import datasets as D  # noqa: E402
from cpp_volume_rendering_amd import screen_tiles as T  # noqa: E402
from cpp_volume_rendering_amd.renderer import Camera, Device, build_tf_rgbt, make_frame  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--size", type=int, default=512)
    ap.add_argument("--res", type=int, default=1024)
    ap.add_argument("--tile", type=int, default=32)
    ap.add_argument("--ranks", default="1,2,4,8")
    ap.add_argument("--quads", default="0,10,25,50,100")
    ap.add_argument("--frames", type=int, default=40)
    ap.add_argument("--fmt", type=int, default=1)
    a = ap.parse_args()
    n, W = a.size, a.res
    vol = D.marschner_lobb_u8(n)
    s = torch.cuda.Stream()
    streams2 = [torch.cuda.Stream(), torch.cuda.Stream()]
    L = N.lib()
    dev = Device(0)
    dev.set_volume(vol, D.voxel_scale(n))
    dev.set_transfer_function(build_tf_rgbt(D.BONSAI_TF_RGB, D.BONSAI_TF_ALPHA))
    dev.set_stream(s.cuda_stream)
    cam = Camera(**D.INITIAL_STATE_CAMERA)
    from cpp_volume_rendering_amd.renderer import RayCasting1Pass
    params = N.Rc1passParams()
    params.step = 0.5
    params.apply_gradient_shading = 0
    res = []
    dtype = torch.float16 if a.fmt == 1 else torch.float32
    for nr in [int(x) for x in a.ranks.split(",")]:
        for rank in sorted({0, nr - 1}):
            if nr == 1:
                frame = make_frame(cam, W, W)
                npx = W * W
            else:
                frame = make_frame(cam, W, W, a.tile, rank, nr)
                npx = T.tiles_for_rank(W, W, a.tile, rank, nr) * a.tile * a.tile
            buf = torch.zeros((npx, 4), dtype=dtype, device="cuda")
            ref = None
            for q in [int(x) for x in a.quads.split(",")]:
                L.cvr_set_option(dev.handle, b"quad", q)
                out = N.Output(buf.data_ptr(), None, None, 1, a.fmt)
                with torch.cuda.stream(s):
                    for _ in range(12):
                        N.check(L.cvr_render_rc1pass(dev.handle, ctypes.byref(frame),
                                                     ctypes.byref(params), ctypes.byref(out)),
                                "render", dev.handle)
                    s.synchronize()
                    img = buf.cpu().numpy().copy()
                    ok = True if ref is None else bool(np.array_equal(img.view(np.uint16 if a.fmt else np.uint32), ref.view(np.uint16 if a.fmt else np.uint32)))
                    if ref is None:
                        ref = img
                    # back-to-back wall time and host time per call (twice: the first
                    # pass after a configuration change may include one-time work)
                    walls = []
                    for rep in range(2):
                        s.synchronize()
                        t0 = time.perf_counter()
                        host = 0.0
                        for _ in range(a.frames):
                            h0 = time.perf_counter()
                            N.check(L.cvr_render_rc1pass(dev.handle, ctypes.byref(frame),
                                                         ctypes.byref(params), ctypes.byref(out)),
                                    "render", dev.handle)
                            host += time.perf_counter() - h0
                        s.synchronize()
                        walls.append((time.perf_counter() - t0) / a.frames * 1e3)
                    wall = walls[-1]
                    # two streams alternating (frames overlap on the device)
                    buf2 = torch.zeros_like(buf)
                    out2 = N.Output(buf2.data_ptr(), None, None, 1, a.fmt)
                    w2 = []
                    for rep in range(2):
                        torch.cuda.synchronize()
                        t0 = time.perf_counter()
                        for i in range(a.frames):
                            dev.set_stream(streams2[i & 1].cuda_stream)
                            N.check(L.cvr_render_rc1pass(dev.handle, ctypes.byref(frame),
                                                         ctypes.byref(params),
                                                         ctypes.byref(out if i & 1 else out2)),
                                    "render", dev.handle)
                        torch.cuda.synchronize()
                        w2.append((time.perf_counter() - t0) / a.frames * 1e3)
                    dev.set_stream(s.cuda_stream)
                    img2 = buf2.cpu().numpy()
                    ok = ok and bool(np.array_equal(img2.view(np.uint16 if a.fmt else np.uint32), ref.view(np.uint16 if a.fmt else np.uint32)))
                    L.cvr_set_option(dev.handle, b"kernel_timing", a.frames)
                    for _ in range(a.frames):
                        N.check(L.cvr_render_rc1pass(dev.handle, ctypes.byref(frame),
                                                     ctypes.byref(params), ctypes.byref(out)),
                                "render", dev.handle)
                    s.synchronize()
                    kt = (ctypes.c_float * a.frames)()
                    nk = ctypes.c_int()
                    N.check(L.cvr_read_kernel_times(dev.handle, kt, a.frames, ctypes.byref(nk)),
                            "kt", dev.handle)
                    L.cvr_set_option(dev.handle, b"kernel_timing", 0)
                r = {"nranks": nr, "rank": rank, "quad": q, "kernel_ms": round(float(np.mean(kt[:nk.value])), 4),
                     "kernel_min_ms": round(float(np.min(kt[:nk.value])), 4),
                     "frame_ms": round(wall, 4), "frame_ms_first_pass": round(walls[0], 4),
                     "frame_ms_2streams": round(w2[-1], 4),
                     "host_us_per_call": round(host / a.frames * 1e6, 1),
                     "bit_equal": ok}
                print(json.dumps(r), flush=True)
                res.append(r)
    L.cvr_set_option(dev.handle, b"quad", 0)
    os.makedirs("gpurun_out", exist_ok=True)
    with open("gpurun_out/split_probe.json", "w") as f:
        json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
