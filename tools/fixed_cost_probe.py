#!/usr/bin/env python3
"""The rc1pass march's per-frame fixed cost: lone-frame kernel times (library HIP
events, one render stream, the learned order) of views whose rays do little work —
every ray missing the box, every ray ending after 8 samples (the camera inside
opaque material, camera state 5) — beside the headline view, at several viewport
sizes.  With the work per ray near zero, the kernel time is the cost of the
workgroups themselves (launch, TF fill, ray set-up, stores, tail).
Prints one JSON object.  Usage: python tools/fixed_cost_probe.py [--frames 40]"""
import argparse
import ctypes
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from cpp_volume_rendering_amd import _native as N  # noqa: E402
from cpp_volume_rendering_amd import datasets as D  # noqa: E402
from cpp_volume_rendering_amd.renderer import (Camera, Device, build_tf_rgbt,  # noqa: E402
                                               make_frame, read_camera_state)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--size", type=int, default=512)
    ap.add_argument("--frames", type=int, default=40)
    ap.add_argument("--res", default="512,1024,2048")
    a = ap.parse_args()
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    path = os.path.join(root, "tests", "golden", "list_camera_states")
    views = {"miss": Camera(eye=(0.0, 0.0, 2000.0), center=(0.0, 0.0, 4000.0), up=(0.0, 1.0, 0.0)),
             "inside8": read_camera_state(path, 5),
             "headline": read_camera_state(path, 0),
             "far_flower": read_camera_state(path, 15)}
    L = N.lib()
    dev = Device(0)
    dev.set_volume(D.marschner_lobb_u8(a.size), D.voxel_scale(a.size))
    dev.set_transfer_function(build_tf_rgbt(D.BONSAI_TF_RGB, D.BONSAI_TF_ALPHA))
    s = torch.cuda.Stream()
    dev.set_stream(s.cuda_stream)
    total = torch.zeros((1,), dtype=torch.int64, device="cuda")
    p = N.Rc1passParams()

    def kernel_times(k):
        kt = (ctypes.c_float * max(k, 1))()
        nk = ctypes.c_int()
        N.check(L.cvr_read_kernel_times(dev.handle, kt, k, ctypes.byref(nk)), "kt", dev.handle)
        return list(kt[:nk.value])

    N.check(L.cvr_set_option(dev.handle, b"kernel_timing", 4096), "opt", dev.handle)
    res = {"volume": a.size, "frames": a.frames, "rows": []}
    for W in (int(x) for x in a.res.split(",")):
        img = torch.zeros((W, W, 4), dtype=torch.float16, device="cuda")

        def render(f, count=False):
            out = N.Output(img.data_ptr(), None, total.data_ptr() if count else None, 1,
                           N.FORMAT_RGBA16F)
            N.check(L.cvr_render_rc1pass(dev.handle, ctypes.byref(f), ctypes.byref(p),
                                         ctypes.byref(out)), "render", dev.handle)

        for name, cam in views.items():
            f = make_frame(cam, W, W)
            total.zero_()
            render(f, True)
            torch.cuda.synchronize()
            smp = int(total.item())
            for _ in range(100):
                render(f)
            torch.cuda.synchronize()
            kernel_times(0)
            for _ in range(a.frames):
                render(f)
            torch.cuda.synchronize()
            kt = kernel_times(a.frames)
            row = {"res": W, "view": name, "samples": smp, "tiles": (W // 8) ** 2,
                   "kernel_ms_median": round(float(np.median(kt)), 5),
                   "kernel_ms_min": round(float(np.min(kt)), 5)}
            res["rows"].append(row)
            print(json.dumps(row), file=sys.stderr, flush=True)
    dev.close()
    print(json.dumps(res))


if __name__ == "__main__":
    main()
