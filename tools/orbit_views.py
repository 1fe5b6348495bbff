#!/usr/bin/env python3
"""Per-view kernel times of the rc1pass march over the 24 reference camera states
(data/#list_camera_states): each view rendered repeatedly (static: the LPT order and
XCD bands learned on the same view) and the views cycled one per frame (orbit: the
order always comes from the previous, different view).  One render stream, kernel
times from the library's HIP events.  Prints one JSON object.
Usage: python tools/orbit_views.py [--size 512] [--res 1024] [--frames 30]"""
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
    ap.add_argument("--res", type=int, default=1024)
    ap.add_argument("--frames", type=int, default=30)
    ap.add_argument("--orders", default="1,0,2", help="tile_order modes to measure")
    ap.add_argument("--stale-deg", type=int, default=-1, help="library option stale_deg (-1: default)")
    ap.add_argument("--smooth", default="0,1,3,10,30", help="degrees per frame of smooth orbits")
    a = ap.parse_args()
    n, W = a.size, a.res
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    path = os.path.join(root, "tests", "golden", "list_camera_states")
    cnt = ctypes.c_int()
    N.check(N.lib().cvr_read_camera_state(path.encode(), 0, N.Camera(), None, 0, cnt), "cams")
    cams = [read_camera_state(path, i) for i in range(cnt.value)]
    L = N.lib()
    dev = Device(0)
    dev.set_volume(D.marschner_lobb_u8(n), D.voxel_scale(n))
    dev.set_transfer_function(build_tf_rgbt(D.BONSAI_TF_RGB, D.BONSAI_TF_ALPHA))
    s = torch.cuda.Stream()
    dev.set_stream(s.cuda_stream)
    img = torch.zeros((W, W, 4), dtype=torch.float16, device="cuda")
    total = torch.zeros((1,), dtype=torch.int64, device="cuda")
    frames = [make_frame(c, W, W) for c in cams]
    p = N.Rc1passParams()

    def render(f, count=False):
        out = N.Output(img.data_ptr(), None, total.data_ptr() if count else None, 1,
                       N.FORMAT_RGBA16F)
        N.check(L.cvr_render_rc1pass(dev.handle, ctypes.byref(f), ctypes.byref(p),
                                     ctypes.byref(out)), "render", dev.handle)

    def kernel_times(k):
        kt = (ctypes.c_float * max(k, 1))()
        nk = ctypes.c_int()
        N.check(L.cvr_read_kernel_times(dev.handle, kt, k, ctypes.byref(nk)), "kt", dev.handle)
        return list(kt[:nk.value])

    samples = []
    for f in frames:
        total.zero_()
        render(f, True)
        torch.cuda.synchronize()
        samples.append(int(total.item()))
    for _ in range(200):                       # clocks
        render(frames[0])
    torch.cuda.synchronize()
    N.check(L.cvr_set_option(dev.handle, b"kernel_timing", 4096), "opt", dev.handle)
    if a.stale_deg >= 0:
        N.check(L.cvr_set_option(dev.handle, b"stale_deg", a.stale_deg), "opt", dev.handle)
    kernel_times(0)
    res = {"volume": n, "viewport": [W, W], "views": len(frames),
           "stale_deg": L.cvr_get_option(dev.handle, b"stale_deg"),
           "mean_samples": int(np.mean(samples)), "modes": {}}
    rows = [{"view": i, "samples": samples[i]} for i in range(len(frames))]
    # tile_order 1 (LPT from the previous frame), 0 (XCD bands), 2 (interleaved)
    for mode in (int(x) for x in a.orders.split(",")):
        N.check(L.cvr_set_option(dev.handle, b"tile_order", mode), "opt", dev.handle)
        static = []
        for f in frames:
            for _ in range(a.frames):
                render(f)
            torch.cuda.synchronize()
            static.append(float(np.median(kernel_times(a.frames)[a.frames // 3:])))
        rounds = max(3, a.frames // 3)
        for _ in range(rounds):
            for f in frames:
                render(f)
        torch.cuda.synchronize()
        kt = np.array(kernel_times(rounds * len(frames))).reshape(rounds, len(frames))
        orbit = [float(x) for x in np.median(kt[1:], axis=0)]
        for i in range(len(frames)):
            rows[i][f"static_o{mode}_ms"] = round(static[i], 4)
            rows[i][f"orbit_o{mode}_ms"] = round(orbit[i], 4)
        res["modes"][f"o{mode}"] = {"static_mean_ms": round(float(np.mean(static)), 4),
                                    "orbit_mean_ms": round(float(np.mean(orbit)), 4)}
    # smooth orbits: the headline camera rotated about the volume's y axis by `deg`
    # per frame (the order always comes from a view `deg` away)
    if a.smooth:
        import math
        c0 = D.INITIAL_STATE_CAMERA
        ex, ey, ez = c0["eye"]
        res["smooth"] = {}
        for deg in (float(x) for x in a.smooth.split(",")):
            nfr = 48
            orb = []
            for k in range(nfr):
                t = math.radians(deg * k)
                cam = Camera(eye=(ex * math.cos(t) + ez * math.sin(t), ey,
                                  -ex * math.sin(t) + ez * math.cos(t)),
                             center=c0["center"], up=c0["up"])
                orb.append(make_frame(cam, W, W))
            out = {}
            for mode in (int(x) for x in a.orders.split(",")):
                N.check(L.cvr_set_option(dev.handle, b"tile_order", mode), "opt", dev.handle)
                for f in orb:
                    render(f)
                torch.cuda.synchronize()
                kernel_times(0)
                for f in orb:
                    render(f)
                torch.cuda.synchronize()
                out[f"o{mode}_mean_ms"] = round(float(np.mean(kernel_times(nfr))), 4)
            res["smooth"][f"{deg:g}deg"] = out
    dev.close()
    res["rows"] = rows
    print(json.dumps(res))


if __name__ == "__main__":
    main()
