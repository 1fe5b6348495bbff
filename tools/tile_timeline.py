#!/usr/bin/env python3
"""Per-tile timeline of one rc1pass frame (tile_stats diagnostics): how long each
8x8 tile ran, its longest ray, when it started, and how many tiles were in flight
over time.  Saves gpurun_out/tile_timeline_<tag>.npz and prints a summary."""
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
from cpp_volume_rendering_amd.renderer import Camera, Device, build_tf_rgbt, make_frame  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--size", type=int, default=512)
    ap.add_argument("--res", type=int, default=1024)
    ap.add_argument("--order", type=int, default=1)
    ap.add_argument("--boost", type=int, default=5)
    ap.add_argument("--batch", type=int, default=4)
    ap.add_argument("--quad", type=int, default=0)
    ap.add_argument("--keep", type=int, default=0, help="render only the longest N entries per band")
    ap.add_argument("--cell-skip", type=int, default=2)
    ap.add_argument("--tag", default="run")
    a = ap.parse_args()
    n, W = a.size, a.res
    dev = Device(0)
    L = N.lib()
    for k, v in (("tile_order", a.order), ("boost", a.boost),
                 ("batch", a.batch), ("quad", a.quad), ("debug_keep", a.keep), ("tile_stats", 1),
                 ("cell_skip", a.cell_skip)):
        N.check(L.cvr_set_option(dev.handle, k.encode(), v), k)
    dev.set_volume(D.marschner_lobb_u8(n), D.voxel_scale(n))
    dev.set_transfer_function(build_tf_rgbt(D.BONSAI_TF_RGB, D.BONSAI_TF_ALPHA))
    s = torch.cuda.Stream()
    dev.set_stream(s.cuda_stream)
    frame = make_frame(Camera(**D.INITIAL_STATE_CAMERA), W, W)
    p = N.Rc1passParams()
    img = torch.zeros((W, W, 4), dtype=torch.float32, device="cuda")
    out = N.Output(img.data_ptr(), None, None, 1)
    def render(n):
        for _ in range(n):
            N.check(L.cvr_render_rc1pass(dev.handle, ctypes.byref(frame), ctypes.byref(p),
                                         ctypes.byref(out)), "render", dev.handle)
        s.synchronize()

    def stats():
        nt = ctypes.c_int()
        N.check(L.cvr_copy_tile_stats(dev.handle, None, 0, ctypes.byref(nt)), "stats")
        st = np.zeros((nt.value, 4), np.uint64)
        N.check(L.cvr_copy_tile_stats(dev.handle, st.ctypes.data, nt.value, ctypes.byref(nt)),
                "stats")
        return st

    render(4)
    before = stats()
    render(1)
    st = stats()
    ran = np.nonzero(st[:, 0] != before[:, 0])[0]   # tiles the last frame rendered
    st = st[ran]
    t0 = st[:, 0].min()
    start = (st[:, 0] - t0).astype(np.float64) / 100.0   # us
    end = (st[:, 1] - t0).astype(np.float64) / 100.0
    dur = end - start
    iters = st[:, 2].astype(np.float64)
    span = end.max()
    grid = np.linspace(0, span, 200)
    inflight = np.array([np.sum((start <= g) & (end > g)) for g in grid])
    top = np.argsort(-dur)[:10]
    us_per_iter = dur[iters > 20] / iters[iters > 20]
    os.makedirs("gpurun_out", exist_ok=True)
    np.savez(f"gpurun_out/tile_timeline_{a.tag}.npz", stats=st)
    summ = {
        "tag": a.tag, "tiles": int(len(ran)), "span_us": round(float(span), 2),
        "tile_dur_us": {"mean": round(float(dur.mean()), 2), "p50": round(float(np.median(dur)), 2),
                        "p99": round(float(np.percentile(dur, 99)), 2), "max": round(float(dur.max()), 2)},
        "us_per_iteration": {"p10": round(float(np.percentile(us_per_iter, 10)), 4),
                             "p50": round(float(np.median(us_per_iter)), 4),
                             "p90": round(float(np.percentile(us_per_iter, 90)), 4)},
        "longest_tiles": [{"tile": int(ran[i]), "start_us": round(float(start[i]), 1),
                           "dur_us": round(float(dur[i]), 1), "iters": int(iters[i])} for i in top],
        "inflight_profile": [int(x) for x in inflight[::10]],
        "last_start_us": round(float(start.max()), 1),
    }
    print(json.dumps(summ, indent=1))


if __name__ == "__main__":
    main()
