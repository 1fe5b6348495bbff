#!/usr/bin/env python3
"""A/B timing of rc1pass kernel variants in ONE process, interleaved rounds
(methodology rule 24).  Every variant's image is checked bit-equal to the first
variant's.  Variant syntax: b<batch>o<tile_order>p<boost%>q<quad%>[c<tile_cost>][w<max waves/CU>][m<macro shift, 0 off>][s<skip_min_pct>][a<async_order>][i<order_interval>], e.g. b4o1p5q0a0i4.
Usage: python tools/ab_rc1pass.py [--size 512] [--res 1024] [--variants ...]"""
import argparse
import ctypes
import json
import os
import re
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from cpp_volume_rendering_amd import _native as N  # noqa: E402
from cpp_volume_rendering_amd import datasets as D  # noqa: E402
from cpp_volume_rendering_amd.renderer import Camera, Device, build_tf_rgbt, make_frame  # noqa: E402


def parse_variant(v):
    m = re.fullmatch(r"(?:L1)?b(\d)o(\d)p(\d+)q(\d+)(?:c(\d))?(?:w(\d+))?(?:m(\d))?(?:s(\d+))?(?:a(\d))?(?:i(\d+))?", v)
    if not m:
        raise ValueError(f"bad variant {v}")
    g = m.groups()
    d = (-1, -1, -1, -1, -1, -1)   # tile_cost, max_waves_cu, macro, skip_min_pct, async_order,
                                   # order_interval (-1: library default)
    return tuple(int(x) for x in g[:4]) + tuple(int(x) if x is not None else dflt
                                                for x, dflt in zip(g[4:], d))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--size", type=int, default=512)
    ap.add_argument("--res", type=int, default=1024)
    ap.add_argument("--field", default="ml")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--frames", type=int, default=20)
    ap.add_argument("--variants", default="b4o1p5q0,b2o1p5q0,b4o1p0q0,b4o0p0q0,b4o1p5q10")
    ap.add_argument("--phong", action="store_true")
    ap.add_argument("--tf-alpha", type=float, default=1.0, help="scale of the TF alpha points")
    ap.add_argument("--no-total", action="store_true", help="time frames without the sample counter")
    a = ap.parse_args()
    n, W = a.size, a.res
    vol = D.marschner_lobb_u8(n) if a.field == "ml" else D.blobs_u8(n)
    variants = a.variants.split(",")
    parsed = {v: parse_variant(v) for v in variants}
    s = torch.cuda.Stream()
    L0 = N.lib()
    dev = Device(0)
    dev.set_volume(vol, D.voxel_scale(n))
    dev.set_transfer_function(build_tf_rgbt(D.BONSAI_TF_RGB, tuple(
        (al * a.tf_alpha, iso) for al, iso in D.BONSAI_TF_ALPHA)))
    if a.phong:
        dev.set_gradient(1)
    dev.set_stream(s.cuda_stream)
    # library defaults, restored for the options a variant leaves unspecified
    defaults = {k: L0.cvr_get_option(dev.handle, k.encode())
                for k in ("tile_cost", "max_waves_cu", "macro", "skip_min_pct", "async_order",
                          "order_interval")}
    frame = make_frame(Camera(**D.INITIAL_STATE_CAMERA), W, W)
    p = N.Rc1passParams()
    p.apply_gradient_shading = int(a.phong)
    p.ka, p.kd, p.ks, p.shininess = 0.5, 0.5, 0.8, 30.0
    p.ispecular[:] = [1, 1, 1]
    p.light_pos[:] = list(D.LIGHT_LIST0_POSITION)
    img = torch.zeros((W, W, 4), dtype=torch.float32, device="cuda")
    tot = torch.zeros(1, dtype=torch.int64, device="cuda")
    out = N.Output(img.data_ptr(), None, tot.data_ptr(), 1)
    out_nt = N.Output(img.data_ptr(), None, None, 1)
    L = N.lib()

    def run(dev, frames, o=out):
        for _ in range(frames):
            N.check(L.cvr_render_rc1pass(dev.handle, ctypes.byref(frame), ctypes.byref(p),
                                         ctypes.byref(o)), "render", dev.handle)

    res = {v: [] for v in variants}
    ref_img = None
    S = None
    for _ in range(a.rounds):
        for v in variants:
            b, o, boost, quad, cost, mw, macro, skip, asy, oint = parsed[v]
            N.check(L.cvr_set_option(dev.handle, b"batch", b), "opt")
            N.check(L.cvr_set_option(dev.handle, b"tile_order", o), "opt")
            N.check(L.cvr_set_option(dev.handle, b"boost", boost), "opt")
            N.check(L.cvr_set_option(dev.handle, b"quad", quad), "opt")
            for key, val in (("tile_cost", cost), ("max_waves_cu", mw), ("macro", macro),
                             ("skip_min_pct", skip), ("async_order", asy),
                             ("order_interval", oint)):
                N.check(L.cvr_set_option(dev.handle, key.encode(),
                                         val if val >= 0 else defaults[key]), key)
            with torch.cuda.stream(s):
                run(dev, 3)   # warm up + learn the order
                tot.zero_()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(s)
                run(dev, a.frames, out_nt if a.no_total else out)
                e1.record(s)
            s.synchronize()
            res[v].append(e0.elapsed_time(e1) / a.frames)
            cur = img.cpu().numpy()
            if ref_img is None:
                ref_img = cur
                if a.no_total:
                    tot.zero_()
                    run(dev, 1)
                    torch.cuda.synchronize()
                    S = int(tot.item())
                else:
                    S = int(tot.item()) // a.frames
            else:
                assert np.array_equal(cur.view(np.uint32), ref_img.view(np.uint32)), f"{v} differs"
    rows = []
    for v in variants:
        med = float(np.median(res[v]))
        rows.append({"variant": v, "median_ms": round(med, 4), "min_ms": round(min(res[v]), 4),
                     "gsamples_s": round(S / med / 1e6, 1)})
    print(json.dumps({"size": n, "res": W, "field": a.field, "phong": a.phong,
                      "samples_per_frame": S, "rows": rows}, indent=1))


if __name__ == "__main__":
    main()
