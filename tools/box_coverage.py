#!/usr/bin/env python3
"""Screen coverage of the volume's box for the 24 reference camera states
(data/#list_camera_states): per view, the fraction of pixels whose ray line meets
the box (the slab test of ray_setup in float64), of 8x8 tiles holding such a pixel,
and of tiles inside the hit pixels' bounding rectangle -- what culling tiles
outside the box's screen projection could save (DESIGN §5″).  CPU only.
Usage: python tools/box_coverage.py [--size 512] [--res 1024]"""
import argparse
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from cpp_volume_rendering_amd.renderer import read_camera_state  # noqa: E402


def basis(eye, center, up):
    eye, c, up = (np.asarray(v, float) for v in (eye, center, up))
    f = c - eye
    f /= np.linalg.norm(f)
    s = np.cross(f, up)
    s /= np.linalg.norm(s)
    return s, np.cross(s, f), f


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--size", type=int, default=512)
    ap.add_argument("--res", type=int, default=1024)
    a = ap.parse_args()
    W = a.res
    hg = np.full(3, a.size / 2.0)
    path = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                        "tests", "golden", "list_camera_states")
    px = (np.arange(W) + 0.5) / W * 2 - 1
    vx, vy = np.meshgrid(px, px)
    rows = []
    for i in range(24):
        cam = read_camera_state(path, i)
        s, u, f = basis(cam.eye, cam.center, cam.up)
        th = np.tan(np.radians(cam.fovy_deg) / 2)
        d = (vx * th)[..., None] * s + (vy * th)[..., None] * u + f
        d /= np.linalg.norm(d, axis=-1, keepdims=True)
        e = np.asarray(cam.eye, float)
        with np.errstate(divide="ignore", invalid="ignore"):
            inv = 1 / d
            ta, tb = inv * (-hg - e), inv * (hg - e)
        hit = np.min(np.maximum(ta, tb), -1) > np.max(np.minimum(ta, tb), -1)
        tiles = hit.reshape(W // 8, 8, W // 8, 8).any(axis=(1, 3))
        ys, xs = np.nonzero(tiles)
        rect = (np.ptp(xs) + 1) * (np.ptp(ys) + 1) / tiles.size if len(xs) else 0.0
        rows.append({"view": i, "hit_pixels": round(float(hit.mean()), 4),
                     "hit_tiles": round(float(tiles.mean()), 4), "rect_tiles": round(float(rect), 4),
                     "eye_inside": bool(np.all(np.abs(e) < hg))})
    print(json.dumps({"volume": a.size, "res": W, "rows": rows}))


if __name__ == "__main__":
    main()
