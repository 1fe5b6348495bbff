#!/usr/bin/env python3
"""Lines per wave-load of the rc1pass march under different cell orders (CPU model).

Not product code.  For a camera of the headline workload it places every sample
of every ray (one lane per ray, 8x8 pixel tiles, lanes at the same sample index
march together -- the per-cell skip keeps them there, raymarch.hip march_ray CS 3)
and counts, per wave-load (tile, sample index), how many distinct 128-B lines the
64 lanes' 16-B cells fall in, for cell orders in bricks of bx x by x bz cells per
line (8 x 1 x 1 = today's x-fastest cell8 grid).  Ray lengths come from the
oracle's per-pixel sample counts (ERT included).  Positions are float32 numpy,
approximate to ~1e-4 texels: a statistic, not a parity claim.

  python tests/models/line_sim.py [--res 1024] [--size 512] [--camera N]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)


def lookat_dirs(eye, center, up, W, H, fovy_deg=45.0):
    eye = np.asarray(eye, np.float64)
    f = np.asarray(center, np.float64) - eye
    f /= np.linalg.norm(f)
    s = np.cross(f, np.asarray(up, np.float64))
    s /= np.linalg.norm(s)
    u = np.cross(s, f)
    t = np.tan(np.radians(fovy_deg) / 2)
    px = (np.arange(W) + 0.5) / W * 2 - 1
    py = (np.arange(H) + 0.5) / H * 2 - 1
    vx, vy = np.meshgrid(px * t * (W / H), py * t)
    d = vx[..., None] * s + vy[..., None] * u + f
    return d / np.linalg.norm(d, axis=-1, keepdims=True)


SHAPES = [(8, 1, 1), (4, 2, 1), (4, 1, 2), (2, 4, 1), (2, 2, 2), (2, 1, 4), (1, 8, 1),
          (1, 4, 2), (1, 2, 4), (1, 1, 8)]


def run(cam, W, n, counts, step=0.5, shapes=SHAPES):
    H = W
    hg = n / 2.0
    eye = np.asarray(cam["eye"], np.float64)
    d = lookat_dirs(cam["eye"], cam["center"], cam["up"], W, H)
    inv = 1.0 / d
    ta = inv * (-hg - eye)
    tb = inv * (hg - eye)
    tnear = np.maximum(np.minimum(ta, tb).max(-1), 0.0)
    o = eye + d * tnear[..., None] + hg - 0.5          # texel coordinates at the entry
    ty, tx = H // 8, W // 8
    res = {s: [0, 0] for s in shapes}                  # distinct lines, quad-lines
    seg64 = [0]
    nwl = 0
    for r0 in range(0, ty, 8):                          # 8 tile rows at a time
        r1 = min(ty, r0 + 8)
        sl = slice(r0 * 8, r1 * 8)
        c = counts[sl].astype(np.int64)
        kmax = int(c.max())
        if kmax == 0:
            continue
        # lane layout: tile (TY, TX), lane = ly * 8 + lx
        cc = c.reshape(r1 - r0, 8, tx, 8).transpose(0, 2, 1, 3).reshape(-1, 64)
        oo = o[sl].reshape(r1 - r0, 8, tx, 8, 3).transpose(0, 2, 1, 3, 4).reshape(-1, 64, 3)
        dd = d[sl].reshape(r1 - r0, 8, tx, 8, 3).transpose(0, 2, 1, 3, 4).reshape(-1, 64, 3)
        ntile = cc.shape[0]
        for k0 in range(0, kmax, 64):
            ks = np.arange(k0, min(kmax, k0 + 64))
            act = cc[:, None, :] > ks[None, :, None]              # tile, k, lane
            if not act.any():
                continue
            t = (ks + 0.5) * step
            p = oo[:, None, :, :] + dd[:, None, :, :] * t[None, :, None, None]
            ijk = np.floor(p).astype(np.int64) + 1                # cell index, 0..n
            ijk = np.clip(ijk, 0, n)
            grp = (np.arange(ntile)[:, None] * 64 + (ks - k0)[None, :])   # tile, k
            grp = np.broadcast_to(grp[..., None], act.shape)[act]
            quad = np.broadcast_to(np.arange(64)[None, None, :] // 4, act.shape)[act]
            cell = ijk[act]
            nwl += len(np.unique(grp))
            for s in shapes:
                bx, by, bz = s
                lx, ly, lz = cell[:, 0] // bx, cell[:, 1] // by, cell[:, 2] // bz
                line = (lz * ((n + 8) // by + 1) + ly) * ((n + 8) // bx + 1) + lx
                key = grp.astype(np.int64) * (1 << 28) + line
                res[s][0] += len(np.unique(key))
                keyq = (grp.astype(np.int64) * 16 + quad) * (1 << 28) + line
                res[s][1] += len(np.unique(keyq))
            seg = (cell[:, 2] * (n + 1) + cell[:, 1]) * ((n + 4) // 4 + 1) + cell[:, 0] // 4
            seg64[0] += len(np.unique(grp.astype(np.int64) * (1 << 30) + seg))
    return {"wave_loads": nwl,
            "lines_per_wave_load": {f"{s[0]}x{s[1]}x{s[2]}": round(res[s][0] / nwl, 3) for s in shapes},
            "quad_lines_per_wave_load": {f"{s[0]}x{s[1]}x{s[2]}": round(res[s][1] / nwl, 3)
                                         for s in shapes},
            "x_fastest_64B_segments_per_wave_load": round(seg64[0] / nwl, 3)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--res", type=int, default=1024)
    ap.add_argument("--size", type=int, default=512)
    ap.add_argument("--camera", type=int, default=-1, help="index into list_camera_states (-1: Initial State)")
    a = ap.parse_args()
    import oracle as O
    from cpp_volume_rendering_amd import datasets as D
    from cpp_volume_rendering_amd.renderer import build_tf_rgbt, read_camera_state
    vol = D.marschner_lobb_u8(a.size)
    tf = build_tf_rgbt(D.BONSAI_TF_RGB, D.BONSAI_TF_ALPHA)
    if a.camera < 0:
        cam = dict(D.INITIAL_STATE_CAMERA)
    else:
        c = read_camera_state(os.path.join(ROOT, "tests", "golden", "list_camera_states"), a.camera)
        cam = dict(eye=c.eye, center=c.center, up=c.up)
    _, cnt, S = O.render_rc1pass(O.volume_r16f(vol), D.voxel_scale(a.size), tf, cam, a.res, a.res,
                                 O.default_step(D.voxel_scale(a.size)))
    out = run(cam, a.res, a.size, cnt)
    out.update({"camera": cam, "samples": S, "res": a.res, "size": a.size})
    print(json.dumps(out))


if __name__ == "__main__":
    main()
