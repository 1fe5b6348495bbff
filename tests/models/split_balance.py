#!/usr/bin/env python3
"""Per-rank work of the screen-tile split, from the oracle's per-pixel sample counts
(512^3 ML, 1024^2, bonsai TF; camera 'Initial State' and the other states of
data/#list_camera_states): samples per rank, max/mean over ranks, for the tile -> rank
assignments 'mod' (tile t -> t mod N, row-major) and 'rot s' (row ty rotated by s*ty
tiles before t mod N; with N | tiles-per-row that is rank (tx + s*ty) mod N).  CPU only.
Usage: python tests/models/split_balance.py [--tile 32,16] [--ranks 2,4,8] [--views 0,3,7]"""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from cpp_volume_rendering_amd import datasets as D  # noqa: E402
from cpp_volume_rendering_amd.renderer import read_camera_state  # noqa: E402
from oracle import oracle as O  # noqa: E402


def counts(view=0, n=512, W=1024):
    cache = f"/tmp/split_counts_v{view}.npy"
    if os.path.exists(cache):
        return np.load(cache)
    vox = D.marschner_lobb_u8(n)
    tf = O.tf_rgbt(O.tf_table_double(D.BONSAI_TF_RGB, D.BONSAI_TF_ALPHA))
    c = read_camera_state(os.path.join(ROOT, "tests", "golden", "list_camera_states"), view)
    cam = dict(eye=tuple(c.eye), center=tuple(c.center), up=tuple(c.up))
    _, cnt, _ = O.render_rc1pass(O.volume_r16f(vox), D.voxel_scale(n), tf, cam, W, W, 0.5)
    np.save(cache, cnt)
    return cnt


def rank_of_tiles(ntx, nty, N, s):
    """rank of every row-major tile: virtual index ty*ntx + (tx + s*ty) mod ntx, mod N."""
    t = np.arange(ntx * nty)
    tx, ty = t % ntx, t // ntx
    return (ty * ntx + (tx + s * ty) % ntx) % N


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--tile", default="32,16")
    ap.add_argument("--ranks", default="2,4,8")
    ap.add_argument("--views", default="0,3,7,12")
    ap.add_argument("--shifts", default="0,1,3,5")
    a = ap.parse_args()
    views = [int(v) for v in a.views.split(",")]
    cnts = {v: counts(v).astype(np.int64) for v in views}
    for T in [int(x) for x in a.tile.split(",")]:
        for N in [int(x) for x in a.ranks.split(",")]:
            for s in [int(x) for x in a.shifts.split(",")]:
                row = []
                for v in views:
                    cnt = cnts[v]
                    H, W = cnt.shape
                    ntx, nty = W // T, H // T
                    per = cnt.reshape(nty, T, ntx, T).sum(axis=(1, 3)).reshape(-1)
                    work = np.bincount(rank_of_tiles(ntx, nty, N, s), weights=per, minlength=N)
                    row.append(work.max() / work.mean())
                print(f"tile {T:2d} N {N} shift {s}: max/mean per view "
                      + " ".join(f"{x:.4f}" for x in row) + f"  worst {max(row):.4f}")
