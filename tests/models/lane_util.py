#!/usr/bin/env python3
"""Lane utilisation of the one-ray-per-lane march from ray lengths alone: the
oracle's per-pixel sample counts of the headline frame, grouped by 8x8 wave tile;
a wave runs as long as its longest ray, so the filled lane-slots are sum(count) /
(64 * max(count)) per tile (and the same in 4-sample batches).  The bound on what
refilling finished lanes with new rays (persistent lanes) could recover (DESIGN §5″).
CPU only (the oracle, ~4 s on 8 threads).  Usage: python tests/models/lane_util.py"""
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import oracle as O  # noqa: E402  (test infrastructure: the checker, used here as a CPU model)
from cpp_volume_rendering_amd import datasets as D  # noqa: E402


def main():
    n, W = 512, 1024
    O.lib()
    vol = D.marschner_lobb_u8(n)
    sc = D.voxel_scale(n)
    tf = O.tf_rgbt(O.tf_table_double(D.BONSAI_TF_RGB, D.BONSAI_TF_ALPHA))
    _, cnt, total = O.render_rc1pass(O.volume_r16f(vol), sc, tf, dict(D.INITIAL_STATE_CAMERA), W, W,
                                     O.default_step(sc))
    c = cnt.reshape(W // 8, 8, W // 8, 8).transpose(0, 2, 1, 3).reshape(-1, 64).astype(np.int64)
    b = (c + 3) // 4
    print(json.dumps({"samples": int(total), "tiles": int(c.shape[0]),
                      "lane_util_samples": round(float(c.sum() / (64 * c.max(1)).sum()), 4),
                      "lane_util_batches": round(float(b.sum() / (64 * b.max(1)).sum()), 4)}))


if __name__ == "__main__":
    main()
