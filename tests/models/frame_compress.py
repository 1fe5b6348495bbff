#!/usr/bin/env python3
"""How far a lossless per-tile code would shrink the multi-GPU gather: the headline
frame (RGBA16F, the oracle's image) cut into the split's 16x16 tiles; per tile and
channel, the fp16 bit patterns minus the tile's minimum, stored at the bit width of
the largest difference (+ a 16-bit base and a 5-bit width per channel).  The
gather moves 8 B per pixel today.  Prints one JSON object."""
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import oracle as O  # noqa: E402  (test infrastructure, here as a CPU model of the frame)
from cpp_volume_rendering_amd import datasets as D  # noqa: E402


def main():
    n, W, T = 512, 1024, 16
    O.lib()
    vol = D.marschner_lobb_u8(n)
    sc = D.voxel_scale(n)
    tf = O.tf_rgbt(O.tf_table_double(D.BONSAI_TF_RGB, D.BONSAI_TF_ALPHA))
    rgba, _, _ = O.render_rc1pass(O.volume_r16f(vol), sc, tf, dict(D.INITIAL_STATE_CAMERA), W, W,
                                  O.default_step(sc))
    h = rgba.astype(np.float16).view(np.uint16).astype(np.int64)
    tiles = h.reshape(W // T, T, W // T, T, 4).transpose(0, 2, 1, 3, 4).reshape(-1, T * T, 4)
    span = tiles.max(axis=1) - tiles.min(axis=1)
    bits = np.where(span == 0, 0, np.floor(np.log2(np.maximum(span, 1))) + 1)
    comp_bits = float((bits.sum(axis=1) * T * T + 4 * (16 + 5)).sum())
    raw_bits = float(tiles.size * 16)
    print(json.dumps({"tile": T, "tiles": int(tiles.shape[0]),
                      "ratio": round(raw_bits / comp_bits, 2),
                      "mean_bits_per_channel": [round(float(b), 2) for b in bits.mean(axis=0)],
                      "constant_channel_tiles": [round(float(x), 3) for x in (span == 0).mean(axis=0)]}))


if __name__ == "__main__":
    main()
