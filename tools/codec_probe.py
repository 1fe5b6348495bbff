#!/usr/bin/env python3
"""The per-tile code (cvr_encode_tiles / cvr_decode_tiles) on the headline frame's
screen-tile shares: for N ranks, every rank's packed RGBA16F tiles (16x16 tiles,
the diagonal lattice of the split) rendered on one GPU, encoded and decoded, with
the stream bytes against the raw 8 B per pixel and the kernel times (HIP events,
median of repeats).  The projection needs the bytes into rank 0.
Prints one JSON object.  Usage: python tools/codec_probe.py [--ranks 2,4,8]"""
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
from cpp_volume_rendering_amd import screen_tiles as T  # noqa: E402
from cpp_volume_rendering_amd.renderer import Camera, Device, build_tf_rgbt, make_frame  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ranks", default="2,4,8")
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    n, W, tile = 512, 1024, 16
    L = N.lib()
    dev = Device(0)
    dev.set_volume(D.marschner_lobb_u8(n), D.voxel_scale(n))
    dev.set_transfer_function(build_tf_rgbt(D.BONSAI_TF_RGB, D.BONSAI_TF_ALPHA))
    s = torch.cuda.Stream()
    dev.set_stream(s.cuda_stream)
    cam = Camera(**D.INITIAL_STATE_CAMERA)
    res = {"res": W, "tile": tile, "rows": []}
    p = N.Rc1passParams()
    e0, e1, e2 = (torch.cuda.Event(enable_timing=True) for _ in range(3))
    for nr in (int(x) for x in a.ranks.split(",")):
        raw = coded = 0
        enc_ms, dec_ms = [], []
        for r in range(nr):
            k = T.tiles_for_rank(W, W, tile, r, nr)
            tiles = torch.zeros((k, tile, tile, 4), dtype=torch.float16, device="cuda")
            out = N.Output(tiles.data_ptr(), None, None, 1, N.FORMAT_RGBA16F)
            frame = make_frame(cam, W, W, tile, r, nr)
            N.check(L.cvr_render_rc1pass(dev.handle, ctypes.byref(frame), ctypes.byref(p), ctypes.byref(out)),
                    "render", h := dev.handle)
            stream = torch.zeros(L.cvr_tile_code_bound(tile, k) // 4, dtype=torch.int32, device="cuda")
            nbytes = torch.zeros(1, dtype=torch.int64, device="cuda")
            back = torch.zeros_like(tiles)
            for _ in range(a.reps):
                with torch.cuda.stream(s):
                    e0.record(s)
                    N.check(L.cvr_encode_tiles(h, tiles.data_ptr(), tile, k, stream.data_ptr(), nbytes.data_ptr()),
                            "encode", h)
                    e1.record(s)
                    N.check(L.cvr_decode_tiles(h, stream.data_ptr(), tile, k, back.data_ptr()), "decode", h)
                    e2.record(s)
                s.synchronize()
                enc_ms.append(e0.elapsed_time(e1))
                dec_ms.append(e1.elapsed_time(e2))
            assert torch.equal(back.view(torch.int16), tiles.view(torch.int16)), (nr, r)
            raw += tiles.numel() * 2
            coded += int(nbytes.item())
        res["rows"].append({"ranks": nr, "raw_bytes": raw, "coded_bytes": coded,
                            "ratio": round(raw / coded, 2),
                            "encode_ms_median_per_rank": round(float(np.median(enc_ms)), 4),
                            "decode_ms_median_per_rank": round(float(np.median(dec_ms)), 4)})
        print(json.dumps(res["rows"][-1]), file=sys.stderr, flush=True)
    dev.close()
    print(json.dumps(res))


if __name__ == "__main__":
    main()
