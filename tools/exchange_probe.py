#!/usr/bin/env python3
"""The coded multi-GPU exchange's costs, measured on one GPU (DESIGN §7b projection).

Part A, a render rank: its share of the headline frame (512^3 ML, 1024^2, 16^2 tiles
on the diagonal lattice of an S-way split) rendered L frames per launch on D streams
with B buffer sets, each group followed on its stream by the exchange's one-launch
encode (cvr_encode_tiles with option encode_onepass), steady state (F frames, best
of 3).  Prints ms per frame with and without the encode, and the coded bytes of one
group against the raw 8 B per pixel.

Part B, rank 0: N contexts of this process joined by the in-process transport
(cvr_comm_init_local) push K groups through cvr_gather_tiles_n exactly as the
bench's ranks do (ranks 1..N-1 encode pre-rendered shares, rank 0 pulls the coded
streams and decodes every frame into its own image in one launch); run it under
`rocprofv3 --kernel-trace --stats` for the encode / decode kernel durations (on a
real node the encodes run on the other GPUs).  Prints the host time of one
cvr_gather_tiles_n call on a render rank and on rank 0.

Usage: python tools/exchange_probe.py [--ranks 2,4,8] [--frames 96] [--part AB]"""
import os
import sys

os.environ.setdefault("GPU_MAX_HW_QUEUES", "32")
import argparse  # noqa: E402
import ctypes  # noqa: E402
import json  # noqa: E402
import time  # noqa: E402

import torch  # noqa: E402

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from cpp_volume_rendering_amd import _native as N  # noqa: E402
from cpp_volume_rendering_amd import datasets as D  # noqa: E402
from cpp_volume_rendering_amd import screen_tiles as T  # noqa: E402
from cpp_volume_rendering_amd.renderer import Camera, Device, build_tf_rgbt, make_frame  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--ranks", default="2,4,8")
ap.add_argument("--frames", type=int, default=96)
ap.add_argument("--flp", type=int, default=4, help="frames per launch and per exchange")
ap.add_argument("--streams", type=int, default=4)
ap.add_argument("--sets", type=int, default=16)
ap.add_argument("--groups", type=int, default=24, help="part B: exchange groups pushed")
ap.add_argument("--part", default="AB")
ap.add_argument("--out", default="")
a = ap.parse_args()

n, W, tile, G = 512, 1024, 16, a.flp
L = N.lib()
tf = build_tf_rgbt(D.BONSAI_TF_RGB, D.BONSAI_TF_ALPHA)
vol, scale = D.marschner_lobb_u8(n), D.voxel_scale(n)
dev = Device(0)
dev.set_volume(vol, scale)
dev.set_transfer_function(tf)
h = dev.handle
cam = Camera(**D.INITIAL_STATE_CAMERA)
p = N.Rc1passParams()
res = []


def emit(d):
    print(json.dumps(d), flush=True)
    res.append(d)


def render_share(S, srank, bufs, totals=None):
    """One launch of G frames of split rank srank (of S) into bufs (G x tpr tiles)."""
    frs = (N.Frame * G)(*[make_frame(cam, W, W, tile, srank, S) for _ in range(G)])
    outs = (N.Output * G)(*[N.Output(bufs[j].data_ptr(), None, None, 1, N.FORMAT_RGBA16F)
                            for j in range(G)])
    N.check(L.cvr_render_rc1pass_frames(h, frs, G, ctypes.byref(p), outs), "render", h)


splits = []
for nr in (int(x) for x in a.ranks.split(",")):
    # the bench's root choice (bench.split_defaults): idle root at N >= 4; both measured
    splits.append((nr, True))
    if nr >= 3:
        splits.append((nr, False))

if "A" in a.part:
    N.check(L.cvr_set_option(h, b"encode_onepass", 1), "opt", h)
    for nr, root_renders in splits:
        S = nr if root_renders else nr - 1          # render ranks of the split
        srank = 0                                   # split rank 0: the largest share
        tpr = T.max_tiles_per_rank(W, W, tile, S)
        k = T.tiles_for_rank(W, W, tile, srank, S)
        streams = [torch.cuda.Stream() for _ in range(a.streams)]
        packed = [torch.zeros((G, tpr, tile, tile, 4), dtype=torch.float16, device="cuda")
                  for _ in range(a.sets)]
        code = [torch.zeros(L.cvr_tile_code_bound(tile, G * tpr) // 4, dtype=torch.int32,
                            device="cuda") for _ in range(a.sets)]
        nbytes = torch.zeros(a.sets, dtype=torch.int64, device="cuda")
        done = [None] * a.sets
        for enc in (False, True):
            best = 1e9
            for rep in range(3):
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                for i in range(a.frames // G):
                    s = streams[i % len(streams)]
                    kset = i % a.sets
                    if done[kset] is not None:
                        s.wait_event(done[kset])
                    L.cvr_set_stream(h, ctypes.c_void_p(s.cuda_stream))
                    render_share(S, srank, packed[kset])
                    if enc:
                        # the group's tiles are contiguous when k == tpr (G frames x k)
                        N.check(L.cvr_encode_tiles(h, packed[kset].data_ptr(), tile, G * tpr,
                                                   code[kset].data_ptr(),
                                                   nbytes[kset:kset + 1].data_ptr()), "encode", h)
                    ev = torch.cuda.Event()
                    ev.record(s)
                    done[kset] = ev
                torch.cuda.synchronize()
                best = min(best, (time.perf_counter() - t0) / (a.frames // G * G) * 1e3)
                done = [None] * a.sets
            emit(dict(part="A", nranks=nr, root_renders=root_renders, render_ranks=S,
                      tiles_per_rank=k, frames_per_launch=G, streams=a.streams, sets=a.sets,
                      frames=a.frames, encode=enc, ms_per_frame=round(best, 5)))
        raw = G * tpr * tile * tile * 8
        emit(dict(part="A", nranks=nr, root_renders=root_renders, coded_bytes_per_group=int(nbytes[0].item()),
                  raw_bytes_per_group=raw, ratio=round(raw / max(1, int(nbytes[0].item())), 2)))
    N.check(L.cvr_set_option(h, b"encode_onepass", 0), "opt", h)

if "B" in a.part:
    for nr, root_renders in splits:
        if nr < 2:
            continue
        idle = not root_renders
        S = nr - 1 if idle else nr
        tpr = T.max_tiles_per_rank(W, W, tile, S)
        # every render rank's share rendered once (rank 0's too when it renders)
        shares = []
        for r in range(S):
            b = torch.zeros((G, tpr, tile, tile, 4), dtype=torch.float16, device="cuda")
            render_share(S, r, b)
            shares.append(b)
        torch.cuda.synchronize()
        ctxs = [dev] + [Device(0) for _ in range(nr - 1)]
        try:
            arr = (ctypes.c_void_p * nr)(*[c.handle.value for c in ctxs])
            N.check(L.cvr_comm_init_local(arr, nr), "init_local")
            for c in ctxs:
                for kk, v in (("split_streams", a.streams), ("gather_sets", a.sets),
                              ("gather_root_idle", int(idle)), ("exchange_code", 1)):
                    N.check(L.cvr_set_option(c.handle, kk.encode(), v), kk, c.handle)
            streams = [[torch.cuda.Stream() for _ in range(a.streams)] for _ in range(nr)]
            gathered = [torch.zeros((nr, G, tpr, tile, tile, 4), dtype=torch.float16, device="cuda")
                        for _ in range(a.sets)]
            if root_renders:
                for gb in gathered:
                    gb[0].copy_(shares[0])
            images = [torch.zeros((W, W, 4), dtype=torch.float16, device="cuda") for _ in range(G)]
            imgs = (ctypes.c_void_p * G)(*[im.data_ptr() for im in images])
            torch.cuda.synchronize()
            host_r, host_0 = [], []
            t0 = time.perf_counter()
            for g in range(a.groups):
                for r in list(range(1, nr)) + [0]:
                    c = ctxs[r]
                    srank = r - 1 if idle else r
                    fr = make_frame(cam, W, W, tile, max(srank, 0), S)
                    N.check(L.cvr_set_stream(c.handle, streams[r][g % a.streams].cuda_stream), "s", c.handle)
                    buf = gathered[g % a.sets] if r == 0 else shares[srank]
                    th = time.perf_counter()
                    N.check(L.cvr_gather_tiles_n(c.handle, ctypes.byref(fr), G,
                                                 None if (r == 0 and idle) else buf.data_ptr(), tpr,
                                                 N.FORMAT_RGBA16F,
                                                 gathered[g % a.sets].data_ptr() if r == 0 else None,
                                                 imgs if r == 0 else None), "gather", c.handle)
                    (host_0 if r == 0 else host_r).append(time.perf_counter() - th)
            cur = torch.cuda.current_stream()
            for c in ctxs:
                L.cvr_set_stream(c.handle, ctypes.c_void_p(cur.cuda_stream))
                N.check(L.cvr_gather_sync(c.handle), "sync", c.handle)
            torch.cuda.synchronize()
            wall = time.perf_counter() - t0
            # the last group's frames against a one-context render of the whole frame
            full = torch.zeros((W, W, 4), dtype=torch.float16, device="cuda")
            L.cvr_set_stream(h, ctypes.c_void_p(cur.cuda_stream))
            N.check(L.cvr_render_rc1pass(h, ctypes.byref(make_frame(cam, W, W)), ctypes.byref(p),
                                         ctypes.byref(N.Output(full.data_ptr(), None, None, 1,
                                                               N.FORMAT_RGBA16F))), "full", h)
            torch.cuda.synchronize()
            exact = all(torch.equal(im.view(torch.int16), full.view(torch.int16)) for im in images)
            host_r.sort()
            host_0.sort()
            emit(dict(part="B", nranks=nr, root_renders=root_renders, groups=a.groups,
                      frames_per_group=G, bit_exact=exact,
                      host_us_render_rank_call_median=round(1e6 * host_r[len(host_r) // 2], 1)
                      if host_r else None,
                      host_us_rank0_call_median=round(1e6 * host_0[len(host_0) // 2], 1),
                      wall_ms_per_frame_all_ranks_on_one_gpu=round(wall / (a.groups * G) * 1e3, 4)))
        finally:
            for c in ctxs[1:]:
                c.close()
            N.check(L.cvr_comm_destroy(h), "destroy", h)

if a.out:
    json.dump(res, open(a.out, "w"), indent=1)
dev.close()
