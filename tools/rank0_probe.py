#!/usr/bin/env python3
"""Rank 0's whole frame loop at N ranks, emulated on one GPU: rank 0's
share of the headline frame (512^3 ML, 1024^2) rendered L frames per launch
(cvr_render_rc1pass_frames) into its block of the gather buffer, then on a
separate communication stream the other N-1 ranks' bytes LANDING in the gather
buffer (a device-to-device copy of the same size stands in for RCCL's receive;
the xGMI transfer time itself is not on one GPU and is bounded separately) and
the unpack of every frame into the image (cvr_unpack_tiles_device_n), with the
render stream of a buffer set waiting for its previous exchange, as
cvr_gather_tiles_n orders them.  Host calls included.  Prints ms per frame with
and without the exchange, for F frames (20 = the driver's command; 96 = steady).
Usage: python tools/rank0_probe.py [--nranks 8] [--streams 4] [--frames-per-launch 4]
       [--frames 20,96] [--out FILE]"""
import os
import sys

os.environ["GPU_MAX_HW_QUEUES"] = (sys.argv[sys.argv.index("--hwq") + 1]
                                   if "--hwq" in sys.argv else "32")
import argparse  # noqa: E402
import ctypes  # noqa: E402
import json  # noqa: E402
import time  # noqa: E402

import torch  # noqa: E402

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from cpp_volume_rendering_amd import _native as N  # noqa: E402
from cpp_volume_rendering_amd import datasets as D  # noqa: E402
from cpp_volume_rendering_amd import screen_tiles as T  # noqa: E402
from cpp_volume_rendering_amd.renderer import (Camera, DataManager, RayCasting1Pass,  # noqa: E402
                                               RC1PConeTracingDirOcclusionShading,
                                               RC1PExtinctionBasedShading, RenderingParameters,
                                               build_ext_lut, build_tf_rgbt, make_frame)

ap = argparse.ArgumentParser()
ap.add_argument("--nranks", type=int, default=8)
ap.add_argument("--streams", default="4")
ap.add_argument("--frames-per-launch", default="4")
ap.add_argument("--frames", default="20,96")
ap.add_argument("--tile", type=int, default=16)
ap.add_argument("--hwq", default="32")
ap.add_argument("--out", default="")
ap.add_argument("--sets", default="0", help="buffer sets (0: one per stream); a set is reused "
                "after its previous exchange")
ap.add_argument("--reserve-cus", default="0",
                help="render streams created with a CU mask that leaves this many CUs "
                     "(the mask's top bits) to the exchange (hipExtStreamCreateWithCUMask)")
ap.add_argument("--render-nranks", default="0",
                help="rank 0 renders its share of a split over this many ranks (0: --nranks; "
                     "-1: renders nothing, a gather-only root) -- a lighter root share")
ap.add_argument("--renderer", choices=["rc1pass", "dos", "ebs"], default="rc1pass",
                help="dos / ebs: configs 4 / 5 (one frame per launch)")
ap.add_argument("--parts", default="both", choices=["both", "copy", "unpack"],
                help="which part of the emulated exchange runs (diagnostics)")
a = ap.parse_args()

n, W = (1024, 1024) if a.renderer == "ebs" else ((512, 2048) if a.renderer == "dos" else (512, 1024))
dm = DataManager()
dm.SetVolume(D.marschner_lobb_u8(n), D.voxel_scale(n))
dm.SetTransferFunction(build_tf_rgbt(D.BONSAI_TF_RGB, D.BONSAI_TF_ALPHA),
                       build_tf_rgbt(D.BONSAI_TF_RGB, D.BONSAI_TF_ALPHA, extinction_input=True))
if a.renderer == "dos":                      # bench.py --renderer dos (config 4)
    r = RC1PConeTracingDirOcclusionShading(0)
    r.glsl_apply_shadow = True
elif a.renderer == "ebs":                    # bench.py --renderer ebs (config 5)
    dm.SetExtinctionTable(build_ext_lut(D.BONSAI_TF_RGB, D.BONSAI_TF_ALPHA))
    r = RC1PExtinctionBasedShading(0)
else:
    r = RayCasting1Pass(0)
r.SetExternalResources(dm, RenderingParameters(W, W, light_position=D.LIGHT_LIST0_POSITION))
assert r.Init(W, W)
cam = Camera(**D.INITIAL_STATE_CAMERA)
r.PrepareRender(cam)
L = N.lib()
h = r.device.handle
NR, tile = a.nranks, a.tile
tpr = T.max_tiles_per_rank(W, W, tile, NR)
frame = make_frame(cam, W, W, tile, 0, NR)
comm = torch.cuda.Stream(priority=-1)
res = []
import itertools  # noqa: E402
_hip = ctypes.CDLL("libamdhip64.so")
NCU = torch.cuda.get_device_properties(0).multi_processor_count


def masked_stream(reserve):
    """A HIP stream whose kernels run on all CUs but the mask's top `reserve` bits."""
    if reserve <= 0:
        return torch.cuda.Stream()
    words = (NCU + 31) // 32
    bits = [1 if i < NCU - reserve else 0 for i in range(words * 32)]
    mask = (ctypes.c_uint32 * words)(*[sum(bits[w * 32 + b] << b for b in range(32)) for w in range(words)])
    st = ctypes.c_void_p()
    rc = _hip.hipExtStreamCreateWithCUMask(ctypes.byref(st), ctypes.c_uint32(words), mask)
    assert rc == 0, f"hipExtStreamCreateWithCUMask: {rc}"
    return torch.cuda.ExternalStream(st.value)


for G, ns, nsets, rsv, rn in itertools.product([int(x) for x in a.frames_per_launch.split(",")],
                                               [int(x) for x in a.streams.split(",")],
                                               [int(x) for x in a.sets.split(",")],
                                               [int(x) for x in a.reserve_cus.split(",")],
                                               [int(x) for x in a.render_nranks.split(",")]):
    if True:
        rframe = make_frame(cam, W, W, tile, 0, rn if rn > 0 else NR)
        pool = [masked_stream(rsv) for _ in range(ns)]
        nsets = nsets or ns
        # buffer set per stream: the gather buffer (NR blocks of G frames) + an image
        gathered = [torch.zeros((NR, G, tpr, tile, tile, 4), dtype=torch.float16, device="cuda")
                    for _ in range(nsets)]
        remote = torch.ones((NR - 1, G, tpr, tile, tile, 4), dtype=torch.float16, device="cuda")
        image = torch.zeros((W, W, 4), dtype=torch.float16, device="cuda")
        # rank 0 renders into the start of its block (a lighter share fits in it)
        outs = [[N.Output(g[0, j].data_ptr(), None, None, 1, N.FORMAT_RGBA16F) for j in range(G)]
                for g in gathered]
        done = [None] * nsets
        for F in [int(x) for x in a.frames.split(",")]:
            for exch in (False, True):
                best = 1e9
                for rep in range(3):
                    torch.cuda.synchronize()
                    t0 = time.perf_counter()
                    for i in range(F // G):
                        k = i % nsets
                        s = pool[i % ns]
                        if done[k] is not None:
                            s.wait_event(done[k])          # the set's previous exchange
                        L.cvr_set_stream(h, ctypes.c_void_p(s.cuda_stream))
                        if rn >= 0 and G > 1:
                            r.render_frames_to([rframe] * G, outs[k])
                        elif rn >= 0:
                            r.render_to(rframe, outs[k][0])
                        if not exch:
                            continue
                        if rn >= 0:
                            ev = torch.cuda.Event()
                            ev.record(s)
                            comm.wait_event(ev)
                        if a.parts != "unpack":
                            with torch.cuda.stream(comm):
                                gathered[k][1:].copy_(remote)   # the other ranks' bytes landing
                        L.cvr_set_stream(h, ctypes.c_void_p(comm.cuda_stream))
                        for j in range(G if a.parts != "copy" else 0):
                            N.check(L.cvr_unpack_tiles_device_n(h, ctypes.byref(frame),
                                                                gathered[k].data_ptr(), tpr, G, j,
                                                                N.FORMAT_RGBA16F, image.data_ptr()),
                                    "unpack", h)
                        d = torch.cuda.Event()
                        d.record(comm)
                        done[k] = d
                    torch.cuda.synchronize()
                    best = min(best, (time.perf_counter() - t0) / (F // G * G) * 1e3)
                    done = [None] * nsets
                line = dict(nranks=NR, render_nranks=rn, frames_per_launch=G, streams=ns, sets=nsets,
                            reserve_cus=rsv,
                            frames=F,
                            exchange=exch,
                            parts=a.parts,
                            ms_per_frame=round(best, 5),
                            inbound_bytes_per_frame=(NR - 1) * tpr * tile * tile * 8)
                print(json.dumps(line), flush=True)
                res.append(line)
if a.out:
    json.dump(res, open(a.out, "w"), indent=1)
