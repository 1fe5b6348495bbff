#!/usr/bin/env python3
"""Per-rank cost of the N-way screen split, measured on one GPU: renders rank r's
share of the headline frame (512^3 ML, 1024^2) F times over D rotated streams, for
every rank r, and prints ms per frame per rank and the max over ranks (the bench
takes the max over ranks).  --renderer dos|ebs: configs 4/5 instead (512^3 at 2048^2,
1024^3 at 1024^2).  Gathers are not included.
Usage: python tools/overlap_probe.py [--nranks 1,2,4,8] [--tile 16] [--streams 4]
       [--quad 0] [--frames 32] [--renderer rc1pass]"""
import os
import sys
# hardware queues: 8 as bench.py (--hwq N overrides), set before HIP initialises
os.environ["GPU_MAX_HW_QUEUES"] = (sys.argv[sys.argv.index("--hwq") + 1]
                                   if "--hwq" in sys.argv else "8")
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
ap.add_argument("--nranks", default="1,2,4,8")
ap.add_argument("--tile", default="16")
ap.add_argument("--quad", default="0")
ap.add_argument("--frames", type=int, default=32)
ap.add_argument("--streams", default="4")
ap.add_argument("--ranks", default="all", help="'all' or a comma list of ranks")
ap.add_argument("--renderer", choices=["rc1pass", "dos", "ebs"], default="rc1pass")
ap.add_argument("--out", default="")
ap.add_argument("--hwq", default="8")
ap.add_argument("--frames-per-launch", type=int, default=1,
                help="a CVR_PROBE_FRAMES=G library build (CVR_LIB_OVERRIDE): each call marches G frames")
ap.add_argument("--tile-order", type=int, default=-1, help="rc1pass tile_order option (-1: default)")
ap.add_argument("--interleave", default="-1",
                help="comma list of launch_interleave settings (-1: library default)")
ap.add_argument("--boost", default="-1", help="rc1pass: comma list of boost percentages (-1: library default)")
a = ap.parse_args()

n, W = (1024, 1024) if a.renderer == "ebs" else ((512, 2048) if a.renderer == "dos" else (512, 1024))
vol = D.marschner_lobb_u8(n)
dm = DataManager()
dm.SetVolume(vol, D.voxel_scale(n))
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
r.PrepareRender(Camera(**D.INITIAL_STATE_CAMERA))
L = N.lib()
handle = r.device.handle


def render(frame, out):
    r.render_to(frame, out)


res = []
import itertools  # noqa: E402
for q, bst, il in itertools.product([int(x) for x in a.quad.split(",")], [int(x) for x in a.boost.split(",")],
                                   [int(x) for x in a.interleave.split(",")]):
    if a.renderer == "rc1pass":
        L.cvr_set_option(handle, b"quad", q)
        if bst >= 0:
            L.cvr_set_option(handle, b"boost", bst)
        if a.tile_order >= 0:
            L.cvr_set_option(handle, b"tile_order", a.tile_order)
        if il >= 0:
            L.cvr_set_option(handle, b"launch_interleave", il)
    for nr in [int(x) for x in a.nranks.split(",")]:
        for tile in [int(x) for x in a.tile.split(",")]:
            ranks = range(nr) if a.ranks == "all" else [int(x) for x in a.ranks.split(",") if int(x) < nr]
            for ns in [int(x) for x in a.streams.split(",")]:
                pool = [torch.cuda.Stream() for _ in range(ns)]
                per = []
                for rk in ranks:
                    frame = make_frame(Camera(**D.INITIAL_STATE_CAMERA), W, W, tile, rk, nr) \
                        if nr > 1 else make_frame(Camera(**D.INITIAL_STATE_CAMERA), W, W)
                    npx = T.tiles_for_rank(W, W, tile, rk, nr) * tile * tile if nr > 1 else W * W
                    G = a.frames_per_launch
                    real_mf = G > 1 and "CVR_LIB_OVERRIDE" not in os.environ   # else a probe build
                    nb = ns * (G if real_mf else 1)
                    bufs = [torch.zeros((npx, 4), dtype=torch.float16, device="cuda") for _ in range(nb)]
                    outs = [N.Output(b.data_ptr(), None, None, 1, 1) for b in bufs]
                    best = 1e9
                    nl = a.frames // G if real_mf else a.frames       # launches
                    for rep in range(3):
                        torch.cuda.synchronize()
                        t0 = time.perf_counter()
                        for i in range(nl):
                            L.cvr_set_stream(handle, ctypes.c_void_p(pool[i % ns].cuda_stream))
                            if real_mf:   # cvr_render_rc1pass_frames: G frames per call
                                k = i % ns
                                r.render_frames_to([frame] * G, outs[k * G:(k + 1) * G])
                            else:
                                render(frame, outs[i % ns])
                        torch.cuda.synchronize()
                        best = min(best, (time.perf_counter() - t0) / (nl * G) * 1e3)
                    per.append(best)
                line = dict(renderer=a.renderer, frames_per_launch=a.frames_per_launch, tile_order=a.tile_order,
                            interleave=il,
                            lib=os.environ.get("CVR_LIB_OVERRIDE", "in-tree"), nranks=nr, tile=tile, quad=q, boost=bst, streams=ns, hwq=int(a.hwq),
                            ms_per_rank=[round(x, 5) for x in per], max_ms=round(max(per), 5),
                            mean_ms=round(sum(per) / len(per), 5),
                            max_over_mean=round(max(per) / (sum(per) / len(per)), 4))
                print(json.dumps(line), flush=True)
                res.append(line)
if a.out:
    with open(a.out, "w") as f:
        json.dump(res, f, indent=1)
