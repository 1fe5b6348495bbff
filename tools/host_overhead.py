#!/usr/bin/env python3
"""Host cost of one frame of the screen-tile split's submit path (render +
cvr_gather_tiles), measured with a one-rank communicator on one GPU: the time the
host spends issuing F frames (the GPU runs behind), per frame.  At 8 GPUs a rank's
frame takes ~23 us of GPU time, so the host path must stay below that.
Usage: python tools/host_overhead.py [--frames 200]"""
import argparse
import ctypes
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from cpp_volume_rendering_amd import _native as N  # noqa: E402
from cpp_volume_rendering_amd import datasets as D  # noqa: E402
from cpp_volume_rendering_amd.renderer import Camera, Device, build_tf_rgbt, make_frame  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--frames", type=int, default=200)
a = ap.parse_args()
L = N.lib()
dev = Device(0)
dev.set_volume(D.marschner_lobb_u8(64), D.voxel_scale(64))
dev.set_transfer_function(build_tf_rgbt(D.BONSAI_TF_RGB, D.BONSAI_TF_ALPHA))
uid = ctypes.create_string_buffer(N.COMM_ID_BYTES)
N.check(L.cvr_comm_unique_id(uid), "uid")
N.check(L.cvr_comm_init(dev.handle, 1, 0, uid.raw), "init", dev.handle)
N.check(L.cvr_set_option(dev.handle, b"split_streams", 4), "opt", dev.handle)
W = H = 256
streams = [torch.cuda.Stream() for _ in range(4)]
bufs = [torch.zeros((H, W, 4), dtype=torch.float16, device="cuda") for _ in range(4)]
img = torch.zeros((H, W, 4), dtype=torch.float16, device="cuda")
frame = make_frame(Camera(**D.INITIAL_STATE_CAMERA), W, H)
p = N.Rc1passParams()
outs = [N.Output(b.data_ptr(), None, None, 1, N.FORMAT_RGBA16F) for b in bufs]
sptr = [s.cuda_stream for s in streams]
fr, pr = ctypes.byref(frame), ctypes.byref(p)
for rep in range(3):
    torch.cuda.synchronize()
    t_render = t_gather = 0.0
    t0 = time.perf_counter()
    for n in range(a.frames):
        k = n % 4
        L.cvr_set_stream(dev.handle, sptr[k])
        h0 = time.perf_counter()
        L.cvr_render_rc1pass(dev.handle, fr, pr, ctypes.byref(outs[k]))
        h1 = time.perf_counter()
        L.cvr_gather_tiles(dev.handle, fr, bufs[k].data_ptr(), 0, N.FORMAT_RGBA16F,
                           bufs[k].data_ptr(), img.data_ptr())
        h2 = time.perf_counter()
        t_render += h1 - h0
        t_gather += h2 - h1
    t_host = time.perf_counter() - t0
    torch.cuda.synchronize()
    t_all = time.perf_counter() - t0
    print(f"rep {rep}: host {t_host / a.frames * 1e6:.1f} us/frame (render call "
          f"{t_render / a.frames * 1e6:.1f}, gather call {t_gather / a.frames * 1e6:.1f}); "
          f"with GPU {t_all / a.frames * 1e6:.1f} us/frame", flush=True)
# The bench's form since round 4: 4 frames per cvr_render_rc1pass_frames call and one
# cvr_gather_tiles_n per 4 frames (host cost per frame = the two calls / 4)
G = 4
blk = [torch.zeros((G, H, W, 4), dtype=torch.float16, device="cuda") for _ in range(4)]
frames4 = (N.Frame * G)(*([frame] * G))
outs4 = [(N.Output * G)(*[N.Output(b[j].data_ptr(), None, None, 1, N.FORMAT_RGBA16F)
                          for j in range(G)]) for b in blk]
imgs4 = (ctypes.c_void_p * G)(*([img.data_ptr()] * G))
ngroups = max(1, a.frames // G)
for rep in range(3):
    torch.cuda.synchronize()
    t_render = t_gather = 0.0
    t0 = time.perf_counter()
    for n in range(ngroups):
        k = n % 4
        L.cvr_set_stream(dev.handle, sptr[k])
        h0 = time.perf_counter()
        L.cvr_render_rc1pass_frames(dev.handle, frames4, G, pr, outs4[k])
        h1 = time.perf_counter()
        L.cvr_gather_tiles_n(dev.handle, fr, G, blk[k].data_ptr(), 0, N.FORMAT_RGBA16F,
                             blk[k].data_ptr(), imgs4)
        h2 = time.perf_counter()
        t_render += h1 - h0
        t_gather += h2 - h1
    t_host = time.perf_counter() - t0
    torch.cuda.synchronize()
    t_all = time.perf_counter() - t0
    nf = ngroups * G
    print(f"rep {rep}, {G} frames per call: host {t_host / nf * 1e6:.1f} us/frame (render call "
          f"{t_render / ngroups * 1e6:.1f} us, gather call {t_gather / ngroups * 1e6:.1f} us per "
          f"{G} frames); with GPU {t_all / nf * 1e6:.1f} us/frame", flush=True)
N.check(L.cvr_comm_destroy(dev.handle), "destroy", dev.handle)
