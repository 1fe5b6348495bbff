"""GPU checks of the frame formats and of the screen-tile split's device side.

* RGBA16F output (the reference's own framebuffer: imageStore into an RGBA16F
  image, ray_marching_1p.comp:174-176) is the RGBA32F composite rounded to
  nearest even, bit for bit, for every renderer path that stores a pixel.
* The device unpack moves RGBA16F pixels exactly like RGBA32F ones.
* The native RCCL gather (cvr_comm_init / cvr_gather_tiles) with two ranks: on a
  one-GPU box both ranks share the device; RCCL may refuse that (duplicate GPU),
  in which case the test is skipped and the path is exercised by the driver's
  multi-GPU bench, which checks the gathered frame bit for bit against a
  one-GPU render (bench.py, multi_gpu_bit_exact_vs_1gpu_frame).
"""
import ctypes
import os
import socket

import numpy as np
import pytest

from cpp_volume_rendering_amd import _native as N
from cpp_volume_rendering_amd import datasets as D
from cpp_volume_rendering_amd import screen_tiles as T
from cpp_volume_rendering_amd.renderer import Camera, Device, make_frame

pytestmark = pytest.mark.gpu

INITIAL = D.INITIAL_STATE_CAMERA


@pytest.fixture(scope="module")
def dev():
    import torch
    assert torch.cuda.is_available(), "GPU tests need a HIP device"
    d = Device(0)
    yield d
    d.close()


def _render(dev, fmt, W, H, phong=False, tile=0, rank=0, nranks=1, cam=INITIAL):
    frame = make_frame(Camera(**cam), W, H, tile, rank, nranks)
    p = N.Rc1passParams()
    p.step = 0.0
    p.apply_gradient_shading = int(phong)
    p.ka, p.kd, p.ks, p.shininess = 0.5, 0.5, 0.8, 30.0
    p.ispecular[:] = [1.0, 1.0, 1.0]
    p.light_pos[:] = list(D.LIGHT_LIST0_POSITION)
    if nranks > 1:
        k = T.tiles_for_rank(W, H, tile, rank, nranks)
        shape = (k, tile, tile, 4)
    else:
        shape = (H, W, 4)
    img = np.zeros(shape, np.float16 if fmt == N.FORMAT_RGBA16F else np.float32)
    out = N.Output(img.ctypes.data, None, None, 0, fmt)
    N.check(N.lib().cvr_render_rc1pass(dev.handle, ctypes.byref(frame), ctypes.byref(p),
                                       ctypes.byref(out)), "render", dev.handle)
    return img


@pytest.mark.parametrize("phong", [False, True])
def test_rgba16f_is_rounded_rgba32f(dev, bonsai_tf, phong):
    vol = D.marschner_lobb_u8(64)
    dev.set_volume(vol, D.voxel_scale(64))
    dev.set_transfer_function(bonsai_tf)
    dev.set_gradient(N.GRADIENT_FINITE_DIFFERENCES if phong else N.GRADIENT_NONE)
    W, H = 120, 88
    f32 = _render(dev, N.FORMAT_RGBA32F, W, H, phong)
    f16 = _render(dev, N.FORMAT_RGBA16F, W, H, phong)
    assert np.array_equal(f16.view(np.uint16), f32.astype(np.float16).view(np.uint16))
    assert (f32[..., 3] > 0).mean() > 0.3        # a real image, not a cleared frame


def test_bad_format_rejected(dev, bonsai_tf):
    vol = D.marschner_lobb_u8(32)
    dev.set_volume(vol, D.voxel_scale(32))
    dev.set_transfer_function(bonsai_tf)
    frame = make_frame(Camera(**INITIAL), 16, 16)
    p = N.Rc1passParams()
    img = np.zeros((16, 16, 4), np.float32)
    out = N.Output(img.ctypes.data, None, None, 0, 7)
    st = N.lib().cvr_render_rc1pass(dev.handle, ctypes.byref(frame), ctypes.byref(p),
                                    ctypes.byref(out))
    assert st == N.CVR_ERR_ARG


@pytest.mark.parametrize("nranks,tile", [(3, 32), (2, 16)])
def test_rgba16f_tiles_unpack(dev, bonsai_tf, nranks, tile):
    import torch
    vol = D.marschner_lobb_u8(64)
    dev.set_volume(vol, D.voxel_scale(64))
    dev.set_transfer_function(bonsai_tf)
    dev.set_gradient(N.GRADIENT_NONE)
    W, H = 100, 72
    full = _render(dev, N.FORMAT_RGBA16F, W, H)
    tpr = T.max_tiles_per_rank(W, H, tile, nranks)
    packed_all = np.zeros((nranks, tpr, tile, tile, 4), np.float16)
    for r in range(nranks):
        p = _render(dev, N.FORMAT_RGBA16F, W, H, tile=tile, rank=r, nranks=nranks)
        packed_all[r, :p.shape[0]] = p
    host = T.unpack(packed_all, W, H, tile, nranks)
    assert np.array_equal(host.view(np.uint16), full.view(np.uint16))
    d_packed = torch.from_numpy(packed_all).cuda()
    d_img = torch.zeros((H, W, 4), dtype=torch.float16, device="cuda")
    frame = make_frame(Camera(**INITIAL), W, H, tile, 0, nranks)
    dev.set_stream(torch.cuda.current_stream().cuda_stream)
    N.check(N.lib().cvr_unpack_tiles_device(dev.handle, ctypes.byref(frame), d_packed.data_ptr(),
                                            tpr, N.FORMAT_RGBA16F, d_img.data_ptr()),
            "unpack", dev.handle)
    torch.cuda.synchronize()
    dev.set_stream(None)
    assert np.array_equal(d_img.cpu().numpy().view(np.uint16), full.view(np.uint16))


def test_screen_tile_split_single_rank(bonsai_tf):
    """world 1: ScreenTileSplit renders the whole frame into its image (RGBA16F)."""
    import torch
    from cpp_volume_rendering_amd.renderer import (DataManager, RayCasting1Pass,
                                                   RenderingParameters)
    dm = DataManager()
    dm.SetVolume(D.marschner_lobb_u8(48), D.voxel_scale(48))
    dm.SetTransferFunction(bonsai_tf)
    r = RayCasting1Pass(0)
    r.SetExternalResources(dm, RenderingParameters(80, 64))
    assert r.Init(80, 64)
    cam = Camera(**INITIAL)
    r.PrepareRender(cam)
    sp = T.ScreenTileSplit(r, tile=32, fmt=N.FORMAT_RGBA16F)
    assert sp.transport == "none"
    img = sp.render(cam)
    torch.cuda.synchronize()
    r.Redraw()
    torch.cuda.synchronize()
    want = r.rgba.cpu().numpy().astype(np.float16)
    assert np.array_equal(img.cpu().numpy().view(np.uint16), want.view(np.uint16))
    sp.close()
    r.Clean()


CAMS = [dict(INITIAL), dict(INITIAL, eye=(-300.0, 120.0, 380.0)),
        dict(INITIAL, eye=(0.0, -400.0, 200.0))]


def _rccl_worker(rank, world, port, q, root_renders=True):
    import torch
    import torch.distributed as dist
    from cpp_volume_rendering_amd.renderer import (DataManager, RayCasting1Pass,
                                                   RenderingParameters, build_tf_rgbt)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        torch.cuda.set_device(0)
        W, H = 200, 136
        dm = DataManager()
        dm.SetVolume(D.marschner_lobb_u8(64), D.voxel_scale(64))
        dm.SetTransferFunction(build_tf_rgbt(D.BONSAI_TF_RGB, D.BONSAI_TF_ALPHA))
        r = RayCasting1Pass(0)
        r.SetExternalResources(dm, RenderingParameters(W, H))
        assert r.Init(W, H)
        r.PrepareRender(Camera(**INITIAL))
        try:
            sp = T.ScreenTileSplit(r, tile=32, fmt=N.FORMAT_RGBA16F, transport="rccl",
                                   root_renders=root_renders)
        except N.CvrError as e:
            if rank == 0:
                q.put(("skip", str(e)))
            return
        ok = True
        seq = [0, 1, 2, 0]
        for ci in seq:
            sp.submit(Camera(**CAMS[ci]))
        img = sp.flush()
        torch.cuda.synchronize()
        if rank == 0:
            full = torch.zeros_like(img)
            r.render_to(make_frame(Camera(**CAMS[seq[-1]]), W, H),
                        N.Output(full.data_ptr(), None, None, 1, N.FORMAT_RGBA16F))
            torch.cuda.synchronize()
            ok = bool(torch.equal(full.view(torch.int16), img.view(torch.int16)))
            q.put(("ok" if ok else "mismatch", ""))
        sp.close()
        r.Clean()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,root_renders", [(2, True), (3, False)])
def test_rccl_gather_ranks_one_gpu(world, root_renders):
    """world ranks on one GPU through the native RCCL gather; (3, False) is the idle
    root of bench.py --gpus 8 (rank 0 gathers only, ranks 1..2 render the split
    over 2): rank 0's image equals its own full render bit for bit.  Skipped where
    RCCL refuses several ranks on one device."""
    import multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    procs = [ctx.Process(target=_rccl_worker, args=(r, world, port, q, root_renders))
             for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=90)
    alive = [p for p in procs if p.is_alive()]
    for p in alive:
        p.kill()
        p.join(5)
    status, detail = q.get(timeout=10) if not q.empty() or not alive else ("hung", "")
    if status == "skip":
        pytest.skip(f"RCCL refused {world} ranks on one GPU: {detail}")
    assert not alive, "RCCL gather workers hung"
    assert status == "ok"
    assert [p.exitcode for p in procs] == [0] * world


@pytest.mark.parametrize("nstreams", [4, 16])
def test_rccl_one_rank_gather_pipeline(dev, bonsai_tf, nstreams):
    """A one-rank communicator through cvr_comm_init / cvr_gather_tiles (ncclGather in
    place + copy), frames rotated over n streams with split_streams = n (16: the
    bench's default at 8 GPUs): after cvr_gather_sync the image holds the last
    frame, bit-equal to a direct render."""
    import torch
    L = N.lib()
    vol = D.marschner_lobb_u8(64)
    dev.set_volume(vol, D.voxel_scale(64))
    dev.set_transfer_function(bonsai_tf)
    dev.set_gradient(N.GRADIENT_NONE)
    uid = ctypes.create_string_buffer(N.COMM_ID_BYTES)
    N.check(L.cvr_comm_unique_id(uid), "uid")
    N.check(L.cvr_comm_init(dev.handle, 1, 0, uid.raw), "cvr_comm_init", dev.handle)
    try:
        N.check(L.cvr_set_option(dev.handle, b"split_streams", nstreams), "opt", dev.handle)
        W, H = 160, 120
        streams = [torch.cuda.Stream() for _ in range(nstreams)]
        bufs = [torch.zeros((H, W, 4), dtype=torch.float16, device="cuda") for _ in range(nstreams)]
        img = torch.zeros((H, W, 4), dtype=torch.float16, device="cuda")
        p = N.Rc1passParams()
        seq = [0, 1, 2, 0, 1, 2, 1] * (3 if nstreams > 4 else 1)
        for n, ci in enumerate(seq):
            k = n % nstreams
            frame = make_frame(Camera(**CAMS[ci]), W, H)
            dev.set_stream(streams[k].cuda_stream)
            out = N.Output(bufs[k].data_ptr(), None, None, 1, N.FORMAT_RGBA16F)
            N.check(L.cvr_render_rc1pass(dev.handle, ctypes.byref(frame), ctypes.byref(p),
                                         ctypes.byref(out)), "render", dev.handle)
            N.check(L.cvr_gather_tiles(dev.handle, ctypes.byref(frame), bufs[k].data_ptr(), 0,
                                       N.FORMAT_RGBA16F, bufs[k].data_ptr(), img.data_ptr()),
                    "cvr_gather_tiles", dev.handle)
        dev.set_stream(torch.cuda.current_stream().cuda_stream)
        N.check(L.cvr_gather_sync(dev.handle), "sync", dev.handle)
        torch.cuda.synchronize()
        want = _render(dev, N.FORMAT_RGBA16F, W, H, cam=CAMS[seq[-1]])
        assert np.array_equal(img.cpu().numpy().view(np.uint16), want.view(np.uint16))
    finally:
        N.check(L.cvr_set_option(dev.handle, b"split_streams", 1), "opt", dev.handle)
        N.check(L.cvr_comm_destroy(dev.handle), "cvr_comm_destroy", dev.handle)
        dev.set_stream(None)


def test_grouped_unpack_matches_full_frames(dev, bonsai_tf):
    """A grouped exchange's layout (rank r's frame j at slot (r*G + j)*tpr), built on
    one GPU from per-rank renders of G different cameras, unpacks frame j to the
    whole frame j bit for bit (cvr_unpack_tiles_device_n)."""
    import torch
    vol = D.marschner_lobb_u8(64)
    dev.set_volume(vol, D.voxel_scale(64))
    dev.set_transfer_function(bonsai_tf)
    dev.set_gradient(N.GRADIENT_NONE)
    W, H, tile, nranks, G = 100, 72, 32, 3, 3
    tpr = T.max_tiles_per_rank(W, H, tile, nranks)
    gathered = np.zeros((nranks, G, tpr, tile, tile, 4), np.float16)
    for r in range(nranks):
        for j in range(G):
            p = _render(dev, N.FORMAT_RGBA16F, W, H, tile=tile, rank=r, nranks=nranks, cam=CAMS[j])
            gathered[r, j, :p.shape[0]] = p
    d_g = torch.from_numpy(gathered).cuda()
    frame = make_frame(Camera(**INITIAL), W, H, tile, 0, nranks)
    dev.set_stream(torch.cuda.current_stream().cuda_stream)
    for j in range(G):
        img = torch.zeros((H, W, 4), dtype=torch.float16, device="cuda")
        N.check(N.lib().cvr_unpack_tiles_device_n(dev.handle, ctypes.byref(frame), d_g.data_ptr(),
                                                  tpr, G, j, N.FORMAT_RGBA16F, img.data_ptr()),
                "unpack_n", dev.handle)
        torch.cuda.synchronize()
        want = _render(dev, N.FORMAT_RGBA16F, W, H, cam=CAMS[j])
        assert np.array_equal(img.cpu().numpy().view(np.uint16), want.view(np.uint16)), j
    dev.set_stream(None)


def test_rccl_one_rank_grouped_gather(dev, bonsai_tf):
    """cvr_gather_tiles_n with a one-rank communicator: G frames rendered into one
    block, one ncclGather, each frame delivered to its own image."""
    import torch
    L = N.lib()
    vol = D.marschner_lobb_u8(64)
    dev.set_volume(vol, D.voxel_scale(64))
    dev.set_transfer_function(bonsai_tf)
    dev.set_gradient(N.GRADIENT_NONE)
    uid = ctypes.create_string_buffer(N.COMM_ID_BYTES)
    N.check(L.cvr_comm_unique_id(uid), "uid")
    N.check(L.cvr_comm_init(dev.handle, 1, 0, uid.raw), "cvr_comm_init", dev.handle)
    try:
        W, H, G = 128, 96, 3
        blk = torch.zeros((G, H, W, 4), dtype=torch.float16, device="cuda")
        imgs_t = [torch.zeros((H, W, 4), dtype=torch.float16, device="cuda") for _ in range(G)]
        imgs = (ctypes.c_void_p * G)(*[t.data_ptr() for t in imgs_t])
        dev.set_stream(torch.cuda.current_stream().cuda_stream)
        p = N.Rc1passParams()
        frame = None
        for j in range(G):
            frame = make_frame(Camera(**CAMS[j]), W, H)
            out = N.Output(blk[j].data_ptr(), None, None, 1, N.FORMAT_RGBA16F)
            N.check(L.cvr_render_rc1pass(dev.handle, ctypes.byref(frame), ctypes.byref(p),
                                         ctypes.byref(out)), "render", dev.handle)
        N.check(L.cvr_gather_tiles_n(dev.handle, ctypes.byref(frame), G, blk.data_ptr(), 0,
                                     N.FORMAT_RGBA16F, blk.data_ptr(), imgs), "gather_n",
                dev.handle)
        N.check(L.cvr_gather_sync(dev.handle), "sync", dev.handle)
        torch.cuda.synchronize()
        for j in range(G):
            want = _render(dev, N.FORMAT_RGBA16F, W, H, cam=CAMS[j])
            assert np.array_equal(imgs_t[j].cpu().numpy().view(np.uint16), want.view(np.uint16)), j
    finally:
        N.check(L.cvr_comm_destroy(dev.handle), "cvr_comm_destroy", dev.handle)
        dev.set_stream(None)


@pytest.mark.parametrize("nstreams,nsets", [(4, 16), (2, 8), (4, 4)])
def test_rccl_one_rank_buffer_sets(dev, bonsai_tf, nstreams, nsets):
    """More exchange buffer sets than render streams (option gather_sets, the bench's
    N > 1 default 4 per stream): groups of G = 4 frames rendered in one launch
    (cvr_render_rc1pass_frames) into set g % B on stream g % D, exchanged with
    cvr_gather_tiles_n into images of their own.  Cameras change every frame, so a
    render that overwrote a set before its exchange had read it would deliver
    another frame's pixels: every frame of every group is checked bit for bit."""
    import torch
    L = N.lib()
    vol = D.marschner_lobb_u8(64)
    dev.set_volume(vol, D.voxel_scale(64))
    dev.set_transfer_function(bonsai_tf)
    dev.set_gradient(N.GRADIENT_NONE)
    uid = ctypes.create_string_buffer(N.COMM_ID_BYTES)
    N.check(L.cvr_comm_unique_id(uid), "uid")
    N.check(L.cvr_comm_init(dev.handle, 1, 0, uid.raw), "cvr_comm_init", dev.handle)
    try:
        N.check(L.cvr_set_option(dev.handle, b"split_streams", nstreams), "opt", dev.handle)
        N.check(L.cvr_set_option(dev.handle, b"gather_sets", nsets), "opt", dev.handle)
        W, H, G, ngroups = 96, 80, 4, 3 * nsets // 2
        streams = [torch.cuda.Stream() for _ in range(nstreams)]
        sets = [torch.zeros((G, H, W, 4), dtype=torch.float16, device="cuda") for _ in range(nsets)]
        imgs_t = [[torch.zeros((H, W, 4), dtype=torch.float16, device="cuda") for _ in range(G)]
                  for _ in range(ngroups)]
        p = N.Rc1passParams()
        cams = []
        for g in range(ngroups):
            k = g % nsets
            dev.set_stream(streams[g % nstreams].cuda_stream)
            frames = []
            for j in range(G):
                c = dict(CAMS[(g * G + j) % len(CAMS)])
                c["eye"] = tuple(e + 3.0 * ((g * G + j) // len(CAMS)) for e in c["eye"])
                cams.append(c)
                frames.append(make_frame(Camera(**c), W, H))
            fa = (N.Frame * G)(*frames)
            oa = (N.Output * G)(*[N.Output(sets[k][j].data_ptr(), None, None, 1, N.FORMAT_RGBA16F)
                                  for j in range(G)])
            N.check(L.cvr_render_rc1pass_frames(dev.handle, fa, G, ctypes.byref(p), oa), "frames",
                    dev.handle)
            imgs = (ctypes.c_void_p * G)(*[t.data_ptr() for t in imgs_t[g]])
            N.check(L.cvr_gather_tiles_n(dev.handle, ctypes.byref(frames[0]), G, sets[k].data_ptr(), 0,
                                         N.FORMAT_RGBA16F, sets[k].data_ptr(), imgs), "gather_n",
                    dev.handle)
        dev.set_stream(torch.cuda.current_stream().cuda_stream)
        N.check(L.cvr_gather_sync(dev.handle), "sync", dev.handle)
        torch.cuda.synchronize()
        for g in range(ngroups):
            for j in range(G):
                want = _render(dev, N.FORMAT_RGBA16F, W, H, cam=cams[g * G + j])
                assert np.array_equal(imgs_t[g][j].cpu().numpy().view(np.uint16),
                                      want.view(np.uint16)), (g, j)
    finally:
        N.check(L.cvr_set_option(dev.handle, b"split_streams", 1), "opt", dev.handle)
        N.check(L.cvr_set_option(dev.handle, b"gather_sets", 0), "opt", dev.handle)
        N.check(L.cvr_comm_destroy(dev.handle), "cvr_comm_destroy", dev.handle)
        dev.set_stream(None)
