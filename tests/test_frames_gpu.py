"""Several frames in one ray-march launch (cvr_render_rc1pass_frames):
every frame of a multi-frame launch equals the same frame rendered by its own
cvr_render_rc1pass call bit for bit (RGBA and per-pixel counts), and the
launch's total is the sum of the frames' totals.  One case is checked against
the oracle directly.  Cases: one camera repeated, distinct cameras from the
reference's camera list (data/#list_camera_states), Blinn-Phong, a screen-tile
share (packed tiles), the learned launch order, the skip modes, filter_bits 8,
and the argument errors."""
import ctypes
import os

import numpy as np
import pytest

from cpp_volume_rendering_amd import _native as N
from cpp_volume_rendering_amd import datasets as D
from cpp_volume_rendering_amd import screen_tiles as T
from cpp_volume_rendering_amd.renderer import Camera, Device, make_frame, read_camera_state

pytestmark = pytest.mark.gpu

INITIAL = D.INITIAL_STATE_CAMERA


def _params(phong=False):
    p = N.Rc1passParams()
    p.step = 0.0
    p.apply_gradient_shading = int(phong)
    p.ka, p.kd, p.ks, p.shininess = 0.5, 0.5, 0.8, 30.0
    p.ispecular[:] = [1.0, 1.0, 1.0]
    p.light_pos[:] = list(D.LIGHT_LIST0_POSITION)
    return p


def _pixels(W, H, tile, rank, nranks):
    return T.tiles_for_rank(W, H, tile, rank, nranks) * tile * tile if nranks > 1 else W * H


def _render(d, frames, p, W, H, tile=0, rank=0, nranks=1, batched=True, fmt=N.FORMAT_RGBA32F):
    """frames rendered in one launch (batched) or one call each; returns the per-frame
    (rgba bits, counts) as numpy arrays and the total(s)."""
    import torch
    npx = _pixels(W, H, tile, rank, nranks)
    dt = torch.float32 if fmt == N.FORMAT_RGBA32F else torch.float16
    rgba = [torch.zeros((npx, 4), dtype=dt, device="cuda") for _ in frames]
    cnt = [torch.zeros((npx,), dtype=torch.int32, device="cuda") for _ in frames]
    totals = [torch.zeros((1,), dtype=torch.int64, device="cuda") for _ in frames]
    L = N.lib()
    if batched:
        outs = [N.Output(rgba[i].data_ptr(), cnt[i].data_ptr(),
                         totals[0].data_ptr() if i == 0 else None, 1, fmt)
                for i in range(len(frames))]
        fa = (N.Frame * len(frames))(*frames)
        oa = (N.Output * len(frames))(*outs)
        N.check(L.cvr_render_rc1pass_frames(d.handle, fa, len(frames), ctypes.byref(p), oa),
                "frames", d.handle)
    else:
        for i, f in enumerate(frames):
            o = N.Output(rgba[i].data_ptr(), cnt[i].data_ptr(), totals[i].data_ptr(), 1, fmt)
            N.check(L.cvr_render_rc1pass(d.handle, ctypes.byref(f), ctypes.byref(p), ctypes.byref(o)),
                    "single", d.handle)
    torch.cuda.synchronize()
    view = torch.int32 if fmt == N.FORMAT_RGBA32F else torch.int16
    return ([r.view(view).cpu().numpy() for r in rgba], [c.cpu().numpy() for c in cnt],
            [int(t.item()) for t in totals])


def _setup(d, vol, scale, tf, gmode=0):
    d.set_volume(vol, scale)
    d.set_transfer_function(tf)
    d.set_gradient(gmode)


def _camera_list(golden_dir, idx):
    path = os.path.join(golden_dir, "list_camera_states")
    return [read_camera_state(path, i) for i in idx]


def _compare(d, frames, p, W, H, what, **kw):
    # warm the launch order on the single-frame path first (same view), then compare
    _render(d, frames[:1], p, W, H, batched=False, **kw)
    one_rgba, one_cnt, one_tot = _render(d, frames, p, W, H, batched=False, **kw)
    mf_rgba, mf_cnt, mf_tot = _render(d, frames, p, W, H, batched=True, **kw)
    for i in range(len(frames)):
        assert np.array_equal(mf_cnt[i], one_cnt[i]), f"{what}: frame {i} counts"
        assert np.array_equal(mf_rgba[i], one_rgba[i]), f"{what}: frame {i} rgba"
    assert mf_tot[0] == sum(one_tot), f"{what}: launch total {mf_tot[0]} vs {sum(one_tot)}"
    return mf_rgba, mf_cnt


@pytest.fixture(scope="module")
def dev():
    import torch
    assert torch.cuda.is_available(), "GPU tests need a HIP device"
    d = Device(0)
    yield d
    d.close()


@pytest.mark.parametrize("nf", [2, 4, 8])
def test_frames_same_camera(dev, bonsai_tf, nf):
    _setup(dev, D.marschner_lobb_u8(96), D.voxel_scale(96), bonsai_tf)
    W, H = 160, 136
    frames = [make_frame(Camera(**INITIAL), W, H) for _ in range(nf)]
    _compare(dev, frames, _params(), W, H, f"same camera x{nf}")


def test_frames_distinct_cameras(dev, bonsai_tf, golden_dir):
    """Four of the reference's camera states in one launch (views far apart: no
    shared launch order) and four nearby views (one order)."""
    _setup(dev, D.marschner_lobb_u8(96), D.voxel_scale(96), bonsai_tf)
    W, H = 144, 144
    cams = _camera_list(golden_dir, [0, 3, 9, 17])
    _compare(dev, [make_frame(c, W, H) for c in cams], _params(), W, H, "camera list")
    near = []
    for k in range(4):
        c = Camera(**INITIAL)
        c.eye = (256.0 + 2.0 * k, 256.0, 512.0 - k)
        near.append(make_frame(c, W, H))
    _compare(dev, near, _params(), W, H, "nearby cameras")


def test_frames_match_oracle(dev, oracle, bonsai_tf, golden_dir):
    vol = D.marschner_lobb_u8(64)
    scale = D.voxel_scale(64)
    _setup(dev, vol, scale, bonsai_tf)
    W, H = 96, 80
    cams = _camera_list(golden_dir, [0, 5, 11])
    rgba, cnt = _compare(dev, [make_frame(c, W, H) for c in cams], _params(), W, H, "oracle case")
    v16 = oracle.volume_r16f(vol)
    for i, c in enumerate(cams):
        ref = oracle.render_rc1pass(v16, scale, bonsai_tf, dict(eye=c.eye, center=c.center, up=c.up,
                                                                fovy_deg=c.fovy_deg),
                                    W, H, oracle.default_step(scale))
        assert np.array_equal(cnt[i].reshape(H, W), ref[1].astype(np.int32)), f"frame {i} counts"
        assert np.array_equal(rgba[i].reshape(H, W, 4),
                              np.ascontiguousarray(ref[0]).view(np.int32)), f"frame {i} rgba"


def test_frames_phong(dev, bonsai_tf):
    _setup(dev, D.marschner_lobb_u8(64), D.voxel_scale(64), bonsai_tf, gmode=N.GRADIENT_FINITE_DIFFERENCES)
    W, H = 128, 112
    frames = [make_frame(Camera(**INITIAL), W, H) for _ in range(3)]
    _compare(dev, frames, _params(phong=True), W, H, "phong")


@pytest.mark.parametrize("nranks,tile", [(8, 16), (3, 32)])
def test_frames_screen_tile_share(dev, bonsai_tf, nranks, tile):
    _setup(dev, D.marschner_lobb_u8(96), D.voxel_scale(96), bonsai_tf)
    W, H = 256, 192
    for rank in (0, nranks - 1):
        frames = [make_frame(Camera(**INITIAL), W, H, tile, rank, nranks) for _ in range(4)]
        _compare(dev, frames, _params(), W, H, f"rank {rank}/{nranks}", tile=tile, rank=rank,
                 nranks=nranks, fmt=N.FORMAT_RGBA16F)


@pytest.mark.parametrize("opt,val", [("tile_order", 0), ("tile_order", 2), ("cell_skip", 0),
                                     ("cell_skip", 2), ("quad", 10), ("filter_bits", 8),
                                     ("batch", 2), ("launch_interleave", 0), ("band_cap", 100),
                                     ("band_cap", 200)])
def test_frames_options(bonsai_tf, opt, val):
    d = Device(0)
    try:
        N.check(N.lib().cvr_set_option(d.handle, opt.encode(), val), opt, d.handle)
        _setup(d, D.marschner_lobb_u8(96), D.voxel_scale(96), bonsai_tf)
        W, H = 160, 160
        frames = [make_frame(Camera(**INITIAL), W, H) for _ in range(4)]
        for _ in range(3):   # the learned order (tile_order 1 / quad) is in use by now
            _compare(d, frames, _params(), W, H, f"{opt}={val}")
    finally:
        d.close()


def test_frames_argument_errors(dev, bonsai_tf):
    import torch
    _setup(dev, D.marschner_lobb_u8(32), D.voxel_scale(32), bonsai_tf)
    L = N.lib()
    p = _params()
    W, H = 64, 48
    buf = [torch.zeros((W * H, 4), dtype=torch.float32, device="cuda") for _ in range(17)]
    outs = (N.Output * 17)(*[N.Output(b.data_ptr(), None, None, 1, N.FORMAT_RGBA32F) for b in buf])
    frames = (N.Frame * 17)(*[make_frame(Camera(**INITIAL), W, H) for _ in range(17)])
    assert L.cvr_render_rc1pass_frames(dev.handle, frames, 0, ctypes.byref(p), outs) == N.CVR_ERR_ARG
    # at most 16 frames per launch
    assert L.cvr_render_rc1pass_frames(dev.handle, frames, 17, ctypes.byref(p), outs) == N.CVR_ERR_ARG
    bad = (N.Frame * 2)(make_frame(Camera(**INITIAL), W, H), make_frame(Camera(**INITIAL), W, H + 1))
    assert L.cvr_render_rc1pass_frames(dev.handle, bad, 2, ctypes.byref(p), outs) == N.CVR_ERR_ARG
    host = np.zeros((H, W, 4), np.float32)
    ho = (N.Output * 2)(N.Output(host.ctypes.data, None, None, 0, N.FORMAT_RGBA32F), outs[1])
    assert L.cvr_render_rc1pass_frames(dev.handle, frames, 2, ctypes.byref(p), ho) == N.CVR_ERR_ARG
    tot = torch.zeros((1,), dtype=torch.int64, device="cuda")
    t1 = (N.Output * 2)(outs[0], N.Output(buf[1].data_ptr(), None, tot.data_ptr(), 1, N.FORMAT_RGBA32F))
    assert L.cvr_render_rc1pass_frames(dev.handle, frames, 2, ctypes.byref(p), t1) == N.CVR_ERR_ARG
    mixed = (N.Output * 2)(outs[0], N.Output(buf[1].data_ptr(), None, None, 1, N.FORMAT_RGBA16F))
    assert L.cvr_render_rc1pass_frames(dev.handle, frames, 2, ctypes.byref(p), mixed) == N.CVR_ERR_ARG
    # one frame through the batch entry is the plain call
    assert L.cvr_render_rc1pass_frames(dev.handle, frames, 1, ctypes.byref(p), outs) == N.CVR_OK


def test_screen_split_world1_launch_groups(bonsai_tf, golden_dir):
    """ScreenTileSplit at world 1 with frames_per_launch 4 over 3 streams (bench.py's
    N = 1 default): 10 frames of distinct cameras submitted, every image checked
    after its launch group completes against the frame rendered alone."""
    import torch
    from cpp_volume_rendering_amd.renderer import (DataManager, RayCasting1Pass,
                                                   RenderingParameters)
    vol = D.marschner_lobb_u8(64)
    dm = DataManager()
    dm.SetVolume(vol, D.voxel_scale(64))
    dm.SetTransferFunction(bonsai_tf, bonsai_tf)
    r = RayCasting1Pass(0)
    W, H = 96, 80
    r.SetExternalResources(dm, RenderingParameters(W, H, light_position=D.LIGHT_LIST0_POSITION))
    assert r.Init(W, H)
    cams = _camera_list(golden_dir, [0, 1, 2, 3, 5, 9, 11, 17, 21, 23])
    try:
        sp = T.ScreenTileSplit(r, W, H, fmt=N.FORMAT_RGBA16F, streams=3, frames_per_launch=4)
        assert sp.L == 4 and len(sp._images) == 12
        r.PrepareRender(cams[0])
        for c in cams:
            sp.submit(c)
        sp.flush()
        torch.cuda.synchronize()
        for n, c in enumerate(cams):
            img = sp._images[sp._image_index(n)].clone()
            ref = torch.zeros_like(img)
            r.render_to(make_frame(c, W, H), N.Output(ref.data_ptr(), None, None, 1, N.FORMAT_RGBA16F))
            torch.cuda.synchronize()
            assert torch.equal(img.view(torch.int16), ref.view(torch.int16)), f"frame {n}"
    finally:
        r.Clean()
