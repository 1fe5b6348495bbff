"""The prefetched emission-absorption march (option "prefetch", raymarch.hip
march_ray_pf: the next batch's cell loads as LDS-DMA during the current batch's
composite, the TF in LDS as RGBA16F) against the plain march and the oracle, bit
for bit: RGBA floats, per-pixel sample counts and frame totals.  Cases: the
rc1pass parity set (non-Phong: ragged, anisotropic, u16, sparse, all-zero,
one pixel, camera inside = clamped positions, dense TF = the range-checked exp),
reference camera states, every cell_skip mode on the headline field, packed
screen-tile shares and multi-frame launches."""
import ctypes

import numpy as np
import pytest

from cpp_volume_rendering_amd import _native as N
from cpp_volume_rendering_amd import datasets as D
from cpp_volume_rendering_amd.renderer import Camera, Device, make_frame, read_camera_state

from test_rc1pass_gpu import CASES, INITIAL, assert_bitexact, case_tf, gpu_render, oracle_render

pytestmark = pytest.mark.gpu

EA_CASES = sorted(k for k, c in CASES.items() if not c.get("phong"))


def _dev(prefetch):
    d = Device(0)
    N.check(N.lib().cvr_set_option(d.handle, b"prefetch", prefetch), "prefetch", d.handle)
    assert N.lib().cvr_get_option(d.handle, b"prefetch") == prefetch
    return d


@pytest.mark.parametrize("name", EA_CASES)
def test_prefetch_bitexact_vs_oracle(oracle, bonsai_tf, name):
    c = CASES[name]
    vol = c["vol"]()
    tf = case_tf(c, bonsai_tf)
    cam = c.get("cam", INITIAL)
    d = _dev(1)
    try:
        for rep in range(2):   # the second frame runs under the learned launch order
            rgba, cnt, total = gpu_render(d, vol, c["scale"], tf, cam, c["W"], c["H"],
                                          step=c.get("step", 0.0), set_data=(rep == 0))
        o_rgba, o_cnt, o_S = oracle_render(oracle, vol, c["scale"], tf, cam, c["W"], c["H"],
                                           step=c.get("step", 0.0))
        assert_bitexact(cnt, o_cnt, f"{name} counts")
        assert_bitexact(rgba, o_rgba, f"{name} rgba")
        assert total == o_S
    finally:
        d.close()


def test_prefetch_cell_skip_modes_and_cameras(bonsai_tf, golden_dir):
    """cell_skip 1..4 on the headline field (and the long-ray TF) and eight reference
    camera states: prefetch 1 == prefetch 0, bit for bit."""
    import os
    vol = D.marschner_lobb_u8(160)
    sc = D.voxel_scale(160)
    W = H = 192
    path = os.path.join(golden_dir, "list_camera_states")
    cams = [INITIAL] + [read_camera_state(path, i) for i in (1, 3, 4, 11, 14, 15, 21)]
    cams = [c if isinstance(c, dict) else dict(eye=c.eye, center=c.center, up=c.up) for c in cams]
    a, b = _dev(0), _dev(1)
    try:
        for tfs in (1.0, 0.02):
            tf = bonsai_tf.copy(); tf[:, 3] *= tfs
            first = True
            for cs in (1, 2, 3, 4):
                for d in (a, b):
                    N.check(N.lib().cvr_set_option(d.handle, b"cell_skip", cs), "cell_skip", d.handle)
                for ci, cam in enumerate(cams if cs == 3 else cams[:2]):
                    ra = gpu_render(a, vol, sc, tf, cam, W, H, set_data=first)
                    rb = gpu_render(b, vol, sc, tf, cam, W, H, set_data=first)
                    first = False
                    what = f"tf x{tfs} cell_skip {cs} camera {ci}"
                    assert_bitexact(rb[1], ra[1], what + " counts")
                    assert_bitexact(rb[0], ra[0], what + " rgba")
                    assert rb[2] == ra[2], what
    finally:
        a.close()
        b.close()


@pytest.mark.parametrize("nranks,tile", [(3, 16), (8, 32)])
def test_prefetch_screen_tiles(bonsai_tf, nranks, tile):
    vol = D.marschner_lobb_u8(96)
    sc = D.voxel_scale(96)
    W, H = 160, 144
    a, b = _dev(0), _dev(1)
    try:
        for r in range(nranks):
            ra = gpu_render(a, vol, sc, bonsai_tf, INITIAL, W, H, tile=tile, rank=r, nranks=nranks,
                            set_data=(r == 0))
            rb = gpu_render(b, vol, sc, bonsai_tf, INITIAL, W, H, tile=tile, rank=r, nranks=nranks,
                            set_data=(r == 0))
            assert_bitexact(rb[1], ra[1], f"rank {r}/{nranks} counts")
            assert_bitexact(rb[0], ra[0], f"rank {r}/{nranks} rgba")
    finally:
        a.close()
        b.close()


def test_prefetch_multi_frame_launch(bonsai_tf, golden_dir):
    """Four frames in one launch (cvr_render_rc1pass_frames, the bench's form), the same
    camera and four distinct reference states: prefetch 1 == prefetch 0."""
    import os
    import torch
    vol = D.marschner_lobb_u8(128)
    sc = D.voxel_scale(128)
    W = H = 160
    path = os.path.join(golden_dir, "list_camera_states")
    sets = [[Camera(**INITIAL)] * 4, [read_camera_state(path, i) for i in (0, 4, 11, 14)]]
    res = {}
    for pf in (0, 1):
        d = _dev(pf)
        try:
            d.set_volume(vol, sc)
            d.set_transfer_function(bonsai_tf)
            for si, cams in enumerate(sets):
                frames = (N.Frame * 4)(*[make_frame(c, W, H) for c in cams])
                for rep in range(2):
                    bufs = [torch.zeros((H, W, 4), dtype=torch.float16, device="cuda") for _ in range(4)]
                    cnts = [torch.zeros((H, W), dtype=torch.int32, device="cuda") for _ in range(4)]
                    total = torch.zeros((1,), dtype=torch.int64, device="cuda")
                    torch.cuda.synchronize()
                    outs = (N.Output * 4)(*[N.Output(bufs[j].data_ptr(), cnts[j].data_ptr(),
                                                     total.data_ptr() if j == 0 else None, 1,
                                                     N.FORMAT_RGBA16F) for j in range(4)])
                    p = N.Rc1passParams()
                    N.check(N.lib().cvr_render_rc1pass_frames(d.handle, frames, 4, ctypes.byref(p), outs),
                            "frames", d.handle)
                    torch.cuda.synchronize()
                res[(pf, si)] = ([b.view(torch.int16).cpu().numpy() for b in bufs],
                                 [c.cpu().numpy() for c in cnts], int(total.item()))
        finally:
            d.close()
    for si in range(len(sets)):
        for j in range(4):
            assert np.array_equal(res[(1, si)][1][j], res[(0, si)][1][j]), f"set {si} frame {j} counts"
            assert np.array_equal(res[(1, si)][0][j], res[(0, si)][0][j]), f"set {si} frame {j} rgba"
        assert res[(1, si)][2] == res[(0, si)][2]
