"""GPU parity at BASELINE.json's own configuration sizes (configs 2-5), through the C-ABI.

The smaller parity suites exercise every code path at toy sizes; these run the
configured sizes, whose indexing and allocation sizes (a 6.5 GiB gradient grid at
512^3, 159-section shadow cones at 2048^2, a 1026^3 SAT of 4.3 GB with 289 wavefront
launches and a 17.3 GiB cell4 copy) no toy case reaches:

  * C2: a 256^3 u8 volume written as a reference `.raw` file
    (name.<bytes>.<W>x<H>x<D>.raw, reader.cpp:162-225), read back by cvr_read_raw,
    rendered at 1024^2: the whole frame against the oracle, bit for bit.
  * C3: 512^3 at 1024^2 with finite-difference gradients and Blinn-Phong: the whole
    frame against the oracle (RGBA bits and per-pixel iteration counts).
  * C4: 512^3 at 2048^2, directional occlusion with cone AO + point-light cone
    shadows (dosrcrenderer.cpp:44-59, 111-113): the 128^3 extinction pyramid level 0
    against the oracle, a 128-row band of the frame bit for bit, and the full-frame
    sample count against the oracle's count over the same march.
  * C5: 1024^3 extinction SAT (ebsrenderer.cpp:624-723) + EBS frame at 1024^2: every
    plane of the 1026^3 float SAT against the reference recurrence (streamed over z,
    oracle.sat_planes), and bands of the frame bit for bit: the centre band and the
    bands richest in finite shaded pixels (at least 5,000 of them; most of the frame
    is inf/NaN through the reference's float-SAT cancellation).
Tolerance 0 throughout (CVR-SPEC).
"""
import ctypes
import math
import os

import numpy as np
import pytest

from cpp_volume_rendering_amd import _native as N
from cpp_volume_rendering_amd import datasets as D
from cpp_volume_rendering_amd.renderer import (Camera, DataManager, Device, default_cone_params,
                                               make_frame)

from test_dos_gpu import LIGHT0, cone_tables, gpu_dos
from test_ebs import lib_ext_lut
from test_ebs_gpu import LIGHT_FWD, LIGHT_POS, ebs_params, gpu_ebs
from test_rc1pass_gpu import assert_bitexact, gpu_render

pytestmark = pytest.mark.gpu

INITIAL = D.INITIAL_STATE_CAMERA


@pytest.fixture()
def fresh_dev():
    import torch
    assert torch.cuda.is_available(), "GPU tests need a HIP device"
    d = Device(0)
    yield d
    d.close()
    torch.cuda.empty_cache()


def test_c2_raw_256_at_1024(fresh_dev, oracle, bonsai_tf, tmp_path):
    vol = D.marschner_lobb_u8(256)
    path = os.path.join(str(tmp_path), D.raw_name("ml", vol))
    D.write_raw(path, vol)
    assert path.endswith("ml.1.256x256x256.raw")
    dm = DataManager()
    dm.ReadVolume(path, scale=D.voxel_scale(256))
    assert dm.volume.shape == (256, 256, 256) and np.array_equal(dm.volume, vol)
    sc = D.voxel_scale(256)
    g_rgba, g_cnt, g_S = gpu_render(fresh_dev, dm.volume, sc, bonsai_tf, INITIAL, 1024, 1024)
    o_rgba, o_cnt, o_S = oracle.render_rc1pass(oracle.volume_r16f(vol), sc, bonsai_tf, INITIAL,
                                               1024, 1024, oracle.default_step(sc))
    assert_bitexact(g_cnt, o_cnt, "C2 counts")
    assert_bitexact(g_rgba, o_rgba, "C2 rgba")
    assert g_S == o_S > 10_000_000


def test_c3_phong_fd_512_at_1024(fresh_dev, oracle, bonsai_tf):
    vol = D.marschner_lobb_u8(512)
    sc = D.voxel_scale(512)
    light = D.LIGHT_LIST0_POSITION
    g_rgba, g_cnt, g_S = gpu_render(fresh_dev, vol, sc, bonsai_tf, INITIAL, 1024, 1024,
                                    phong=True, gmode=N.GRADIENT_FINITE_DIFFERENCES, light=light)
    grad = oracle.gradient(vol, "fd")
    o_rgba, o_cnt, o_S = oracle.render_rc1pass(oracle.volume_r16f(vol), sc, bonsai_tf, INITIAL,
                                               1024, 1024, oracle.default_step(sc), grad=grad,
                                               phong=True, light=light)
    del grad
    assert_bitexact(g_cnt, o_cnt, "C3 counts")
    assert_bitexact(g_rgba, o_rgba, "C3 rgba")
    assert g_S == o_S


def test_c4_dos_512_at_2048(fresh_dev, oracle, bonsai_tf, bonsai_tf_rgba):
    n, W = 512, 2048
    vol = D.marschner_lobb_u8(n)
    sc = D.voxel_scale(n)
    res = (128, 128, 128)
    fresh_dev.set_volume(vol, sc)
    fresh_dev.set_transfer_function(bonsai_tf)
    fresh_dev.set_gradient(0)
    fresh_dev.set_extinction_volume(bonsai_tf_rgba, res, 1.0)
    occ, sdw = default_cone_params(True), default_cone_params(False)
    diag = math.sqrt(sum((n * s) ** 2 for s in sc))
    t_occ, t_sdw = cone_tables(occ, diag, 0.50), cone_tables(sdw, diag, 0.75)
    # the reference's section counts at these defaults
    assert list(t_occ.counts) == [1, 17, 0] and list(t_sdw.counts) == [159, 0, 0]
    step = oracle.default_step(sc)
    g_rgba, g_cnt, g_S = gpu_dos(fresh_dev, INITIAL, W, W, step, occ, sdw, apply_shadow=True,
                                 shadow_type=0)
    v16 = oracle.volume_r16f(vol)
    levels = oracle.ext_volume(v16, sc, bonsai_tf_rgba, res)
    got_levels = fresh_dev.extinction_levels()
    assert len(got_levels) == len(levels) == 8
    for L, (g, w) in enumerate(zip(got_levels, levels)):
        assert_bitexact(g, w, f"C4 extinction level {L}")
    rows = (W // 2 - 64, W // 2 + 64)
    o_rgba, o_cnt, _ = oracle.render_dos(v16, sc, bonsai_tf, levels, INITIAL, W, W, step, t_occ,
                                         t_sdw, apply_shadow=True, shadow_type=0, light=LIGHT0,
                                         rows=rows)
    assert_bitexact(g_cnt[rows[0]:rows[1]], o_cnt[rows[0]:rows[1]], "C4 band counts")
    assert_bitexact(g_rgba[rows[0]:rows[1]], o_rgba[rows[0]:rows[1]], "C4 band rgba")
    assert o_rgba[rows[0]:rows[1], :, 3].max() > 0.5
    # the whole frame's iteration counts: shading never changes opacity, so the
    # plain march's counts (cheap on the CPU) are the DOS frame's counts
    _, e_cnt, e_S = oracle.render_rc1pass(v16, sc, bonsai_tf, INITIAL, W, W, step)
    assert_bitexact(g_cnt, e_cnt, "C4 full-frame counts")
    assert g_S == e_S > 300_000_000


def test_c5_sat_and_ebs_1024(fresh_dev, oracle, bonsai_tf):
    n, W = 1024, 1024
    vol = D.marschner_lobb_u8(n)
    sc = D.voxel_scale(n)
    lut = lib_ext_lut(1)
    fresh_dev.set_volume(vol, sc)
    fresh_dev.set_transfer_function(bonsai_tf)
    fresh_dev.set_gradient(0)
    fresh_dev.set_extinction_sat(lut)
    sat = fresh_dev.extinction_sat()
    assert sat.shape == (n + 2, n + 2, n + 2)
    # every plane of the GPU SAT against the reference recurrence (one streamed pass)
    want = oracle.sat_planes(vol, lut, range(n + 2))
    assert_bitexact(sat, want, "C5 SAT")
    del want
    v16 = oracle.volume_r16f(vol)
    step = oracle.default_step(sc)
    p = ebs_params(step=step)
    g_rgba, g_cnt, g_S = gpu_ebs(fresh_dev, INITIAL, W, W, p)
    # At 1024^3 most shaded pixels are inf/NaN (the reference's float-SAT cancellation,
    # DESIGN §5c), so the centre band compares mostly NaN with NaN.  Compare the centre
    # band AND the bands richest in finite shaded pixels, and require thousands of
    # those to match bit for bit.
    bands, n_fin = oracle.finite_shaded_bands(g_rgba, 32, need=8000, max_bands=4)
    bands = sorted(set(bands) | {(W // 2 - 32, W // 2 + 32)})
    compared = 0
    for rows in bands:
        o_rgba, o_cnt, _ = oracle.render_ebs(v16, sc, bonsai_tf, sat, INITIAL, W,
                                             W, step, light=LIGHT_POS, light_forward=LIGHT_FWD,
                                             rows=rows)
        assert_bitexact(g_cnt[rows[0]:rows[1]], o_cnt[rows[0]:rows[1]], f"C5 band {rows} counts")
        assert_bitexact(g_rgba[rows[0]:rows[1]], o_rgba[rows[0]:rows[1]], f"C5 band {rows} rgba")
        ob = o_rgba[rows[0]:rows[1]]
        compared += int((np.isfinite(ob).all(-1) & (ob[..., 3] > 0)).sum())
    print(f"C5: bands {bands}, {compared} finite shaded pixels compared bit for bit")
    assert compared >= 5000, f"only {compared} finite shaded pixels in the compared bands"
    _, e_cnt, e_S = oracle.render_rc1pass(v16, sc, bonsai_tf, INITIAL, W, W, step)
    assert_bitexact(g_cnt, e_cnt, "C5 full-frame counts")
    assert g_S == e_S
    # the plain float SAT (sat_layout 1: no 17 GiB cell4 copy; its +1 reads at the far
    # corner stay inside the padding, cvr_sat_layout_check): the same frame, bit for bit
    from cpp_volume_rendering_amd import _native as N
    N.check(N.lib().cvr_set_option(fresh_dev.handle, b"sat_layout", 1), "sat_layout", fresh_dev.handle)
    try:
        p_rgba, p_cnt, p_S = gpu_ebs(fresh_dev, INITIAL, W, W, p)
        assert_bitexact(p_cnt, g_cnt, "C5 plain-SAT counts")
        assert_bitexact(p_rgba, g_rgba, "C5 plain-SAT rgba")
        assert p_S == g_S
    finally:
        N.lib().cvr_set_option(fresh_dev.handle, b"sat_layout", 0)


def test_view_matrix_frame_equals_lookat_frame(fresh_dev, bonsai_tf):
    """cvr_frame.use_view (the adapters pass vis::Camera::LookAt directly): with the matrix
    the library would build itself, the frame is the same bit for bit."""
    vol = D.marschner_lobb_u8(64)
    sc = D.voxel_scale(64)
    cam = Camera(**INITIAL)
    view = (ctypes.c_float * 16)()
    tanh = ctypes.c_float()
    N.check(N.lib().cvr_camera_lookat(ctypes.byref(cam.to_c()), view, ctypes.byref(tanh)), "lookat")
    fresh_dev.set_volume(vol, sc)
    fresh_dev.set_transfer_function(bonsai_tf)
    imgs = []
    for use_view in (0, 1):
        f = make_frame(cam, 96, 80)
        if use_view:
            f.use_view = 1
            f.view[:] = list(view)
            f.camera.center[:] = [0.0, 0.0, 0.0]   # ignored
            f.camera.center[0] = 1e6
        rgba = np.zeros((80, 96, 4), np.float32)
        out = N.Output(rgba.ctypes.data, None, None, 0)
        p = N.Rc1passParams()
        N.check(N.lib().cvr_render_rc1pass(fresh_dev.handle, ctypes.byref(f), ctypes.byref(p),
                                           ctypes.byref(out)), "render", fresh_dev.handle)
        imgs.append(rgba)
    assert_bitexact(imgs[1], imgs[0], "use_view")
    assert imgs[0][..., 3].max() > 0.5
