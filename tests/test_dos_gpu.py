"""GPU parity of the directional-occlusion renderer (rc1pdosct) against the CPU oracle.

Two stages, each bit-exact (tolerance 0) under CVR-SPEC:
  * the extinction-coefficient pyramid (extcoefvolumegenerator.cpp:230-408) built by
    ext_level_kernel / ext_to_tau_kernel vs oracle.ext_volume, every level;
  * the cone-traced frame (ray_bbox_marching.comp:607-734) vs oracle.render_dos on
    the same pyramid, for occlusion, shadows (point / spot / directional), Blinn-Phong
    and the 7-ray cone packing.
The cone tables both sides use come from cvr_build_cone_tables, which is pinned
against the reference's own ConeGaussianSampler (tests/test_cones.py).  The GLSL
stages themselves cannot run here (no GL), so their restatement is pinned by
construction only ("Parity pinning").
"""
import ctypes
import math

import numpy as np
import pytest

from cpp_volume_rendering_amd import _native as N
from cpp_volume_rendering_amd import datasets as D
from cpp_volume_rendering_amd.renderer import Camera, Device, default_cone_params, make_frame

from test_rc1pass_gpu import assert_bitexact

pytestmark = pytest.mark.gpu

INITIAL = D.INITIAL_STATE_CAMERA
LIGHT0 = dict(position=(-206.873, -51.0699, 557.011), forward=(-0.346883, -0.0856335, 0.933991),
              up=(-0.0298143, 0.996327, 0.0802758), right=(0.937434, -0.0, 0.348162),
              spot_angle_deg=20.0)


@pytest.fixture(scope="module")
def dev():
    import torch
    assert torch.cuda.is_available(), "GPU tests need a HIP device"
    d = Device(0)
    yield d
    d.close()


def cone_tables(params, diag, frac):
    p = N.ConeParams.from_buffer_copy(params)
    if p.covered_distance <= 0:
        p.covered_distance = float(np.float32(diag * np.float32(frac)))
    t = N.ConeTables()
    N.check(N.lib().cvr_build_cone_tables(ctypes.byref(p), 1.0, ctypes.byref(t)), "cones")
    return t


def setup(dev, vol, scale, tf, tf_rgba, res, sigma0=1.0, gmode=0):
    dev.set_volume(vol, scale)
    dev.set_transfer_function(tf)
    dev.set_gradient(gmode)
    dev.set_extinction_volume(tf_rgba, res, sigma0)


def gpu_dos(dev, cam, W, H, step, occ, sdw, apply_occlusion=True, apply_shadow=False,
            shadow_type=0, light=LIGHT0, phong=False, shading=(0.5, 0.5, 0.8, 30.0)):
    p = N.DosParams()
    p.step = step
    p.apply_gradient_shading = int(phong)
    p.ka, p.kd, p.ks, p.shininess = shading
    p.ispecular[:] = [1.0, 1.0, 1.0]
    p.light.position[:] = list(light["position"])
    p.light.forward[:] = list(light["forward"])
    p.light.up[:] = list(light["up"])
    p.light.right[:] = list(light["right"])
    p.light.spot_angle_deg = light["spot_angle_deg"]
    p.apply_occlusion, p.apply_shadow, p.shadow_type = int(apply_occlusion), int(apply_shadow), shadow_type
    p.occlusion, p.shadow = occ, sdw
    frame = make_frame(Camera(**cam), W, H)
    rgba = np.zeros((H, W, 4), np.float32)
    cnt = np.zeros((H, W), np.uint32)
    total = np.zeros(1, np.uint64)
    out = N.Output(rgba.ctypes.data, cnt.ctypes.data, total.ctypes.data, 0)
    N.check(N.lib().cvr_render_dosct(dev.handle, ctypes.byref(frame), ctypes.byref(p),
                                     ctypes.byref(out)), "cvr_render_dosct", dev.handle)
    return rgba, cnt, int(total[0])


@pytest.mark.parametrize("res,sigma0", [((40, 32, 24), 1.0), ((32, 32, 32), 1.5),
                                        ((128, 128, 128), 1.0)])
def test_extinction_pyramid_bitexact(dev, oracle, bonsai_tf, bonsai_tf_rgba, res, sigma0):
    vol = D.marschner_lobb_u8(48)[:, :, :44].copy()
    scale = (10.0, 10.5, 9.0)
    setup(dev, vol, scale, bonsai_tf, bonsai_tf_rgba, res, sigma0)
    got = dev.extinction_levels()
    want = oracle.ext_volume(oracle.volume_r16f(vol), scale, bonsai_tf_rgba, res, sigma0)
    assert len(got) == len(want) == int(math.log2(max(res))) + 1
    for L, (g, w) in enumerate(zip(got, want)):
        assert g.shape == w.shape == tuple(oracle.ext_level_dims(res, L)[::-1])
        assert_bitexact(g, w, f"level {L}")
    assert np.isfinite(got[0]).all() and (got[0] >= 0).all()
    assert got[0].max() > 0


def _occ7():
    c = default_cone_params(True)
    c.half_angle_deg, c.max_packing, c.covered_distance = 30.0, 2, 300.0
    return c


DOS_CASES = {
    "occlusion": dict(),
    "shadow_point": dict(apply_shadow=True, shadow_type=0),
    "shadow_spot": dict(apply_shadow=True, shadow_type=1),
    "shadow_dir": dict(apply_shadow=True, shadow_type=2),
    "shadow_only": dict(apply_occlusion=False, apply_shadow=True, shadow_type=0),
    "phong_fd": dict(apply_shadow=True, phong=True, gmode=1),
    "occ7_ragged": dict(occ=_occ7, W=77, H=53),
    "inside": dict(cam=dict(eye=(10.0, -20.0, 30.0), center=(100.0, 50.0, -200.0),
                            up=(0.0, 1.0, 0.0)), W=64, H=48),
}


@pytest.mark.parametrize("name", sorted(DOS_CASES))
def test_dosct_bitexact_vs_oracle(dev, oracle, bonsai_tf, bonsai_tf_rgba, name):
    c = DOS_CASES[name]
    n = 48
    vol = D.marschner_lobb_u8(n)
    scale = D.voxel_scale(n)
    res = (64, 64, 64)
    gmode = c.get("gmode", 0)
    setup(dev, vol, scale, bonsai_tf, bonsai_tf_rgba, res, gmode=gmode)
    diag = math.sqrt(sum((n * s) ** 2 for s in scale))
    occ = c["occ"]() if "occ" in c else default_cone_params(True)
    sdw = default_cone_params(False)
    W, H = c.get("W", 96), c.get("H", 80)
    cam = c.get("cam", INITIAL)
    step = oracle.default_step(scale)
    kw = dict(apply_occlusion=c.get("apply_occlusion", True),
              apply_shadow=c.get("apply_shadow", False), shadow_type=c.get("shadow_type", 0),
              phong=c.get("phong", False))
    g_rgba, g_cnt, g_total = gpu_dos(dev, cam, W, H, step, occ, sdw, **kw)

    levels = oracle.ext_volume(oracle.volume_r16f(vol), scale, bonsai_tf_rgba, res)
    for L, (g, w) in enumerate(zip(dev.extinction_levels(), levels)):
        assert_bitexact(g, w, f"level {L}")
    grad = oracle.gradient(vol, "fd") if gmode == 1 else None
    o_rgba, o_cnt, o_total = oracle.render_dos(
        oracle.volume_r16f(vol), scale, bonsai_tf, levels, cam, W, H, step,
        cone_tables(occ, diag, 0.50), cone_tables(sdw, diag, 0.75), light=LIGHT0, grad=grad,
        **kw)
    assert_bitexact(g_cnt, o_cnt, f"{name} counts")
    assert_bitexact(g_rgba, o_rgba, f"{name} rgba")
    assert g_total == o_total == int(o_cnt.sum())
    assert o_rgba[..., 3].max() > 0.5          # the frame is not empty


def test_dosct_occlusion_darkens(dev, bonsai_tf, bonsai_tf_rgba):
    """Occlusion only attenuates: every RGB channel <= the unoccluded march's."""
    vol = D.marschner_lobb_u8(48)
    scale = D.voxel_scale(48)
    setup(dev, vol, scale, bonsai_tf, bonsai_tf_rgba, (64, 64, 64))
    occ, sdw = default_cone_params(True), default_cone_params(False)
    g, _, _ = gpu_dos(dev, INITIAL, 96, 80, 0.0, occ, sdw)
    p = N.Rc1passParams()
    p.ka, p.kd, p.ks, p.shininess = 0.5, 0.5, 0.8, 30.0
    rgba = np.zeros((80, 96, 4), np.float32)
    out = N.Output(rgba.ctypes.data, None, None, 0)
    N.check(N.lib().cvr_render_rc1pass(dev.handle, ctypes.byref(make_frame(Camera(**INITIAL), 96, 80)),
                                       ctypes.byref(p), ctypes.byref(out)), "rc1pass", dev.handle)
    assert (g[..., :3] <= rgba[..., :3] + 1e-6).all()
    assert g[..., :3].sum() < rgba[..., :3].sum()


def test_dosct_errors(bonsai_tf):
    d = Device(0)
    try:
        vol = D.sphere_u8(16)
        d.set_volume(vol, (1.0, 1.0, 1.0))
        d.set_transfer_function(bonsai_tf)
        p = N.DosParams()
        p.occlusion, p.shadow = default_cone_params(True), default_cone_params(False)
        p.apply_occlusion = 1
        img = np.zeros((8, 8, 4), np.float32)
        out = N.Output(img.ctypes.data, None, None, 0)
        fr = make_frame(Camera(**INITIAL), 8, 8)
        st = N.lib().cvr_render_dosct(d.handle, ctypes.byref(fr), ctypes.byref(p), ctypes.byref(out))
        assert st == N.CVR_ERR_STATE            # no extinction volume yet
        d.set_extinction_volume(bonsai_tf, (8, 8, 8))
        p.shadow_type = 7
        p.apply_shadow = 1
        st = N.lib().cvr_render_dosct(d.handle, ctypes.byref(fr), ctypes.byref(p), ctypes.byref(out))
        assert st == N.CVR_ERR_ARG
        with pytest.raises(N.CvrError):
            d.set_extinction_volume(bonsai_tf, (0, 8, 8))
    finally:
        d.close()


@pytest.mark.parametrize("nranks,tile", [(2, 32), (3, 16)])
def test_dosct_screen_tiles_match_full_frame(dev, bonsai_tf, bonsai_tf_rgba, nranks, tile):
    """Multi-GPU split of the shaded renderer: packed per-rank tiles equal the full frame."""
    from cpp_volume_rendering_amd import screen_tiles as T
    vol = D.marschner_lobb_u8(48)
    scale = D.voxel_scale(48)
    setup(dev, vol, scale, bonsai_tf, bonsai_tf_rgba, (64, 64, 64))
    occ, sdw = default_cone_params(True), default_cone_params(False)
    W, H = 100, 72
    full, full_cnt, full_total = gpu_dos(dev, INITIAL, W, H, 0.0, occ, sdw, apply_shadow=True)
    tpr = T.max_tiles_per_rank(W, H, tile, nranks)
    packed = np.zeros((nranks, tpr, tile, tile, 4), np.float32)
    tot = 0
    for r in range(nranks):
        p = N.DosParams()
        p.ka, p.kd, p.ks, p.shininess = 0.5, 0.5, 0.8, 30.0
        p.ispecular[:] = [1.0, 1.0, 1.0]
        for f in ("position", "forward", "up", "right"):
            getattr(p.light, f)[:] = list(LIGHT0[f])
        p.light.spot_angle_deg = LIGHT0["spot_angle_deg"]
        p.apply_occlusion, p.apply_shadow = 1, 1
        p.occlusion, p.shadow = occ, sdw
        k = T.tiles_for_rank(W, H, tile, r, nranks)
        rgba = np.zeros((k, tile, tile, 4), np.float32)
        total = np.zeros(1, np.uint64)
        out = N.Output(rgba.ctypes.data, None, total.ctypes.data, 0)
        fr = make_frame(Camera(**INITIAL), W, H, tile, r, nranks)
        N.check(N.lib().cvr_render_dosct(dev.handle, ctypes.byref(fr), ctypes.byref(p),
                                         ctypes.byref(out)), "dosct tiles", dev.handle)
        packed[r, :k] = rgba
        tot += int(total[0])
    assert tot == full_total
    assert_bitexact(T.unpack(packed, W, H, tile, nranks), full, "dos tiles")


@pytest.mark.parametrize("name", ["occlusion", "shadow_spot", "phong_fd", "occ7_ragged", "inside"])
def test_dosct_flat_equals_per_wave(dev, bonsai_tf, bonsai_tf_rgba, name):
    """Flat shading (the default: one job list, shaded by its own grid and folded per
    pixel, shaded_march.h) against the per-wave deferred kernel, bit for bit, for
    several XCD chunk groupings, counts included."""
    c = DOS_CASES[name]
    n = 48
    vol = D.marschner_lobb_u8(n)
    scale = D.voxel_scale(n)
    setup(dev, vol, scale, bonsai_tf, bonsai_tf_rgba, (64, 64, 64), gmode=c.get("gmode", 0))
    occ = c["occ"]() if "occ" in c else default_cone_params(True)
    sdw = default_cone_params(False)
    W, H = c.get("W", 96), c.get("H", 80)
    kw = dict(apply_occlusion=c.get("apply_occlusion", True),
              apply_shadow=c.get("apply_shadow", False), shadow_type=c.get("shadow_type", 0),
              phong=c.get("phong", False))
    L = N.lib()
    step = 0.5 / math.sqrt(3.0)
    try:
        L.cvr_set_option(dev.handle, b"shade_flat", 0)
        ref = gpu_dos(dev, c.get("cam", INITIAL), W, H, step, occ, sdw, **kw)
        L.cvr_set_option(dev.handle, b"shade_flat", 1)
        for group in (1, 8, 64):
            L.cvr_set_option(dev.handle, b"flat_group", group)
            got = gpu_dos(dev, c.get("cam", INITIAL), W, H, step, occ, sdw, **kw)
            assert_bitexact(got[1], ref[1], f"{name} counts (group {group})")
            assert_bitexact(got[0], ref[0], f"{name} rgba (group {group})")
            assert got[2] == ref[2]
    finally:
        L.cvr_set_option(dev.handle, b"shade_flat", 1)
        L.cvr_set_option(dev.handle, b"flat_group", 8)


def _dos_params(occ, sdw, step, apply_shadow=True):
    p = N.DosParams()
    p.step = step
    p.ka, p.kd, p.ks, p.shininess = 0.5, 0.5, 0.8, 30.0
    p.ispecular[:] = [1.0, 1.0, 1.0]
    for k in ("position", "forward", "up", "right"):
        getattr(p.light, k)[:] = list(LIGHT0[k])
    p.light.spot_angle_deg = LIGHT0["spot_angle_deg"]
    p.apply_occlusion, p.apply_shadow, p.shadow_type = 1, int(apply_shadow), 0
    p.occlusion, p.shadow = occ, sdw
    return p


FAR = dict(eye=(700.0, 600.0, 1400.0), center=(0.0, 0.0, 0.0), up=(0.0, 1.0, 0.0))


def test_dosct_flat_fallback_and_growth(dev, bonsai_tf, bonsai_tf_rgba):
    """The flat pipeline without host round trips (shaded_march.h launch_shaded_flat): a
    stream's job-list set is sized from its earlier frames' totals; a frame with more jobs
    than the set holds is rendered by the per-wave kernel, chosen on the device, and the
    set grows for the frames after it.  Every frame equals the per-wave kernel bit for
    bit: far view (sizes the set), near view (does not fit: fallback), near again (grown),
    and near with debug_flat_limit = 1 (fallback forced)."""
    n = 48
    vol = D.marschner_lobb_u8(n)
    scale = D.voxel_scale(n)
    setup(dev, vol, scale, bonsai_tf, bonsai_tf_rgba, (64, 64, 64))
    occ, sdw = default_cone_params(True), default_cone_params(False)
    W, H = 96, 80
    step = 0.5 / math.sqrt(3.0)
    L = N.lib()
    try:
        L.cvr_set_option(dev.handle, b"shade_flat", 0)
        ref = {k: gpu_dos(dev, cam, W, H, step, occ, sdw, apply_shadow=True)
               for k, cam in (("far", FAR), ("near", INITIAL))}
        assert ref["near"][0][..., 3].sum() > 4 * ref["far"][0][..., 3].sum()
        L.cvr_set_option(dev.handle, b"shade_flat", 1)
        d2 = Device(0)   # a fresh context: its stream's set starts empty
        try:
            setup(d2, vol, scale, bonsai_tf, bonsai_tf_rgba, (64, 64, 64))
            caps = []
            for k, lim in (("far", 0), ("near", 0), ("near", 0), ("far", 0), ("near", 1)):
                N.check(L.cvr_set_option(d2.handle, b"debug_flat_limit", lim), "limit")
                got = gpu_dos(d2, FAR if k == "far" else INITIAL, W, H, step, occ, sdw,
                              apply_shadow=True)
                assert_bitexact(got[1], ref[k][1], f"{k} counts (limit {lim})")
                assert_bitexact(got[0], ref[k][0], f"{k} rgba (limit {lim})")
                assert got[2] == ref[k][2]
                caps.append(L.cvr_get_option(d2.handle, b"flat_cap_kjobs"))
            assert caps[2] > caps[1] >= caps[0] > 0, caps   # grew after the near frame
        finally:
            d2.close()
    finally:
        L.cvr_set_option(dev.handle, b"shade_flat", 1)


def test_dosct_frames_in_flight_on_streams(bonsai_tf, bonsai_tf_rgba):
    """Device outputs on three render streams, frames submitted back to back with no
    host synchronisation in between (each stream has its own job-list set): every frame
    equals the per-wave kernel's image of its view bit for bit."""
    import torch
    n = 48
    vol = D.marschner_lobb_u8(n)
    scale = D.voxel_scale(n)
    dev = Device(0)
    setup(dev, vol, scale, bonsai_tf, bonsai_tf_rgba, (64, 64, 64))
    occ, sdw = default_cone_params(True), default_cone_params(False)
    W, H = 96, 80
    step = 0.5 / math.sqrt(3.0)
    cams = [INITIAL, FAR, dict(eye=(-300.0, 120.0, 420.0), center=(0.0, 0.0, 0.0), up=(0.0, 1.0, 0.0))]
    L = N.lib()
    L.cvr_set_option(dev.handle, b"shade_flat", 0)
    ref = [gpu_dos(dev, c, W, H, step, occ, sdw, apply_shadow=True)[0] for c in cams]
    L.cvr_set_option(dev.handle, b"shade_flat", 1)
    streams = [torch.cuda.Stream() for _ in range(3)]
    p = _dos_params(occ, sdw, step)
    # the images are zeroed on torch's stream: let that finish before the renders
    outs = [torch.zeros((H, W, 4), dtype=torch.float32, device="cuda") for _ in range(12)]
    torch.cuda.synchronize()
    try:
        for i in range(12):
            s = streams[i % 3]
            img = outs[i]
            dev.set_stream(s.cuda_stream)
            frame = make_frame(Camera(**cams[i % 3]), W, H)
            o = N.Output(img.data_ptr(), None, None, 1)
            N.check(L.cvr_render_dosct(dev.handle, ctypes.byref(frame), ctypes.byref(p),
                                       ctypes.byref(o)), "render", dev.handle)
        torch.cuda.synchronize()
        for i, img in enumerate(outs):
            assert_bitexact(img.cpu().numpy(), ref[i % 3], f"frame {i} (stream {i % 3})")
    finally:
        dev.close()
