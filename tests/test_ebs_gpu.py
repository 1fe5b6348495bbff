"""GPU parity of the extinction-based shading renderer (rc1pextbsd) against the CPU
oracle, bit for bit (tolerance 0):
  * the summed-area table built on the GPU by the skewed wavefront (sat.hip) vs
    the oracle's literal SummedAreaTable3D<double>::BuildSAT (itself pinned against
    the reference's own build, tests/test_ebs.py), as float;
  * the shaded frame (ebs_ray_bbox_marching.comp:498-625) vs oracle.render_ebs on
    that SAT: ambient occlusion, point / directional shadows, Blinn-Phong.
"""
import ctypes
import math

import numpy as np
import pytest

from cpp_volume_rendering_amd import _native as N
from cpp_volume_rendering_amd import datasets as D
from cpp_volume_rendering_amd.renderer import Camera, Device, make_frame

from test_rc1pass_gpu import assert_bitexact
from test_ebs import lib_ext_lut

pytestmark = pytest.mark.gpu

INITIAL = D.INITIAL_STATE_CAMERA
LIGHT_POS = (-206.873, -51.0699, 557.011)
LIGHT_FWD = (-0.346883, -0.0856335, 0.933991)


@pytest.fixture(scope="module")
def dev():
    import torch
    assert torch.cuda.is_available(), "GPU tests need a HIP device"
    d = Device(0)
    yield d
    d.close()


def gpu_sat(dev, vox, scale=(1.0, 1.0, 1.0)):
    dev.set_volume(vox, scale)
    lut = lib_ext_lut(vox.dtype.itemsize)
    N.check(N.lib().cvr_set_extinction_sat(dev.handle, N.fptr(lut), lut.shape[0]), "sat", dev.handle)
    dims = (ctypes.c_int * 3)()
    N.check(N.lib().cvr_copy_extinction_sat(dev.handle, None, 0, dims), "sat dims", dev.handle)
    out = np.zeros((dims[2], dims[1], dims[0]), np.float32)
    N.check(N.lib().cvr_copy_extinction_sat(dev.handle, N.fptr(out), out.size, dims), "sat copy",
            dev.handle)
    return out, lut


@pytest.mark.parametrize("shape,bpv", [((4, 5, 6), 1), ((23, 29, 37), 1), ((70, 17, 9), 1),
                                       ((33, 40, 20), 2), ((96, 96, 96), 1)])
def test_sat_bitexact_vs_reference_recurrence(dev, oracle, shape, bpv):
    rng = np.random.default_rng(sum(shape) + bpv)
    if bpv == 1:
        vox = rng.integers(0, 256, shape, dtype=np.uint8)
    else:
        vox = rng.integers(0, 65536, shape, dtype=np.uint16)
    got, lut = gpu_sat(dev, vox)
    want = oracle.sat_build(vox, lut).astype(np.float32)
    assert got.shape == want.shape == tuple(s + 2 for s in shape)
    assert_bitexact(got, want, f"SAT {shape}")
    assert got.max() > 0


def test_sat_of_ml_field_matches_oracle(dev, oracle):
    vox = D.marschner_lobb_u8(64)
    got, lut = gpu_sat(dev, vox, D.voxel_scale(64))
    assert_bitexact(got, oracle.sat_build(vox, lut).astype(np.float32), "SAT ml64")


def ebs_params(step=0.0, apply_occlusion=True, apply_shadow=True, shadow_type=0, phong=False,
               shells=15, radius=1.0, angle=1.0, interval=2.0, initial=2.0, weight=1.0,
               max_distance=0.0):
    p = N.EbsParams()
    p.step = step
    p.apply_gradient_shading = int(phong)
    p.ka, p.kd, p.ks, p.shininess = 0.5, 0.5, 0.8, 30.0
    p.ispecular[:] = [1.0, 1.0, 1.0]
    p.light_pos[:] = list(LIGHT_POS)
    p.light_forward[:] = list(LIGHT_FWD)
    p.apply_occlusion, p.occlusion_shells, p.occlusion_radius = int(apply_occlusion), shells, radius
    p.apply_shadow, p.shadow_type = int(apply_shadow), shadow_type
    p.shadow_cone_angle_deg, p.shadow_sample_interval = angle, interval
    p.shadow_initial_step, p.shadow_ui_weight, p.shadow_max_distance = initial, weight, max_distance
    return p


def gpu_ebs(dev, cam, W, H, p, tile=0, rank=0, nranks=1):
    frame = make_frame(Camera(**cam), W, H, tile, rank, nranks)
    rgba = np.zeros((H, W, 4), np.float32)
    cnt = np.zeros((H, W), np.uint32)
    total = np.zeros(1, np.uint64)
    out = N.Output(rgba.ctypes.data, cnt.ctypes.data, total.ctypes.data, 0)
    N.check(N.lib().cvr_render_extbsd(dev.handle, ctypes.byref(frame), ctypes.byref(p),
                                      ctypes.byref(out)), "cvr_render_extbsd", dev.handle)
    return rgba, cnt, int(total[0])


EBS_CASES = {
    "defaults_point": dict(),
    "occlusion_only": dict(apply_shadow=False),
    "shadow_only": dict(apply_occlusion=False),
    "directional": dict(shadow_type=1),
    "phong": dict(phong=True),
    "wide_cone": dict(angle=12.0, interval=3.0, initial=1.0, weight=0.7, shells=6, radius=1.5,
                      max_distance=150.0),
    # cone angles past 44 deg take the IEEE division for the cone edges (ebs.hip
    # cone_div): the edge's axis component d can reach 0 near 90 deg
    "cone_60": dict(angle=60.0, max_distance=60.0),
    "cone_89": dict(angle=89.0, max_distance=40.0, apply_occlusion=False),
    "ragged_inside": dict(W=57, H=43, cam=dict(eye=(10.0, -20.0, 30.0), center=(100.0, 50.0, -200.0),
                                            up=(0.0, 1.0, 0.0))),
}


@pytest.mark.parametrize("name", sorted(EBS_CASES))
def test_ebs_bitexact_vs_oracle(dev, oracle, bonsai_tf, name):
    c = dict(EBS_CASES[name])
    n = 40
    vol = D.marschner_lobb_u8(n)
    scale = D.voxel_scale(n)
    W, H = c.pop("W", 80), c.pop("H", 64)
    cam = c.pop("cam", INITIAL)
    phong = c.get("phong", False)
    sat, lut = gpu_sat(dev, vol, scale)
    dev.set_transfer_function(bonsai_tf)
    dev.set_gradient(1 if phong else 0)
    step = oracle.default_step(scale)
    p = ebs_params(step=step, **c)
    g_rgba, g_cnt, g_total = gpu_ebs(dev, cam, W, H, p)
    want_sat = oracle.sat_build(vol, lut).astype(np.float32)
    assert_bitexact(sat, want_sat, "SAT")
    o_rgba, o_cnt, o_total = oracle.render_ebs(
        oracle.volume_r16f(vol), scale, bonsai_tf, want_sat, cam, W, H, step,
        apply_occlusion=p.apply_occlusion, occ_shells=p.occlusion_shells,
        occ_radius=p.occlusion_radius, apply_shadow=p.apply_shadow, shadow_type=p.shadow_type,
        cone_angle_deg=p.shadow_cone_angle_deg, interval=p.shadow_sample_interval,
        initial_step=p.shadow_initial_step, ui_weight=p.shadow_ui_weight,
        max_distance=(p.shadow_max_distance if p.shadow_max_distance > 0 else None),
        light=LIGHT_POS, light_forward=LIGHT_FWD,
        grad=oracle.gradient(vol, "fd") if phong else None, phong=phong)
    assert_bitexact(g_cnt, o_cnt, f"{name} counts")
    assert_bitexact(g_rgba, o_rgba, f"{name} rgba")
    assert g_total == o_total == int(o_cnt.sum())
    assert o_rgba[..., 3].max() > 0.5


def test_ebs_errors(bonsai_tf):
    d = Device(0)
    try:
        d.set_volume(D.sphere_u8(16), (1.0, 1.0, 1.0))
        d.set_transfer_function(bonsai_tf)
        p = ebs_params()
        img = np.zeros((8, 8, 4), np.float32)
        out = N.Output(img.ctypes.data, None, None, 0)
        fr = make_frame(Camera(**INITIAL), 8, 8)
        L = N.lib()
        assert L.cvr_render_extbsd(d.handle, ctypes.byref(fr), ctypes.byref(p), ctypes.byref(out)) == N.CVR_ERR_STATE
        lut = lib_ext_lut(1)
        assert L.cvr_set_extinction_sat(d.handle, N.fptr(lut), 255) == N.CVR_ERR_ARG
        N.check(L.cvr_set_extinction_sat(d.handle, N.fptr(lut), 256), "sat", d.handle)
        p.shadow_type = 2
        assert L.cvr_render_extbsd(d.handle, ctypes.byref(fr), ctypes.byref(p), ctypes.byref(out)) == N.CVR_ERR_ARG
    finally:
        d.close()


@pytest.mark.parametrize("nranks,tile", [(2, 32), (3, 16), (8, 32)])
def test_ebs_screen_tiles_match_full_frame(dev, bonsai_tf, nranks, tile):
    """Multi-GPU split of the EBS renderer (config 5 runs over 8 GPUs): every rank's packed
    tiles, unpacked, equal the 1-GPU frame bit for bit, and the sample counts add up."""
    from cpp_volume_rendering_amd import screen_tiles as T
    n = 40
    vol = D.marschner_lobb_u8(n)
    gpu_sat(dev, vol, D.voxel_scale(n))
    dev.set_transfer_function(bonsai_tf)
    dev.set_gradient(0)
    p = ebs_params()
    W, H = 100, 72
    full, _, full_total = gpu_ebs(dev, INITIAL, W, H, p)
    tpr = T.max_tiles_per_rank(W, H, tile, nranks)
    packed = np.zeros((nranks, tpr, tile, tile, 4), np.float32)
    tot = 0
    for r in range(nranks):
        k = T.tiles_for_rank(W, H, tile, r, nranks)
        rgba = np.zeros((k, tile, tile, 4), np.float32)
        total = np.zeros(1, np.uint64)
        out = N.Output(rgba.ctypes.data, None, total.ctypes.data, 0)
        fr = make_frame(Camera(**INITIAL), W, H, tile, r, nranks)
        N.check(N.lib().cvr_render_extbsd(dev.handle, ctypes.byref(fr), ctypes.byref(p),
                                          ctypes.byref(out)), "extbsd tiles", dev.handle)
        packed[r, :k] = rgba
        tot += int(total[0])
    assert tot == full_total
    assert_bitexact(T.unpack(packed, W, H, tile, nranks), full, "ebs tiles")


@pytest.mark.parametrize("name", ["defaults_point", "phong", "directional", "ragged_inside"])
def test_ebs_flat_equals_per_wave(dev, bonsai_tf, name):
    """Flat shading (the default) against the per-wave deferred kernel, bit for bit,
    counts included, for several XCD chunk groupings and a screen-tile share."""
    c = dict(EBS_CASES[name])
    n = 40
    vol = D.marschner_lobb_u8(n)
    scale = D.voxel_scale(n)
    W, H = c.pop("W", 80), c.pop("H", 64)
    cam = c.pop("cam", INITIAL)
    gpu_sat(dev, vol, scale)
    dev.set_transfer_function(bonsai_tf)
    dev.set_gradient(1 if c.get("phong", False) else 0)
    p = ebs_params(step=0.5 / math.sqrt(3.0), **c)
    L = N.lib()
    try:
        for tile, rank, nranks in ((0, 0, 1), (16, 1, 3)):
            L.cvr_set_option(dev.handle, b"shade_flat", 0)
            ref = gpu_ebs(dev, cam, W, H, p, tile, rank, nranks)
            L.cvr_set_option(dev.handle, b"shade_flat", 1)
            for group in (1, 8, 64):
                L.cvr_set_option(dev.handle, b"flat_group", group)
                got = gpu_ebs(dev, cam, W, H, p, tile, rank, nranks)
                assert_bitexact(got[1], ref[1], f"{name} counts (group {group}, split {nranks})")
                assert_bitexact(got[0], ref[0], f"{name} rgba (group {group}, split {nranks})")
                assert got[2] == ref[2]
    finally:
        L.cvr_set_option(dev.handle, b"shade_flat", 1)
        L.cvr_set_option(dev.handle, b"flat_group", 8)


def test_ebs_flat_fallback_growth_and_streams(bonsai_tf):
    """EBS through the flat pipeline without host round trips: a far view sizes the
    stream's set, a near view does not fit (device-side per-wave fallback), the set grows;
    then frames on three streams in flight with device outputs.  All bit-exact with the
    per-wave kernel."""
    import torch
    n = 40
    vol = D.marschner_lobb_u8(n)
    scale = D.voxel_scale(n)
    far = dict(eye=(700.0, 600.0, 1400.0), center=(0.0, 0.0, 0.0), up=(0.0, 1.0, 0.0))
    cams = [far, INITIAL, INITIAL, far]
    W, H = 80, 64
    L = N.lib()
    d = Device(0)
    try:
        gpu_sat(d, vol, scale)
        d.set_transfer_function(bonsai_tf)
        p = ebs_params(step=0.5 / math.sqrt(3.0))
        L.cvr_set_option(d.handle, b"shade_flat", 0)
        ref = [gpu_ebs(d, c, W, H, p) for c in (far, INITIAL)]
        L.cvr_set_option(d.handle, b"shade_flat", 1)
        for i, c in enumerate(cams):
            got = gpu_ebs(d, c, W, H, p)
            r = ref[0] if c is far else ref[1]
            assert_bitexact(got[1], r[1], f"frame {i} counts")
            assert_bitexact(got[0], r[0], f"frame {i} rgba")
            assert got[2] == r[2]
        streams = [torch.cuda.Stream() for _ in range(3)]
        # the images are zeroed on torch's stream: let that finish before the renders
        outs = [torch.zeros((H, W, 4), dtype=torch.float32, device="cuda") for _ in range(9)]
        torch.cuda.synchronize()
        for i in range(9):
            img = outs[i]
            d.set_stream(streams[i % 3].cuda_stream)
            frame = make_frame(Camera(**cams[i % 2]), W, H)
            o = N.Output(img.data_ptr(), None, None, 1)
            N.check(L.cvr_render_extbsd(d.handle, ctypes.byref(frame), ctypes.byref(p),
                                        ctypes.byref(o)), "render", d.handle)
        torch.cuda.synchronize()
        for i, img in enumerate(outs):
            assert_bitexact(img.cpu().numpy(), ref[0 if i % 2 == 0 else 1][0], f"stream frame {i}")
    finally:
        d.close()


@pytest.mark.parametrize("name", ["defaults_point", "phong", "directional", "ragged_inside", "cone_60"])
def test_ebs_sat_layouts_bitexact(dev, bonsai_tf, name):
    """The frame read from the plain float SAT (sat_layout 1, its clamped +1 neighbours in
    the zero padding) equals the cell4 copy's frame bit for bit, flat and per-wave, and
    switching back rebuilds the copy."""
    c = dict(EBS_CASES[name])
    n = 40
    vol = D.marschner_lobb_u8(n)
    scale = D.voxel_scale(n)
    W, H = c.pop("W", 80), c.pop("H", 64)
    cam = c.pop("cam", INITIAL)
    gpu_sat(dev, vol, scale)
    dev.set_transfer_function(bonsai_tf)
    dev.set_gradient(1 if c.get("phong", False) else 0)
    p = ebs_params(step=0.5 / math.sqrt(3.0), **c)
    L = N.lib()
    try:
        for flat in (1, 0):
            L.cvr_set_option(dev.handle, b"shade_flat", flat)
            L.cvr_set_option(dev.handle, b"sat_layout", 0)
            ref = gpu_ebs(dev, cam, W, H, p)
            N.check(L.cvr_set_option(dev.handle, b"sat_layout", 1), "sat_layout", dev.handle)
            got = gpu_ebs(dev, cam, W, H, p)
            assert_bitexact(got[1], ref[1], f"{name} counts (flat {flat})")
            assert_bitexact(got[0], ref[0], f"{name} rgba (flat {flat})")
            L.cvr_set_option(dev.handle, b"sat_layout", 0)
            back = gpu_ebs(dev, cam, W, H, p)
            assert_bitexact(back[0], ref[0], f"{name} rgba after switching back (flat {flat})")
    finally:
        L.cvr_set_option(dev.handle, b"shade_flat", 1)
        L.cvr_set_option(dev.handle, b"sat_layout", 0)


def test_ebs_sat_plain_layout_fresh_build(bonsai_tf):
    """sat_layout 1 set before the build: no cell4 copy is made (device bytes), the frame
    equals the cell4 build's, and the scratch can be dropped (sat_keep_scratch 0)."""
    n = 36
    vol = D.marschner_lobb_u8(n)
    scale = D.voxel_scale(n)
    p = ebs_params(step=0.5 / math.sqrt(3.0))
    L = N.lib()
    imgs = []
    for layout in (0, 1):
        d = Device(0)
        try:
            N.check(L.cvr_set_option(d.handle, b"sat_layout", layout), "sat_layout", d.handle)
            N.check(L.cvr_set_option(d.handle, b"sat_keep_scratch", 0), "keep", d.handle)
            gpu_sat(d, vol, scale)
            d.set_transfer_function(bonsai_tf)
            imgs.append(gpu_ebs(d, INITIAL, 64, 48, p))
            gpu_sat(d, vol, scale)            # a rebuild after the scratch was freed
            again = gpu_ebs(d, INITIAL, 64, 48, p)
            assert_bitexact(again[0], imgs[-1][0], f"layout {layout} rebuild")
        finally:
            d.close()
    assert_bitexact(imgs[1][0], imgs[0][0], "plain vs cell4 rgba")
    assert_bitexact(imgs[1][1], imgs[0][1], "plain vs cell4 counts")
