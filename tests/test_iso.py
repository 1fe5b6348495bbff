"""CPU checks of the isosurface oracle and host logic (no GPU): the block table
against a numpy restatement of ComputeBlocksFromVolume
(rc1custompisoadaptrenderer.cpp:20-117), analytic properties of the marches, and
the renderer classes' reference metadata."""
import numpy as np
import pytest

from cpp_volume_rendering_amd import datasets as D


def numpy_blocks(vox, nb):
    d, h, w = vox.shape
    mx = 255.0 if vox.dtype == np.uint8 else 65535.0
    bs = [(n + b - 1) // b for n, b in zip((w, h, d), nb)]
    lo = np.full((nb[2], nb[1], nb[0]), np.finfo(np.float32).max, np.float32)
    hi = np.full_like(lo, -np.finfo(np.float32).max)
    for bz in range(nb[2]):
        for by in range(nb[1]):
            for bx in range(nb[0]):
                blk = vox[bz * bs[2]:min(bz * bs[2] + bs[2], d), by * bs[1]:min(by * bs[1] + bs[1], h),
                          bx * bs[0]:min(bx * bs[0] + bs[0], w)]
                if blk.size:
                    lo[bz, by, bx] = np.float32(blk.min() / mx)
                    hi[bz, by, bx] = np.float32(blk.max() / mx)
    return lo, hi


@pytest.mark.parametrize("nb", [(4, 4, 4), (32, 32, 32), (5, 3, 7)])
def test_block_table_matches_numpy(oracle, nb):
    for vox in (D.marschner_lobb_u8(48)[:, :40, :33].copy(),
                D.marschner_lobb_u8(24).astype(np.uint16) * 257 + 3):
        lo, hi = oracle.iso_blocks(vox, nb)
        n_lo, n_hi = numpy_blocks(vox, nb)
        assert np.array_equal(lo, n_lo) and np.array_equal(hi, n_hi)


def _sphere(n=64):
    return D.sphere_u8(n)


CAM = dict(eye=(0.0, 0.0, 150.0), center=(0.0, 0.0, 0.0), up=(0.0, 1.0, 0.0))


@pytest.mark.parametrize("variant", [0, 1, 2])
def test_iso_sphere_silhouette(oracle, variant):
    """The 0.5 isosurface of the radial ramp is a sphere of radius ~0.45*N*0.5:
    opaque hits (alpha 1, Color rgb) inside its silhouette, none well outside."""
    vox = _sphere(64)
    v16 = oracle.volume_r16f(vox)
    W = H = 96
    rgba, cnt, S, _ = oracle.render_iso(v16, vox, (1.0, 1.0, 1.0), CAM, W, H, variant=variant)
    a = rgba[..., 3]
    assert set(np.unique(a)).issubset({0.0, 1.0})
    hit = a == 1.0
    assert np.allclose(rgba[hit][:, :3], np.float32([0.66, 0.6, 0.05]))
    # projected silhouette radius in pixels
    tanh = np.tan(np.radians(45.0) / 2)
    r_world = 0.45 * 64 * 0.5
    r_px = r_world / (150.0 - r_world) / tanh * (W / 2)
    yy, xx = np.mgrid[0:H, 0:W]
    rr = np.hypot(xx + 0.5 - W / 2, yy + 0.5 - H / 2)
    assert not hit[rr > r_px + 3].any()
    if variant == 2:     # the plain march finds every hit
        assert hit[rr < r_px - 3].all()
    else:                # the block tables miss crossings between blocks (reference behaviour)
        assert hit[rr < r_px - 3].mean() > 0.5
    assert S == int(cnt.sum())


def test_iso_block_skipping_saves_fetches(oracle):
    """Blocks cut the fetches of the adaptive march on a sparse volume."""
    vox = D.blobs_u8(64, count=4)
    v16 = oracle.volume_r16f(vox)
    S = [oracle.render_iso(v16, vox, (1.0, 1.0, 1.0), CAM, 64, 64, variant=v)[2] for v in (0, 1, 2)]
    assert S[1] < S[2] and S[0] <= S[2]


def test_renderer_classes_metadata():
    from cpp_volume_rendering_amd.renderer import (CustomRayCasting1PassIsoAdapt,
                                                   CustomRayCasting1PassIsodfsAdapt,
                                                   RayCasting1PassIsoAdapt)
    for cls, name, nb in ((RayCasting1PassIsoAdapt, "1-Pass - Isosurface Raycaster Adaptive", None),
                          (CustomRayCasting1PassIsoAdapt,
                           "1-Pass - Custom Isosurface Raycaster Adaptive", (4, 4, 4)),
                          (CustomRayCasting1PassIsodfsAdapt, "Empty Sapce Skipping V2", (32, 32, 32))):
        r = cls()
        assert r.GetName() == name and r.GetAbbreviationName() == "iso"
        assert r.m_u_isovalue == pytest.approx(0.5) and r.m_u_step_size_small == pytest.approx(0.05)
        assert r.m_u_step_size_large == pytest.approx(1.0) and r.m_u_step_size_range == pytest.approx(0.1)
        assert tuple(np.float32(r.m_u_color)) == tuple(np.float32([0.66, 0.6, 0.05, 1.0]))
        assert not r.IsPixelMultiScalingSupported()
        if nb:
            assert tuple(r.num_blocks) == nb
        ps = {}
        r.FillParameterSpace(ps)
        assert set(ps) == {"StepSizeSmall", "StepSizeLarge", "StepSizeRange"}
