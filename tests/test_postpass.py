"""CPU checks of the multiscaling post-pass restatement (oracle) and of the
screenshot composite, by the properties the reference's filters have.

The GLSL filters (libs/vis_utils/shader/renderoutputframe/*.comp) cannot run
here (no GL), and the reference holds no outputs of them: the restatement is
"parity unpinned" at the GL boundary (texture() filter weights, texelFetch out
of range = 0 under robust access).  What the reference's own filter math
implies is checked instead: partition of unity of the interpolating kernels,
exact 2x2 averaging of the multisample fetch, the box/hat decimation of a
constant image, the cardinal kernels with their digital prefilter reproducing
constants, and the composite over white.  tests/test_postpass_gpu.py checks the
HIP kernels against this restatement bit for bit.
"""
import numpy as np
import pytest

from cpp_volume_rendering_amd import _native as N

KERNELS = [N.FILTER_BOX, N.FILTER_HAT, N.FILTER_CATMULL_ROM, N.FILTER_MITCHELL_NETRAVALI,
           N.FILTER_CARDINAL_BSPLINE_3, N.FILTER_CARDINAL_OMOMS3]


def _const(h, w, v=(0.25, 0.5, 0.75, 1.0)):
    return np.broadcast_to(np.array(v, np.float16), (h, w, 4)).copy()


def test_multisample_is_2x2_average(oracle):
    rng = np.random.default_rng(1)
    f = rng.random((48, 64, 4)).astype(np.float16)
    out = oracle.multiscale_filter(N.MULTIPLE_RAYS_PER_PIXEL, N.FILTER_HAT, f, 32, 24)
    blocks = f.astype(np.float64).reshape(24, 2, 32, 2, 4).mean(axis=(1, 3))
    assert np.allclose(out.astype(np.float64), blocks, atol=1e-3)


@pytest.mark.parametrize("k", KERNELS)
def test_downscale_constant_interior(oracle, k):
    f = _const(64, 80)
    out = oracle.multiscale_filter(N.DOWN_SCALING_RENDER, k, f, 40, 32).astype(np.float64)
    inner = out[8:-8, 8:-8]
    tol = 0.0 if k in (N.FILTER_BOX, N.FILTER_HAT) else 2e-2
    assert np.abs(inner - np.array([0.25, 0.5, 0.75, 1.0])).max() <= tol


@pytest.mark.parametrize("k", KERNELS)
def test_upscale_constant_interior(oracle, k):
    f = _const(32, 40)
    out = oracle.multiscale_filter(N.UP_SCALING_RENDER, k, f, 80, 64).astype(np.float64)
    inner = out[6:-6, 6:-6]
    assert np.abs(inner - np.array([0.25, 0.5, 0.75, 1.0])).max() <= 4e-3


def test_upscale_cardinal_prefilters_in_place(oracle):
    rng = np.random.default_rng(2)
    f = rng.random((32, 40, 4)).astype(np.float16)
    g = f.copy()
    oracle.multiscale_filter(N.UP_SCALING_RENDER, N.FILTER_HAT, g, 80, 64)
    assert np.array_equal(g.view(np.uint16), f.view(np.uint16))      # hat: frame untouched
    oracle.multiscale_filter(N.UP_SCALING_RENDER, N.FILTER_CARDINAL_BSPLINE_3, g, 80, 64)
    assert not np.array_equal(g.view(np.uint16), f.view(np.uint16))  # the digital prefilter


def test_box_downscale_edges_read_zero_outside(oracle):
    """The hat kernel's support reaches one texel past the frame at the borders;
    texelFetch there reads 0 (robust access), so border pixels darken."""
    f = _const(16, 16, (1.0, 1.0, 1.0, 1.0))
    out = oracle.multiscale_filter(N.DOWN_SCALING_RENDER, N.FILTER_HAT, f, 8, 8).astype(np.float64)
    assert out[4, 4, 0] == 1.0
    assert out[0, 4, 0] == pytest.approx(0.875)        # one row of taps (weight 1/4 of 2) missing
    assert out[0, 0, 0] == pytest.approx(0.875 * 0.875)


def test_screenshot_over_white(oracle):
    f = np.zeros((2, 3, 4), np.float32)
    f[0, 0] = (1.0, 0.0, 0.5, 1.0)        # opaque
    f[0, 1] = (0.2, 0.4, 0.6, 0.0)        # transparent -> white
    f[0, 2] = (1.0, 1.0, 1.0, 0.5)
    f[1, :] = (0.0, 0.0, 0.0, 0.25)
    rgb = oracle.screenshot_rgb8(f)
    assert rgb[0, 0].tolist() == [255, 0, 128]
    assert rgb[0, 1].tolist() == [255, 255, 255]
    assert rgb[0, 2].tolist() == [255, 255, 255]
    assert rgb[1, 0].tolist() == [191, 191, 191]
    from cpp_volume_rendering_amd.renderer import composite_over_white
    assert np.array_equal(rgb, composite_over_white(f))
    assert np.array_equal(oracle.screenshot_rgb8(f.astype(np.float16)),
                          composite_over_white(f.astype(np.float16).astype(np.float32)))


def test_multiscale_resolution():
    import ctypes
    L = N.lib()
    w, h = ctypes.c_int(), ctypes.c_int()
    for mode, want in [(0, (1024, 768)), (1, (2048, 1536)), (2, (2048, 1536)), (3, (512, 384))]:
        assert L.cvr_multiscale_resolution(mode, 1024, 768, ctypes.byref(w), ctypes.byref(h)) == 0
        assert (w.value, h.value) == want
    assert L.cvr_multiscale_resolution(3, 1, 1, ctypes.byref(w), ctypes.byref(h)) != 0
