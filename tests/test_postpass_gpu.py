"""GPU parity of the multiscaling post-pass and the screenshot (postpass.hip via
the C-ABI) against the oracle restatement, bit for bit: every mode x every
kernel on random RGBA16F images and on a rendered frame, and the renderer-level
path (RayCasting1Pass in each multiscaling mode: the frame rendered at the
mode's resolution, filtered to the screen) against oracle frame + oracle filter."""
import ctypes

import numpy as np
import pytest

from cpp_volume_rendering_amd import _native as N
from cpp_volume_rendering_amd import datasets as D

pytestmark = pytest.mark.gpu

KERNELS = list(range(6))


@pytest.fixture(scope="module")
def dev():
    import torch
    from cpp_volume_rendering_amd.renderer import Device
    assert torch.cuda.is_available(), "GPU tests need a HIP device"
    d = Device(0)
    yield d
    d.close()


def gpu_filter(dev, mode, k, frame, sw, sh):
    import torch
    f = torch.from_numpy(frame.copy()).cuda()
    out = torch.zeros((sh, sw, 4), dtype=torch.float16, device="cuda")
    dev.set_stream(torch.cuda.current_stream().cuda_stream)
    N.check(N.lib().cvr_multiscale_filter(dev.handle, mode, k, f.data_ptr(), frame.shape[1],
                                          frame.shape[0], out.data_ptr(), sw, sh),
            "cvr_multiscale_filter", dev.handle)
    torch.cuda.synchronize()
    dev.set_stream(None)
    return out.cpu().numpy(), f.cpu().numpy()


def _eq16(a, b):
    return np.array_equal(a.view(np.uint16), b.view(np.uint16))


def _eq16_nan(a, b):
    """Bit-equal, except that any NaN equals any NaN."""
    na, nb = np.isnan(a), np.isnan(b)
    return np.array_equal(na, nb) and np.array_equal(a.view(np.uint16)[~na], b.view(np.uint16)[~nb])


@pytest.mark.parametrize("mode", [1, 2, 3])
@pytest.mark.parametrize("k", KERNELS)
def test_filters_match_oracle_random(dev, oracle, mode, k):
    rng = np.random.default_rng(10 * mode + k)
    sw, sh = 72, 56
    fw, fh = (sw * 2, sh * 2) if mode < 3 else (sw // 2, sh // 2)
    frame = (rng.random((fh, fw, 4)) * 1.5 - 0.25).astype(np.float16)
    got, gframe = gpu_filter(dev, mode, k, frame, sw, sh)
    oframe = frame.copy()
    want = oracle.multiscale_filter(mode, k, oframe, sw, sh)
    assert _eq16(got, want)
    assert _eq16(gframe, oframe)      # the in-place prefilter (mode 3, cardinal) as well


def test_bad_filter_arguments(dev):
    import torch
    f = torch.zeros((8, 8, 4), dtype=torch.float16, device="cuda")
    o = torch.zeros((16, 16, 4), dtype=torch.float16, device="cuda")
    L = N.lib()
    assert L.cvr_multiscale_filter(dev.handle, 4, 0, f.data_ptr(), 8, 8, o.data_ptr(), 16, 16) != 0
    assert L.cvr_multiscale_filter(dev.handle, 3, 9, f.data_ptr(), 8, 8, o.data_ptr(), 16, 16) != 0
    # cardinal prefilter on lines shorter than its LU factors
    assert L.cvr_multiscale_filter(dev.handle, 3, 4, f.data_ptr(), 8, 8, o.data_ptr(), 16, 16) != 0


@pytest.mark.parametrize("mode", [1, 2, 3])
@pytest.mark.parametrize("k", [N.FILTER_HAT, N.FILTER_CATMULL_ROM, N.FILTER_CARDINAL_OMOMS3])
def test_renderer_multiscaling_matches_oracle(oracle, bonsai_tf, mode, k):
    """RayCasting1Pass in a multiscaling mode == oracle frame (at the render
    resolution, RGBA16F) through the oracle post-pass; its Screenshot == oracle's."""
    import torch
    from cpp_volume_rendering_amd.renderer import (Camera, DataManager, RayCasting1Pass,
                                                   RenderingParameters)
    n, W, H = 64, 96, 80
    vol = D.marschner_lobb_u8(n)
    dm = DataManager()
    dm.SetVolume(vol, D.voxel_scale(n))
    dm.SetTransferFunction(bonsai_tf)
    r = RayCasting1Pass(0)
    r.SetExternalResources(dm, RenderingParameters(W, H))
    r.SetCurrentMultiScalingMode(mode)
    r.SetImageKernelFilter(k)
    assert r.Init(W, H)
    cam = Camera(**D.INITIAL_STATE_CAMERA)
    r.PrepareRender(cam)
    r.Redraw()
    torch.cuda.synchronize()
    rw, rh = (2 * W, 2 * H) if mode < 3 else (W // 2, H // 2)
    assert (r.width, r.height) == (rw, rh)
    frame = r.rgba.cpu().numpy()
    cam_o = dict(D.INITIAL_STATE_CAMERA, aspect=W / H)
    ref, _, _ = oracle.render_rc1pass(oracle.volume_r16f(vol), D.voxel_scale(n), bonsai_tf, cam_o,
                                      rw, rh, oracle.default_step(D.voxel_scale(n)))
    ref16 = ref.astype(np.float16)
    want = oracle.multiscale_filter(mode, k, ref16.copy(), W, H)
    assert _eq16(r.screen.cpu().numpy(), want)
    if mode != 3 or k < 4:
        assert _eq16(frame, ref16)
    assert np.array_equal(r.Screenshot(), oracle.screenshot_rgb8(want))
    r.Clean()


def test_screenshot_rgba32f(dev, oracle):
    import torch
    rng = np.random.default_rng(5)
    f = rng.random((33, 47, 4)).astype(np.float32)
    d = torch.from_numpy(f).cuda()
    rgb = torch.zeros((33, 47, 3), dtype=torch.uint8, device="cuda")
    dev.set_stream(torch.cuda.current_stream().cuda_stream)
    N.check(N.lib().cvr_screenshot_rgb8(dev.handle, d.data_ptr(), N.FORMAT_RGBA32F, 47, 33,
                                        rgb.data_ptr()), "screenshot", dev.handle)
    torch.cuda.synchronize()
    dev.set_stream(None)
    assert np.array_equal(rgb.cpu().numpy(), oracle.screenshot_rgb8(f))


@pytest.mark.parametrize("mode,sw,sh", [(2, 16, 16), (2, 17, 19), (2, 1500, 16), (2, 16, 2700),
                                        (2, 21000, 16), (3, 1024, 1024), (3, 34, 38),
                                        (2, 65, 129), (2, 8000, 16), (3, 34, 130), (2, 16, 88)])
@pytest.mark.parametrize("k", [N.FILTER_CARDINAL_BSPLINE_3, N.FILTER_CARDINAL_OMOMS3])
def test_digital_filter_shapes(dev, oracle, mode, sw, sh, k):
    """The cardinal kernels' recursive digital filter (LDS-staged lines cut into 64-element
    segments, 16/8/4/2/1 lines per workgroup by line length, the global-memory kernel past
    ~8900 elements) on ragged, tiny and long lines: bit for bit with the oracle, including
    the in-place prefilter of mode 3."""
    rng = np.random.default_rng(sw * 7 + sh + k)
    fw, fh = (sw * 2, sh * 2) if mode < 3 else (max(1, sw // 2), max(1, sh // 2))
    frame = (rng.random((fh, fw, 4)) * 1.5 - 0.25).astype(np.float16)
    got, gframe = gpu_filter(dev, mode, k, frame, sw, sh)
    oframe = frame.copy()
    want = oracle.multiscale_filter(mode, k, oframe, sw, sh)
    assert _eq16(got, want)
    assert _eq16(gframe, oframe)


def _spec_frames():
    """Frames aimed at the segment-parallel digital filter: constant lines (their rounded
    recursion can settle into a 2-cycle, so warm-ups do not agree and segments are redone
    in order), signed zeros, non-finite values and values whose bound leaves binary16
    (whole workgroups sequential), and plain random data."""
    rng = np.random.default_rng(77)
    fh, fw = 260, 300
    out = {}
    out["const_rows"] = np.repeat(rng.random((fh, 1, 4)), fw, axis=1).astype(np.float16)
    out["const_cols"] = np.repeat(rng.random((1, fw, 4)), fh, axis=0).astype(np.float16)
    z = np.zeros((fh, fw, 4), np.float16)
    z[:, ::3] = np.float16(-0.0)
    z[::7, ::5] = np.float16(1e-7)
    out["signed_zeros"] = z
    f = (rng.random((fh, fw, 4)) * 2 - 1).astype(np.float16)
    f[100, 17, 2] = np.float16(np.inf)
    f[3, 250, 0] = np.float16(np.nan)
    out["nonfinite"] = f
    out["huge"] = (rng.random((fh, fw, 4)) * 60000 - 30000).astype(np.float16)
    out["near_max"] = np.where(rng.random((fh, fw, 4)) < 0.01, 65000.0,
                               rng.random((fh, fw, 4))).astype(np.float16)
    b = (rng.random((fh, fw, 4)) < 0.5).astype(np.float16)
    b[:, 130:170] = np.float16(0.5)
    out["blocks"] = b
    return out


@pytest.mark.parametrize("name", sorted(_spec_frames()))
@pytest.mark.parametrize("k", [N.FILTER_CARDINAL_BSPLINE_3, N.FILTER_CARDINAL_OMOMS3])
def test_digital_filter_speculation_cases(dev, oracle, name, k):
    """The in-place prefilter (mode 3) on frames that drive the segment-parallel filter
    through its redo and sequential paths: bit for bit with the sequential oracle."""
    frame = _spec_frames()[name]
    fh, fw = frame.shape[:2]
    got, gframe = gpu_filter(dev, 3, k, frame, fw * 2, fh * 2)
    oframe = frame.copy()
    want = oracle.multiscale_filter(3, k, oframe, fw * 2, fh * 2)
    # a recursion that overflows makes inf - inf: the sign of that fresh NaN is the
    # hardware's (x86: negative default NaN, gfx950: positive), not part of CVR-SPEC
    assert _eq16_nan(gframe, oframe)
    assert _eq16_nan(got, want)
    if name in ("const_rows", "const_cols", "blocks", "signed_zeros"):
        assert _eq16(gframe, oframe) and _eq16(got, want)


@pytest.mark.parametrize("ratio", [3, 5])
@pytest.mark.parametrize("k", KERNELS)
def test_downscale_ratios(dev, oracle, ratio, k):
    """Kernel decimation at other frame/screen ratios: the LDS-window kernel where its taps
    and window fit (ratio 3: box, hat), the global-memory kernel otherwise; bit for bit."""
    rng = np.random.default_rng(100 * ratio + k)
    sw, sh = 40, 33
    frame = (rng.random((sh * ratio, sw * ratio, 4)) * 1.5 - 0.25).astype(np.float16)
    got, _ = gpu_filter(dev, 2, k, frame, sw, sh)
    want = oracle.multiscale_filter(2, k, frame.copy(), sw, sh)
    assert _eq16(got, want)


@pytest.mark.parametrize("k", [N.FILTER_CARDINAL_BSPLINE_3, N.FILTER_CARDINAL_OMOMS3])
def test_digital_filter_unaligned_frame(dev, oracle, k):
    """A frame that starts 8 B past a 16-B boundary: the row pass stages single pixels
    instead of pixel pairs; same bits."""
    import torch
    rng = np.random.default_rng(31 + k)
    fh, fw = 40, 52
    frame = (rng.random((fh, fw, 4)) * 1.5 - 0.25).astype(np.float16)
    buf = torch.zeros(fh * fw * 4 + 4, dtype=torch.float16, device="cuda")
    buf[4:] = torch.from_numpy(frame.reshape(-1)).cuda()
    out = torch.zeros((2 * fh, 2 * fw, 4), dtype=torch.float16, device="cuda")
    dev.set_stream(torch.cuda.current_stream().cuda_stream)
    N.check(N.lib().cvr_multiscale_filter(dev.handle, 3, k, buf.data_ptr() + 8, fw, fh,
                                          out.data_ptr(), 2 * fw, 2 * fh), "filter", dev.handle)
    torch.cuda.synchronize()
    dev.set_stream(None)
    oframe = frame.copy()
    want = oracle.multiscale_filter(3, k, oframe, 2 * fw, 2 * fh)
    assert _eq16(buf[4:].cpu().numpy().reshape(fh, fw, 4), oframe)
    assert _eq16(out.cpu().numpy(), want)


@pytest.mark.parametrize("k", [N.FILTER_BOX, N.FILTER_HAT])
def test_downscale_lds_budget_boundary(dev, oracle, k):
    """Frame/screen ratio 4.8: the hat kernel's LDS window (90 x 91 pixels, 65,520 B) plus
    the kernel's static weight tables no longer fit 64 KiB, so the launch takes the
    global-memory kernel instead of failing; the box kernel's window still fits.  Bit for
    bit either way."""
    rng = np.random.default_rng(4800 + k)
    sw, sh, fw, fh = 40, 33, 192, 158
    frame = (rng.random((fh, fw, 4)) * 1.5 - 0.25).astype(np.float16)
    got, _ = gpu_filter(dev, 2, k, frame, sw, sh)
    want = oracle.multiscale_filter(2, k, frame.copy(), sw, sh)
    assert _eq16(got, want)
