"""State changes while frames are in flight on other streams.

The reference changes its transfer function (or volume) between frames and calls
Init again (renderingmanager.cpp:1050-1127, rc1prenderer.cpp:50-70); GL orders that
change after every draw already issued.  Here frames may still be queued on any of
the non-blocking streams a caller rotates (screen_tiles.ScreenTileSplit), so every
state setter drains the device before it writes or frees state frames read
(cvr_api.cpp QUIESCE).  Each test queues frames on 3 non-blocking streams behind a
spin kernel (so they are certainly still pending), changes the state, renders the
next frame, and checks every in-flight frame against the oracle with the OLD state
and the next frame against the oracle with the NEW state, bit for bit."""
import ctypes

import numpy as np
import pytest

from cpp_volume_rendering_amd import _native as N
from cpp_volume_rendering_amd import datasets as D
from cpp_volume_rendering_amd.renderer import Camera, Device, make_frame

pytestmark = pytest.mark.gpu

W = H = 96
SPIN_CYCLES = 20_000_000        # ~10 ms of torch.cuda._sleep per stream


def _render_on(dev, stream, frame, buf):
    dev.set_stream(stream.cuda_stream)
    out = N.Output(buf.data_ptr(), None, None, 1, N.FORMAT_RGBA32F)
    p = N.Rc1passParams()
    N.check(N.lib().cvr_render_rc1pass(dev.handle, ctypes.byref(frame), ctypes.byref(p),
                                       ctypes.byref(out)), "render", dev.handle)


def _oracle(oracle, vol, scale, tf, cam):
    ref = oracle.render_rc1pass(oracle.volume_r16f(vol), scale, tf,
                                dict(eye=cam.eye, center=cam.center, up=cam.up), W, H,
                                oracle.default_step(scale))
    return np.ascontiguousarray(ref[0]).view(np.int32)


def _in_flight(dev, frames_per_stream=3):
    """3 non-blocking streams, each: a spin kernel, then frames_per_stream frames."""
    import torch
    streams = [torch.cuda.Stream() for _ in range(3)]
    cam = Camera(**D.INITIAL_STATE_CAMERA)
    frame = make_frame(cam, W, H)
    # the outputs (and the next frame's) are zeroed on the default stream, which the
    # non-blocking render streams do not wait for: zero them all, then synchronise
    bufs = [torch.zeros((H, W, 4), dtype=torch.float32, device="cuda")
            for _ in range(3 * frames_per_stream + 1)]
    torch.cuda.synchronize()
    for k, s in enumerate(streams):
        with torch.cuda.stream(s):
            torch.cuda._sleep(SPIN_CYCLES)
        for j in range(frames_per_stream):
            _render_on(dev, s, frame, bufs[k * frames_per_stream + j])
    return streams, cam, frame, bufs[:-1], bufs[-1]


@pytest.mark.parametrize("what", ["tf", "volume"])
def test_state_change_with_frames_in_flight(oracle, bonsai_tf, what):
    import torch
    n = 48
    vol = D.marschner_lobb_u8(n)
    scale = D.voxel_scale(n)
    dev = Device(0)
    try:
        dev.set_volume(vol, scale)
        dev.set_transfer_function(bonsai_tf)
        # warm: the skip flags and launch order exist before the frames queue up
        s0 = torch.cuda.Stream()
        _render_on(dev, s0, make_frame(Camera(**D.INITIAL_STATE_CAMERA), W, H),
                   torch.zeros((H, W, 4), dtype=torch.float32, device="cuda"))
        torch.cuda.synchronize()
        streams, cam, frame, bufs, nxt = _in_flight(dev)
        # the state change, issued while every queued frame is still pending
        if what == "tf":
            alpha = tuple((a * 0.25, i) for a, i in D.BONSAI_TF_ALPHA)
            new_tf = oracle.tf_rgbt(oracle.tf_table_double(D.BONSAI_TF_RGB, alpha))
            dev.set_transfer_function(new_tf)
            new_vol, new_scale = vol, scale
        else:
            new_vol = (vol.astype(np.int32) * 3 // 4).astype(np.uint8)   # another volume
            new_tf, new_scale = bonsai_tf, scale
            dev.set_volume(new_vol, new_scale)
        _render_on(dev, streams[0], frame, nxt)
        torch.cuda.synchronize()
        old_ref = _oracle(oracle, vol, scale, bonsai_tf, cam)
        new_ref = _oracle(oracle, new_vol, new_scale, new_tf, cam)
        assert not np.array_equal(old_ref, new_ref)       # the change is visible
        for i, b in enumerate(bufs):
            got = b.cpu().numpy().view(np.int32)
            assert np.array_equal(got, old_ref), f"in-flight frame {i} does not match the old state"
        assert np.array_equal(nxt.cpu().numpy().view(np.int32), new_ref), "next frame"
    finally:
        dev.close()


def _render_kind(dev, stream, kind, frame, buf, p):
    dev.set_stream(stream.cuda_stream)
    out = N.Output(buf.data_ptr(), None, None, 1, N.FORMAT_RGBA32F)
    entry = {"rc1pass": "cvr_render_rc1pass", "dos": "cvr_render_dosct",
             "ebs": "cvr_render_extbsd"}[kind]
    N.check(getattr(N.lib(), entry)(dev.handle, ctypes.byref(frame), ctypes.byref(p),
                                    ctypes.byref(out)), entry, dev.handle)


def _shaded_setup(dev, what, vol, scale, tf, tf_rgba, lut, state):
    """The state a `what` test renders with; state 0 = old, 1 = new."""
    dev.set_volume(vol, scale)
    dev.set_transfer_function(tf)
    if what == "gradient":
        dev.set_gradient(N.GRADIENT_FINITE_DIFFERENCES if state == 0 else N.GRADIENT_SOBEL_FELDMAN)
    elif what == "extinction_volume":
        dev.set_extinction_volume(tf_rgba, (32, 32, 32), 1.0 if state == 0 else 2.0)
    else:
        N.check(N.lib().cvr_set_extinction_sat(dev.handle, N.fptr(lut * (1.0 if state == 0 else 3.0)),
                                               256), "sat", dev.handle)


def _shaded_params(what):
    from cpp_volume_rendering_amd.renderer import default_cone_params
    if what == "gradient":
        p = N.Rc1passParams()
        p.apply_gradient_shading = 1
        p.ka, p.kd, p.ks, p.shininess = 0.5, 0.5, 0.8, 30.0
        p.ispecular[:] = [1.0, 1.0, 1.0]
        p.light_pos[:] = list(D.LIGHT_LIST0_POSITION)
        return "rc1pass", p
    if what == "extinction_volume":
        p = N.DosParams()
        p.ka, p.kd, p.ks, p.shininess = 0.5, 0.5, 0.8, 30.0
        p.light.position[:] = list(D.LIGHT_LIST0_POSITION)
        p.apply_occlusion, p.apply_shadow = 1, 1
        p.occlusion, p.shadow = default_cone_params(True), default_cone_params(False)
        return "dos", p
    from test_ebs_gpu import ebs_params
    return "ebs", ebs_params()


@pytest.mark.parametrize("what", ["gradient", "extinction_volume", "extinction_sat"])
def test_shaded_state_change_with_frames_in_flight(bonsai_tf, bonsai_tf_rgba, what):
    """The same for the other setters that drain the device: the gradient
    under Blinn-Phong frames, the DOS extinction pyramid and the EBS SAT under their
    frames.  References: a fresh context renders each state with nothing in flight."""
    import torch
    n = 40
    vol, scale = D.marschner_lobb_u8(n), D.voxel_scale(n)
    lut = np.zeros(256, np.float32)
    lut[1:] = np.linspace(0.0, 0.05, 255, dtype=np.float32)
    kind, p = _shaded_params(what)
    frame = make_frame(Camera(**D.INITIAL_STATE_CAMERA), W, H)
    refs = []
    for state in (0, 1):
        ref_dev = Device(0)
        try:
            _shaded_setup(ref_dev, what, vol, scale, bonsai_tf, bonsai_tf_rgba, lut, state)
            b = torch.zeros((H, W, 4), dtype=torch.float32, device="cuda")
            torch.cuda.synchronize()
            _render_kind(ref_dev, torch.cuda.current_stream(), kind, frame, b, p)
            torch.cuda.synchronize()
            refs.append(b.cpu().numpy().view(np.int32).copy())
        finally:
            ref_dev.close()
    assert not np.array_equal(refs[0], refs[1])       # the change is visible
    dev = Device(0)
    try:
        _shaded_setup(dev, what, vol, scale, bonsai_tf, bonsai_tf_rgba, lut, 0)
        streams = [torch.cuda.Stream() for _ in range(3)]
        bufs = [torch.zeros((H, W, 4), dtype=torch.float32, device="cuda") for _ in range(7)]
        torch.cuda.synchronize()
        _render_kind(dev, streams[0], kind, frame, bufs[6], p)     # warm (tables, lists)
        torch.cuda.synchronize()
        for k, s in enumerate(streams):
            with torch.cuda.stream(s):
                torch.cuda._sleep(SPIN_CYCLES)
            for j in range(2):
                _render_kind(dev, s, kind, frame, bufs[2 * k + j], p)
        if what == "gradient":
            dev.set_gradient(N.GRADIENT_SOBEL_FELDMAN)
        elif what == "extinction_volume":
            dev.set_extinction_volume(bonsai_tf_rgba, (32, 32, 32), 2.0)
        else:
            N.check(N.lib().cvr_set_extinction_sat(dev.handle, N.fptr(lut * 3.0), 256), "sat",
                    dev.handle)
        _render_kind(dev, streams[0], kind, frame, bufs[6], p)
        torch.cuda.synchronize()
        for i in range(6):
            assert np.array_equal(bufs[i].cpu().numpy().view(np.int32), refs[0]), f"in-flight frame {i}"
        assert np.array_equal(bufs[6].cpu().numpy().view(np.int32), refs[1]), "next frame"
    finally:
        dev.close()


def test_cell_flags_oom_fallback_after_tf_change(oracle, bonsai_tf):
    """the skip flags' scratch runs out (forced by debug_cell_flags_oom)
    after a TF change, while the cells' sign bits still hold the OLD TF's flags: the
    frame renders without the skip, equal to the oracle of the NEW TF bit for bit,
    reports CVR_OK with no error text, and the flags come back after the next TF change."""
    import torch
    n = 48
    vol, scale = D.marschner_lobb_u8(n), D.voxel_scale(n)
    cam = Camera(**D.INITIAL_STATE_CAMERA)
    frame = make_frame(cam, W, H)
    dev = Device(0)
    L = N.lib()
    try:
        dev.set_volume(vol, scale)
        dev.set_transfer_function(bonsai_tf)
        s = torch.cuda.Stream()
        b = torch.zeros((H, W, 4), dtype=torch.float32, device="cuda")
        torch.cuda.synchronize()
        _render_on(dev, s, frame, b)                       # flags of the bonsai TF
        torch.cuda.synchronize()
        assert L.cvr_get_option(dev.handle, b"cell_flags_active") == 1
        N.check(L.cvr_set_option(dev.handle, b"debug_cell_flags_oom", 1), "opt", dev.handle)
        alpha = tuple((a * 0.25, i) for a, i in D.BONSAI_TF_ALPHA)
        new_tf = oracle.tf_rgbt(oracle.tf_table_double(D.BONSAI_TF_RGB, alpha))
        dev.set_transfer_function(new_tf)
        for _ in range(2):                                 # the fallback holds for later frames
            b.zero_()
            torch.cuda.synchronize()
            _render_on(dev, s, frame, b)
            torch.cuda.synchronize()
            assert L.cvr_get_option(dev.handle, b"cell_flags_active") == 0
            assert L.cvr_last_error(dev.handle) in (b"", None)
            assert np.array_equal(b.cpu().numpy().view(np.int32),
                                  _oracle(oracle, vol, scale, new_tf, cam)), "fallback frame"
        N.check(L.cvr_set_option(dev.handle, b"debug_cell_flags_oom", 0), "opt", dev.handle)
        dev.set_transfer_function(bonsai_tf)               # clears the OOM mark: flags rebuilt
        b.zero_()
        torch.cuda.synchronize()
        _render_on(dev, s, frame, b)
        torch.cuda.synchronize()
        assert L.cvr_get_option(dev.handle, b"cell_flags_active") == 1
        assert np.array_equal(b.cpu().numpy().view(np.int32),
                              _oracle(oracle, vol, scale, bonsai_tf, cam))
    finally:
        dev.close()
