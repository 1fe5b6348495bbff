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
