"""GPU parity of the multi-rank exchange and of the single-process multi-device group.

RCCL refuses several ranks on one GPU, so the exchange PROTOCOL the N-GPU bench runs
(cvr_gather_tiles_n: groups of frames per launch, render streams rotated over buffer
sets, the idle root, the coded exchange with its sizes read `exchange_lag` exchanges
late, the partial group at the end) is run here through the library's in-process
device-copy transport (cvr_comm_init_local) with 3 and 8 contexts on the one GPU.
Every gathered frame must equal a one-context render of the whole frame bit for bit.

cvr_create_group (one context over several devices of this process, the plugin's
multi-GPU path) runs with 1, 3 and 8 members on device 0: pixels, per-pixel sample
counts and totals equal one context's, for every renderer family.
"""
import ctypes

import numpy as np
import pytest

from cpp_volume_rendering_amd import _native as N
from cpp_volume_rendering_amd import datasets as D
from cpp_volume_rendering_amd import screen_tiles as T
from cpp_volume_rendering_amd.renderer import Camera, Device, default_cone_params, make_frame

pytestmark = pytest.mark.gpu

INITIAL = D.INITIAL_STATE_CAMERA
CAMS = [dict(INITIAL), dict(INITIAL, eye=(-300.0, 120.0, 380.0)),
        dict(INITIAL, eye=(0.0, -400.0, 200.0)), dict(INITIAL, eye=(420.0, 60.0, -150.0))]


def _params():
    p = N.Rc1passParams()
    p.step = 0.0
    p.ka, p.kd, p.ks, p.shininess = 0.5, 0.5, 0.8, 30.0
    p.ispecular[:] = [1.0, 1.0, 1.0]
    p.light_pos[:] = list(D.LIGHT_LIST0_POSITION)
    return p


def _ctx(vol, scale, tf):
    d = Device(0)
    d.set_volume(vol, scale)
    d.set_transfer_function(tf)
    return d


def _full_frames(vol, scale, tf, cams, W, H, fmt):
    """One context, whole frames (host outputs): the reference images."""
    import torch
    d = _ctx(vol, scale, tf)
    try:
        p = _params()
        out = []
        for cam in cams:
            img = np.zeros((H, W, 4), np.float16 if fmt == N.FORMAT_RGBA16F else np.float32)
            o = N.Output(img.ctypes.data, None, None, 0, fmt)
            fr = make_frame(Camera(**cam), W, H)
            N.check(N.lib().cvr_render_rc1pass(d.handle, ctypes.byref(fr), ctypes.byref(p),
                                               ctypes.byref(o)), "full", d.handle)
            out.append(img)
        torch.cuda.synchronize()
        return out
    finally:
        d.close()


def _bits(a):
    a = np.ascontiguousarray(a)
    return a.view(np.uint16 if a.dtype == np.float16 else np.uint32)


# world, idle root, coded exchange, format, frames per group, streams, buffer sets, lag[, tile]
PROTOCOL = {
    "w3_code": (3, False, 1, N.FORMAT_RGBA16F, 4, 2, 4, -1),
    "w3_code_tile32": (3, False, 1, N.FORMAT_RGBA16F, 4, 2, 4, -1, 32),
    "w8_idle_code_8frames": (8, True, 1, N.FORMAT_RGBA16F, 8, 4, 16, -1),
    "w8_idle_code_16frames": (8, True, 1, N.FORMAT_RGBA16F, 16, 4, 16, -1),  # the N >= 8 default (16 per launch)
    "w3_idle_code": (3, True, 1, N.FORMAT_RGBA16F, 4, 2, 4, -1),
    "w8_idle_code": (8, True, 1, N.FORMAT_RGBA16F, 4, 4, 16, -1),   # bench.py --gpus 8's layout
    "w8_code_lag0": (8, False, 1, N.FORMAT_RGBA16F, 4, 4, 16, 0),
    "w8_idle_code_1stream": (8, True, 1, N.FORMAT_RGBA16F, 2, 1, 2, -1),
    "w3_raw16": (3, True, 0, N.FORMAT_RGBA16F, 4, 2, 4, -1),
    "w3_raw32": (3, False, 1, N.FORMAT_RGBA32F, 3, 2, 4, -1),       # RGBA32F always moves raw tiles
}


@pytest.mark.parametrize("name", list(PROTOCOL))
def test_local_exchange_equals_full_frames(bonsai_tf, name):
    """N contexts on one GPU run the multi-rank exchange of cvr_gather_tiles_n
    (device-copy transport): every frame of 5 groups (the last one partial), rendered
    as 4-frame launches of different cameras on rotated streams, arrives in its own
    image on rank 0 equal to the one-context frame bit for bit."""
    import torch
    world, idle, code, fmt, L, D_, B, lag = PROTOCOL[name][:8]
    tile = PROTOCOL[name][8] if len(PROTOCOL[name]) > 8 else 16
    n = 64
    vol, scale = D.marschner_lobb_u8(n), D.voxel_scale(n)
    W, H = 272, 208                         # 17 x 13 tiles of 16: ragged shares
    nframes = 4 * L + L // 2
    cams = [CAMS[i % len(CAMS)] for i in range(nframes)]
    want = _full_frames(vol, scale, bonsai_tf, CAMS, W, H, fmt)
    ctxs = [_ctx(vol, scale, bonsai_tf) for _ in range(world)]
    L_ = N.lib()
    try:
        arr = (ctypes.c_void_p * world)(*[c.handle.value for c in ctxs])
        N.check(L_.cvr_comm_init_local(arr, world), "cvr_comm_init_local")
        for c in ctxs:
            for k, v in (("split_streams", D_), ("gather_sets", B), ("gather_root_idle", int(idle)),
                         ("exchange_code", code), ("exchange_lag", lag)):
                N.check(L_.cvr_set_option(c.handle, k.encode(), v), k, c.handle)
        sworld = world - 1 if idle else world
        tpr = T.max_tiles_per_rank(W, H, tile, sworld)
        dt = torch.float16 if fmt == N.FORMAT_RGBA16F else torch.float32
        dev = torch.device("cuda", 0)
        streams = [[torch.cuda.Stream(dev) for _ in range(D_)] for _ in range(world)]
        packed = [[torch.zeros((L, tpr, tile, tile, 4), dtype=dt, device=dev) for _ in range(B)]
                  for _ in range(world)]
        gathered = [torch.zeros((world, L, tpr, tile, tile, 4), dtype=dt, device=dev)
                    for _ in range(B)]
        images = [torch.zeros((H, W, 4), dtype=dt, device=dev) for _ in range(nframes)]
        torch.cuda.synchronize()
        p = _params()
        order = list(range(1, world)) + [0]
        g = 0
        for n0 in range(0, nframes, L):
            nb = min(L, nframes - n0)
            for r in order:
                c = ctxs[r]
                srank = max(r - 1, 0) if idle else r
                N.check(L_.cvr_set_stream(c.handle, streams[r][g % D_].cuda_stream), "stream", c.handle)
                renders = not (idle and r == 0)
                buf = gathered[g % B][0] if r == 0 else packed[r][g % B]
                frs = [make_frame(Camera(**cams[n0 + j]), W, H, tile, srank, sworld) for j in range(nb)]
                if renders:
                    fa = (N.Frame * nb)(*frs)
                    oa = (N.Output * nb)(*[N.Output(buf[j].data_ptr(), None, None, 1, fmt)
                                           for j in range(nb)])
                    N.check(L_.cvr_render_rc1pass_frames(c.handle, fa, nb, ctypes.byref(p), oa),
                            "render", c.handle)
                imgs = ((ctypes.c_void_p * nb)(*[images[n0 + j].data_ptr() for j in range(nb)])
                        if r == 0 else None)
                N.check(L_.cvr_gather_tiles_n(c.handle, ctypes.byref(frs[0]), nb,
                                              buf.data_ptr() if renders else None, tpr, fmt,
                                              gathered[g % B].data_ptr() if r == 0 else None, imgs),
                        "cvr_gather_tiles_n", c.handle)
            g += 1
        cur = torch.cuda.current_stream(dev)
        for r in range(world):           # rank 0 first: it posts the exchanges still trailing
            N.check(L_.cvr_set_stream(ctxs[r].handle, cur.cuda_stream), "stream", ctxs[r].handle)
            N.check(L_.cvr_gather_sync(ctxs[r].handle), "cvr_gather_sync", ctxs[r].handle)
        torch.cuda.synchronize()
        for i in range(nframes):
            got = images[i].cpu().numpy()
            ref = want[i % len(CAMS)]
            assert np.array_equal(_bits(got), _bits(ref)), f"{name}: frame {i} differs"
        assert (want[0][..., 3] > 0).mean() > 0.3
    finally:
        for c in ctxs:
            c.close()


def test_local_exchange_order_and_errors(bonsai_tf):
    """The in-process transport needs ranks 1..N-1 to issue an exchange before rank 0
    (CVR_ERR_STATE otherwise, no device work queued on a missing rank) and more buffer
    sets than render streams for its non-root ranks; a group context refuses it."""
    import torch
    n = 32
    vol, scale = D.marschner_lobb_u8(n), D.voxel_scale(n)
    ctxs = [_ctx(vol, scale, bonsai_tf) for _ in range(3)]
    L_ = N.lib()
    try:
        arr = (ctypes.c_void_p * 3)(*[c.handle.value for c in ctxs])
        N.check(L_.cvr_comm_init_local(arr, 3), "init")
        assert L_.cvr_comm_init_local(arr, 3) == N.CVR_ERR_STATE          # already joined
        W = H = 64
        tpr = T.max_tiles_per_rank(W, H, 16, 3)
        dev = torch.device("cuda", 0)
        g = torch.zeros((3, 1, tpr, 16, 16, 4), dtype=torch.float16, device=dev)
        img = torch.zeros((H, W, 4), dtype=torch.float16, device=dev)
        imgs = (ctypes.c_void_p * 1)(img.data_ptr())
        fr = make_frame(Camera(**INITIAL), W, H, 16, 0, 3)
        st = L_.cvr_gather_tiles_n(ctxs[0].handle, ctypes.byref(fr), 1, g[0].data_ptr(), tpr,
                                   N.FORMAT_RGBA16F, g.data_ptr(), imgs)
        assert st == N.CVR_ERR_STATE
        assert b"rank 1" in L_.cvr_last_error(ctxs[0].handle)
        torch.cuda.synchronize()
    finally:
        for c in ctxs:
            c.close()
    grp = Device(devices=[0, 0])
    try:
        a1 = (ctypes.c_void_p * 1)(grp.handle.value)
        assert L_.cvr_comm_init_local(a1, 1) == N.CVR_ERR_STATE
        for k in (b"split_streams", b"gather_sets", b"gather_root_idle", b"exchange_lag"):
            assert L_.cvr_set_option(grp.handle, k, 1) == N.CVR_ERR_ARG
        N.check(L_.cvr_set_option(grp.handle, b"cell_skip", 2), "cell_skip", grp.handle)
        assert L_.cvr_get_option(grp.handle, b"cell_skip") == 2
        assert grp.group_size == 2
    finally:
        grp.close()


def _render_host(dev, entry, frame, params, fmt, W, H):
    img = np.zeros((H, W, 4), np.float16 if fmt == N.FORMAT_RGBA16F else np.float32)
    cnt = np.zeros((H, W), np.uint32)
    total = np.zeros(1, np.uint64)
    out = N.Output(img.ctypes.data, cnt.ctypes.data, total.ctypes.data, 0, fmt)
    N.check(getattr(N.lib(), entry)(dev.handle, ctypes.byref(frame), ctypes.byref(params),
                                    ctypes.byref(out)), entry, dev.handle)
    return img, cnt, int(total[0])


@pytest.mark.parametrize("members", [1, 3, 8])
@pytest.mark.parametrize("fmt", [N.FORMAT_RGBA16F, N.FORMAT_RGBA32F])
def test_group_rc1pass_equals_one_context(bonsai_tf, members, fmt):
    """cvr_create_group over `members` devices (all device 0 here): host outputs with
    counts and total, three cameras, equal one context's render bit for bit."""
    n = 64
    vol, scale = D.marschner_lobb_u8(n), D.voxel_scale(n)
    W, H = 200, 136
    one = _ctx(vol, scale, bonsai_tf)
    grp = Device(devices=[0] * members)
    try:
        assert grp.group_size == members
        grp.set_volume(vol, scale)
        grp.set_transfer_function(bonsai_tf)
        p = _params()
        for cam in CAMS[:3]:
            fr = make_frame(Camera(**cam), W, H)
            a = _render_host(one, "cvr_render_rc1pass", fr, p, fmt, W, H)
            b = _render_host(grp, "cvr_render_rc1pass", fr, p, fmt, W, H)
            assert np.array_equal(_bits(a[0]), _bits(b[0])), "pixels"
            assert np.array_equal(a[1], b[1]), "per-pixel counts"
            assert a[2] == b[2] > 0, "totals"
    finally:
        grp.close()
        one.close()


def test_group_frames_device_outputs(bonsai_tf):
    """cvr_render_rc1pass_frames on a group of 8: four cameras in one call, device
    outputs on the group's stream, the total accumulated over the frames; twice in a
    row (the buffer sets rotate), each frame equal to one context's."""
    import torch
    n = 64
    vol, scale = D.marschner_lobb_u8(n), D.voxel_scale(n)
    W, H = 256, 192
    want = _full_frames(vol, scale, bonsai_tf, CAMS, W, H, N.FORMAT_RGBA16F)
    one = _ctx(vol, scale, bonsai_tf)
    grp = Device(devices=[0] * 8)
    try:
        grp.set_volume(vol, scale)
        grp.set_transfer_function(bonsai_tf)
        dev = torch.device("cuda", 0)
        s = torch.cuda.Stream(dev)
        grp.set_stream(s.cuda_stream)
        p = _params()
        total = torch.zeros((1,), dtype=torch.int64, device=dev)
        want_total = 0
        for cam in CAMS:
            want_total += _render_host(one, "cvr_render_rc1pass", make_frame(Camera(**cam), W, H), p,
                                       N.FORMAT_RGBA16F, W, H)[2]
        for rep in range(2):
            imgs = [torch.zeros((H, W, 4), dtype=torch.float16, device=dev) for _ in CAMS]
            cnts = [torch.zeros((H, W), dtype=torch.int32, device=dev) for _ in CAMS]
            fa = (N.Frame * 4)(*[make_frame(Camera(**c), W, H) for c in CAMS])
            oa = (N.Output * 4)(*[N.Output(imgs[j].data_ptr(), cnts[j].data_ptr(),
                                           total.data_ptr() if j == 0 else None, 1,
                                           N.FORMAT_RGBA16F) for j in range(4)])
            with torch.cuda.stream(s):
                total.zero_()
            N.check(N.lib().cvr_render_rc1pass_frames(grp.handle, fa, 4, ctypes.byref(p), oa),
                    "frames", grp.handle)
            s.synchronize()
            assert int(total.item()) == want_total
            for j in range(4):
                assert np.array_equal(_bits(imgs[j].cpu().numpy()), _bits(want[j])), (rep, j)
                assert int(cnts[j].sum().item()) > 0
    finally:
        grp.close()
        one.close()


def test_group_errors(bonsai_tf):
    """A member that cannot be created (device 99) fails the group's creation
    cleanly, releasing the members made so far; several frames with host outputs
    are refused (a multi-frame launch writes device buffers, as for one context)."""
    L = N.lib()
    h = ctypes.c_void_p()
    devs = (ctypes.c_int * 3)(0, 0, 99)
    assert L.cvr_create_group(devs, 3, ctypes.byref(h)) != N.CVR_OK
    assert not h.value
    vol, scale = D.marschner_lobb_u8(32), D.voxel_scale(32)
    grp = Device(devices=[0, 0])
    try:
        grp.set_volume(vol, scale)
        grp.set_transfer_function(bonsai_tf)
        W, H = 64, 48
        imgs = [np.zeros((H, W, 4), np.float32) for _ in range(2)]
        fa = (N.Frame * 2)(*[make_frame(Camera(**c), W, H) for c in CAMS[:2]])
        oa = (N.Output * 2)(*[N.Output(im.ctypes.data, None, None, 0, N.FORMAT_RGBA32F) for im in imgs])
        st = L.cvr_render_rc1pass_frames(grp.handle, fa, 2, ctypes.byref(_params()), oa)
        assert st == N.CVR_ERR_ARG
        assert b"device outputs" in N.lib().cvr_last_error(grp.handle)
    finally:
        grp.close()


def test_group_dos_ebs_iso_equal_one_context(bonsai_tf, bonsai_tf_rgba):
    """The shaded renderers and the isosurface renderer on a group of 3 equal one
    context (DOS with AO + point-light shadow, EBS defaults, iso variant 0)."""
    from test_dos_gpu import LIGHT0
    from test_ebs_gpu import ebs_params
    n = 40
    vol, scale = D.marschner_lobb_u8(n), D.voxel_scale(n)
    W, H = 120, 88
    devs = [_ctx(vol, scale, bonsai_tf), Device(devices=[0, 0, 0])]
    devs[1].set_volume(vol, scale)
    devs[1].set_transfer_function(bonsai_tf)
    L_ = N.lib()
    try:
        outs = []
        for d in devs:
            d.set_extinction_volume(bonsai_tf_rgba, (32, 32, 32), 1.0)
            lut = np.zeros(256, np.float32)
            lut[1:] = np.linspace(0.0, 0.05, 255, dtype=np.float32)
            N.check(L_.cvr_set_extinction_sat(d.handle, N.fptr(lut), 256), "sat", d.handle)
            fr = make_frame(Camera(**INITIAL), W, H)
            dp = N.DosParams()
            dp.step = 0.0
            dp.ka, dp.kd, dp.ks, dp.shininess = 0.5, 0.5, 0.8, 30.0
            dp.ispecular[:] = [1.0, 1.0, 1.0]
            for k in ("position", "forward", "up", "right"):
                getattr(dp.light, k)[:] = list(LIGHT0[k])
            dp.light.spot_angle_deg = LIGHT0["spot_angle_deg"]
            dp.apply_occlusion, dp.apply_shadow, dp.shadow_type = 1, 1, 0
            dp.occlusion, dp.shadow = default_cone_params(True), default_cone_params(False)
            ip = N.IsoParams()
            L_.cvr_iso_params_default(0, ctypes.byref(ip))
            outs.append([_render_host(d, "cvr_render_dosct", fr, dp, N.FORMAT_RGBA32F, W, H),
                         _render_host(d, "cvr_render_extbsd", fr, ebs_params(), N.FORMAT_RGBA32F, W, H),
                         _render_host(d, "cvr_render_iso", fr, ip, N.FORMAT_RGBA16F, W, H)])
        for name, a, b in zip(("dos", "ebs", "iso"), outs[0], outs[1]):
            assert np.array_equal(_bits(a[0]), _bits(b[0])), name
            assert np.array_equal(a[1], b[1]), name
            assert a[2] == b[2], name
            assert (a[0][..., 3] > 0).mean() > 0.2, name
        # the group's shade counters are its members' sums: equal to one context's
        shs = []
        fr = make_frame(Camera(**INITIAL), W, H)
        for d in devs:
            N.check(L_.cvr_set_option(d.handle, b"shade_counters", 1), "opt", d.handle)
            _render_host(d, "cvr_render_extbsd", fr, ebs_params(), N.FORMAT_RGBA32F, W, H)
            sh = (ctypes.c_uint64 * 3)()
            N.check(L_.cvr_read_shade_counters(d.handle, sh), "shade", d.handle)
            shs.append(list(sh))
        assert shs[0] == shs[1] and shs[0][0] > 0
        assert L_.cvr_device_bytes(devs[1].handle) > 3 * L_.cvr_device_bytes(devs[0].handle) // 2
    finally:
        for d in devs:
            d.close()
