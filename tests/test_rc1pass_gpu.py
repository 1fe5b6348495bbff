"""GPU parity of the rc1pass ray-march (HIP kernel via the C-ABI) against the CPU
oracle.  CVR-SPEC makes the two bit-identical: RGBA floats and per-pixel
iteration counts are compared exactly (tolerance 0).  The image-level gate of
BASELINE.md (|dRGBA| <= 2e-3 for 99.9 % of pixels, max 2e-2, SSIM >= 0.99) is
implied by that and is checked as well on the headline-sized property tests.
"""
import ctypes

import numpy as np
import pytest

from cpp_volume_rendering_amd import _native as N
from cpp_volume_rendering_amd import datasets as D
from cpp_volume_rendering_amd import screen_tiles as T
from cpp_volume_rendering_amd.renderer import Camera, Device, make_frame

pytestmark = pytest.mark.gpu

INITIAL = D.INITIAL_STATE_CAMERA


@pytest.fixture(scope="module")
def dev():
    import torch
    assert torch.cuda.is_available(), "GPU tests need a HIP device"
    d = Device(0)
    yield d
    d.close()


def gpu_render(dev, vol, scale, tf, cam, W, H, step=0.0, phong=False, gmode=0, light=(0, 0, 0),
               shading=(0.5, 0.5, 0.8, 30.0), tile=0, rank=0, nranks=1, set_data=True):
    if set_data:
        dev.set_volume(vol, scale)
        dev.set_transfer_function(tf)
        dev.set_gradient(gmode)
    frame = make_frame(Camera(**cam), W, H, tile, rank, nranks)
    p = N.Rc1passParams()
    p.step = step
    p.apply_gradient_shading = int(phong)
    p.ka, p.kd, p.ks, p.shininess = shading
    p.ispecular[:] = [1.0, 1.0, 1.0]
    p.light_pos[:] = list(light)
    if nranks > 1:
        k = T.tiles_for_rank(W, H, tile, rank, nranks)
        rgba = np.zeros((k, tile, tile, 4), np.float32)
        cnt = np.zeros((k, tile, tile), np.uint32)
    else:
        rgba = np.zeros((H, W, 4), np.float32)
        cnt = np.zeros((H, W), np.uint32)
    total = np.zeros(1, np.uint64)
    out = N.Output(rgba.ctypes.data, cnt.ctypes.data, total.ctypes.data, 0)
    N.check(N.lib().cvr_render_rc1pass(dev.handle, ctypes.byref(frame), ctypes.byref(p),
                                       ctypes.byref(out)), "render", dev.handle)
    return rgba, cnt, int(total[0])


def oracle_render(oracle, vol, scale, tf, cam, W, H, step=0.0, phong=False, gmode=0,
                  light=(0, 0, 0), shading=(0.5, 0.5, 0.8, 30.0)):
    v16 = oracle.volume_r16f(vol)
    grad = None
    if gmode:
        grad = oracle.gradient(vol, "fd" if gmode == 1 else "sobel")
    st = step if step > 0 else oracle.default_step(scale)
    ka, kd, ks, sh = shading
    return oracle.render_rc1pass(v16, scale, tf, cam, W, H, st, grad=grad, phong=phong, ka=ka,
                                 kd=kd, ks=ks, shininess=sh, light=light)


def assert_bitexact(a, b, what):
    a = np.ascontiguousarray(a); b = np.ascontiguousarray(b)
    assert a.shape == b.shape, what
    if a.dtype == np.float32:
        diff = a.view(np.uint32) != b.view(np.uint32)
    else:
        diff = a != b
    n = int(diff.sum())
    if n:
        idx = np.argwhere(diff)[:5]
        raise AssertionError(f"{what}: {n} mismatches, first at {idx.tolist()}: "
                             f"gpu={a[tuple(idx[0])]} oracle={b[tuple(idx[0])]}")


def _ml(n):
    return D.marschner_lobb_u8(n)


CASES = {
    # C1: 64^3 .syn sphere, 256^2, EA only (BASELINE.json configs[0])
    "c1_sphere64": dict(vol=lambda: D.sphere_u8(64), scale=D.voxel_scale(64), W=256, H=256),
    # ragged viewport (not a multiple of the 16x16 block), non-square aspect
    "ml64_ragged": dict(vol=lambda: _ml(64), scale=D.voxel_scale(64), W=203, H=117),
    # non-power-of-two step and anisotropic, non-cubic volume
    "ml_aniso": dict(vol=lambda: _ml(48)[:, :40, :33].copy(), scale=(9.0, 11.5, 7.25), W=160,
                     H=144, step=1.7),
    # 16-bit voxels (GetNormalizedSample /65535)
    "u16": dict(vol=lambda: (_ml(40).astype(np.uint16) * 257 + 3), scale=D.voxel_scale(40),
                W=128, H=128),
    # empty space only: every sample transparent, counts still exact
    "blobs_sparse": dict(vol=lambda: D.blobs_u8(64, count=6), scale=D.voxel_scale(64), W=192,
                         H=192),
    "all_zero": dict(vol=lambda: np.zeros((16, 16, 16), np.uint8), scale=(32.0, 32.0, 32.0),
                     W=64, H=64),
    # 1x1 viewport
    "one_pixel": dict(vol=lambda: _ml(32), scale=D.voxel_scale(32), W=1, H=1),
    # camera inside the volume (tnear clamps to 0, ray_bbox_intersection.comp:224)
    "camera_inside": dict(vol=lambda: _ml(64), scale=D.voxel_scale(64), W=128, H=96,
                          cam=dict(eye=(10.0, -20.0, 30.0), center=(100.0, 50.0, -200.0),
                                   up=(0.0, 1.0, 0.0))),
    # Blinn-Phong with finite-difference and Sobel gradients (config 3 path)
    "phong_fd": dict(vol=lambda: _ml(64), scale=D.voxel_scale(64), W=160, H=160, phong=True,
                     gmode=1, light=D.LIGHT_LIST0_POSITION),
    # opacities so large that -(alpha*h) leaves exp's fast range (range-checked exp path,
    # exp underflows to 0 past -86)
    "dense_tf": dict(vol=lambda: _ml(48), scale=D.voxel_scale(48), W=128, H=112, step=1.7,
                     tf_alpha_scale=400.0),
    "phong_sobel": dict(vol=lambda: _ml(48), scale=D.voxel_scale(48), W=128, H=128, phong=True,
                        gmode=2, light=D.LIGHT_LIST0_POSITION, shading=(0.3, 0.6, 0.5, 12.5)),
    # Blinn-Phong with the camera inside the volume (clamped sample positions, shading
    # jobs rebuilt from the owner's ray on another lane) and a ragged viewport
    "phong_inside": dict(vol=lambda: _ml(64), scale=D.voxel_scale(64), W=101, H=75, phong=True,
                         gmode=1, light=D.LIGHT_LIST0_POSITION,
                         cam=dict(eye=(10.0, -20.0, 30.0), center=(100.0, 50.0, -200.0),
                                  up=(0.0, 1.0, 0.0))),
}


def case_tf(c, tf):
    if "tf_alpha_scale" in c:
        tf = tf.copy()
        tf[:, 3] *= c["tf_alpha_scale"]
    return tf


@pytest.mark.parametrize("name", sorted(CASES))
def test_rc1pass_bitexact_vs_oracle(dev, oracle, bonsai_tf, name):
    c = CASES[name]
    vol = c["vol"]()
    bonsai_tf = case_tf(c, bonsai_tf)
    cam = c.get("cam", INITIAL)
    kw = dict(step=c.get("step", 0.0), phong=c.get("phong", False), gmode=c.get("gmode", 0),
              light=c.get("light", (0, 0, 0)), shading=c.get("shading", (0.5, 0.5, 0.8, 30.0)))
    g_rgba, g_cnt, g_total = gpu_render(dev, vol, c["scale"], bonsai_tf, cam, c["W"], c["H"], **kw)
    o_rgba, o_cnt, o_total = oracle_render(oracle, vol, c["scale"], bonsai_tf, cam, c["W"],
                                           c["H"], **kw)
    assert_bitexact(g_cnt, o_cnt, f"{name} counts")
    assert_bitexact(g_rgba, o_rgba, f"{name} rgba")
    assert g_total == o_total == int(o_cnt.sum())
    if name == "all_zero":
        assert not o_rgba.any()


@pytest.mark.parametrize("cam_index", [0, 1, 2, 3, 5, 9, 11, 17, 21])
def test_reference_camera_states(dev, oracle, bonsai_tf, golden_dir, cam_index):
    """Cameras of data/#list_camera_states (arbitrary up vectors, off-centre targets)."""
    from cpp_volume_rendering_amd.renderer import read_camera_state
    cam = read_camera_state(f"{golden_dir}/list_camera_states", cam_index)
    camd = dict(eye=cam.eye, center=cam.center, up=cam.up)
    vol = _ml(64)
    g = gpu_render(dev, vol, D.voxel_scale(64), bonsai_tf, camd, 96, 80)
    o = oracle_render(oracle, vol, D.voxel_scale(64), bonsai_tf, camd, 96, 80)
    assert_bitexact(g[1], o[1], "counts")
    assert_bitexact(g[0], o[0], "rgba")


@pytest.mark.parametrize("nranks,tile", [(2, 32), (3, 16), (8, 32), (5, 64)])
def test_screen_tiles_match_full_frame(dev, bonsai_tf, nranks, tile):
    """Multi-GPU tile split: packed per-rank tiles, unpacked, equal the 1-GPU frame bit for bit."""
    import torch
    vol = _ml(64)
    W, H = 200, 136
    full, full_cnt, full_total = gpu_render(dev, vol, D.voxel_scale(64), bonsai_tf, INITIAL, W, H)
    tpr = T.max_tiles_per_rank(W, H, tile, nranks)
    packed_all = np.zeros((nranks, tpr, tile, tile, 4), np.float32)
    cnt_all = np.zeros((nranks, tpr, tile, tile), np.uint32)
    tot = 0
    for r in range(nranks):
        rgba, cnt, t = gpu_render(dev, vol, D.voxel_scale(64), bonsai_tf, INITIAL, W, H,
                                  tile=tile, rank=r, nranks=nranks, set_data=False)
        packed_all[r, :rgba.shape[0]] = rgba
        cnt_all[r, :cnt.shape[0]] = cnt
        tot += t
    assert tot == full_total
    assert_bitexact(T.unpack(packed_all, W, H, tile, nranks), full, "host unpack")
    assert_bitexact(T.unpack(cnt_all, W, H, tile, nranks), full_cnt, "host unpack counts")
    # device unpack kernel
    d_packed = torch.from_numpy(packed_all).cuda()
    d_img = torch.zeros((H, W, 4), dtype=torch.float32, device="cuda")
    frame = make_frame(Camera(**INITIAL), W, H, tile, 0, nranks)
    dev.set_stream(torch.cuda.current_stream().cuda_stream)
    N.check(N.lib().cvr_unpack_tiles_device(dev.handle, ctypes.byref(frame), d_packed.data_ptr(),
                                            tpr, N.FORMAT_RGBA32F, d_img.data_ptr()), "unpack",
            dev.handle)
    torch.cuda.synchronize()
    dev.set_stream(None)
    assert_bitexact(d_img.cpu().numpy(), full, "device unpack")


def test_headline_512_properties(dev, oracle, bonsai_tf):
    """512^3 / 1024^2 (the bench workload): deterministic, device/host outputs agree,
    and a band of rows matches the oracle bit for bit (full frame is checked by counts sum)."""
    import torch
    vol = _ml(512)
    sc = D.voxel_scale(512)
    W = H = 1024
    g1, c1, t1 = gpu_render(dev, vol, sc, bonsai_tf, INITIAL, W, H)
    g2, c2, t2 = gpu_render(dev, vol, sc, bonsai_tf, INITIAL, W, H, set_data=False)
    assert_bitexact(g1, g2, "determinism")
    assert t1 == t2 == int(c1.astype(np.uint64).sum())
    # rows through the middle of the image, against the oracle
    v16 = oracle.volume_r16f(vol)
    rows = (500, 524)
    o_rgba, o_cnt, _ = oracle.render_rc1pass(v16, sc, bonsai_tf, INITIAL, W, H,
                                             oracle.default_step(sc), rows=rows)
    assert_bitexact(g1[rows[0]:rows[1]], o_rgba[rows[0]:rows[1]], "rows rgba")
    assert_bitexact(c1[rows[0]:rows[1]], o_cnt[rows[0]:rows[1]], "rows counts")
    # device-output path (what bench.py times) equals the host-output path
    from cpp_volume_rendering_amd.renderer import RayCasting1Pass, DataManager, RenderingParameters
    dm = DataManager(); dm.SetVolume(vol, sc); dm.SetTransferFunction(bonsai_tf)
    r = RayCasting1Pass(0); r.SetExternalResources(dm, RenderingParameters(W, H))
    assert r.Init(W, H)
    r.PrepareRender(Camera(**INITIAL))
    r.Redraw()
    torch.cuda.synchronize()
    assert_bitexact(r.rgba.cpu().numpy(), g1, "renderer device output")
    assert int(r.total.item()) == t1
    r.Clean()


SCHEDULES = [
    dict(tile_order=0, batch=4),
    dict(tile_order=1, quad=10, boost=5, batch=4),
    dict(tile_order=1, quad=100, boost=0, batch=2),
    dict(tile_order=1, quad=0, boost=50, batch=2),
    dict(tile_order=1, quad=35, boost=5, batch=4),
    # macro-cell empty-space skipping forced on (any fraction of empty macro cells;
    # it runs only with the per-cell skip off)
    dict(tile_order=1, batch=4, macro=3, skip_min_pct=0, cell_skip=0),
    dict(tile_order=0, batch=2, macro=2, skip_min_pct=0, cell_skip=0),
    dict(tile_order=1, batch=4, macro=5, skip_min_pct=0, quad=10, cell_skip=0),
    # per-cell skip: off, empty-sample flags only (the default, 2, runs in every other row)
    dict(tile_order=1, batch=4, cell_skip=0, macro=0),
    dict(tile_order=1, batch=2, cell_skip=1),
    dict(tile_order=0, batch=4, cell_skip=1),
    dict(tile_order=1, batch=4, cell_skip=3),
    dict(tile_order=1, batch=2, cell_skip=3, boost=0),
    dict(tile_order=1, batch=4, cell_skip=4),
    dict(tile_order=2, batch=2, cell_skip=4),
    # order built on a side stream (lag 3) / rebuilt every frame
    dict(tile_order=1, batch=4, async_order=1, quad=10),
    dict(tile_order=1, batch=2, order_interval=1, boost=0),
    # screen order interleaved over the XCDs (the fallback of a stale order)
    dict(tile_order=2, batch=4),
    # XCD bands capped near the even share (fewer empty slots; past the cap the
    # bands fall back to even tile counts)
    dict(tile_order=1, batch=4, band_cap=100),
    dict(tile_order=1, batch=4, band_cap=125, quad=10),
]


@pytest.mark.parametrize("sched", range(len(SCHEDULES)))
@pytest.mark.parametrize("name", ["ml64_ragged", "ml_aniso", "phong_fd", "camera_inside",
                                  "blobs_sparse", "dense_tf", "phong_inside"])
def test_schedules_bitexact(oracle, bonsai_tf, name, sched):
    """Every scheduling / march variant (LPT order, quad = 4-lanes-per-ray march for the
    longest tiles, batch size, empty-space skipping) reproduces the oracle bit for bit, on the
    first frame (screen order) and on later frames (learned LPT order + quad tiles)."""
    c = CASES[name]
    opts = SCHEDULES[sched]
    vol = c["vol"]()
    bonsai_tf = case_tf(c, bonsai_tf)
    cam = c.get("cam", INITIAL)
    kw = dict(step=c.get("step", 0.0), phong=c.get("phong", False), gmode=c.get("gmode", 0),
              light=c.get("light", (0, 0, 0)), shading=c.get("shading", (0.5, 0.5, 0.8, 30.0)))
    o_rgba, o_cnt, o_total = oracle_render(oracle, vol, c["scale"], bonsai_tf, cam, c["W"],
                                           c["H"], **kw)
    d = Device(0)
    try:
        for k in ("tile_order", "quad", "boost", "batch", "macro", "skip_min_pct", "async_order",
                  "order_interval", "cell_skip", "band_cap"):
            if k in opts:
                N.check(N.lib().cvr_set_option(d.handle, k.encode(), opts[k]), k)
        for frame in range(5):
            g_rgba, g_cnt, g_total = gpu_render(d, vol, c["scale"], bonsai_tf, cam, c["W"], c["H"],
                                                set_data=(frame == 0), **kw)
            assert_bitexact(g_cnt, o_cnt, f"{name} frame {frame} counts")
            assert_bitexact(g_rgba, o_rgba, f"{name} frame {frame} rgba")
            assert g_total == o_total
    finally:
        d.close()


def _cell_flags(d, n):
    """The skip flags the library wrote into the cells (cvr_copy_cells), as
    (empty bool, q int) arrays over the (n+1)^3 cell grid (z, y, x)."""
    cells = np.zeros(((n + 1) ** 3, 4), np.uint32)
    N.check(N.lib().cvr_copy_cells(d.handle, cells.ctypes.data, cells.nbytes), "copy cells", d.handle)
    empty = (cells[:, 0] >> 31).astype(bool)
    q = ((cells[:, 1] >> 31) | ((cells[:, 2] >> 31) << 1) | ((cells[:, 3] >> 31) << 2)).astype(int)
    return empty.reshape((n + 1,) * 3), q.reshape((n + 1,) * 3), cells


def test_cell_flags_match_host_restatement(oracle, bonsai_tf):
    """The per-cell skip flags (precompute.hip build_cell_flags): EMPTY exactly where every
    density the cell's corners can interpolate to reads only TF entries with tau = 0
    (recomputed here in numpy, with the same 2^-10 margin), and q = min(d, 8) - 1 for the
    chessboard distance d to the nearest non-empty cell (scipy's distance transform, cells
    outside the grid ignored).  The flags change with the TF and vanish with cell_skip 0
    on a new volume; the densities (the low 15 bits of every half) never change."""
    from scipy import ndimage
    n = 40
    vol = D.blobs_u8(n, count=5)
    sc = D.voxel_scale(n)
    d = Device(0)
    try:
        for tf in (bonsai_tf, case_tf(dict(tf_alpha_scale=0.0), bonsai_tf)):
            gpu_render(d, vol, sc, tf, INITIAL, 32, 32)
            empty, q, cells = _cell_flags(d, n)
            v16 = oracle.volume_r16f(vol)
            idx = np.clip(np.arange(n + 1) - 1, 0, n - 1); idx2 = np.clip(np.arange(n + 1), 0, n - 1)

            def mm(f):
                a = f(v16[idx], v16[idx2]); a = f(a[:, idx], a[:, idx2])
                return f(a[:, :, idx], a[:, :, idx2])
            vmin, vmax = mm(np.minimum), mm(np.maximum)
            t16 = tf.astype(np.float16).astype(np.float32)
            tau = np.concatenate([[t16[0, 3]], t16[:, 3], [t16[-1, 3]]])
            pre = np.concatenate([[0], np.cumsum((tau > 0) | np.isnan(tau))])
            fn = np.float32(tf.shape[0])
            kl = np.maximum(np.floor((vmin - np.float32(1 / 1024)) * fn - 0.5).astype(int) + 1, 0)
            kh = np.minimum(np.floor((vmax + np.float32(1 / 1024)) * fn - 0.5).astype(int) + 2,
                            tf.shape[0] + 1)
            want_empty = ~((kl <= kh) & (pre[np.maximum(kh, 0) + 1] - pre[kl] > 0))
            assert np.array_equal(empty, want_empty)
            dist = (ndimage.distance_transform_cdt(want_empty, metric="chessboard")
                    if (~want_empty).any() else np.full(want_empty.shape, 99))   # all empty
            want_q = np.where(want_empty, np.minimum(dist, 8) - 1, 0)
            assert np.array_equal(q, want_q)
            assert want_empty.any()
        # the densities are untouched by the flags
        fresh = Device(0)
        try:
            N.check(N.lib().cvr_set_option(fresh.handle, b"cell_skip", 0), "cell_skip")
            gpu_render(fresh, vol, sc, bonsai_tf, INITIAL, 32, 32)
            e0, q0, c0 = _cell_flags(fresh, n)
            assert not e0.any() and not q0.any()
            assert np.array_equal(c0 & 0x7fff7fff, cells & 0x7fff7fff)
        finally:
            fresh.close()
    finally:
        d.close()


def test_cell_skip_modes_bitexact_headline_band(oracle, bonsai_tf):
    """cell_skip 0 / 1 / 2 / 3 / 4 render the headline field identically (RGBA bits and per-pixel
    counts); a TF change rebuilds the flags (long-ray TF: alpha x 0.02)."""
    vol = _ml(256)
    sc = D.voxel_scale(256)
    W = H = 256
    d = Device(0)
    try:
        for tfs in (1.0, 0.02):
            tf = bonsai_tf.copy(); tf[:, 3] *= tfs
            res = []
            for cs in (0, 1, 2, 3, 4):
                N.check(N.lib().cvr_set_option(d.handle, b"cell_skip", cs), "cell_skip")
                res.append(gpu_render(d, vol, sc, tf, INITIAL, W, H, set_data=(cs == 0)))
            for cs in (1, 2, 3, 4):
                assert_bitexact(res[cs][0], res[0][0], f"cell_skip {cs} rgba (tf x{tfs})")
                assert_bitexact(res[cs][1], res[0][1], f"cell_skip {cs} counts (tf x{tfs})")
                assert res[cs][2] == res[0][2]
            rows = (120, 136)
            o_rgba, o_cnt, _ = oracle.render_rc1pass(oracle.volume_r16f(vol), sc, tf, INITIAL, W, H,
                                                     oracle.default_step(sc), rows=rows)
            assert_bitexact(res[2][0][rows[0]:rows[1]], o_rgba[rows[0]:rows[1]], "rows rgba")
            assert_bitexact(res[2][1][rows[0]:rows[1]], o_cnt[rows[0]:rows[1]], "rows counts")
    finally:
        d.close()


def test_jumping_camera_orders_bitexact(oracle, bonsai_tf):
    """Frames alternating between distant views (the learned order goes stale and
    the frame falls back to interleaved screen order), then holding one view (the
    order is relearned): every frame equals the oracle bit for bit."""
    vol = _ml(64)
    scale = (1.0, 1.0, 1.0)
    cams = [INITIAL, dict(eye=(-80.0, 40.0, -90.0), center=(0.0, 0.0, 0.0), up=(0.0, 1.0, 0.0)),
            dict(eye=(10.0, 120.0, 30.0), center=(2.0, 0.0, 0.0), up=(0.0, 0.0, 1.0))]
    W = H = 96
    ref = [oracle_render(oracle, vol, scale, bonsai_tf, c, W, H) for c in cams]
    d = Device(0)
    try:
        seq = [0, 1, 2, 0, 1, 1, 1, 2, 2, 2, 2, 0, 0]
        for k, i in enumerate(seq):
            g_rgba, g_cnt, g_total = gpu_render(d, vol, scale, bonsai_tf, cams[i], W, H,
                                                set_data=(k == 0))
            assert_bitexact(g_cnt, ref[i][1], f"frame {k} (view {i}) counts")
            assert_bitexact(g_rgba, ref[i][0], f"frame {k} (view {i}) rgba")
            assert g_total == ref[i][2]
    finally:
        d.close()


@pytest.mark.parametrize("nranks,tile", [(3, 16), (8, 32)])
def test_screen_tiles_with_quad_schedule(bonsai_tf, nranks, tile):
    """Packed (multi-GPU) tiles under the LPT + quad schedule equal the full frame."""
    vol = _ml(64)
    W, H = 200, 136
    d = Device(0)
    try:
        N.check(N.lib().cvr_set_option(d.handle, b"quad", 50), "quad")
        full, full_cnt, _ = gpu_render(d, vol, D.voxel_scale(64), bonsai_tf, INITIAL, W, H)
        tpr = T.max_tiles_per_rank(W, H, tile, nranks)
        packed_all = np.zeros((nranks, tpr, tile, tile, 4), np.float32)
        for r in range(nranks):
            for rep in range(4):   # the fourth pass runs with the learned order (lag 3)
                rgba, cnt, _ = gpu_render(d, vol, D.voxel_scale(64), bonsai_tf, INITIAL, W, H,
                                          tile=tile, rank=r, nranks=nranks, set_data=False)
            packed_all[r, :rgba.shape[0]] = rgba
        assert_bitexact(T.unpack(packed_all, W, H, tile, nranks), full, "unpacked")
    finally:
        d.close()


def test_kernel_timing_ring(dev, bonsai_tf):
    """kernel_timing: the library's HIP events around the ray-march launch."""
    vol = _ml(32)
    L = N.lib()
    N.check(L.cvr_set_option(dev.handle, b"kernel_timing", 3), "kernel_timing")
    try:
        for i in range(5):
            gpu_render(dev, vol, D.voxel_scale(32), bonsai_tf, INITIAL, 64, 64, set_data=(i == 0))
        ms = (ctypes.c_float * 8)()
        n = ctypes.c_int()
        N.check(L.cvr_read_kernel_times(dev.handle, ms, 8, ctypes.byref(n)), "read", dev.handle)
        assert n.value == 3 and all(0.0 < ms[i] < 1000.0 for i in range(3))
        N.check(L.cvr_read_kernel_times(dev.handle, ms, 8, ctypes.byref(n)), "read", dev.handle)
        assert n.value == 0
    finally:
        N.check(L.cvr_set_option(dev.handle, b"kernel_timing", 0), "kernel_timing")
    assert L.cvr_read_kernel_times(dev.handle, ms, 8, ctypes.byref(n)) == N.CVR_ERR_STATE


@pytest.mark.parametrize("cap", [100, 130, 200])
def test_band_cap_holds(bonsai_tf, cap):
    """Under the learned launch order every XCD band holds at most band_cap % of an
    even eighth of the tiles (tile_epilogue_kernel moves a balanced boundary the
    least that fits), and every tile runs in exactly one slot: the slots the
    tiles report (tile_stats: block index b -> band b % 8, entry b / 8) are
    distinct and within the band's entries.  The image stays that of the first
    (unordered) frame."""
    W = H = 256
    ntiles = (W // 8) * (H // 8)
    seg_avg = (ntiles + 7) // 8
    cap_tiles = (seg_avg * cap + 99) // 100
    d = Device(0)
    try:
        for k, v in (("tile_order", 1), ("band_cap", cap), ("tile_stats", 1), ("order_interval", 1)):
            N.check(N.lib().cvr_set_option(d.handle, k.encode(), v), k, d.handle)
        vol = D.marschner_lobb_u8(128)
        first = None
        for frame in range(4):
            rgba, cnt, _ = gpu_render(d, vol, D.voxel_scale(128), bonsai_tf, INITIAL, W, H,
                                      set_data=(frame == 0))
            if first is None:
                first = (rgba, cnt)
        assert_bitexact(rgba, first[0], f"cap {cap} ordered rgba")
        assert_bitexact(cnt, first[1], f"cap {cap} ordered counts")
        st = np.zeros(ntiles * 4, np.uint64)
        nt = ctypes.c_int()
        N.check(N.lib().cvr_copy_tile_stats(d.handle, st.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)),
                                            ntiles, ctypes.byref(nt)), "stats", d.handle)
        slots = (st.reshape(-1, 4)[:, 3] >> np.uint64(32)).astype(np.int64)
        assert len(np.unique(slots)) == ntiles
        assert not np.array_equal(slots, np.arange(ntiles)), "the learned order was not in use"
        band, entry = slots & 7, slots >> 3
        per_band = np.bincount(band, minlength=8)
        assert per_band.sum() == ntiles and per_band.max() <= cap_tiles, per_band
        for x in range(8):   # a band's entries are 0 .. n-1, each once
            assert np.array_equal(np.sort(entry[band == x]), np.arange(per_band[x]))
    finally:
        d.close()
