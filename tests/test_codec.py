"""The lossless per-tile code of RGBA16F screen tiles (codec.hip, cvr_encode_tiles /
cvr_decode_tiles).

CPU: a numpy restatement of the stream (tile starts, 3 header words, each
channel's differences from the tile minimum at the bit width of the largest one),
its bound, and its round trip.  GPU (marked): the library's stream equals the
restatement word for word on rendered tiles, random bit patterns, constant tiles
and 32 x 32 tiles, and decodes to the input bit for bit."""
import ctypes

import numpy as np
import pytest

from cpp_volume_rendering_amd import _native as N
from cpp_volume_rendering_amd import datasets as D
from cpp_volume_rendering_amd import screen_tiles as T
from cpp_volume_rendering_amd.renderer import Camera, Device, make_frame


def np_encode(tiles: np.ndarray) -> np.ndarray:
    """tiles: (n, npx, 4) uint16 channel patterns -> the stream (uint32 words)."""
    n, npx, _ = tiles.shape
    words = [np.zeros(n + 1, np.uint32)]
    pos = n + 1
    starts = []
    for t in range(n):
        x = tiles[t].astype(np.uint32)
        base = x.min(axis=0)
        span = x.max(axis=0) - base
        width = [int(s).bit_length() for s in span]
        hdr = np.array([base[0] | (base[1] << 16), base[2] | (base[3] << 16),
                        width[0] | (width[1] << 5) | (width[2] << 10) | (width[3] << 15)], np.uint32)
        body = [hdr]
        for c in range(4):
            w = width[c]
            if not w:
                continue
            nw = (npx * w + 31) // 32
            bits = np.zeros(nw * 32, np.uint8)
            d = x[:, c] - base[c]
            for k in range(w):   # bit k of pixel p at position p * w + k
                bits[np.arange(npx) * w + k] = (d >> k) & 1
            body.append(np.packbits(bits.reshape(-1, 32)[:, ::-1], axis=1).view(">u4").ravel().astype(np.uint32))
        blk = np.concatenate(body)
        starts.append(pos)
        pos += len(blk)
        words.append(blk)
    table = np.array(starts + [pos], np.uint32)
    words[0] = table
    return np.concatenate(words)


def np_decode(stream: np.ndarray, n: int, npx: int) -> np.ndarray:
    out = np.zeros((n, npx, 4), np.uint32)
    for t in range(n):
        s = int(stream[t])
        h0, h1, h2 = (int(v) for v in stream[s:s + 3])
        base = [h0 & 0xffff, h0 >> 16, h1 & 0xffff, h1 >> 16]
        width = [h2 & 31, (h2 >> 5) & 31, (h2 >> 10) & 31, (h2 >> 15) & 31]
        pos = s + 3
        for c in range(4):
            w = width[c]
            if w:
                nw = (npx * w + 31) // 32
                bits = np.unpackbits(stream[pos:pos + nw].astype(">u4").view(np.uint8).reshape(-1, 4),
                                     axis=1)
                bits = bits.reshape(-1, 32)[:, ::-1].ravel()
                idx = np.arange(npx)[:, None] * w + np.arange(w)[None, :]
                d = (bits[idx].astype(np.uint32) << np.arange(w, dtype=np.uint32)[None, :]).sum(axis=1)
                pos += nw
            else:
                d = 0
            out[t, :, c] = base[c] + d
    return out.astype(np.uint16)


def bound_bytes(tile, n):
    npx = tile * tile
    return 4 * (n + 1 + n * (3 + 4 * ((npx * 16 + 31) // 32)))


def _smooth_tiles(n, npx, seed=1):
    rng = np.random.default_rng(seed)
    base = rng.integers(0, 0x7c00, (n, 1, 4))
    return (base + rng.integers(0, 37, (n, npx, 4))).astype(np.uint16)


def test_np_code_round_trip_and_bound():
    for tiles in (_smooth_tiles(5, 256), np.random.default_rng(2).integers(0, 65536, (3, 256, 4)).astype(np.uint16),
                  np.full((4, 256, 4), 0x3c00, np.uint16)):
        st = np_encode(tiles)
        assert st[0] == len(tiles) + 1 and st[len(tiles)] == len(st)
        assert np.array_equal(np_decode(st, len(tiles), 256), tiles)
        assert 4 * len(st) <= bound_bytes(16, len(tiles))
    const = np_encode(np.full((4, 256, 4), 0x3c00, np.uint16))
    assert len(const) == 5 + 4 * 3        # headers only


def test_tile_code_bound_abi():
    L = N.lib()
    assert L.cvr_tile_code_bound(16, 10) == bound_bytes(16, 10)
    assert L.cvr_tile_code_bound(32, 3) == bound_bytes(32, 3)
    assert L.cvr_tile_code_bound(16, 0) == 4
    for bad in ((8, 4), (24, 4), (128, 4), (16, -1)):
        assert L.cvr_tile_code_bound(*bad) == 0


# ---------------------------------------------------------------------------- GPU


@pytest.fixture(scope="module")
def dev():
    import torch
    assert torch.cuda.is_available(), "GPU tests need a HIP device"
    d = Device(0)
    yield d
    d.close()


def _gpu_round_trip(dev, tiles_u16, tile):
    """tiles_u16: (n, tile*tile, 4) uint16 -> (stream words, decoded tiles)."""
    import torch
    n = tiles_u16.shape[0]
    L = N.lib()
    d_tiles = torch.from_numpy(tiles_u16.view(np.int16).copy()).cuda()
    d_stream = torch.zeros(L.cvr_tile_code_bound(tile, n) // 4, dtype=torch.int32, device="cuda")
    d_bytes = torch.zeros(1, dtype=torch.int64, device="cuda")
    d_out = torch.zeros_like(d_tiles)
    dev.set_stream(torch.cuda.current_stream().cuda_stream)
    try:
        N.check(L.cvr_encode_tiles(dev.handle, d_tiles.data_ptr(), tile, n, d_stream.data_ptr(),
                                   d_bytes.data_ptr()), "encode", dev.handle)
        N.check(L.cvr_decode_tiles(dev.handle, d_stream.data_ptr(), tile, n, d_out.data_ptr()),
                "decode", dev.handle)
        torch.cuda.synchronize()
    finally:
        dev.set_stream(None)
    nbytes = int(d_bytes.item())
    stream = d_stream.cpu().numpy().view(np.uint32)[:nbytes // 4]
    return stream, d_out.cpu().numpy().view(np.uint16), nbytes


def _rendered_tiles(dev, bonsai_tf, W, H, tile, rank, nranks):
    vol = D.marschner_lobb_u8(96)
    dev.set_volume(vol, D.voxel_scale(96))
    dev.set_transfer_function(bonsai_tf)
    dev.set_gradient(N.GRADIENT_NONE)
    frame = make_frame(Camera(**D.INITIAL_STATE_CAMERA), W, H, tile, rank, nranks)
    k = T.tiles_for_rank(W, H, tile, rank, nranks)
    img = np.zeros((k, tile, tile, 4), np.float16)
    out = N.Output(img.ctypes.data, None, None, 0, N.FORMAT_RGBA16F)
    p = N.Rc1passParams()
    N.check(N.lib().cvr_render_rc1pass(dev.handle, ctypes.byref(frame), ctypes.byref(p),
                                       ctypes.byref(out)), "render", dev.handle)
    return img.view(np.uint16).reshape(k, tile * tile, 4)


@pytest.mark.gpu
@pytest.mark.parametrize("tile", [16, 32])
def test_gpu_code_rendered_tiles(dev, bonsai_tf, tile):
    tiles = _rendered_tiles(dev, bonsai_tf, 200, 168, tile, 1, 3)
    stream, back, nbytes = _gpu_round_trip(dev, tiles, tile)
    assert np.array_equal(back, tiles)
    assert np.array_equal(stream, np_encode(tiles))
    assert nbytes < tiles.nbytes / 2          # rendered tiles code small


@pytest.mark.gpu
@pytest.mark.parametrize("kind", ["random", "constant", "smooth", "empty"])
def test_gpu_code_patterns(dev, kind):
    rng = np.random.default_rng(7)
    n, tile = 37, 16
    if kind == "random":
        tiles = rng.integers(0, 65536, (n, tile * tile, 4)).astype(np.uint16)
    elif kind == "constant":
        tiles = np.broadcast_to(rng.integers(0, 65536, (n, 1, 4)), (n, tile * tile, 4)).astype(np.uint16)
    elif kind == "smooth":
        tiles = _smooth_tiles(n, tile * tile, seed=3)
    else:
        tiles = np.zeros((0, tile * tile, 4), np.uint16)
    stream, back, nbytes = _gpu_round_trip(dev, tiles, tile)
    assert np.array_equal(back, tiles)
    assert np.array_equal(stream, np_encode(tiles))
    assert nbytes <= bound_bytes(tile, len(tiles))


@pytest.mark.gpu
def test_gpu_code_bad_arguments(dev):
    L = N.lib()
    assert L.cvr_encode_tiles(dev.handle, None, 16, 4, None, None) == N.CVR_ERR_ARG
    assert L.cvr_decode_tiles(dev.handle, None, 8, 4, None) == N.CVR_ERR_ARG


@pytest.mark.gpu
@pytest.mark.parametrize("kind", ["rendered16", "rendered32", "random", "constant", "empty"])
def test_gpu_code_onepass(dev, bonsai_tf, kind):
    """The exchange's one-launch encode (option encode_onepass): tiles claim
    their words with an atomic, so codes follow in claim order, but the stream has the
    same length as the three-launch form, every tile's code is the same words wherever
    it lies, and cvr_decode_tiles restores the tiles bit for bit.  Twice in a row: the
    launch leaves its counters zero for the next one."""
    rng = np.random.default_rng(11)
    tile = 32 if kind == "rendered32" else 16
    npx = tile * tile
    if kind.startswith("rendered"):
        tiles = _rendered_tiles(dev, bonsai_tf, 200, 168, tile, 1, 3)
    elif kind == "random":
        tiles = rng.integers(0, 65536, (29, npx, 4)).astype(np.uint16)
    elif kind == "constant":
        tiles = np.broadcast_to(rng.integers(0, 65536, (29, 1, 4)), (29, npx, 4)).astype(np.uint16)
    else:
        tiles = np.zeros((0, npx, 4), np.uint16)
    want = np_encode(tiles)
    n = tiles.shape[0]
    L = N.lib()
    N.check(L.cvr_set_option(dev.handle, b"encode_onepass", 1), "opt", dev.handle)
    try:
        for _ in range(2):
            stream, back, nbytes = _gpu_round_trip(dev, tiles, tile)
            assert np.array_equal(back, tiles)
            assert nbytes == want.nbytes and int(stream[n]) == len(want)
            for t in range(n):          # tile t's code, wherever it was placed
                s, s0 = int(stream[t]), int(want[t])
                ln = int(want[t + 1]) - s0
                assert np.array_equal(stream[s:s + ln], want[s0:s0 + ln]), t
    finally:
        N.check(L.cvr_set_option(dev.handle, b"encode_onepass", 0), "opt", dev.handle)


@pytest.mark.gpu
def test_gpu_code_onepass_concurrent_streams(dev, bonsai_tf):
    """One-launch encodes on four streams at once: each keeps its counters in its own
    stream's end word and length (an earlier form shared one counter pair per context,
    so concurrent launches claimed each other's words and wrote past their streams)."""
    import torch
    tiles = _rendered_tiles(dev, bonsai_tf, 256, 256, 16, 0, 2)
    n = tiles.shape[0]
    want = np_encode(tiles)
    L = N.lib()
    d_tiles = torch.from_numpy(tiles.view(np.int16).copy()).cuda()
    streams = [torch.cuda.Stream() for _ in range(4)]
    bound = L.cvr_tile_code_bound(16, n)
    outs = [torch.zeros(bound // 4, dtype=torch.int32, device="cuda") for _ in streams]
    lens = [torch.zeros(1, dtype=torch.int64, device="cuda") for _ in streams]
    torch.cuda.synchronize()
    N.check(L.cvr_set_option(dev.handle, b"encode_onepass", 1), "opt", dev.handle)
    try:
        for rep in range(8):
            for s, o, ln in zip(streams, outs, lens):
                dev.set_stream(s.cuda_stream)
                N.check(L.cvr_encode_tiles(dev.handle, d_tiles.data_ptr(), 16, n, o.data_ptr(),
                                           ln.data_ptr()), "encode", dev.handle)
        torch.cuda.synchronize()
    finally:
        dev.set_stream(None)
        N.check(L.cvr_set_option(dev.handle, b"encode_onepass", 0), "opt", dev.handle)
    for o, ln in zip(outs, lens):
        assert int(ln.item()) == want.nbytes
        back = torch.zeros_like(d_tiles)
        N.check(L.cvr_decode_tiles(dev.handle, o.data_ptr(), 16, n, back.data_ptr()), "decode", dev.handle)
        torch.cuda.synchronize()
        assert np.array_equal(back.cpu().numpy().view(np.uint16), tiles)
