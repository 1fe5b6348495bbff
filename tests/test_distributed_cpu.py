"""Multi-process (gloo, CPU) checks of the screen-tile split.

Every rank packs its interleaved tiles of one frame exactly as the device kernel
does (screen_tiles.pack_rank is the host mirror of the packed layout), rank 0
gathers them with screen_tiles.gather_to_root -- the same call bench.py makes
over RCCL -- and unpacks; the result must equal the full frame bit for bit.
The frame is an oracle rendering, so the content is a real ray-cast image
(misses, ERT, ragged edges), and ranks may own different tile counts.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from cpp_volume_rendering_amd import datasets as D
from cpp_volume_rendering_amd import screen_tiles as T


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _frame(W, H):
    import oracle as O
    vol = D.marschner_lobb_u8(24)
    scale = D.voxel_scale(24)
    table = O.tf_table_double(D.BONSAI_TF_RGB, D.BONSAI_TF_ALPHA)
    rgba, cnt, _ = O.render_rc1pass(O.volume_r16f(vol), scale, O.tf_rgbt(table),
                                    D.INITIAL_STATE_CAMERA, W, H, O.default_step(scale))
    return rgba, cnt


def _worker(rank, world, port, W, H, tile, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        rgba, cnt = _frame(W, H)
        tpr = T.max_tiles_per_rank(W, H, tile, world)
        mine = torch.from_numpy(T.pack_rank(rgba, tile, rank, world))
        assert mine.shape[0] == T.tiles_for_rank(W, H, tile, rank, world)
        allp = T.gather_to_root(mine, tpr)
        mine_c = torch.from_numpy(T.pack_rank(cnt.astype(np.int32), tile, rank, world))
        allc = T.gather_to_root(mine_c, tpr)
        if rank == 0:
            img = T.unpack(allp.numpy(), W, H, tile, world)
            counts = T.unpack(allc.numpy(), W, H, tile, world)
            ok = (np.array_equal(img.view(np.uint32), rgba.view(np.uint32))
                  and np.array_equal(counts, cnt.astype(np.int32)))
            q.put(("ok" if ok else "mismatch", int(cnt.sum())))
        else:
            assert allp is None and allc is None
        dist.barrier()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,W,H,tile", [(2, 96, 80, 32), (3, 70, 45, 16), (2, 16, 16, 32),
                                            (4, 128, 96, 16)])
def test_gather_unpack_gloo(world, W, H, tile):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, W, H, tile, q))
             for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=240)
    codes = [p.exitcode for p in procs]
    assert codes == [0] * world, f"worker exit codes {codes}"
    status, samples = q.get(timeout=10)
    assert status == "ok"
    assert samples > 0


def test_tile_partition_covers_frame():
    for W, H, tile, world in [(1024, 1024, 32, 8), (1000, 600, 48, 3), (17, 9, 16, 4)]:
        ntx, nty = T.tile_grid(W, H, tile)
        owned = sum(T.tiles_for_rank(W, H, tile, r, world) for r in range(world))
        assert owned == ntx * nty
        assert T.max_tiles_per_rank(W, H, tile, world) == -(-ntx * nty // world)


CAMS = [dict(D.INITIAL_STATE_CAMERA),
        dict(D.INITIAL_STATE_CAMERA, eye=(-300.0, 120.0, 380.0)),
        dict(D.INITIAL_STATE_CAMERA, eye=(0.0, -400.0, 200.0))]


def _frames(W, H):
    import oracle as O
    vol = D.marschner_lobb_u8(24)
    scale = D.voxel_scale(24)
    table = O.tf_table_double(D.BONSAI_TF_RGB, D.BONSAI_TF_ALPHA)
    out = {}
    for c in CAMS:
        rgba, _, _ = O.render_rc1pass(O.volume_r16f(vol), scale, O.tf_rgbt(table), c, W, H,
                                      O.default_step(scale))
        out[tuple(c["eye"])] = rgba.astype(np.float16)
    return out


def _split_worker(rank, world, port, W, H, tile, q):
    """ScreenTileSplit (torch transport, RGBA16F) over gloo with host mirrors of the
    render (pack_rank of an oracle frame) and the unpack: frames are pipelined, so
    after submit(n) rank 0's image must hold frame n-1, and after flush frame n."""
    from cpp_volume_rendering_amd import _native as N
    from cpp_volume_rendering_amd.renderer import Camera
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        imgs = _frames(W, H)

        def render_fn(frame, out, total):
            eye = tuple(float(v) for v in frame.camera.eye)
            assert frame.rank == rank and frame.nranks == world
            p = T.pack_rank(imgs[eye], tile, rank, world)
            out.zero_()
            out[:p.shape[0]] = torch.from_numpy(p)

        def unpack_fn(frame, gathered, image):
            image.copy_(torch.from_numpy(T.unpack(gathered.numpy(), W, H, tile, world)))

        sp = T.ScreenTileSplit(None, W, H, tile=tile, fmt=N.FORMAT_RGBA16F, device="cpu",
                               render_fn=render_fn, unpack_fn=unpack_fn)
        assert sp.transport == "torch"
        seq = [0, 1, 2, 1, 0]
        ok = True
        for n, ci in enumerate(seq):
            sp.submit(Camera(**CAMS[ci]))
            assert sp.completed == n - 1
            if rank == 0 and n > 0:
                want = imgs[tuple(CAMS[seq[n - 1]]["eye"])]
                ok &= np.array_equal(sp.image.numpy().view(np.uint16), want.view(np.uint16))
        img = sp.flush()
        assert sp.completed == len(seq) - 1
        if rank == 0:
            want = imgs[tuple(CAMS[seq[-1]]["eye"])]
            ok &= np.array_equal(img.numpy().view(np.uint16), want.view(np.uint16))
            q.put("ok" if ok else "mismatch")
        dist.barrier()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,W,H,tile", [(2, 96, 80, 32), (3, 70, 45, 16)])
def test_screen_tile_split_pipeline_gloo(world, W, H, tile):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_split_worker, args=(r, world, port, W, H, tile, q))
             for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=240)
    codes = [p.exitcode for p in procs]
    assert codes == [0] * world, f"worker exit codes {codes}"
    assert q.get(timeout=10) == "ok"


class _FakeStream:
    _n = 0

    def __init__(self):
        _FakeStream._n += 1
        self.cuda_stream = 1000 + _FakeStream._n

    def wait_stream(self, other):
        pass


class _FakeLib:
    """Records the native split path's C calls (cvr_render_* / cvr_gather_tiles_n)."""

    def __init__(self):
        self.calls = []
        self.stream = None

    def cvr_comm_unique_id(self, buf):
        buf.raw = b"\x07" * len(buf.raw)
        return 0

    def cvr_comm_init(self, h, world, rank, uid):
        assert uid == b"\x07" * len(uid)
        self.calls.append(("init", world, rank))
        return 0

    def cvr_set_option(self, h, key, val):
        self.calls.append(("opt", key, val))
        return 0

    def cvr_set_stream(self, h, s):
        self.stream = s
        return 0

    def cvr_render_rc1pass(self, h, fr, params, out):
        self.calls.append(("render", self.stream, out._obj.rgba))
        return 0

    def cvr_render_rc1pass_frames(self, h, frames, n, params, outs):
        self.calls.append(("render_n", self.stream, n, [outs[j].rgba for j in range(n)],
                           [outs[j].total for j in range(n)],
                           [(frames[j].rank, frames[j].nranks) for j in range(n)]))
        return 0

    def cvr_gather_tiles_n(self, h, fr, nframes, buf, tpr, fmt, g, imgs):
        self.calls.append(("gather", self.stream, nframes, buf, g is not None,
                           [imgs[j] for j in range(nframes)] if imgs is not None else None))
        return 0

    def cvr_gather_sync(self, h):
        self.calls.append(("sync",))
        return 0

    def cvr_comm_destroy(self, h):
        self.calls.append(("destroy",))
        return 0


def _native_flow_worker(rank, world, port, q):
    """ScreenTileSplit's native-RCCL fast path (frames rotated over D streams, G frames
    per exchange, a partial group at flush) with the library calls recorded: every
    rank must issue the same gathers, each covering its group's frames in order."""
    from cpp_volume_rendering_amd import _native as N
    from cpp_volume_rendering_amd.renderer import Camera
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        fake = _FakeLib()
        N._lib = fake

        class R:
            _ENTRY = "cvr_render_rc1pass"
            _params = N.Rc1passParams()

            class device:
                handle = 1

                @staticmethod
                def set_stream(s):
                    fake.stream = s

        D_, G = 3, 4
        sp = T.ScreenTileSplit(R(), 96, 64, tile=32, fmt=N.FORMAT_RGBA16F, device="cpu",
                               transport="rccl", streams=D_, frames_per_exchange=G,
                               stream_factory=_FakeStream)
        assert sp._fast is not None and sp.G == G and sp.nbuf == D_
        cam = Camera(**D.INITIAL_STATE_CAMERA)
        nframes = 10
        for _ in range(nframes):
            sp.submit(cam)
        sp.flush()
        renders = [c for c in fake.calls if c[0] == "render"]
        gathers = [c for c in fake.calls if c[0] == "gather"]
        assert len(renders) == nframes
        assert [g[2] for g in gathers] == [4, 4, 2]          # two full groups + the rest
        streams = [s.cuda_stream for s in sp.streams]
        # group q renders and gathers on stream q % D; frame j of a group -> slot j
        for n, rc in enumerate(renders):
            grp, j = divmod(n, G)
            assert rc[1] == streams[grp % D_]
            blk = (sp.gathered[grp % D_][0] if rank == 0 else sp.packed[grp % D_])
            assert rc[2] == blk[j].data_ptr()
        for grp, g in enumerate(gathers):
            assert g[1] == streams[grp % D_]
            assert g[4] == (rank == 0)
        assert ("opt", b"split_streams", D_) in fake.calls
        sp.close()
        assert fake.calls[-1] == ("destroy",)
        q.put(("ok", rank, len(gathers)))
    except Exception as e:   # noqa: BLE001  (reported to the parent)
        q.put(("fail", rank, repr(e)))
        raise
    finally:
        dist.destroy_process_group()


def _native_batch_worker(rank, world, port, q):
    """The same fast path with frames_per_launch = 4: a group's frames render in ONE
    cvr_render_rc1pass_frames call (slots 0..3 of the group's buffer, only frame 0
    with the total), then its gather; the partial group at flush renders its 2."""
    from cpp_volume_rendering_amd import _native as N
    from cpp_volume_rendering_amd.renderer import Camera
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        fake = _FakeLib()
        N._lib = fake

        class R:
            _ENTRY = "cvr_render_rc1pass"
            _params = N.Rc1passParams()

            class device:
                handle = 1

                @staticmethod
                def set_stream(s):
                    fake.stream = s

        D_, L = 3, 4
        sp = T.ScreenTileSplit(R(), 96, 64, tile=32, fmt=N.FORMAT_RGBA16F, device="cpu",
                               transport="rccl", streams=D_, frames_per_exchange=2,
                               stream_factory=_FakeStream, count_samples=True,
                               frames_per_launch=L)
        assert sp._fast is not None and sp.G == L and sp.L == L
        cam = Camera(**D.INITIAL_STATE_CAMERA)
        for _ in range(10):
            sp.submit(cam)
        assert [c[0] for c in fake.calls if c[0] in ("render", "render_n", "gather")] == \
            ["render_n", "gather", "render_n", "gather"]
        sp.flush()
        calls = [c for c in fake.calls if c[0] in ("render", "render_n", "gather")]
        assert [c[0] for c in calls] == ["render_n", "gather"] * 3
        renders = [c for c in calls if c[0] == "render_n"]
        gathers = [c for c in calls if c[0] == "gather"]
        assert [r[2] for r in renders] == [4, 4, 2] and [g[2] for g in gathers] == [4, 4, 2]
        streams = [s.cuda_stream for s in sp.streams]
        for grp, (rc, g) in enumerate(zip(renders, gathers)):
            assert rc[1] == streams[grp % D_] and g[1] == streams[grp % D_]
            blk = (sp.gathered[grp % D_][0] if rank == 0 else sp.packed[grp % D_])
            assert rc[3] == [blk[j].data_ptr() for j in range(rc[2])]
            assert rc[4][0] == sp.total.data_ptr() and not any(rc[4][1:])
        sp.close()
        q.put(("ok", rank, len(gathers)))
    except Exception as e:   # noqa: BLE001  (reported to the parent)
        q.put(("fail", rank, repr(e)))
        raise
    finally:
        dist.destroy_process_group()


def _native_idle_root_worker(rank, world, port, q):
    """root_renders=False (library option gather_root_idle): rank 0 renders nothing and
    only exchanges; ranks 1..N-1 render the split over N-1 render ranks (frame rank =
    rank - 1), 4 frames per launch; every rank issues the same gathers."""
    from cpp_volume_rendering_amd import _native as N
    from cpp_volume_rendering_amd.renderer import Camera
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        fake = _FakeLib()
        N._lib = fake

        class R:
            _ENTRY = "cvr_render_rc1pass"
            _params = N.Rc1passParams()

            class device:
                handle = 1

                @staticmethod
                def set_stream(s):
                    fake.stream = s

        sp = T.ScreenTileSplit(R(), 96, 64, tile=16, fmt=N.FORMAT_RGBA16F, device="cpu",
                               transport="rccl", streams=2, stream_factory=_FakeStream,
                               frames_per_launch=4, buffer_sets=8, root_renders=False)
        assert sp.idle_root and sp.sworld == world - 1 and sp.nbuf == 8
        assert sp.k == (0 if rank == 0 else T.tiles_for_rank(96, 64, 16, rank - 1, world - 1))
        assert sp.tpr_max == T.max_tiles_per_rank(96, 64, 16, world - 1)
        cam = Camera(**D.INITIAL_STATE_CAMERA)
        for _ in range(9):
            sp.submit(cam)
        sp.flush()
        renders = [c for c in fake.calls if c[0] == "render_n"]
        gathers = [c for c in fake.calls if c[0] == "gather"]
        assert [g[2] for g in gathers] == [4, 4, 1]
        if rank == 0:
            assert renders == []
        else:
            assert [r[2] for r in renders] == [4, 4, 1]
            assert all(fr == (rank - 1, world - 1) for r in renders for fr in r[5])
        assert ("opt", b"gather_root_idle", 1) in fake.calls
        assert ("opt", b"gather_sets", 8) in fake.calls
        sp.close()
        q.put(("ok", rank, len(gathers)))
    except Exception as e:   # noqa: BLE001  (reported to the parent)
        q.put(("fail", rank, repr(e)))
        raise
    finally:
        dist.destroy_process_group()


def _native_bench8_worker(rank, world, port, q):
    """Exactly `bench.py --gpus 8`'s default split (bench.split_defaults): 1024^2, 16^2
    tiles, 16 frames per launch and per exchange (coded), 4 render streams, 16 buffer
    sets, an idle root (ranks 1..7 render the split over 7 render ranks), 32 HW queues.
    Every rank must issue the same gathers; each render rank renders its 16-frame
    groups as its own split rank into the group's buffer set, rotated over the 16."""
    G = 16
    os.environ["WORLD_SIZE"] = str(world)       # bench.py reads it at import (HW queues)
    import bench
    from cpp_volume_rendering_amd import _native as N
    from cpp_volume_rendering_amd.renderer import Camera
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        fake = _FakeLib()
        N._lib = fake

        class R:
            _ENTRY = "cvr_render_rc1pass"
            _params = N.Rc1passParams()

            class device:
                handle = 1

                @staticmethod
                def set_stream(s):
                    fake.stream = s

        a = bench.parse(["--gpus", str(world)])
        kw = bench.split_defaults(a, world)
        assert kw == {"streams": 4, "frames_per_exchange": G, "frames_per_launch": G,
                      "buffer_sets": 16, "root_renders": False}, kw
        assert bench.HW_QUEUES == 32 and a.tile == 16 and a.transport == "rccl"
        W = H = 1024
        sp = T.ScreenTileSplit(R(), W, H, tile=a.tile, fmt=N.FORMAT_RGBA16F, device="cpu",
                               transport=a.transport, stream_factory=_FakeStream,
                               count_samples=True, **kw)
        assert sp.idle_root and sp.renders == (rank != 0)
        assert sp.sworld == world - 1 and sp.srank == max(rank - 1, 0)
        assert sp.nbuf == 16 and sp.G == G and sp.L == G and sp.nstreams == 4
        assert sp.k == (0 if rank == 0 else T.tiles_for_rank(W, H, 16, rank - 1, world - 1))
        cam = Camera(**D.INITIAL_STATE_CAMERA)
        nframes = G * 16 + 6            # every buffer set used, then reused, and a partial group
        for _ in range(nframes):
            sp.submit(cam)
        sp.flush()
        renders = [c for c in fake.calls if c[0] == "render_n"]
        gathers = [c for c in fake.calls if c[0] == "gather"]
        sizes = [G] * (nframes // G) + ([nframes % G] if nframes % G else [])
        assert [g[2] for g in gathers] == sizes
        streams = [s.cuda_stream for s in sp.streams]
        bufs = set()
        for grp, g in enumerate(gathers):
            assert g[1] == streams[grp % 4]
            assert g[4] == (rank == 0)
            bufs.add(g[3])
        if rank == 0:
            assert renders == []
        else:
            assert [r[2] for r in renders] == sizes
            assert all(fr == (rank - 1, world - 1) for r in renders for fr in r[5])
            for grp, rc in enumerate(renders):
                assert rc[1] == streams[grp % 4]
            assert len(bufs) == 16          # the 16 sets rotate
        for opt in (("opt", b"gather_root_idle", 1), ("opt", b"gather_sets", 16),
                    ("opt", b"split_streams", 4), ("opt", b"exchange_code", 1)):
            assert opt in fake.calls, opt
        # the coded exchange decodes a group's frames in one launch: rank 0 hands every
        # frame of a group its own image (G distinct), the same G for every group
        if rank == 0:
            imgs = [tuple(g[5]) for g in gathers]
            assert all(len(set(i)) == len(i) for i in imgs)
            assert imgs[0] == tuple(im.data_ptr() for im in sp._images[:G])
            assert all(i == imgs[0][:len(i)] for i in imgs)
        else:
            assert all(g[5] is None for g in gathers)
        sp.close()
        q.put(("ok", rank, len(gathers)))
    except Exception as e:   # noqa: BLE001  (reported to the parent)
        q.put(("fail", rank, repr(e)))
        raise
    finally:
        dist.destroy_process_group()


def _buffer_sets_worker(rank, world, port, q):
    """Buffer sets above the library's limit (CVR_MAX_GATHER_SETS = 64) are clamped to
    the most whole multiples of the streams, never passed on."""
    from cpp_volume_rendering_amd import _native as N
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        fake = _FakeLib()
        N._lib = fake

        class R:
            _ENTRY = "cvr_render_rc1pass"
            _params = N.Rc1passParams()

            class device:
                handle = 1

                @staticmethod
                def set_stream(s):
                    fake.stream = s

        for streams, sets, want in ((16, 64, 64), (16, 80, 64), (13, 52, 52), (20, 80, 60),
                                    (3, 200, 63)):
            fake.calls.clear()
            sp = T.ScreenTileSplit(R(), 64, 64, tile=16, fmt=N.FORMAT_RGBA16F, device="cpu",
                                   transport="rccl", streams=streams, stream_factory=_FakeStream,
                                   buffer_sets=sets)
            assert sp.nbuf == want, (streams, sets, sp.nbuf)
            assert ("opt", b"gather_sets", want) in fake.calls
            sp.close()
        q.put(("ok", rank, 0))
    except Exception as e:   # noqa: BLE001  (reported to the parent)
        q.put(("fail", rank, repr(e)))
        raise
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("worker", ["flow", "batch", "idle_root", "bench8", "buffer_sets"])
def test_native_split_control_flow_gloo(worker):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    target = {"flow": _native_flow_worker, "batch": _native_batch_worker,
              "idle_root": _native_idle_root_worker, "bench8": _native_bench8_worker,
              "buffer_sets": _buffer_sets_worker}[worker]
    world = {"idle_root": 3, "bench8": 8}.get(worker, 2)
    procs = [ctx.Process(target=target, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=240)
    res = [q.get(timeout=10) for _ in range(world)]
    assert all(r[0] == "ok" for r in res), res
    assert [p.exitcode for p in procs] == [0] * world


@pytest.mark.parametrize("W,H,tile,world", [(1024, 1024, 16, 8), (1024, 1024, 32, 4),
                                            (2048, 2048, 16, 8), (100, 72, 16, 3), (70, 45, 16, 2)])
def test_split_tile_is_a_partition(W, H, tile, world):
    """split_tile deals every tile to exactly one rank, with tiles_for_rank tiles each;
    when N divides the tiles per row it is the diagonal lattice (tx + s*ty) mod N."""
    ntx, nty = T.tile_grid(W, H, tile)
    seen = np.zeros((nty, ntx), np.int32)
    owner = np.full((nty, ntx), -1, np.int32)
    for r in range(world):
        for k in range(T.tiles_for_rank(W, H, tile, r, world)):
            tx, ty = T.split_tile(r, world, k, ntx)
            seen[ty, tx] += 1
            owner[ty, tx] = r
    assert (seen == 1).all()
    if ntx % world == 0:
        tx, ty = np.meshgrid(np.arange(ntx), np.arange(nty))
        assert np.array_equal(owner, (tx + T.split_shift(world) * ty) % world)
