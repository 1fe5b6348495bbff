"""Screen-tile split of one frame over the GPUs of a node.

The reference renders on one GPU; pixels are independent, so the framebuffer
is cut into ``tile`` x ``tile`` tiles (16 by default) dealt over the ranks on a
diagonal lattice (``split_tile``: rank (tx + s*ty) mod N when N divides the tiles
per row, s = 3 at N >= 4; interleaved for load balance, since ERT and empty
space skew per-tile cost), every rank keeps a full replica of the volume and
renders its tiles packed contiguously, and rank 0 gathers the packed buffers
over RCCL (xGMI) and scatters them into the image with one small kernel
(cvr_unpack_tiles_device).  The only collective is that gather.

The numpy functions below are the host mirror of the device packing; the CPU
(gloo) tests use them to check the gather/unpack logic without a GPU.
"""
from __future__ import annotations

import ctypes

import numpy as np
import torch
import torch.distributed as dist

from . import _native as N
from .renderer import make_frame


def tile_grid(width: int, height: int, tile: int):
    return (width + tile - 1) // tile, (height + tile - 1) // tile


def tiles_for_rank(width: int, height: int, tile: int, rank: int, nranks: int) -> int:
    ntx, nty = tile_grid(width, height, tile)
    nt = ntx * nty
    return (nt - rank + nranks - 1) // nranks if nt > rank else 0


def split_shift(nranks: int) -> int:
    return 3 if nranks >= 4 else 1


def split_tile(rank: int, nranks: int, k: int, ntx: int) -> tuple[int, int]:
    """(tx, ty) of rank's k-th tile: virtual row-major tile v = rank + k*nranks, whose
    row ty is rotated by split_shift*ty tiles (mirror of cvr::split_tile, cvr_internal.h;
    tests/models/split_balance.py measures the balance)."""
    v = rank + k * nranks
    ty = v // ntx
    tx = (v - ty * ntx - split_shift(nranks) * ty) % ntx
    return tx, ty


def max_tiles_per_rank(width: int, height: int, tile: int, nranks: int) -> int:
    return tiles_for_rank(width, height, tile, 0, nranks)


def pack_rank(image: np.ndarray, tile: int, rank: int, nranks: int) -> np.ndarray:
    """Host mirror of a rank's packed output: (k, tile, tile, C), zero outside the image."""
    h, w = image.shape[:2]
    ntx, _ = tile_grid(w, h, tile)
    k = tiles_for_rank(w, h, tile, rank, nranks)
    out = np.zeros((k, tile, tile) + image.shape[2:], image.dtype)
    for i in range(k):
        tx, ty = split_tile(rank, nranks, i, ntx)
        blk = image[ty * tile:(ty + 1) * tile, tx * tile:(tx + 1) * tile]
        out[i, :blk.shape[0], :blk.shape[1]] = blk
    return out


def unpack(packed_all: np.ndarray, width: int, height: int, tile: int, nranks: int) -> np.ndarray:
    """Host mirror of cvr_unpack_tiles_device: packed_all is (nranks, tpr_max, tile, tile, C)."""
    ntx, _ = tile_grid(width, height, tile)
    out = np.zeros((height, width) + packed_all.shape[4:], packed_all.dtype)
    for r in range(nranks):
        for i in range(tiles_for_rank(width, height, tile, r, nranks)):
            tx, ty = split_tile(r, nranks, i, ntx)
            blk = out[ty * tile:(ty + 1) * tile, tx * tile:(tx + 1) * tile]
            blk[...] = packed_all[r, i, :blk.shape[0], :blk.shape[1]]
    return out


def gather_to_root(packed: torch.Tensor, tpr_max: int, group=None) -> torch.Tensor | None:
    """Gather every rank's packed tiles (padded to tpr_max) on rank 0.

    Returns a (nranks, tpr_max, ...) tensor on rank 0 and None elsewhere.  Works on
    any backend (RCCL on GPUs, gloo on CPU tensors)."""
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    if packed.shape[0] < tpr_max:
        pad = torch.zeros((tpr_max - packed.shape[0],) + tuple(packed.shape[1:]),
                          dtype=packed.dtype, device=packed.device)
        packed = torch.cat([packed, pad], 0)
    if rank == 0:
        bufs = [torch.empty_like(packed) for _ in range(world)]
        dist.gather(packed, gather_list=bufs, dst=0, group=group)
        return torch.stack(bufs, 0)
    dist.gather(packed, dst=0, group=group)
    return None


def _copy_frame(f):
    g = N.Frame()
    ctypes.pointer(g)[0] = f
    return g


class CommUnavailable(N.CvrError):
    """The library's RCCL communicator could not be created (cvr_comm_init failed):
    the only error a caller may answer by falling back to torch's dist.gather.
    Option and argument errors are CvrError and mean a wrong configuration."""


class ScreenTileSplit:
    """One renderer's frames split over the ranks of a process group.

    Every rank holds a replica of the renderer's device data (volume, TF, gradient,
    extinction pyramid or SAT) and renders its interleaved ``tile`` x ``tile`` screen
    tiles packed contiguously; rank 0 gathers the packed buffers (RCCL over xGMI; gloo
    on CPU) and unpacks them into ``image``.  Pixels travel as ``fmt``: RGBA16F by
    default, the reference's own frame format (imageStore into the RGBA16F image,
    ray_marching_1p.comp:174-176), which halves the gather; RGBA32F keeps the exact
    composite.

    Frames are pipelined.  ``submit`` launches frame n's tiles and its gather
    (asynchronous); buffer sets rotate (see ``streams``).  ``flush`` completes everything
    submitted (the current stream waits for it); afterwards ``image`` holds frame
    ``completed`` for work queued on the current stream.  ``render`` = submit + flush.
    (With the torch transport, frame n-1 is already complete after submit(n).)

    ``streams`` = D (default 4 on GPUs): frame n renders on stream n % D with buffer
    set n % D, so D consecutive frames also overlap on the device (a frame's longest
    tiles no longer idle the GPU at its end).  At world 1 the frames rotate D images.
    Streams sharing a hardware queue serialise: give the process enough queues
    (GPU_MAX_HW_QUEUES, bench.py sets 8).

    ``frames_per_launch`` = L > 1 (rc1pass with the library render only): L
    consecutive frames render in ONE launch (cvr_render_rc1pass_frames), issued when
    the L-th is submitted (or at flush); at world > 1 the launch is the exchange group
    (frames_per_exchange = L).  At world 1 the groups rotate over the D streams with
    L images each.

    Transport ``"rccl"`` (default on GPUs at world > 1): the library's own
    communicator (cvr_comm_init, id broadcast over the process group) and
    cvr_gather_tiles, two C calls per frame; rank 0 renders straight into its block
    of the gather buffer.  ``code`` (default): RGBA16F exchanges move the lossless
    per-tile code instead of raw tiles (library option exchange_code),
    and every frame of an exchange group gets its own image on rank 0.  ``"torch"``: ``dist.gather`` of the process group (any
    backend; the gloo tests), one stream, with ``render_fn(frame, out_tensor,
    total_tensor_or_None)`` and ``unpack_fn(frame, gathered, image)`` defaulting to
    the library (renderer.render_to, cvr_unpack_tiles_device); the CPU tests pass
    host mirrors."""

    def __init__(self, renderer=None, width: int = None, height: int = None, tile: int = 16,
                 fmt: int = N.FORMAT_RGBA16F, group=None, device=None, render_fn=None,
                 unpack_fn=None, count_samples: bool = False, transport: str = None,
                 streams: int = None, frames_per_exchange: int = 1, stream_factory=None,
                 frames_per_launch: int = 1, buffer_sets: int = 0, root_renders: bool = True,
                 code: bool = True):
        self.r = renderer
        self.code = bool(code)      # native transport: RGBA16F exchanges move the per-tile code
        self.width = width if width is not None else renderer.width
        self.height = height if height is not None else renderer.height
        self.tile = tile
        self.fmt = fmt
        self.group = group
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        self.rank = dist.get_rank(group) if dist.is_initialized() else 0
        if device is None:
            device = torch.device("cuda", renderer._device_index)
        self.device = torch.device(device)
        self.render_fn = render_fn or self._render_lib
        self.unpack_fn = unpack_fn or self._unpack_lib
        dtype = torch.float16 if fmt == N.FORMAT_RGBA16F else torch.float32
        w, h = self.width, self.height
        self.split = self.world > 1
        custom = render_fn is not None or unpack_fn is not None
        if transport is None:
            transport = "rccl" if self.device.type == "cuda" and not custom else "torch"
        self.transport = transport if self.split else "none"
        if streams is None:
            streams = 4 if self.device.type == "cuda" and self.transport != "torch" else 1
        if self.transport == "torch":
            streams = 1
        self.nstreams = streams
        # stream_factory: tests drive the native path's control flow with stand-in
        # streams on CPU
        mk = stream_factory or (lambda: torch.cuda.Stream(self.device))
        self.streams = [mk() for _ in range(streams)] if streams > 1 else None
        # root_renders=False (native transport, world >= 3): rank 0 only gathers and
        # unpacks; ranks 1..N-1 render the split over N-1 render ranks (library
        # option gather_root_idle)
        self.idle_root = not root_renders and self.split and self.world >= 3
        if self.idle_root and (self.transport != "rccl" or render_fn is not None or
                               self.streams is None):
            raise ValueError("root_renders=False needs the native transport, the library "
                             "render and >= 2 streams")
        self.sworld = self.world - 1 if self.idle_root else self.world     # the render split
        self.srank = max(self.rank - 1, 0) if self.idle_root else self.rank
        self.renders = not (self.idle_root and self.rank == 0)
        self.k = (tiles_for_rank(w, h, tile, self.srank, self.sworld)
                  if self.split and self.renders else 0)
        self.tpr_max = max_tiles_per_rank(w, h, tile, self.sworld) if self.split else 0
        # frames per launch: rc1pass through the library's own render call only
        self.L = max(1, int(frames_per_launch))
        if (self.L > 1 and (render_fn is not None or renderer is None or
                            getattr(renderer, "_ENTRY", "") != "cvr_render_rc1pass")):
            self.L = 1
        if self.split and self.L > 1:
            frames_per_exchange = self.L
        # buffer sets: frame n uses set n % nbuf (one per stream; two for one stream).
        # With the native transport, G = frames_per_exchange consecutive frames share
        # one set (one slot each), render on its stream and travel in ONE gather.
        self.nbuf = max(2, streams)
        if buffer_sets > self.nbuf:
            # more buffer sets than streams (a multiple of them): a render stream then
            # waits for the exchange that used its next set rounds earlier, not for
            # its own last one (library option gather_sets)
            self.nbuf = -(-int(buffer_sets) // streams) * streams
            # the library holds the end events of the last MAX_GATHER_SETS exchanges
            # (cvr.h CVR_MAX_GATHER_SETS): the most whole multiples of the streams
            if self.nbuf > N.MAX_GATHER_SETS:
                self.nbuf = max(streams, N.MAX_GATHER_SETS // streams * streams)
        self.G = max(1, int(frames_per_exchange)) if (self.transport == "rccl" and
                                                       self.streams is not None) else 1
        if self.split and self.G == 1:
            self.L = 1
        # rank 0's images: world 1 rotates D x L; a native split gives every frame of an
        # exchange group its own image (the coded exchange decodes the group's frames in
        # one launch, so they cannot share one), the torch transport one
        nimg = (streams * self.L if not self.split else
                (self.G if self.transport == "rccl" and self.streams is not None else 1))
        self._images = ([torch.zeros((h, w, 4), dtype=dtype, device=self.device)
                         for _ in range(nimg)] if self.rank == 0 else None)
        self._batch = []            # frames of the open launch (L > 1)
        if self.split:
            # padded to tpr_max tiles (gather needs equal sizes); padding stays zero
            self.packed = [torch.zeros((self.G, self.tpr_max, tile, tile, 4), dtype=dtype,
                                       device=self.device) for _ in range(self.nbuf)]
            self.gathered = ([torch.zeros((self.world, self.G, self.tpr_max, tile, tile, 4),
                                          dtype=dtype, device=self.device)
                              for _ in range(self.nbuf)]
                             if self.rank == 0 else None)
        self.total = (torch.zeros((1,), dtype=torch.int64, device=self.device)
                      if count_samples else None)
        self.submitted = 0
        self.completed = -1
        self._pending = []          # [(frame_no, slot, work, frame)]
        self._fkey = None
        self._fresh = True          # next submit makes the render streams wait for the caller
        self._comm = False
        if self.transport == "rccl":
            self._init_comm()
        # fast path (library render + RCCL gather): per-slot C arguments built once,
        # so a frame costs a few ctypes calls on the host
        self._fast = None
        if self.transport == "rccl" and render_fn is None and self.streams is not None:
            L = N.lib()
            h = self.r.device.handle
            slots = []
            for i in range(self.nbuf):
                g = self.gathered[i] if self.rank == 0 else None
                blk = g[0] if self.rank == 0 else self.packed[i]     # (G, tpr, T, T, 4)
                outs = [N.Output(blk[j].data_ptr(), None,
                                 self.total.data_ptr() if self.total is not None and
                                 (self.L == 1 or j == 0) else None, 1,
                                 fmt) for j in range(self.G)]
                slots.append((self.streams[i % self.nstreams].cuda_stream, outs, blk.data_ptr(),
                              g.data_ptr() if g is not None else None))
            imgs = (ctypes.c_void_p * self.G)(*([self._images[j].data_ptr() for j in range(self.G)]
                                                 if self.rank == 0 else [None] * self.G))
            self._fast = (L, h, getattr(L, self.r._ENTRY), ctypes.byref(self.r._params), imgs,
                          slots)
            self._group = 0      # frames rendered into the open exchange group
        self._xg = 0             # exchange groups issued (the library's exchange count)
        self._last_j = 0         # rank 0: image of the last exchanged frame

    def _image_index(self, n):
        """World 1: the image of frame n (launch group g = n // L on stream g % D)."""
        if self.L == 1:
            return n % len(self._images)
        return ((n // self.L) % self.nstreams) * self.L + n % self.L

    @property
    def image(self):
        """Rank 0: the frame ``completed`` (None on other ranks)."""
        if self._images is None:
            return None
        if self.split:
            return self._images[self._last_j if self._fast is not None else 0]
        return self._images[self._image_index(max(self.completed, 0))]

    def _init_comm(self):
        L = N.lib()
        buf = ctypes.create_string_buffer(N.COMM_ID_BYTES)
        if self.rank == 0:
            N.check(L.cvr_comm_unique_id(buf), "cvr_comm_unique_id")
        on_dev = dist.get_backend(self.group) == "nccl"
        t = torch.tensor(list(buf.raw), dtype=torch.uint8,
                         device=self.device if on_dev else "cpu")
        dist.broadcast(t, src=0, group=self.group)
        uid = bytes(t.cpu().tolist())
        h = self.r.device.handle
        try:
            N.check(L.cvr_comm_init(h, self.world, self.rank, uid), "cvr_comm_init", h)
        except N.CvrError as e:
            raise CommUnavailable(e.status, "cvr_comm_init", str(e)) from e
        self._comm = True
        N.check(L.cvr_set_option(h, b"split_streams", self.nstreams), "split_streams", h)
        N.check(L.cvr_set_option(h, b"gather_sets", self.nbuf), "gather_sets", h)
        N.check(L.cvr_set_option(h, b"gather_root_idle", int(self.idle_root)), "gather_root_idle", h)
        N.check(L.cvr_set_option(h, b"exchange_code", int(self.code)), "exchange_code", h)

    def close(self):
        if self._comm:
            self.flush()
            N.check(N.lib().cvr_comm_destroy(self.r.device.handle), "cvr_comm_destroy",
                    self.r.device.handle)
            self._comm = False

    # -- library defaults ---------------------------------------------------
    def _render_lib(self, frame, out_tensor, total):
        out = N.Output(out_tensor.data_ptr(), None,
                       total.data_ptr() if total is not None else None, 1, self.fmt)
        self.r.render_to(frame, out)

    def _unpack_lib(self, frame, gathered, image):  # torch transport
        N.check(N.lib().cvr_unpack_tiles_device(self.r.device.handle, ctypes.byref(frame),
                                                gathered.data_ptr(), self.tpr_max, self.fmt,
                                                image.data_ptr()),
                "cvr_unpack_tiles_device", self.r.device.handle)

    # -- frames ---------------------------------------------------------------
    def _stream_for(self, n):
        """The render stream of frame n, made current on the renderer's context."""
        cur = torch.cuda.current_stream(self.device) if self.device.type == "cuda" else None
        if self.streams is None:
            s = cur
        else:
            if self._fresh:
                for st in self.streams:     # see everything the caller queued before
                    st.wait_stream(cur)
                self._fresh = False
            s = self.streams[n % self.nstreams]
        if s is not None and self.r is not None:
            self.r.device.set_stream(s.cuda_stream)
        return s

    def submit(self, camera):
        """Render this rank's tiles of one frame and start their gather."""
        n = self.submitted
        frame = self._frame_for(camera)
        if self.L > 1:
            # the launch group's frames are rendered together when the last arrives
            self._batch.append(_copy_frame(frame))
            self.submitted += 1
            if len(self._batch) == self.L:
                self._launch_batch()
            return
        self._stream_for(n)
        if not self.split:
            self.render_fn(frame, self._images[n % len(self._images)], self.total)
            self.submitted += 1
            self.completed = n if self.streams is None else n - 1
            return
        slot = n % self.nbuf
        if self._fast is not None:
            L, h, entry, params, imgs, slots = self._fast
            if self._fresh:
                self._stream_for(n)
            G = self.G
            # the open exchange group: its buffer set (and stream) follow the library's
            # own exchange count, its frames fill slots 0, 1, ... (a flush may close a
            # group early, so frame numbers need not align with groups)
            sptr, outs, buf, g = slots[self._xg % self.nbuf]
            j = self._group
            L.cvr_set_stream(h, sptr)
            if self.renders:
                st = entry(h, ctypes.byref(frame), params, ctypes.byref(outs[j]))
                if st:
                    N.check(st, self.r._ENTRY, h)
            self._group = j + 1
            if self._group == G:
                self._exchange(G, n)
            self.submitted += 1
            self.completed = n - 1
            return
        if self.transport == "rccl":
            # the library orders this render after the gather of frame n-2 (same slot)
            h = self.r.device.handle
            g = self.gathered[slot] if self.rank == 0 else None
            buf = g[0, 0] if self.rank == 0 else self.packed[slot][0]
            self.render_fn(frame, buf, self.total)
            N.check(N.lib().cvr_gather_tiles(h, ctypes.byref(frame), buf.data_ptr(), self.tpr_max,
                                             self.fmt, g.data_ptr() if g is not None else None,
                                             self._images[0].data_ptr() if self.rank == 0
                                             else None),
                    "cvr_gather_tiles", h)
            self.submitted += 1
            self.completed = n - 1
            return
        # the slot's previous frame (n-2) was completed before frame n-1 was submitted
        # returned, so its gather no longer reads packed[slot]
        self.render_fn(frame, self.packed[slot][0], self.total)
        gl = [g[0] for g in self.gathered[slot].unbind(0)] if self.rank == 0 else None
        work = dist.gather(self.packed[slot][0], gather_list=gl, dst=0, group=self.group,
                           async_op=True)
        self._pending.append((n, slot, work, frame))
        self.submitted += 1
        while len(self._pending) > 1:
            self._complete_oldest()

    def _launch_batch(self):
        """Render the open launch group (frames submitted - len(batch) .. submitted - 1)
        in one cvr_render_rc1pass_frames call on the group's stream; at world > 1
        start its gather."""
        frames, self._batch = self._batch, []
        nb = len(frames)
        n0 = self.submitted - nb
        g = self._xg if self.split else n0 // self.L
        self._stream_for(g)
        if not self.split:
            outs = [N.Output(self._images[self._image_index(n0 + j)].data_ptr(), None,
                             self.total.data_ptr() if (self.total is not None and j == 0) else None,
                             1, self.fmt) for j in range(nb)]
            self.r.render_frames_to(frames, outs)
            self.completed = n0 + nb - 1 if self.streams is None else n0 - 1
            return
        L, h, entry, params, imgs, slots = self._fast
        sptr, outs, buf, gb = slots[g % self.nbuf]
        L.cvr_set_stream(h, sptr)
        if self.renders:
            fa = (N.Frame * nb)(*frames)
            oa = (N.Output * nb)(*outs[:nb])
            st = L.cvr_render_rc1pass_frames(h, fa, nb, params, oa)
            if st:
                N.check(st, "cvr_render_rc1pass_frames", h)
        self._frame = frames[-1]
        self._exchange(nb, n0 + nb - 1)
        self.completed = n0 - 1

    def _exchange(self, nframes, n_last):
        """Gather the open group's `nframes` frames, the last of which is frame
        `n_last`, in one ncclGather on the group's stream."""
        L, h, entry, params, imgs, slots = self._fast
        sptr, outs, buf, g = slots[self._xg % self.nbuf]
        L.cvr_set_stream(h, sptr)
        st = L.cvr_gather_tiles_n(h, ctypes.byref(self._frame), nframes, buf, self.tpr_max,
                                  self.fmt, g, imgs if self.rank == 0 else None)
        if st:
            N.check(st, "cvr_gather_tiles_n", h)
        self._group = 0
        self._xg += 1
        self._last_j = nframes - 1       # the image of the group's last frame

    def _frame_for(self, camera):
        """This rank's cvr_frame for `camera` (cached while the camera is unchanged)."""
        key = (tuple(camera.eye), tuple(camera.center), tuple(camera.up), camera.fovy_deg,
               camera.aspect)
        if key != self._fkey:
            self._frame = (make_frame(camera, self.width, self.height, self.tile, self.srank,
                                      self.sworld) if self.split else
                           make_frame(camera, self.width, self.height))
            self._fkey = key
        return self._frame

    def _complete_oldest(self):
        n, slot, work, frame = self._pending.pop(0)
        work.wait()       # the current stream waits for the gather (RCCL) / host waits (gloo)
        if self.rank == 0:
            self.unpack_fn(frame, self.gathered[slot][:, 0], self._images[0])
        self.completed = n

    def flush(self):
        """Complete every submitted frame: work queued on the current stream afterwards
        sees the last frame in `image`."""
        if self._batch:
            self._launch_batch()                              # a partly filled launch group
        if self._fast is not None and self._group:
            self._exchange(self._group, self.submitted - 1)   # a partly filled group
        if self.device.type == "cuda":
            cur = torch.cuda.current_stream(self.device)
            if self.streams is not None:
                for st in self.streams:
                    cur.wait_stream(st)
            if self.r is not None:
                self.r.device.set_stream(cur.cuda_stream)
            if self.transport == "rccl" and self.submitted:
                N.check(N.lib().cvr_gather_sync(self.r.device.handle), "cvr_gather_sync",
                        self.r.device.handle)
        self._fresh = True
        while self._pending:
            self._complete_oldest()
        self.completed = self.submitted - 1
        return self.image

    def render(self, camera):
        self.submit(camera)
        return self.flush()


class TiledRc1pass(ScreenTileSplit):
    """ScreenTileSplit of a RayCasting1Pass with RGBA32F pixels (the exact composite)
    and a per-frame sample total; ``render(camera)`` returns the image on rank 0 and
    this rank's packed tiles elsewhere."""

    def __init__(self, renderer, tile: int = 16):
        super().__init__(renderer, tile=tile, fmt=N.FORMAT_RGBA32F, count_samples=True,
                         streams=1)

    def render(self, camera, stream=None, gather: bool = True):
        s = stream if stream is not None else torch.cuda.current_stream(self.r._device_index)
        self.r.Update(camera)
        self.r.device.set_stream(s.cuda_stream)
        with torch.cuda.stream(s):
            self.total.zero_()
            if not gather and self.split:
                frame = make_frame(camera, self.width, self.height, self.tile, self.rank,
                                   self.world)
                self.render_fn(frame, self.packed[0][0], self.total)
                return self.packed[0][0][:self.k]
            img = super().render(camera)
        return img if self.rank == 0 else self.packed[(self.submitted - 1) % self.nbuf][0][:self.k]
