"""Screen-tile split of one frame over the GPUs of a node.

The reference renders on one GPU; pixels are independent, so the framebuffer
is cut into ``tile`` x ``tile`` tiles, tile t (row-major over the tile grid)
belongs to rank ``t % nranks`` (interleaved for load balance: ERT and empty
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


def max_tiles_per_rank(width: int, height: int, tile: int, nranks: int) -> int:
    return tiles_for_rank(width, height, tile, 0, nranks)


def pack_rank(image: np.ndarray, tile: int, rank: int, nranks: int) -> np.ndarray:
    """Host mirror of a rank's packed output: (k, tile, tile, C), zero outside the image."""
    h, w = image.shape[:2]
    ntx, _ = tile_grid(w, h, tile)
    k = tiles_for_rank(w, h, tile, rank, nranks)
    out = np.zeros((k, tile, tile) + image.shape[2:], image.dtype)
    for i in range(k):
        t = rank + i * nranks
        tx, ty = t % ntx, t // ntx
        blk = image[ty * tile:(ty + 1) * tile, tx * tile:(tx + 1) * tile]
        out[i, :blk.shape[0], :blk.shape[1]] = blk
    return out


def unpack(packed_all: np.ndarray, width: int, height: int, tile: int, nranks: int) -> np.ndarray:
    """Host mirror of cvr_unpack_tiles_device: packed_all is (nranks, tpr_max, tile, tile, C)."""
    ntx, _ = tile_grid(width, height, tile)
    out = np.zeros((height, width) + packed_all.shape[4:], packed_all.dtype)
    for r in range(nranks):
        for i in range(tiles_for_rank(width, height, tile, r, nranks)):
            t = r + i * nranks
            tx, ty = t % ntx, t // ntx
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


class TiledRc1pass:
    """Renders one frame of a RayCasting1Pass split over the ranks of a process group.

    Each rank owns a replica of the renderer's device data; ``render`` launches this
    rank's tiles, gathers to rank 0 over the default group and unpacks there."""

    def __init__(self, renderer, tile: int = 32):
        self.r = renderer
        self.tile = tile
        self.world = dist.get_world_size() if dist.is_initialized() else 1
        self.rank = dist.get_rank() if dist.is_initialized() else 0
        w, h = renderer.width, renderer.height
        self.k = tiles_for_rank(w, h, tile, self.rank, self.world)
        self.tpr_max = max_tiles_per_rank(w, h, tile, self.world)
        dev = torch.device("cuda", renderer._device_index)
        self.packed = torch.zeros((self.tpr_max, tile, tile, 4), dtype=torch.float32, device=dev)
        self.total = torch.zeros((1,), dtype=torch.int64, device=dev)
        self.image = (torch.zeros((h, w, 4), dtype=torch.float32, device=dev)
                      if self.rank == 0 else None)

    def render(self, camera, stream=None, gather: bool = True):
        r = self.r
        s = stream if stream is not None else torch.cuda.current_stream(r._device_index)
        frame = make_frame(camera, r.width, r.height, self.tile, self.rank, self.world)
        r.Update(camera)
        r.device.set_stream(s.cuda_stream)
        out = N.Output(self.packed.data_ptr(), None, self.total.data_ptr(), 1)
        N.check(N.lib().cvr_render_rc1pass(r.device.handle, ctypes.byref(frame),
                                           ctypes.byref(r._params), ctypes.byref(out)),
                "cvr_render_rc1pass", r.device.handle)
        if not gather or self.world == 1:
            return self.packed
        allp = gather_to_root(self.packed, self.tpr_max)
        if self.rank == 0:
            N.check(N.lib().cvr_unpack_tiles_device(r.device.handle, ctypes.byref(frame),
                                                    allp.data_ptr(), self.tpr_max,
                                                    self.image.data_ptr()),
                    "cvr_unpack_tiles_device", r.device.handle)
            self._keep = allp      # keep the gather buffer alive until the stream passes it
        return self.image
