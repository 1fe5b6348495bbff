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


@pytest.mark.parametrize("world,W,H,tile", [(2, 96, 80, 32), (3, 70, 45, 16), (2, 16, 16, 32)])
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
