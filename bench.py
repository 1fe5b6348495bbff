#!/usr/bin/env python3
"""Headline benchmark: rc1pass ray-march, Msamples/s at 1024^2 on a 512^3 volume.

Workload (BASELINE.json metric, SURVEY.md §8d "512^3 EA"): Marschner-Lobb field
(alpha 0.25, f_M 6) quantised to u8, 512^3, voxel scale 1 (world box +-256),
data/tf1dcp/bonsai_01.tf1d, camera "Initial State", 1024x1024, default step
0.5/sqrt(3)*|scale| = 0.5, emission-absorption (no Phong).  Synthetic data,
generated here; the volume is resident in HBM before timing starts.

A step = one full frame: every ray of the 1024^2 image marched to its exit or
ERT break.  Samples (the work unit S) = the reference's loop iterations
(ray_marching_1p.comp:124-172, transparent samples included), counted by the
kernel itself.  value = (S summed over ranks) * steps / (max-over-ranks time).

N > 1 (torchrun, one process per GPU): screen-tile split — every rank owns a
replica of the volume, renders its interleaved 32x32 tiles, rank 0 gathers the
packed tiles over RCCL and unpacks them (that gather is inside the timed region).
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from cpp_volume_rendering_amd import _native as N  # noqa: E402
from cpp_volume_rendering_amd import datasets as D  # noqa: E402
from cpp_volume_rendering_amd import screen_tiles as T  # noqa: E402
from cpp_volume_rendering_amd.renderer import (Camera, DataManager, RayCasting1Pass,  # noqa: E402
                                               RenderingParameters, build_tf_rgbt, make_frame)

HBM_PEAK_GBS = 8000.0    # MI355X HBM3E, /opt/skills/guides/MI355X_MICROARCH.md (spec)


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=50)
    p.add_argument("--warmup", type=int, default=5)
    p.add_argument("--size", type=int, default=512)
    p.add_argument("--res", type=int, default=1024)
    p.add_argument("--tile", type=int, default=32)
    p.add_argument("--field", choices=["ml", "blobs"], default="ml")
    p.add_argument("--phong", action="store_true")
    p.add_argument("--cpu-seconds", type=float, default=12.0)
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--pmc", default=os.path.join(ROOT, "profiles", "pmc_rc1pass.json"))
    return p.parse_args()


def cpu_baseline(vol, scale, tf, cam, W, H, seconds):
    """The CPU oracle (C++/OpenMP restatement of ray_marching_1p.comp; the reference has
    no CPU ray-caster) on the host cores: whole frames of the same workload, repeated
    until `seconds` of wall time are spent (each frame starts from the centre band of
    rows and grows outward, so a partial last frame is still a representative sample),
    plus a 1-thread figure on a shorter sample."""
    import oracle as O
    threads = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or (os.cpu_count() or 1)
    v16 = O.volume_r16f(vol)
    step = O.default_step(scale)
    rows_per_chunk = 16
    y = H // 2 - rows_per_chunk // 2
    order = []
    for k in range(H // rows_per_chunk + 2):
        off = ((k + 1) // 2) * (1 if k % 2 else -1) * rows_per_chunk
        yy = y + off
        if 0 <= yy and yy + rows_per_chunk <= H and yy not in order:
            order.append(yy)

    def run(nthreads, budget):
        S = rows = 0
        t0 = time.perf_counter()
        while True:
            for yy in order:
                _, _, s = O.render_rc1pass(v16, scale, tf, cam, W, H, step,
                                           rows=(yy, yy + rows_per_chunk), threads=nthreads)
                S += s
                rows += rows_per_chunk
                if time.perf_counter() - t0 >= budget:
                    return S, rows, time.perf_counter() - t0

    S, rows, dt = run(threads, seconds)
    S1, rows1, dt1 = run(1, max(2.0, seconds / 4))
    return {"value": round(S / dt / 1e6, 3), "unit": "Msamples/s", "cores": threads,
            "kind": "port",
            "sample": f"{rows} image rows ({rows / H:.1f} frames, centre band outward) of the "
                      f"same {W}x{H} frame, {S} samples in {dt:.1f} s on {threads} threads; "
                      f"C++/OpenMP oracle (no CPU ray-caster exists in the reference)",
            "single_thread_value": round(S1 / dt1 / 1e6, 3),
            "single_thread_sample": f"{rows1} rows, {S1} samples in {dt1:.1f} s"}


def load_traffic(path, workload_key):
    try:
        with open(path) as f:
            d = json.load(f)
        if d.get("workload_key") != workload_key:
            return None
        return d.get("hbm_bytes_per_launch")
    except (OSError, ValueError):
        return None


def main():
    a = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    else:
        torch.cuda.set_device(0)

    n, W = a.size, a.res
    H = W
    vol = D.marschner_lobb_u8(n) if a.field == "ml" else D.blobs_u8(n)
    scale = D.voxel_scale(n)
    tf = build_tf_rgbt(D.BONSAI_TF_RGB, D.BONSAI_TF_ALPHA)
    cam = Camera(**D.INITIAL_STATE_CAMERA)

    dm = DataManager()
    dm.SetVolume(vol, scale)
    dm.SetTransferFunction(tf)
    if a.phong:
        dm.SetGradientType(N.GRADIENT_FINITE_DIFFERENCES)
    rp = RenderingParameters(W, H, light_position=D.LIGHT_LIST0_POSITION)
    r = RayCasting1Pass(local if world > 1 else 0)
    r.m_apply_gradient_shading = a.phong
    r.SetExternalResources(dm, rp)
    assert r.Init(W, H)
    r.PrepareRender(cam)

    dev = torch.device("cuda", local if world > 1 else 0)
    stream = torch.cuda.current_stream(dev)
    r.device.set_stream(stream.cuda_stream)
    tile = a.tile
    if world > 1:
        frame = make_frame(cam, W, H, tile, rank, world)
        k = T.tiles_for_rank(W, H, tile, rank, world)
        tpr = T.max_tiles_per_rank(W, H, tile, world)
        out_buf = torch.zeros((tpr, tile, tile, 4), dtype=torch.float32, device=dev)
        image = torch.zeros((H, W, 4), dtype=torch.float32, device=dev) if rank == 0 else None
        pixels = k * tile * tile
    else:
        frame = make_frame(cam, W, H)
        out_buf = r.rgba
        pixels = W * H
    total = torch.zeros((1,), dtype=torch.int64, device=dev)
    L = N.lib()
    fptr, pptr = ctypes.byref(frame), ctypes.byref(r._params)
    out = N.Output(out_buf.data_ptr(), None, total.data_ptr(), 1)

    def step_once():
        N.check(L.cvr_render_rc1pass(r.device.handle, fptr, pptr, ctypes.byref(out)),
                "cvr_render_rc1pass", r.device.handle)

    def gather_once():
        if world > 1:
            allp = T.gather_to_root(out_buf, tpr)
            if rank == 0:
                N.check(L.cvr_unpack_tiles_device(r.device.handle, fptr, allp.data_ptr(), tpr,
                                                  image.data_ptr()), "unpack", r.device.handle)

    # samples per frame (this rank), counted by the kernel
    step_once()
    torch.cuda.synchronize(dev)
    S_rank = int(total.item())

    for _ in range(a.warmup):
        step_once()
        gather_once()
    torch.cuda.synchronize(dev)

    # The timed region renders without the sample counter (S is the kernel's own
    # count from the frame above, checked again after timing) and without the
    # library's timing events (an event record between kernels costs ~5 us).
    out_nt = N.Output(out_buf.data_ptr(), None, None, 1)
    fptr_nt = ctypes.byref(out_nt)

    def step_timed():
        N.check(L.cvr_render_rc1pass(r.device.handle, fptr, pptr, fptr_nt),
                "cvr_render_rc1pass", r.device.handle)

    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for i in range(a.steps):
        step_timed()
        gather_once()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    t1 = time.perf_counter()
    elapsed = t1 - t0

    # Kernel-only time for the roofline: HIP events the library records on its
    # own stream around the ray-march launch (kernel_timing), in a separate pass.
    N.check(L.cvr_set_option(r.device.handle, b"kernel_timing", a.steps), "kernel_timing",
            r.device.handle)
    total.zero_()
    for i in range(a.steps):
        step_once()
    torch.cuda.synchronize(dev)
    kt = (ctypes.c_float * a.steps)()
    nkt = ctypes.c_int()
    N.check(L.cvr_read_kernel_times(r.device.handle, kt, a.steps, ctypes.byref(nkt)),
            "cvr_read_kernel_times", r.device.handle)
    assert nkt.value == a.steps
    kern_ms = float(np.mean(kt[:nkt.value]))
    assert int(total.item()) == S_rank * a.steps, "sample count changed between frames"
    batch = L.cvr_get_option(r.device.handle, b"batch")
    macro = L.cvr_get_option(r.device.handle, b"macro")

    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        s = torch.tensor([S_rank], dtype=torch.int64, device=dev)
        dist.all_reduce(s, op=dist.ReduceOp.SUM)
        S_all = int(s.item())
    else:
        S_all = S_rank

    if rank == 0:
        msps = S_all * a.steps / elapsed / 1e6
        ms_per_step = elapsed / a.steps * 1e3
        # algorithmic bytes per launch: 8 trilinear corners x 1 B (u8 input)
        # per sample + float4 output per pixel (+ 48 B per sample for the Phong gradient,
        # counted on every sample as an upper bound of the shaded ones)
        b_alg = 8 * 1 * S_rank + 16 * pixels + (48 * S_rank if a.phong else 0)
        achieved = b_alg / (kern_ms * 1e-3) / 1e9
        wkey = f"rc1pass_{a.field}{n}_{W}x{H}{'_phong' if a.phong else ''}"
        roof = {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
                "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                "traffic": load_traffic(a.pmc, wkey),
                "kernel": f"rc1pass_tile_kernel<{batch}, {str(a.phong).lower()}, *, false, true>",
                "kernel_ms": round(kern_ms, 4),
                "bytes_alg_per_launch": b_alg, "samples_per_launch": S_rank}
        res = {
            "metric": "Msamples/s (rays x steps), rc1pass ray-march, 512^3 volume at 1024^2",
            "value": round(msps, 2),
            "unit": "Msamples/s",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": round(ms_per_step, 4),
            "fps": round(1000.0 / ms_per_step, 1),
            "higher_is_better": True,
            "scaling": "strong",   # one fixed frame split over the GPUs
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic",
            "config": {"workload": f"rc1pass emission-absorption, Marschner-Lobb {n}^3 u8 "
                                   f"({a.field}), {W}x{H}, bonsai_01.tf1d, camera "
                                   f"'Initial State', step 0.5, ERT 0.99"
                                   + (", Blinn-Phong FD gradient" if a.phong else ""),
                       "volume": n, "viewport": [W, H], "samples_per_frame": S_all,
                       "parallelism": f"screen tiles {tile}x{tile} over {world} GPU(s)"
                                      if world > 1 else "1 GPU",
                       "storage": "cell8 fp16 (16 B/cell, x-fastest)",
                       "empty_space_skip": f"macro cells 2^{macro}, auto (on at >= 15 % empty)"
                                           if macro > 0 else "off"},
            "roofline": roof,
        }
        if world == 1 and not a.no_cpu_baseline:
            res["cpu_baseline"] = cpu_baseline(vol, scale, tf, D.INITIAL_STATE_CAMERA, W, H,
                                               a.cpu_seconds)
        print(json.dumps(res))
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    r.Clean()


if __name__ == "__main__":
    main()
