#!/usr/bin/env python3
"""Headline benchmark: rc1pass ray-march, Msamples/s at 1024^2 on a 512^3 volume.

(--renderer dos: BASELINE.json config 4 instead, the directional-occlusion renderer
with cone AO + cone shadows at 2048^2; --renderer ebs: config 5, the extinction-SAT
precompute + extinction-based shading on 1024^3.  Secondary lines, not the headline.)

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


def _launch_ranks_if_needed():
    """`bench.py --gpus N` with N > 1 outside a launcher: start N rank processes with
    torch.distributed.run (127.0.0.1 rendezvous) as a CHILD process, before this process
    touches HIP, and exit with its status; rank 0's JSON line reaches stdout directly.
    Under a launcher (WORLD_SIZE set) --gpus must equal WORLD_SIZE."""
    pre = argparse.ArgumentParser(add_help=False)
    pre.add_argument("--gpus", type=int, default=1)
    known, _ = pre.parse_known_args()
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is not None:
        if int(env_world) != known.gpus:
            sys.exit(f"bench.py: --gpus {known.gpus} but WORLD_SIZE={env_world}")
        return
    if known.gpus <= 1:
        return
    import socket
    import subprocess
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={known.gpus}", "--master-addr", "127.0.0.1",
           "--master-port", str(port), os.path.abspath(__file__), *sys.argv[1:]]
    sys.exit(subprocess.call(cmd))


if __name__ == "__main__":
    _launch_ranks_if_needed()

# Frames in flight run on separate HIP streams; HIP maps streams onto at most
# GPU_MAX_HW_QUEUES hardware queues per process (4 by default), and streams that
# share a queue serialise.  8 queues keep 4 render streams + RCCL's apart.  Set
# unconditionally (not setdefault), before torch initialises HIP, so the bench runs
# the configuration DESIGN §7 measured whatever the box's environment holds; the
# value is reported in config.hw_queues.
# Default by world size (WORLD_SIZE is set by the launcher before this process
# starts): the frames in flight need a queue each, one per render stream and the
# RCCL stream (32 at 8 ranks: 16 streams; DESIGN §7, profiles/r03_s25_*).
_WS = int(os.environ.get("WORLD_SIZE", "1"))


def _hw_queues_arg() -> int:
    """--hw-queues N / --hw-queues=N, read before torch initialises HIP (argparse
    proper runs later); 0 = the default by world size.  The box refuses more than 32."""
    pre = argparse.ArgumentParser(add_help=False)
    pre.add_argument("--hw-queues", type=int, default=0)
    known, _ = pre.parse_known_args()
    if known.hw_queues and not 1 <= known.hw_queues <= 32:
        sys.exit(f"bench.py: --hw-queues must be in 1..32 (got {known.hw_queues})")
    return known.hw_queues


HW_QUEUES = _hw_queues_arg() or (32 if _WS >= 8 else (24 if _WS >= 4 else 8))
os.environ["GPU_MAX_HW_QUEUES"] = str(HW_QUEUES)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from cpp_volume_rendering_amd import _native as N  # noqa: E402
from cpp_volume_rendering_amd import datasets as D  # noqa: E402
from cpp_volume_rendering_amd import screen_tiles as T  # noqa: E402
from cpp_volume_rendering_amd.renderer import (CustomRayCasting1PassIsoAdapt,  # noqa: E402
                                               CustomRayCasting1PassIsodfsAdapt,
                                               RayCasting1PassIsoAdapt)
from cpp_volume_rendering_amd.renderer import (Camera, DataManager, RayCasting1Pass,  # noqa: E402
                                               RC1PConeTracingDirOcclusionShading,
                                               RC1PExtinctionBasedShading, RenderingParameters,
                                               build_ext_lut, build_tf_rgbt, make_frame,
                                               read_camera_state)

HBM_PEAK_GBS = 8000.0    # MI355X HBM3E, /opt/skills/guides/MI355X_MICROARCH.md (spec)
# aggregate L2 bandwidth of the 8 XCDs (MI355X_MICROARCH.md "L2 (per XCD)": ~34.5 TB/s):
# the bound for EBS, whose 32-B SAT fetches (2.2 TB per 1024^3 frame) are served by
# L1/L2/MALL, not HBM (PMC: ~220 GB of HBM traffic per frame)
L2_PEAK_GBS = 34500.0
# The pipes of one CU at the peak engine clock (MI355X_MICROARCH.md; under load DVFS
# gives some of it back, the PMC record's effective clock says how much):
CLOCK_GHZ = 2.4
N_CU, N_SIMD = 256, 1024
# a wave64 VALU instruction issues over 2 cycles per SIMD (constants table)
VALU_PEAK_GWIPS = N_SIMD * CLOCK_GHZ / 2.0
# the texture-data return path: 64 B/clk per CU, one 1-KiB dwordx4 wave-load per 16 clk
# (tools/ta_probe.hip: 16.5 clk for any wave-load whose lanes share lines in runs, L1-hot)
VMEM_PEAK_GBS = N_CU * 64 * CLOCK_GHZ


def pipe_roofline(kern_ms, fpl, pmc, live_wave_loads):
    """The rc1pass march's roofline on the pipe that binds.  Two pipes
    are priced for one launch of `fpl` frames over its kernel time:
      * vmem: dwordx4 wave-loads x 1 KiB through the L1 -> VGPR return path (64 B/clk/CU);
      * valu: VALU wave-instructions x 2 issue cycles per SIMD.
    Counts come from the PMC record of this library build (per launch of the record's
    frames, scaled to `fpl`); without one, the vmem pipe uses the kernel's own count of
    its march rounds (live_wave_loads).  `bound` is the pipe with the larger fraction."""
    t = kern_ms * 1e-3
    rec_fpl = (pmc.get("frames_per_launch") or 4) if pmc else None
    pipes = {}
    wl, src = None, None
    if pmc.get("sq_insts_vmem_rd"):
        wl, src = pmc["sq_insts_vmem_rd"] * fpl / rec_fpl, "PMC SQ_INSTS_VMEM_RD"
    elif live_wave_loads:
        wl, src = live_wave_loads, "kernel count: K x march rounds + TF staging loads"
    if wl:
        pipes["vmem"] = {"achieved": round(wl * 1024 / t / 1e9, 1), "peak": VMEM_PEAK_GBS,
                         "unit": "GB/s", "wave_loads_per_launch": int(wl), "count": src}
    if pmc.get("valu_wave_insts"):
        v = pmc["valu_wave_insts"] * fpl / rec_fpl
        pipes["valu"] = {"achieved": round(v / t / 1e9, 2), "peak": VALU_PEAK_GWIPS,
                         "unit": "G wave-instr/s", "wave_insts_per_launch": int(v),
                         "count": "PMC SQ_INSTS_VALU"}
    for p in pipes.values():
        p["frac"] = round(p["achieved"] / p["peak"], 4)
    if not pipes:
        return {}
    bound = max(pipes, key=lambda k: pipes[k]["frac"])
    out = {"bound": bound, "achieved": pipes[bound]["achieved"], "peak": pipes[bound]["peak"],
           "unit": pipes[bound]["unit"], "frac": pipes[bound]["frac"], "pipes": pipes}
    if pmc.get("td_busy_frac_per_cu") is not None and pmc.get("td_tc_stall_frac_per_cu") is not None:
        out["vmem_detail"] = {
            "td_busy_per_cu": round(pmc["td_busy_frac_per_cu"], 3),
            "td_stalled_on_cache_per_cu": round(pmc["td_tc_stall_frac_per_cu"], 3),
            "td_work_clk_per_wave_load": round(pmc.get("td_work_cycles_per_wave_load", 0), 2),
            "coalesced_clk_per_wave_load": 16,
            "tcp_accesses_per_wave_load": round(pmc.get("tcp_accesses_per_wave_load", 0), 2),
            "coalesced_tcp_accesses": 16,
            "l1_miss_requests_per_wave_load": round(pmc.get("l1_miss_requests_per_wave_load", 0), 2),
            "what": "TD busy = its own work + cycles stalled waiting for L1 misses (TD_TC_STALL); "
                    "per wave-load the work is the coalesced cost, the stall is miss latency "
                    "(DESIGN §5)"}
    if pmc.get("effective_clock_ghz_under_pmc"):
        out["effective_clock_ghz_under_pmc"] = round(pmc["effective_clock_ghz_under_pmc"], 3)
    return out


def parse(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=0,
                   help="default 200 (iso*: 20, dos: 5, ebs: 2)")
    p.add_argument("--warmup", type=int, default=-1,
                   help="default 20 (iso*: 3, dos/ebs: 1)")
    p.add_argument("--size", type=int, default=0, help="volume N^3 (default 512; ebs 1024)")
    p.add_argument("--res", type=int, default=0, help="viewport (default 1024; dos 2048)")
    p.add_argument("--renderer", choices=["rc1pass", "dos", "ebs", "iso", "isodfs", "isoadapt"],
                   default="rc1pass",
                   help="iso / isodfs / isoadapt: the isosurface ray-casters (variants 0 / 1 / 2)")
    p.add_argument("--tile", type=int, default=16,
                   help="screen-tile side of the N > 1 split (16: diagonal lattice, DESIGN §7)")
    p.add_argument("--field", choices=["ml", "blobs"], default="ml")
    p.add_argument("--phong", action="store_true")
    p.add_argument("--tile-order", type=int, default=-1, choices=[-1, 0, 1, 2],
                   help="rc1pass launch order: 0 XCD bands, 1 learned LPT (default), 2 interleaved")
    p.add_argument("--launch-interleave", type=int, default=-1,
                   help="multi-frame launches: 1 deals the frames' launch-order entries "
                        "interleaved, 0 frame after frame (-1: library default)")
    p.add_argument("--skip-min-pct", type=int, default=-1,
                   help="empty-space skipping when >= this %% of macro cells are empty (101: off; "
                        "-1: the library default)")
    p.add_argument("--cell-skip", type=int, default=-1, choices=[-1, 0, 1, 2, 3, 4],
                   help="rc1pass per-cell skip: 0 off, 1 empty-sample flags, 2 + distance skip "
                        "(-1: the library default, 3: + the distance skip when every lane can)")
    p.add_argument("--batch", type=int, default=0, choices=[0, 2, 4],
                   help="rc1pass samples per lane per memory round trip (0 = auto: 4, 2 with Phong)")
    p.add_argument("--cpu-seconds", type=float, default=12.0)
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--format", choices=["rgba16f", "rgba32f"], default="rgba16f",
                   help="frame format: RGBA16F (the reference's framebuffer) or RGBA32F")
    p.add_argument("--hw-queues", type=int, default=0,
                   help="GPU_MAX_HW_QUEUES for this process, set before HIP initialises "
                        "(default: 8; 24 at 4 GPUs, 32 at >= 8)")
    p.add_argument("--streams", type=int, default=0,
                   help="render streams, rotated per launch (default with multi-frame launches: "
                        "3, 4 at N > 1; one frame per launch: 4, 12 at 4 GPUs, 16 at >= 8)")
    p.add_argument("--exchange-frames", type=int, default=0,
                   help="frames per gather at N > 1 (default: 2 at >= 4 GPUs, else 1; "
                        "the launch group with --frames-per-launch > 1)")
    p.add_argument("--frames-per-launch", type=int, default=0,
                   help="rc1pass: consecutive frames rendered in ONE launch "
                        "(cvr_render_rc1pass_frames, 1..16; default 4, other renderers 1)")
    p.add_argument("--buffer-sets", type=int, default=0,
                   help="N > 1: exchange buffer sets rotated over the render streams (default 4 per "
                        "stream: a render waits for the exchange of its set 4 rounds back)")
    p.add_argument("--root-renders", type=int, default=-1, choices=[-1, 0, 1],
                   help="N > 1: 0 = rank 0 only gathers and unpacks, ranks 1..N-1 render the split "
                        "(-1: 0 for rc1pass at >= 4 GPUs, else 1; DESIGN §7a)")
    p.add_argument("--quad", type=int, default=-1,
                   help="quad (4 lanes per ray) share of the longest tiles, %% (default 0)")
    p.add_argument("--exchange-code", type=int, default=1, choices=[0, 1],
                   help="N > 1, RGBA16F: 1 = the exchange moves the lossless per-tile code "
                        "(one encode launch per group on the render ranks, one fused decode "
                        "on rank 0; DESIGN §7b), 0 = raw tiles (one ncclGather)")
    p.add_argument("--transport", choices=["rccl", "torch"], default="rccl",
                   help="N > 1 gather: the library's RCCL communicator or dist.gather")
    p.add_argument("--shade-flat", type=int, default=-1, choices=[-1, 0, 1],
                   help="dos/ebs: 1 flat job list (library default), 0 per-wave shading batches")
    p.add_argument("--sat-layout", type=int, default=-1, choices=[-1, 0, 1],
                   help="ebs: the SAT the frame reads, 0 the cell4 copy, 1 the plain float SAT "
                        "(-1: the library default)")
    p.add_argument("--flat-group", type=int, default=0,
                   help="dos/ebs flat shading: 64-job chunks per XCD turn (0: library default)")
    p.add_argument("--postpass", action="store_true",
                   help="also time the multiscaling post-pass filters on this workload's frame")
    p.add_argument("--no-cadence", action="store_true",
                   help="rc1pass, 1 GPU: skip the plugin-cadence lines (one frame per call on one "
                        "stream: the static view and the 24-state orbit)")
    p.add_argument("--pmc", default=os.path.join(ROOT, "profiles", "pmc_rc1pass.json"))
    p.add_argument("--orbit", action="store_true",
                   help="move the camera every frame through the reference's camera states "
                        "(tests/golden/list_camera_states = data/#list_camera_states), so the "
                        "LPT/band schedule never replays one view")
    p.add_argument("--tf-alpha", type=float, default=1.0,
                   help="scale of bonsai_01.tf1d's alpha control points (0.02: long rays)")
    p.add_argument("--settle-ms", type=float, default=150.0,
                   help="untimed frames before the warmup until this much wall time has passed "
                        "(GPU clocks ramp over the first ~100 ms of load)")
    p.add_argument("--opt", action="append", default=[], metavar="KEY=VALUE",
                   help="extra cvr_set_option (repeatable; e.g. band_cap=150), recorded in "
                        "config.options")
    p.add_argument("--dry-run", action="store_true",
                   help="launcher rehearsal without a GPU: the ranks join a gloo group and "
                        "rank 0 prints the world size (tests/test_bench_launch.py)")
    return p.parse_args(argv)


def split_defaults(a, world):
    """The screen split bench.py runs for these arguments at this world size (the
    defaults of --frames-per-launch, --streams, --buffer-sets, --exchange-frames,
    --root-renders), as ScreenTileSplit keyword arguments.  Shared with the world-8
    control-flow test (tests/test_distributed_cpu.py), so the test runs exactly the
    N = 8 default path."""
    # Frames per launch (and per exchange) at N > 1, from the length of the run: a
    # share of one frame is a fraction of a GPU residency, so a launch lasts as long
    # as its longest rays and more frames per launch amortise that tail in a long run
    # (7-way share with the encode, steady state: 0.0135 / 0.0121-0.0124 /
    # 0.0118-0.0121 ms per frame at 4 / 8 / 16 frames; N = 2 / 4: -4 / -6 % at 16),
    # while a short run needs several launches in flight on its streams (a 16-frame
    # burst: 0.0147 / 0.0161 / 0.0180 ms at 4 / 8 / 16; tools/exchange_probe.py,
    # profiles/r06/s41, s43, s44).  So: the largest power of two up to 16
    # that leaves two launches per render stream (4 streams): 4 frames for the
    # driver's 20-step runs, 16 from 128 steps on.  One GPU keeps 4.
    steps = a.steps or 200
    fpl_n = 4
    while fpl_n < 16 and steps // (2 * 4) >= 2 * fpl_n:
        fpl_n *= 2
    fpl = (a.frames_per_launch if a.frames_per_launch > 0 else
           ((fpl_n if world >= 2 else 4) if a.renderer == "rc1pass" else 1))
    streams = a.streams or ((4 if world >= 2 else 3) if fpl > 1 else
                            (16 if world >= 8 else (12 if world >= 4 else 4)))
    # fewer, larger exchanges at high N: one gather's host + launch cost (~18 us
    # on rank 0) would otherwise rival a rank's share of the frame (~23 us at N = 8)
    gx = fpl if fpl > 1 else (a.exchange_frames or (2 if world >= 4 else 1))
    # Rank 0's share of the exchange is one fused decode per group of every render
    # rank's coded tiles (tools/exchange_probe.py: ~14-19 us per 4-frame
    # group at N = 4 and 8).  At N = 8 an idle root leaves 7 render ranks whose
    # share (0.0124-0.0135 ms per frame with the encode) beats an 8-way share plus
    # the decode on rank 0 (~0.0128 + ~0.004); at N = 4 three render ranks lose a
    # quarter of the GPUs (0.0289 ms) against 4-way + decode (~0.022 + ~0.0035), so
    # the root renders below 8 ranks and only gathers from 8 on
    root_renders = (a.root_renders == 1 or world < 8 or a.renderer != "rc1pass"
                    or a.transport != "rccl") if a.root_renders != 0 else False
    return {"streams": streams, "frames_per_exchange": gx, "frames_per_launch": fpl,
            "buffer_sets": a.buffer_sets or 4 * streams, "root_renders": root_renders}


def dry_run(world, rank, a):
    """The N-rank control flow without a GPU (gloo): every rank packs its tiles of the
    workload's viewport (a pixel-id image, through screen_tiles' host mirror of the
    device packing), rank 0 gathers and unpacks them, and checks that every pixel
    arrived exactly once (tests/test_bench_launch.py)."""
    n, W = a.size or (1024 if a.renderer == "ebs" else 512), a.res or (2048 if a.renderer == "dos" else 1024)
    ids = np.arange(1, W * W + 1, dtype=np.int32).reshape(W, W, 1)
    tiles = [T.tiles_for_rank(W, W, a.tile, r, world) for r in range(world)]
    exact = True
    if world > 1:
        dist.init_process_group("gloo")
        ranks = [None] * world
        dist.all_gather_object(ranks, rank)
        mine = torch.from_numpy(T.pack_rank(ids, a.tile, rank, world))
        allp = T.gather_to_root(mine, T.max_tiles_per_rank(W, W, a.tile, world))
        if rank == 0:
            exact = bool(np.array_equal(T.unpack(allp.numpy(), W, W, a.tile, world), ids))
        dist.destroy_process_group()
    else:
        ranks = [0]
    if rank == 0:
        print(json.dumps({"dry_run": True, "n_gpus": world, "ranks": ranks,
                          "renderer": a.renderer, "volume": n, "viewport": [W, W],
                          "tile": a.tile, "tiles_per_rank": tiles, "gather_exact": exact,
                          "hw_queues": int(os.environ["GPU_MAX_HW_QUEUES"])}))


def cpu_baseline(vol, scale, tf, cam, W, H, seconds, dos=None, ebs=None, gpu_rgba=None,
                 phong=None, half=False, iso=None):
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
    if dos is not None:
        levels = O.ext_volume(v16, scale, dos["tf_rgba"], dos["res"], threads=threads)
    grad = O.gradient(vol, "fd") if phong is not None else None

    def render_rows_full(y0, y1, nthreads):
        if iso is not None:
            return O.render_iso(v16, vol, scale, cam, W, H, variant=iso["variant"], grad=grad,
                                phong=phong is not None,
                                light=phong["light"] if phong is not None else (0, 0, 0),
                                rows=(y0, y1), threads=nthreads)
        if dos is not None:
            return O.render_dos(v16, scale, tf, levels, cam, W, H, step, dos["occ"], dos["sdw"],
                                apply_shadow=True, light=dos["light"], rows=(y0, y1),
                                threads=nthreads)
        if ebs is not None:
            return O.render_ebs(v16, scale, tf, ebs["sat"], cam, W, H, step,
                                light=ebs["light"], light_forward=ebs["forward"],
                                rows=(y0, y1), threads=nthreads)
        if phong is not None:
            return O.render_rc1pass(v16, scale, tf, cam, W, H, step, grad=grad, phong=True,
                                    light=phong["light"], rows=(y0, y1), threads=nthreads)
        return O.render_rc1pass(v16, scale, tf, cam, W, H, step, rows=(y0, y1),
                                threads=nthreads)

    def render_rows(y0, y1, nthreads):
        return render_rows_full(y0, y1, nthreads)[2]
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
                S += render_rows(yy, yy + rows_per_chunk, nthreads)
                rows += rows_per_chunk
                if time.perf_counter() - t0 >= budget:
                    return S, rows, time.perf_counter() - t0

    S, rows, dt = run(threads, seconds)
    S1, rows1, dt1 = run(1, max(2.0, seconds / 4))
    extra = {}
    if ebs is not None:
        # the reference's SAT build (serial BuildSAT, restated) on a 256^3 sub-volume
        sub = np.ascontiguousarray(vol[:256, :256, :256])
        t0 = time.perf_counter()
        O.sat_build(sub, ebs["lut"])
        dts = time.perf_counter() - t0
        extra = {"sat_build_Mcells_s": round((sub.shape[0] + 2) * (sub.shape[1] + 2) *
                                             (sub.shape[2] + 2) / dts / 1e6, 2),
                 "sat_build_sample": f"serial BuildSAT restatement, {sub.shape[::-1]} voxels "
                                     f"in {dts:.2f} s (1 thread, as the reference)"}
    if gpu_rgba is not None:
        # the checker: this frame's GPU image against the oracle on a band of rows
        # (the whole frame for rc1pass), as float bits and as eval.py's SSIM
        from cpp_volume_rendering_amd.ssim import ssim_rgba
        band = H if (dos is None and ebs is None) else (64 if dos is not None else 32)
        y0 = H // 2 - band // 2
        if ebs is not None:
            # the band richest in finite shaded pixels: at 1024^3 most of the EBS frame
            # is inf/NaN (float-SAT cancellation), and a centre band compares NaN with NaN
            best, _ = O.finite_shaded_bands(gpu_rgba, band, need=1, max_bands=1)
            y0 = best[0][0] if best else y0
        ref = render_rows_full(y0, y0 + band, threads)[0][y0:y0 + band]
        if half:   # the RGBA16F frame: the oracle's float composite rounded to nearest even
            ref = ref.astype(np.float16).astype(np.float32)
        got = gpu_rgba[y0:y0 + band]
        fin = np.isfinite(ref).all(-1)
        extra["parity"] = {
            "rows": [y0, y0 + band],
            "finite_px": int(fin.sum()),
            "finite_shaded_px": int((fin & (ref[..., 3] > 0)).sum()),
            "bit_exact": bool(np.array_equal(got.view(np.uint32), ref.view(np.uint32))),
            "max_abs_diff": float(np.nan_to_num(np.abs(got.astype(np.float64) - ref), nan=0.0,
                                                posinf=0.0).max()),
            # non-finite pixels (NaN/inf in the same channels on both sides count as equal)
            "nonfinite_px": int((~np.isfinite(ref)).any(-1).sum()),
            "ssim_rgb8_vs_oracle": round(ssim_rgba(got, ref), 6),
            "what": "GPU frame vs the CPU oracle (CVR-SPEC" + (", rounded to RGBA16F" if half else "")
                    + ") on these rows; SSIM as eval.py "
                    "(magick compare -metric SSIM, tests/test_ssim.py) of the screenshots"}
    return {**extra, "value": round(S / dt / 1e6, 3), "unit": "Msamples/s", "cores": threads,
            "kind": "port",
            "sample": f"{rows} image rows ({rows / H:.1f} frames, centre band outward) of the "
                      f"same {W}x{H} frame, {S} samples in {dt:.1f} s on {threads} threads; "
                      f"C++/OpenMP oracle (no CPU ray-caster exists in the reference), built "
                      f"g++ -O2 -march=x86-64-v3 -ffp-contract=off (oracle/Makefile; not BASELINE.md's "
                      f"-O3 -march=native: GCC -O3 vectorisation drops a float narrowing the "
                      f"CVR-SPEC table build needs)"
                      + ("; extinction pyramid built outside the timed sample" if dos else "")
                      + ("; shading only, on the GPU-built SAT (bit-identical to the oracle's, "
                         "tests/test_ebs_gpu.py)" if ebs else ""),
            "single_thread_value": round(S1 / dt1 / 1e6, 3),
            "single_thread_sample": f"{rows1} rows, {S1} samples in {dt1:.1f} s"}


def cone_tables_for(params, n, scale, frac):
    """The cone tables cvr_render_dosct builds (covered distance <= 0: diagonal * frac)."""
    p = N.ConeParams.from_buffer_copy(params)
    if p.covered_distance <= 0:
        diag = float(np.sqrt(sum((n * float(s)) ** 2 for s in scale)))
        p.covered_distance = float(np.float32(diag * np.float32(frac)))
    t = N.ConeTables()
    N.check(N.lib().cvr_build_cone_tables(ctypes.byref(p), 1.0, ctypes.byref(t)), "cones")
    return t


def cone_fetches(r, n, scale):
    """Trilinear extinction fetches per cone: n1 + 3 n3 + 7 n7 (occlusion, shadow)."""
    out = []
    for params, frac in ((r.sampler_occlusion, 0.50), (r.sampler_shadow, 0.75)):
        t = cone_tables_for(params, n, scale, frac)
        out.append(t.counts[0] + 3 * t.counts[1] + 7 * t.counts[2])
    return out


def lib_sha16():
    """The running libcvr.so's build: the first 16 hex digits of its sha256."""
    import hashlib
    with open(N.lib()._name, "rb") as f:
        return hashlib.sha256(f.read()).hexdigest()[:16]


def load_pmc(path, workload_key, kernel, sha):
    """The PMC record (tools/pmc_record.py) of this exact workload, dominant kernel and
    library build: `path` or any profiles/pmc_<renderer>*.json beside it; {} if none.
    A record counted on another build or kernel is not this run's and is never used."""
    import glob
    stem = os.path.splitext(path)[0]
    for f in [path] + sorted(glob.glob(stem + "_*.json")):
        try:
            with open(f) as fh:
                d = json.load(fh)
        except (OSError, ValueError):
            continue
        if (d.get("workload_key") == workload_key and d.get("kernel") == kernel
                and d.get("lib_sha16") == sha):
            return d
    return {}


def cadence_lines(r, dev, W, H, fmt, cam, S_static, reps=100):
    """The plugin's own cadence: ONE frame per cvr_render_rc1pass call
    on ONE stream, as HipRayCasting1Pass::Redraw issues it once per
    RenderingManager::Display (renderingmanager.cpp:199-208, rc1prenderer.cpp:140-151),
    each frame RGBA16F into a device buffer.  Two lines: the static headline view
    (the launch order learned on it) and an orbit through the reference's 24 camera
    states (data/#list_camera_states), one state per frame, so no frame's order was
    learned on its own view.  Host wall time between synchronisations over `reps`
    frames; kernel times from the library's HIP events on the same stream."""
    L = N.lib()
    h = r.device.handle
    s = torch.cuda.Stream(dev)
    r.device.set_stream(s.cuda_stream)
    img = torch.zeros((H, W, 4), dtype=torch.float16 if fmt == N.FORMAT_RGBA16F else torch.float32,
                      device=dev)
    total = torch.zeros((1,), dtype=torch.int64, device=dev)
    out = N.Output(img.data_ptr(), None, None, 1, fmt)
    out_cnt = N.Output(img.data_ptr(), None, total.data_ptr(), 1, fmt)
    path = os.path.join(ROOT, "tests", "golden", "list_camera_states")
    ncam = ctypes.c_int()
    N.check(L.cvr_read_camera_state(path.encode(), 0, N.Camera(), None, 0, ncam), "camera list")
    orbit = [make_frame(read_camera_state(path, i), W, H) for i in range(ncam.value)]
    S_orbit = []
    for f in orbit:                  # samples of each state, counted by the kernel
        total.zero_()
        r.render_to(f, out_cnt)
        torch.cuda.synchronize(dev)
        S_orbit.append(int(total.item()))
    res = {}
    for name, frames, S in (("static", [make_frame(cam, W, H)], [S_static]), ("orbit", orbit, S_orbit)):
        n = reps if name == "static" else 2 * len(frames)
        for i in range(max(20, len(frames))):          # warm: clocks, the slot's launch order
            r.render_to(frames[i % len(frames)], out)
        torch.cuda.synchronize(dev)
        N.check(L.cvr_set_option(h, b"kernel_timing", n), "kernel_timing", h)
        t0 = time.perf_counter()
        for i in range(n):
            r.render_to(frames[i % len(frames)], out)
        torch.cuda.synchronize(dev)
        dt = time.perf_counter() - t0
        kt = (ctypes.c_float * n)()
        nkt = ctypes.c_int()
        N.check(L.cvr_read_kernel_times(h, kt, n, ctypes.byref(nkt)), "kernel times", h)
        N.check(L.cvr_set_option(h, b"kernel_timing", 0), "kernel_timing", h)
        Sn = sum(S[i % len(S)] for i in range(n))
        kms = float(np.mean(kt[:nkt.value]))
        res[name] = {"frames": n, "ms_per_frame": round(dt / n * 1e3, 4),
                     "fps": round(n / dt, 1),
                     "Msamples_s": round(Sn / dt / 1e6, 2),
                     "kernel_ms_mean": round(kms, 4),
                     "kernel_Msamples_s": round(Sn / n / (kms * 1e-3) / 1e6, 2),
                     "samples_per_frame_mean": int(round(Sn / n))}
        if name == "orbit":
            res[name]["samples_per_state"] = S_orbit
    res["what"] = ("one cvr_render_rc1pass call per frame on one stream, RGBA16F device output "
                   "(the plugin's Redraw cadence; the adapter's HIP-GL interop copy of the "
                   "frame is not included: no GL here); static = camera 'Initial State', orbit "
                   "= the reference's camera states in order, one per frame")
    return res


def postpass_bench(r, dev, W, H, reps):
    """The step after the march: RenderFrameToScreen's multiscaling
    filters, timed with HIP events on the context stream.  Modes 1-2 filter a (2W, 2H)
    RGBA16F frame of this workload to the W x H screen, mode 3 a (W/2, H/2) one; the
    frames are rendered here by the same renderer.  Algorithmic bytes: 8 B per frame pixel
    read + 8 B per screen pixel written (+ 2 x 16 B per pixel of the image the cardinal
    kernels' digital filter sweeps in place, twice)."""
    L = N.lib()
    cur = torch.cuda.current_stream(dev)
    r.device.set_stream(cur.cuda_stream)
    cam = Camera(**D.INITIAL_STATE_CAMERA, aspect=W / H)
    out = []
    screen = torch.zeros((H, W, 4), dtype=torch.float16, device=dev)
    for mode, kern in [(1, 1), (2, 1), (2, 2), (2, 4), (3, 1), (3, 2), (3, 5)]:
        fw, fh = (2 * W, 2 * H) if mode < 3 else (W // 2, H // 2)
        frame = torch.zeros((fh, fw, 4), dtype=torch.float16, device=dev)
        r.render_to(make_frame(cam, fw, fh), N.Output(frame.data_ptr(), None, None, 1,
                                                      N.FORMAT_RGBA16F))
        work = frame.clone()
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        for i in range(reps + 2):
            if i == 2:
                ev[0].record(cur)
            if mode == 3 and kern >= 4:      # the prefilter runs in place: restore the frame
                work.copy_(frame)
            N.check(L.cvr_multiscale_filter(r.device.handle, mode, kern, work.data_ptr(), fw, fh,
                                            screen.data_ptr(), W, H), "filter", r.device.handle)
        ev[1].record(cur)
        torch.cuda.synchronize(dev)
        ms = ev[0].elapsed_time(ev[1]) / reps
        swept = (W * H if mode == 2 else fw * fh) if kern >= 4 else 0
        b = 8 * fw * fh + 8 * W * H + 2 * 16 * swept
        out.append({"mode": mode, "kernel": kern, "frame": [fw, fh], "ms": round(ms, 4),
                    "bytes_alg": b, "GB_s": round(b / (ms * 1e-3) / 1e9, 1)})
    return {"screen": [W, H], "filters": out,
            "what": "cvr_multiscale_filter (postpass.hip); mode 1 multisample, 2 downscale, "
                    "3 upscale; kernel 1 hat, 2 Catmull-Rom, 4 cardinal B-spline, 5 o-MOMS; "
                    "mode 3 with a cardinal kernel includes restoring the frame (in-place prefilter)"}


def main():
    a = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if a.dry_run:
        return dry_run(world, rank, a)
    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    else:
        torch.cuda.set_device(0)

    dos = a.renderer == "dos"
    ebs = a.renderer == "ebs"
    iso_variant = {"iso": 0, "isodfs": 1, "isoadapt": 2}.get(a.renderer)
    iso = iso_variant is not None
    shaded = dos or ebs
    # sub-millisecond frames: enough untimed frames for the clocks to settle
    # (5 warmup frames measured ~8 % slower than 20) and a timed region of ~25 ms
    a.steps = a.steps or (5 if dos else (2 if ebs else (20 if iso else 200)))
    a.warmup = a.warmup if a.warmup >= 0 else (1 if shaded else (3 if iso else 20))
    n, W = a.size or (1024 if ebs else 512), a.res or (2048 if dos else 1024)
    H = W
    vol = D.marschner_lobb_u8(n) if a.field == "ml" else D.blobs_u8(n)
    scale = D.voxel_scale(n)
    # --tf-alpha scales the TF's alpha control points (0.02: rays rarely reach the ERT
    # threshold and stream the whole volume -- the long-ray, HBM-bound line)
    alpha_cp = tuple((a_ * a.tf_alpha, iso_) for a_, iso_ in D.BONSAI_TF_ALPHA)
    tf = build_tf_rgbt(D.BONSAI_TF_RGB, alpha_cp)
    # GenerateTexture_1D_RGBA of the same TF (alpha = opacity) for the extinction pyramid
    tf_rgba = build_tf_rgbt(D.BONSAI_TF_RGB, alpha_cp, extinction_input=True)
    cam = Camera(**D.INITIAL_STATE_CAMERA)
    cams = [cam]
    if a.orbit:
        path = os.path.join(ROOT, "tests", "golden", "list_camera_states")
        cnt = ctypes.c_int()
        N.check(N.lib().cvr_read_camera_state(path.encode(), 0, N.Camera(), None, 0, cnt),
                "camera list")
        cams = [read_camera_state(path, i) for i in range(cnt.value)]

    dm = DataManager()
    dm.SetVolume(vol, scale)
    dm.SetTransferFunction(tf, tf_rgba)
    if a.phong:
        dm.SetGradientType(N.GRADIENT_FINITE_DIFFERENCES)
    rp = RenderingParameters(W, H, light_position=D.LIGHT_LIST0_POSITION)
    sat_ms = None
    if dos:
        r = RC1PConeTracingDirOcclusionShading(local if world > 1 else 0)
        r.glsl_apply_shadow = True        # config 4: cone AO + cone shadows (point light)
    elif ebs:
        dm.SetExtinctionTable(build_ext_lut(D.BONSAI_TF_RGB, alpha_cp))
        r = RC1PExtinctionBasedShading(local if world > 1 else 0)
    elif iso:
        r = (CustomRayCasting1PassIsoAdapt, CustomRayCasting1PassIsodfsAdapt,
             RayCasting1PassIsoAdapt)[iso_variant](local if world > 1 else 0)
    else:
        r = RayCasting1Pass(local if world > 1 else 0)
    r.m_apply_gradient_shading = a.phong
    r.SetExternalResources(dm, rp)
    assert r.Init(W, H)
    r.PrepareRender(cam)
    if ebs and a.sat_layout >= 0:
        N.check(N.lib().cvr_set_option(r.device.handle, b"sat_layout", a.sat_layout), "sat_layout",
                r.device.handle)
    if ebs:
        # the SAT precompute on its own (Init built it once already): GPU wall time
        torch.cuda.synchronize()
        t_sat = time.perf_counter()
        r.device.set_extinction_sat(dm.ext_lut)
        sat_ms = (time.perf_counter() - t_sat) * 1e3

    dev = torch.device("cuda", local if world > 1 else 0)
    stream = torch.cuda.current_stream(dev)
    r.device.set_stream(stream.cuda_stream)
    tile = a.tile
    fmt = N.FORMAT_RGBA16F if a.format == "rgba16f" else N.FORMAT_RGBA32F
    # the frame (its tiles on this rank at N > 1): render, RCCL gather to rank 0, unpack
    # the per-GPU share of the frame shrinks with N while its longest rays do not:
    # at 8 GPUs a rank's frame is ~14 us of throughput and ~50 us of latency, so
    # more frames fly (16 streams: 0.0188 ms per rank frame against 0.030 with 4
    # streams and quad 10 %, which the deeper pipeline no longer needs)
    quad = a.quad if a.quad >= 0 else 0
    # Several frames per launch (rc1pass): one launch fills the GPU with 4 frames'
    # waves, so a frame's tail overlaps the next frame inside the launch and rank 0's
    # host pays one call per 4 frames.  Measured (profiles/r04/s11_*, s12_*):
    # the driver's 20-frame command at N = 1, 0.0808 ms per frame (1 frame per launch,
    # 4 streams) -> 0.0778 (4 per launch, 3 streams); rank shares at N = 8 over 20
    # frames 0.0254 -> 0.0154 ms, in steady state 0.0224 -> 0.0122-0.0131 ms
    if a.renderer != "rc1pass" and a.frames_per_launch > 1:
        sys.exit("bench.py: --frames-per-launch > 1 needs --renderer rc1pass")
    if a.frames_per_launch > 16:
        sys.exit("bench.py: --frames-per-launch must be in 1..16")
    SD = split_defaults(a, world)
    FPL = a.frames_per_launch = SD["frames_per_launch"]
    a.streams = SD["streams"]
    if a.renderer == "rc1pass":
        N.check(N.lib().cvr_set_option(r.device.handle, b"quad", quad), "quad", r.device.handle)
        if a.batch:
            N.check(N.lib().cvr_set_option(r.device.handle, b"batch", a.batch), "batch", r.device.handle)
        if a.tile_order >= 0:
            N.check(N.lib().cvr_set_option(r.device.handle, b"tile_order", a.tile_order), "tile_order",
                    r.device.handle)
        if a.cell_skip >= 0:
            N.check(N.lib().cvr_set_option(r.device.handle, b"cell_skip", a.cell_skip), "cell_skip",
                    r.device.handle)
        if a.launch_interleave >= 0:
            N.check(N.lib().cvr_set_option(r.device.handle, b"launch_interleave", a.launch_interleave),
                    "launch_interleave", r.device.handle)
        if a.skip_min_pct >= 0:
            N.check(N.lib().cvr_set_option(r.device.handle, b"skip_min_pct", a.skip_min_pct),
                    "skip_min_pct", r.device.handle)
    for kv in a.opt:
        k, _, v = kv.partition("=")
        N.check(N.lib().cvr_set_option(r.device.handle, k.encode(), int(v)), k, r.device.handle)
    if shaded and a.shade_flat >= 0:
        N.check(N.lib().cvr_set_option(r.device.handle, b"shade_flat", a.shade_flat), "shade_flat",
                r.device.handle)
    if shaded and a.flat_group > 0:
        N.check(N.lib().cvr_set_option(r.device.handle, b"flat_group", a.flat_group), "flat_group",
                r.device.handle)
    try:
        root_renders = SD["root_renders"]

        def make_split(root):
            return T.ScreenTileSplit(r, W, H, tile=tile, fmt=fmt, device=dev,
                                     transport=a.transport if world > 1 else None,
                                     streams=SD["streams"],
                                     frames_per_exchange=SD["frames_per_exchange"],
                                     frames_per_launch=FPL, buffer_sets=SD["buffer_sets"],
                                     root_renders=root, code=bool(a.exchange_code))
        split = make_split(root_renders)

        def preflight(sp):
            # one frame through the exchange must equal rank 0's own render of the
            # whole frame (the N > 1 paths have not run on hardware before the
            # driver's multi-GPU run)
            sp.render(cam)
            ok = torch.ones((1,), dtype=torch.int32, device=dev)
            if rank == 0:
                full = torch.zeros_like(sp.image)
                r.render_to(make_frame(cam, W, H), N.Output(full.data_ptr(), None, None, 1, fmt))
                torch.cuda.synchronize(dev)
                view = torch.int16 if fmt else torch.int32
                ok[0] = int(torch.equal(full.view(view), sp.image.view(view)))
            dist.broadcast(ok, src=0)
            return bool(int(ok.item()))

        if world > 1 and a.transport == "rccl":
            # fall back one step at a time: a rendering root, then raw tiles
            while not preflight(split):
                if not root_renders:
                    what, instead, root_renders = "the idle-root exchange", "a rendering root", True
                elif a.exchange_code:
                    what, instead, a.exchange_code = "the coded exchange", "raw tiles", 0
                else:
                    raise RuntimeError("the multi-GPU exchange does not reproduce the frame")
                print(f"rank {rank}: {what} did not reproduce the frame; using {instead}",
                      file=sys.stderr)
                split.close()
                split = make_split(root_renders)
    except T.CommUnavailable as e:     # no native communicator: torch's dist.gather instead
        # (only cvr_comm_init failures land here: an option the library rejects is a
        # configuration error and ends the bench)
        if world == 1 or a.transport != "rccl":
            raise
        print(f"rank {rank}: native RCCL gather unavailable ({e}); using dist.gather",
              file=sys.stderr)
        a.transport = "torch"
        split = T.ScreenTileSplit(r, W, H, tile=tile, fmt=fmt, device=dev, transport="torch")
    renders = split.renders if world > 1 else True       # False: rank 0 only gathers
    if world > 1:
        frames = [make_frame(c, W, H, tile, split.srank, split.sworld) for c in cams]
        k = split.k
        pixels = k * tile * tile
        out_buf = split.packed[0]
    else:
        frames = [make_frame(c, W, H) for c in cams]
        pixels = W * H
        out_buf = split.image
    total = torch.zeros((1,), dtype=torch.int64, device=dev)
    L = N.lib()
    out = N.Output(out_buf.data_ptr(), None, total.data_ptr(), 1, fmt)

    def step_once(i=0):
        r.render_to(frames[i % len(frames)], out)

    # samples per frame (this rank) and camera, counted by the kernel; for the shaded
    # renderers also the shaded / shadow-lit samples and the secondary fetches
    # (rc1pass: [0] Phong-shaded samples, [1] samples the per-cell skip stepped over)
    count_shaded = not iso
    if count_shaded:
        N.check(L.cvr_set_option(r.device.handle, b"shade_counters", 1), "opt", r.device.handle)
    S_cam = []
    shade = (ctypes.c_uint64 * 3)()
    for i in range(len(frames)):
        if not renders:
            S_cam.append(0)
            continue
        total.zero_()
        step_once(i)
        torch.cuda.synchronize(dev)
        S_cam.append(int(total.item()))
        if count_shaded:
            sh = (ctypes.c_uint64 * 3)()
            N.check(L.cvr_read_shade_counters(r.device.handle, sh), "shade", r.device.handle)
            for q in range(3):
                shade[q] += sh[q]
    if count_shaded:
        N.check(L.cvr_set_option(r.device.handle, b"shade_counters", 0), "opt", r.device.handle)
        for q in range(3):     # per frame, averaged over the camera cycle
            shade[q] = shade[q] // len(frames)
    # the timed frames cycle through the cameras: samples of frame i = S_cam[i % ncam]
    S_rank_steps = sum(S_cam[i % len(S_cam)] for i in range(a.steps))
    S_rank = int(round(S_rank_steps / a.steps))       # mean samples per frame

    # clock settle: untimed frames until the GPU has been busy for settle_ms
    settle = 0
    t_settle = time.perf_counter()
    while (time.perf_counter() - t_settle) * 1e3 < a.settle_ms:
        for _ in range(8):
            split.submit(cams[settle % len(cams)])
            settle += 1
        split.flush()
        torch.cuda.synchronize(dev)
    for i in range(a.warmup):
        split.submit(cams[i % len(cams)])
    split.flush()
    torch.cuda.synchronize(dev)

    # The timed region renders without the sample counter (S is the kernel's own
    # count from the frame above, checked again after timing) and without the
    # library's timing events (an event record between kernels costs ~5 us).
    # Frames are pipelined at N > 1: frame i+1 renders while frame i is gathered.
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for i in range(a.steps):
        split.submit(cams[i % len(cams)])
    split.flush()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    t1 = time.perf_counter()
    elapsed = t1 - t0

    # multi-GPU check: rank 0 renders the whole frame itself; the gathered image
    # must equal it bit for bit
    split_exact = None
    if world > 1 and rank == 0:
        full = torch.zeros_like(split.image)
        last_cam = cams[(a.steps - 1) % len(cams)]
        r.render_to(make_frame(last_cam, W, H), N.Output(full.data_ptr(), None, None, 1, fmt))
        torch.cuda.synchronize(dev)
        split_exact = bool(torch.equal(full.view(torch.int16 if fmt else torch.int32),
                                       split.image.view(torch.int16 if fmt else torch.int32)))

    # Kernel-only time for the roofline: HIP events the library records on its
    # own stream around the ray-march launch (kernel_timing), in a separate pass.
    # With multi-frame launches the pass times the same launches as the timed region:
    # floor(steps / FPL) launches of FPL frames (the roofline's bytes are per launch).
    n_launch = max(1, a.steps // FPL)
    N.check(L.cvr_set_option(r.device.handle, b"kernel_timing", n_launch if renders else 0),
            "kernel_timing", r.device.handle)
    total.zero_()
    if not renders:
        S_timed = 0
    elif FPL > 1:
        mf_bufs = [out_buf] + [torch.empty_like(out_buf) for _ in range(FPL - 1)]
        mf_outs = [N.Output(mf_bufs[j].data_ptr(), None, total.data_ptr() if j == 0 else None, 1, fmt)
                   for j in range(FPL)]
        for k in range(n_launch):
            r.render_frames_to([frames[(k * FPL + j) % len(frames)] for j in range(FPL)], mf_outs)
        S_timed = sum(S_cam[i % len(S_cam)] for i in range(n_launch * FPL))
    else:
        for i in range(a.steps):
            step_once(i)
        S_timed = S_rank_steps
    torch.cuda.synchronize(dev)
    kern_ms = 0.0
    if renders:
        kt = (ctypes.c_float * n_launch)()
        nkt = ctypes.c_int()
        N.check(L.cvr_read_kernel_times(r.device.handle, kt, n_launch, ctypes.byref(nkt)),
                "cvr_read_kernel_times", r.device.handle)
        assert nkt.value == n_launch
        kern_ms = float(np.mean(kt[:nkt.value]))
    assert int(total.item()) == S_timed, "sample count changed between frames"
    S_launch = int(round(S_timed / n_launch))            # samples per launch (FPL frames)
    roof_src = "this rank"
    if world > 1 and split.idle_root:
        # an idle root renders nothing: the roofline is rank 1's share (same launches)
        v = torch.tensor([kern_ms, S_launch, pixels, shade[0], shade[1], shade[2]],
                         dtype=torch.float64, device=dev)
        dist.broadcast(v, src=1)
        kern_ms, S_launch, pixels = float(v[0]), int(v[1]), int(v[2])
        for q in range(3):
            shade[q] = int(v[3 + q])
        roof_src = "rank 1 (rank 0 only gathers)"
    batch = L.cvr_get_option(r.device.handle, b"batch") or (2 if a.phong else 4)   # 0 = auto
    macro = L.cvr_get_option(r.device.handle, b"macro")

    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        s = torch.tensor([S_rank_steps], dtype=torch.int64, device=dev)
        dist.all_reduce(s, op=dist.ReduceOp.SUM)
        S_all_steps = int(s.item())
    else:
        S_all_steps = S_rank_steps
    S_all = int(round(S_all_steps / a.steps))

    if rank == 0:
        msps = S_all_steps / elapsed / 1e6
        ms_per_step = elapsed / a.steps * 1e3
        # algorithmic bytes per launch: 8 trilinear corners x 1 B (u8 input)
        # per sample + the output pixel (RGBA16F 8 B, RGBA32F 16 B) (+ 48 B per shaded
        # sample for the Phong gradient: 8 corners x 3 fp16, counted by the kernel)
        px_bytes = 8 if fmt == N.FORMAT_RGBA16F else 16
        # (iso: 8 B per volume fetch + the pixel; the <= 1 gradient fetch per hit is left out)
        b_alg = (8 * 1 * S_launch + FPL * px_bytes * pixels
                 + (FPL * 48 * int(shade[0]) if count_shaded and a.phong else 0))
        fetches = int(shade[2])
        if dos:
            # + 8 fp16 corners (16 B) per trilinear extinction fetch the kernel issues.
            # The reference evaluates shade[0]*f_occ + shade[1]*f_sdw taps; those whose
            # CONSIDER_BORDERS factor is exactly 0 are skipped (not fetched), so they
            # count in the reference-work rate but not in the roofline's bytes.
            f_occ, f_sdw = cone_fetches(r, n, scale)
            ref_taps = shade[0] * f_occ + shade[1] * f_sdw
            assert 0 < fetches <= ref_taps
            b_alg += 16 * fetches
        elif ebs:
            # + 8 float corners (32 B) per trilinear SAT fetch
            b_alg += 32 * fetches
        achieved = b_alg / (kern_ms * 1e-3) / 1e9
        wkey = (f"{a.renderer}_{a.field}{n}_{W}x{H}{'_phong' if a.phong else ''}"
                f"{'_orbit' if a.orbit else ''}"
                f"{f'_alpha{a.tf_alpha:g}' if a.tf_alpha != 1.0 else ''}")
        flat = shaded and N.lib().cvr_get_option(r.device.handle, b"shade_flat") == 1
        kname = ("flat_shade_kernel<DosShader> (+ shaded_jobs_kernel x2, flat_fold_kernel)" if dos and flat else
                 "flat_shade_kernel<EbsShaderT> (+ shaded_jobs_kernel x2, flat_fold_kernel)" if ebs and flat else
                 "shaded_march_kernel<DosShader>" if dos else
                 "shaded_march_kernel<EbsShader>" if ebs else
                 f"iso_tile_kernel<{iso_variant}, {str(a.phong).lower()}>" if iso else
                 f"rc1pass_tile_kernel<{batch}, {str(a.phong).lower()}, *, false, true, *>")
        # DOS and EBS move their secondary fetches (DOS: 85 GB of pyramid corners per
        # frame, a 37 MiB pyramid; EBS: ~2 TB of SAT corners) through the vector-memory
        # pipe from L1/L2/MALL, far above what HBM could serve at these frame times:
        # their roofline is the L2's, with the HBM figures (PMC traffic) beside it
        peak = L2_PEAK_GBS if shaded else HBM_PEAK_GBS
        sha = lib_sha16()
        pmc = load_pmc(a.pmc.replace("rc1pass", a.renderer), wkey, kname, sha)
        roof = {"bound": "l2" if shaded else "hbm", "achieved": round(achieved, 1), "peak": peak,
                "unit": "GB/s", "frac": round(achieved / peak, 4),
                "traffic": pmc.get("hbm_bytes_per_launch"),
                "kernel": kname,
                "kernel_ms": round(kern_ms, 4),
                "frames_per_launch": FPL, "share": roof_src,
                "bytes_alg_per_launch": b_alg, "samples_per_launch": S_launch,
                # the same bytes over the frame time of the timed region (frames in
                # flight overlap, so a frame takes less than one launch's duration)
                "frac_frame": round(b_alg / FPL / (ms_per_step * 1e-3) / 1e9 / peak, 4)}
        if shaded:
            roof["alg_over_hbm_peak"] = round(achieved / HBM_PEAK_GBS, 4)
        else:
            # "an *effective* bandwidth" -- B_alg counts 8 corners per
            # sample of the reference's loop; most of them come from L1/L2 (traffic
            # below is what HBM served), so frac near or above 1 means the march is
            # past the HBM roofline of its algorithmic bytes (VALU issue and vector-
            # memory latency bound it)
            roof["definition"] = "effective: B_alg / launch time (SURVEY 8d); HBM bytes in traffic"
        if ebs:
            # the vector-memory pipe: 2 dwordx4 wave-loads (2 x 1 KiB) per 64 SAT fetches,
            # against 256 CUs x one 1-KiB wave-load per 16 clocks (64 B/clk per CU L1) at
            # 2.4 GHz; PMC: the texture-data unit's busy share per CU (pmc_ebs.json)
            vm = 2 * fetches / 64 / (kern_ms * 1e-3)
            vm_peak = 256 * 2.4e9 / 16
            roof["vmem_dwordx4_per_s"] = round(vm, 1)
            roof["vmem_peak_dwordx4_per_s"] = vm_peak
            roof["vmem_frac"] = round(vm / vm_peak, 4)
        if shaded and pmc.get("kernel_ns_avg_under_pmc") and pmc.get("valu_wave_insts"):
            # the shade kernel's own pipes (the counters and the duration of the same
            # dispatches under PMC; the frame's other kernels are ~15 % of it): the
            # roofline on the pipe that binds, beside the L2 figure
            t_pmc = pmc["kernel_ns_avg_under_pmc"] * 1e-9
            pipes = {"valu": {"frac": round(pmc["valu_wave_insts"] / t_pmc / 1e9 / VALU_PEAK_GWIPS, 4),
                              "count": "PMC SQ_INSTS_VALU of flat_shade_kernel"}}
            if pmc.get("sq_insts_vmem_rd"):
                pipes["vmem"] = {"frac": round(pmc["sq_insts_vmem_rd"] * 1024 / t_pmc / 1e9 / VMEM_PEAK_GBS, 4),
                                 "count": "PMC SQ_INSTS_VMEM_RD of flat_shade_kernel"}
            if ("vmem" in pipes and pmc.get("td_tc_stall_frac_per_cu") is not None
                    and pmc.get("td_busy_frac_per_cu") is not None):
                pipes["vmem"]["td_busy_per_cu"] = round(pmc["td_busy_frac_per_cu"], 3)
                pipes["vmem"]["td_stalled_on_cache_per_cu"] = round(pmc["td_tc_stall_frac_per_cu"], 3)
            roof["shade_kernel_pipes"] = pipes
            roof["shade_kernel_bound"] = max(pipes, key=lambda k: pipes[k]["frac"])
        # the counters of the same workload's dominant kernel on this library build
        # (rocprofv3 --pmc, committed under profiles/): which pipe is busy, VALU per
        # sample, the bytes written
        if pmc.get("td_busy_frac_per_cu") is not None:
            roof["pmc"] = {"td_busy_per_cu": round(pmc["td_busy_frac_per_cu"], 3),
                           "ta_busy_per_cu": round(pmc["ta_busy_frac_per_cu"], 3),
                           "valu_issue_per_simd": round(pmc["valu_issue_frac_per_simd"], 3),
                           "l2_hit_rate": round(pmc["tcc_hit_rate"], 3),
                           "write_bytes_per_launch": int(pmc["write_bytes_per_launch"])}
            if pmc.get("valu_per_sample") is not None:
                roof["pmc"]["valu_per_sample"] = round(pmc["valu_per_sample"], 1)
            if a.renderer == "rc1pass" and not a.phong:
                roof["pmc"]["scratch_bytes_per_launch_est"] = max(
                    0, int(pmc["write_bytes_per_launch"]) - FPL * px_bytes * pixels)
            roof["pmc"]["kernel_ns_under_pmc"] = pmc.get("kernel_ns_avg_under_pmc")
            roof["pmc"]["record"] = f"profiles/pmc_{a.renderer}*.json, lib {sha}"
        if roof["traffic"]:
            # the bytes HBM actually served (PMC) at the kernel's own time: where the
            # algorithmic figure is mostly served from L1/L2 (frac > 1 for EBS), this
            # is the quantity the HBM roofline bounds
            roof["traffic_GBs"] = round(roof["traffic"] / (kern_ms * 1e-3) / 1e9, 1)
            roof["traffic_frac"] = round(roof["traffic_GBs"] / HBM_PEAK_GBS, 4)
        if a.phong and count_shaded:
            roof["phong_shaded_samples"] = int(shade[0])
        if a.renderer == "rc1pass":
            # the per-cell skip (cell_skip 2-4) steps over samples in empty space without
            # a load: they count in S (the reference's loop iterations) but fetch nothing;
            # the same roofline on the bytes actually fetched, beside it
            skipped = int(shade[1]) * FPL
            b_fetch = b_alg - 8 * skipped
            roof.update({"skipped_samples": skipped, "fetched_samples": S_launch - skipped,
                         "bytes_fetched_per_launch": b_fetch,
                         "achieved_fetched": round(b_fetch / (kern_ms * 1e-3) / 1e9, 1),
                         "frac_fetched": round(b_fetch / (kern_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)})
            # SURVEY §8(d)'s figure (B_alg over the launch time against the HBM peak) is an
            # effective bandwidth, not a roofline: most of B_alg is served by L1/L2 and
            # it exceeds 1 on cache-friendly views.  Kept as effective_frac; the roofline
            # proper is the busier of the vmem and VALU pipes (pipe_roofline)
            eff = roof["frac"]
            live_wl = None
            if not a.phong and shade[2]:
                ntiles_frame = pixels // 64
                tf_loads = -(-(len(tf) + 2) // 64)
                live_wl = FPL * (batch * int(shade[2]) + ntiles_frame * tf_loads)
            pr = pipe_roofline(kern_ms, FPL, pmc, live_wl)
            if pr:
                roof.update(pr)
                roof["effective_bound"] = "hbm (SURVEY 8d effective bandwidth)"
                roof["effective_achieved"] = round(achieved, 1)
                roof["effective_frac"] = eff
                roof["effective_frac_frame"] = roof.pop("frac_frame")
                roof["definition"] = ("frac: the busier pipe of the march (vmem: wave-loads x 1 KiB "
                                      "vs 64 B/clk/CU; valu: wave-instructions x 2 clk per SIMD), "
                                      "at the 2.4 GHz peak clock; effective_frac: B_alg / launch "
                                      "time / 8 TB/s (SURVEY 8d, not a roofline when > 1); "
                                      "traffic_frac: PMC HBM bytes / launch time / 8 TB/s")
        if dos:
            roof.update({"shaded_samples": shade[0], "shadow_lit_samples": shade[1],
                         "cone_fetches_per_shaded": [f_occ, f_sdw],
                         "secondary_fetches": fetches,
                         "reference_taps": ref_taps,
                         "skipped_zero_border_taps": ref_taps - fetches,
                         "reference_taps_per_s": round(ref_taps / (kern_ms * 1e-3), 1)})
        elif ebs:
            roof.update({"shaded_samples": shade[0], "shadow_chains": shade[1],
                         "sat_fetches": fetches,
                         "sat_fetches_per_shaded": round(fetches / max(1, shade[0]), 1)})
        metric = ("Msamples/s (rays x steps), Dir. Occlusion Shading (cone AO + cone shadows), "
                  f"{n}^3 volume at {W}^2" if dos else
                  "Msamples/s (rays x steps), Extinction-Based Shading (SAT AO + SAT shadows), "
                  f"{n}^3 volume at {W}^2" if ebs else
                  f"Msamples/s (volume fetches), isosurface ray-caster '{r.GetName()}', "
                  f"{n}^3 volume at {W}^2" if iso else
                  f"Msamples/s (rays x steps), rc1pass ray-march, {n}^3 volume at {W}^2")
        res = {
            "metric": metric,
            "value": round(msps, 2),
            "unit": "Msamples/s",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": round(ms_per_step, 4),
            "fps": round(1000.0 / ms_per_step, 1),
            # fps and ms_per_step are throughput: frames overlap on the device (one
            # static view, split.nstreams launches of frames_per_launch frames in
            # flight); a frame is delivered when its launch ends, so its latency is
            # about roofline.kernel_ms (its launch, with the other launches in flight)
            "frame_latency_ms_approx": None,
            "higher_is_better": True,
            "scaling": "strong",   # one fixed frame split over the GPUs
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic",
            "config": {"workload": (f"rc1pdosct cone AO (20 deg, <=3 rays) + point-light cone "
                                    f"shadows (0.5 deg), extinction pyramid 128^3, " if dos else
                                    f"rc1pextbsd SAT AO (15 shells) + point-light SAT box-chain "
                                    f"shadows (1 deg cone), extinction SAT {n + 2}^3, " if ebs else
                                    f"{r.GetName()} (isovalue 0.5, steps 0.05/1.0/0.1, blocks "
                                    f"{tuple(r.num_blocks) if iso_variant != 2 else 'none'}), "
                                    if iso else
                                    f"rc1pass emission-absorption, ")
                                   + f"Marschner-Lobb {n}^3 u8 "
                                   f"({a.field}), {W}x{H}, bonsai_01.tf1d"
                                   + (f" (alpha x{a.tf_alpha:g})" if a.tf_alpha != 1.0 else "")
                                   + ", "
                                   + (f"camera orbit: the {len(cams)} states of "
                                      f"data/#list_camera_states, one per frame" if a.orbit
                                      else "camera 'Initial State'")
                                   + ("" if iso else ", step 0.5, ERT 0.99")
                                   + (", Blinn-Phong FD gradient" if a.phong else ""),
                       "volume": n, "viewport": [W, H], "samples_per_frame": S_all,
                       "workload_key": wkey, "lib_sha16": sha,
                       **({"options": dict(kv.partition("=")[::2] for kv in a.opt)} if a.opt else {}),
                       "settle_frames": settle,
                       "parallelism": f"screen tiles {tile}x{tile} over {world} GPU(s)"
                                      if world > 1 else "1 GPU",
                       "storage": "cell8 fp16 (16 B/cell, x-fastest; skip flags in the sign bits)"
                                  + ((", SAT " + ("plain float" if N.lib().cvr_get_option(
                                      r.device.handle, b"sat_layout") == 1 else "cell4 float4"))
                                     if ebs else ""),
                       "frame_format": a.format,
                       "frames_in_flight": split.nstreams * FPL,
                       "frames_per_launch": FPL,
                       "render_streams": split.nstreams,
                       "hw_queues": int(os.environ["GPU_MAX_HW_QUEUES"]),
                       "quad_pct": quad if a.renderer == "rc1pass" else 0,
                       "shading": ("flat job list" if N.lib().cvr_get_option(r.device.handle, b"shade_flat")
                                   else "per-wave batches") if shaded else None,
                       "empty_space_skip": f"macro cells 2^{macro}, auto (on at >= 15 % empty)"
                                           if macro > 0 else "off"},
            "roofline": roof,
        }
        res["frame_latency_ms_approx"] = round(kern_ms, 4)
        if world > 1:
            coded = a.transport == "rccl" and a.exchange_code and a.format == "rgba16f"
            res["config"]["gather"] = ((f"{a.transport}: per-tile code of each rank's {a.format} tiles "
                                        f"({split.G} frame(s) per exchange: one encode launch, sizes "
                                        f"first, grouped ncclSend/ncclRecv, one decode launch into "
                                        f"the images on rank 0), " if coded else
                                        f"{a.transport}: packed {a.format} tiles to rank 0 "
                                        f"({split.G} frame(s) per ncclGather) + unpack of every "
                                        f"frame, ")
                                       + f"{split.nstreams} render streams, {split.nbuf} "
                                       f"buffer sets, "
                                       + ("rank 0 only gathers (N - 1 render ranks)"
                                          if split.idle_root else "every rank renders"))
            res["multi_gpu_bit_exact_vs_1gpu_frame"] = split_exact
        if ebs:
            cells = (n + 2) ** 3
            sat_gpu_ms = N.lib().cvr_get_option(r.device.handle, b"sat_build_us") / 1e3
            res["precompute"] = {"sat_ms": round(sat_ms, 2), "sat_cells": cells,
                                 "sat_gpu_ms": round(sat_gpu_ms, 2),
                                 "sat_Mcells_s": round(cells / (sat_gpu_ms * 1e-3) / 1e6, 1),
                                 "what": "GenerateExtinctionSAT3DTex + BuildSAT on the GPU "
                                         "(double, reference recurrence, bit-exact): sat_ms = wall "
                                         "time of cvr_set_extinction_sat incl. freeing and "
                                         "allocating the SAT buffers, sat_gpu_ms = HIP-event time "
                                         "of the build + cell4 expansion kernels"}
        if a.postpass and world == 1:
            res["postpass"] = postpass_bench(r, dev, W, H, a.steps)
        if world == 1 and a.renderer == "rc1pass" and not a.orbit and not a.no_cadence:
            res["plugin_cadence"] = cadence_lines(r, dev, W, H, fmt, cam, S_cam[0])
        if world == 1 and not a.no_cpu_baseline:
            dos_cfg = None
            if dos:
                dos_cfg = {"tf_rgba": tf_rgba, "res": r.ext_res,
                           "occ": cone_tables_for(r.sampler_occlusion, n, scale, 0.50),
                           "sdw": cone_tables_for(r.sampler_shadow, n, scale, 0.75),
                           "light": {"position": rp.light_position,
                                     "forward": rp.light_forward, "up": rp.light_up,
                                     "right": rp.light_right,
                                     "spot_angle_deg": rp.spot_light_angle}}
            ebs_cfg = None
            if ebs:
                ebs_cfg = {"sat": r.device.extinction_sat(), "lut": dm.ext_lut,
                           "light": rp.light_position, "forward": rp.light_forward}
            gpu_img = split.image.float().cpu().numpy() if world == 1 else None
            phong_cfg = {"light": rp.light_position} if a.phong else None
            res["cpu_baseline"] = cpu_baseline(vol, scale, tf, D.INITIAL_STATE_CAMERA, W, H,
                                               a.cpu_seconds, dos_cfg, ebs_cfg, gpu_img, phong_cfg,
                                               half=fmt == N.FORMAT_RGBA16F,
                                               iso={"variant": iso_variant} if iso else None)
            if "parity" in res["cpu_baseline"]:
                res["parity"] = res["cpu_baseline"].pop("parity")
        print(json.dumps(res))
    split.close()
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    r.Clean()


if __name__ == "__main__":
    main()
