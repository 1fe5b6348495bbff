#!/usr/bin/env python3
"""How well can a launch order be predicted for a NEW view without marching it?
(CPU model, not product code; VERDICT r04 #4.)

For each of the reference's camera states it takes the oracle's per-pixel sample
counts at the headline workload, forms each 8x8 tile's cost (its longest ray, the
march's critical path), and list-schedules the tiles onto `slots` concurrent wave
slots (the GPU's 8192 at 8 waves/SIMD) in several orders:
  * lpt      : true costs, longest first (what a learned order on the same view gives)
  * interleave: screen order (the library's fallback without an order)
  * chord    : predicted by the geometric chord length of the tile's centre ray
               through the volume box (no marching)
  * coarse   : predicted by the tile's centre ray marched at a coarse step (P x the
               step, alpha-only composite to ERT), i.e. a probe kernel's estimate
Reports the makespan of each (in "samples" of critical path) relative to lpt.

  python tests/models/order_predict_sim.py [--res 1024] [--size 512] [--cams 0,4,11,14]
"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)


def list_schedule(cost, order, slots):
    """Greedy: tiles start in `order` whenever a slot frees; returns the makespan."""
    import heapq
    free = [0.0] * slots
    heapq.heapify(free)
    end = 0.0
    for t in order:
        s = heapq.heappop(free)
        e = s + cost[t]
        end = max(end, e)
        heapq.heappush(free, e)
    return end


def tile_costs(cnt, W, H):
    return cnt.reshape(H // 8, 8, W // 8, 8).max(axis=(1, 3)).reshape(-1).astype(np.float64)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--res", type=int, default=1024)
    ap.add_argument("--size", type=int, default=512)
    ap.add_argument("--cams", default="")
    ap.add_argument("--slots", type=int, default=8192)
    ap.add_argument("--coarse", type=int, default=8)
    a = ap.parse_args()
    import oracle as O
    from cpp_volume_rendering_amd import datasets as D
    from cpp_volume_rendering_amd.renderer import build_tf_rgbt, read_camera_state
    n, W = a.size, a.res
    vol = D.marschner_lobb_u8(n)
    sc = D.voxel_scale(n)
    v16 = O.volume_r16f(vol)
    tf = build_tf_rgbt(D.BONSAI_TF_RGB, D.BONSAI_TF_ALPHA)
    st = O.default_step(sc)
    path = os.path.join(ROOT, "tests", "golden", "list_camera_states")
    idx = [int(x) for x in a.cams.split(",")] if a.cams else list(range(24))
    rows = []
    for i in idx:
        c = read_camera_state(path, i)
        cam = dict(eye=c.eye, center=c.center, up=c.up)
        _, cnt, S = O.render_rc1pass(v16, sc, tf, cam, W, W, st)
        cost = tile_costs(cnt, W, W)
        # the probe: the tiles' centre rays at 1/8 resolution (pixel centres = tile
        # centres) with a coarse step; its per-ray counts x coarse = the estimate
        _, cc, _ = O.render_rc1pass(v16, sc, tf, cam, W // 8, W // 8, st * a.coarse)
        est_coarse = cc.reshape(-1).astype(np.float64) * a.coarse
        # chord: the probe at a step so large that every ray takes 1 + chord / step
        # samples... simply the geometric chord of the centre ray (the count of an
        # all-transparent march): an empty TF renders the chord lengths
        zero_tf = tf.copy()
        zero_tf[:, 3] = 0.0
        _, ch, _ = O.render_rc1pass(v16, sc, zero_tf, cam, W // 8, W // 8, st)
        est_chord = ch.reshape(-1).astype(np.float64)
        nt = cost.size
        lpt = np.argsort(-cost, kind="stable")
        inter = np.arange(nt)
        res = {"view": i, "samples": S, "tiles": nt,
               "max_tile": float(cost.max()), "sum_over_slots": float(cost.sum() / a.slots)}
        base = list_schedule(cost, lpt, a.slots)
        res["lpt"] = round(base, 1)
        for name, order in (("interleave", inter), ("chord", np.argsort(-est_chord, kind="stable")),
                            ("coarse", np.argsort(-est_coarse, kind="stable"))):
            res[name] = round(list_schedule(cost, order, a.slots) / base, 3)
        res["spearman_coarse"] = round(float(np.corrcoef(np.argsort(np.argsort(cost)),
                                                         np.argsort(np.argsort(est_coarse)))[0, 1]), 3)
        res["spearman_chord"] = round(float(np.corrcoef(np.argsort(np.argsort(cost)),
                                                        np.argsort(np.argsort(est_chord)))[0, 1]), 3)
        rows.append(res)
        print(json.dumps(res), flush=True)
    print(json.dumps({"mean": {k: round(float(np.mean([r[k] for r in rows])), 3)
                               for k in ("interleave", "chord", "coarse")}}))


if __name__ == "__main__":
    main()
