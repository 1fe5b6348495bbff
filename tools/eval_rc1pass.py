#!/usr/bin/env python3
"""The reference's only published hot-path table, reproduced: the RayCasting1Pass
StepSize sweep of Evaluation.md:32-51 (FillParameterSpace, rc1prenderer.cpp:225-229:
StepSize 0.2 .. 2.0 by 0.1), run through evaluation.run_evaluation (the
RenderingManager sweep, renderingmanager.cpp:261-317 / 805-857) on this build.

Evaluation.md does not state its hardware, dataset, viewport or camera.  Two
workloads are swept: the bench's headline (512^3 Marschner-Lobb u8, 1024^2) and the
reference's plausible defaults (a 256^3 volume at 768^2: Bonsai is a missing blob,
so a 256^3 Marschner-Lobb field stands in).  Both with bonsai_01.tf1d and the
camera "Initial State".  Writes <out>/<tag>/eval.csv (+ img/) and prints one JSON
object with the sweep beside the reference's column.
Usage: python tools/eval_rc1pass.py [--out gpurun_out/eval_rc1pass] [--frames 100]"""
import argparse
import ctypes
import csv
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import numpy as np  # noqa: E402

from cpp_volume_rendering_amd import _native as N  # noqa: E402
from cpp_volume_rendering_amd import datasets as D  # noqa: E402
from cpp_volume_rendering_amd import evaluation as E  # noqa: E402
from cpp_volume_rendering_amd.renderer import (Camera, DataManager, RayCasting1Pass,  # noqa: E402
                                               RenderingParameters, build_tf_rgbt)

# Evaluation.md:34-51 (StepSize -> TimePerFrame ms), hardware/dataset unstated
REFERENCE_MS = {0.2: 18.95, 0.3: 13.61, 0.4: 10.87, 0.5: 9.22, 0.6: 8.03, 0.7: 7.31, 0.8: 6.64,
                0.9: 6.17, 1.0: 5.76, 1.1: 5.47, 1.2: 5.20, 1.3: 5.01, 1.4: 4.72, 1.5: 4.60,
                1.6: 4.46, 1.7: 4.27, 1.8: 4.25, 1.9: 4.12}


def sweep(tag, n, w, h, out, frames):
    dm = DataManager()
    dm.SetVolume(D.marschner_lobb_u8(n), D.voxel_scale(n), name=f"ml{n}")
    dm.SetTransferFunction(build_tf_rgbt(D.BONSAI_TF_RGB, D.BONSAI_TF_ALPHA))
    r = RayCasting1Pass()
    r.SetExternalResources(dm, RenderingParameters(w, h))
    assert r.Init(w, h)
    cam = Camera(**D.INITIAL_STATE_CAMERA)
    s = torch.cuda.Stream()
    # warm the clocks and the launch order on the default step before the sweep
    r.PrepareRender(cam)
    for _ in range(200):
        r.Redraw(s, count_samples=False)
    torch.cuda.synchronize()
    d = os.path.join(out, tag)
    # the ray-march kernel's own time per sample point (HIP events around each launch)
    L = N.lib()
    N.check(L.cvr_set_option(r.device.handle, b"kernel_timing", frames), "kernel_timing")
    kms = []

    def on_sample(i, values):
        kt = (ctypes.c_float * frames)()
        nk = ctypes.c_int()
        N.check(L.cvr_read_kernel_times(r.device.handle, kt, frames, ctypes.byref(nk)),
                "cvr_read_kernel_times")
        kms.append(float(np.mean(kt[:nk.value])))

    N.check(L.cvr_read_kernel_times(r.device.handle, None, 0, ctypes.byref(ctypes.c_int())),
            "reset kernel times")
    path = E.run_evaluation(r, cam, d, frames_per_sample=frames, stream=s, on_sample=on_sample)
    rows = list(csv.DictReader(open(path)))
    r.Clean()
    return [{"StepSize": float(x["StepSize"]), "ms": float(x["TimePerFrame (ms)"]),
             "fps": float(x["FramesPerSecond"]), "kernel_ms": round(k, 4)}
            for x, k in zip(rows, kms)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default="gpurun_out/eval_rc1pass")
    ap.add_argument("--frames", type=int, default=100)
    a = ap.parse_args()
    res = {"source": "Evaluation.md:32-51 (hardware, dataset, viewport, camera unstated)",
           "frames_per_sample": a.frames, "sweeps": {}}
    for tag, n, w, h in (("ml512_1024", 512, 1024, 1024), ("ml256_768", 256, 768, 768)):
        rows = sweep(tag, n, w, h, a.out, a.frames)
        for row in rows:
            ref = REFERENCE_MS.get(round(row["StepSize"], 1))
            row["reference_ms"] = ref
            row["speedup_vs_reference"] = round(ref / row["ms"], 1) if ref else None
        res["sweeps"][tag] = {"volume": n, "viewport": [w, h], "rows": rows}
    print(json.dumps(res))


if __name__ == "__main__":
    main()
