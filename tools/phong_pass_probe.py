#!/usr/bin/env python3
"""Shading passes of the Blinn-Phong march (bench.py --phong's frame), counted by a
probe build (-DCVR_PROBE_SHADE_PASSES, tools/build_variant.sh; CVR_LIB_OVERRIDE):
per wave and batch, the passes today's inline shading runs (one per batch slot j
where any lane shades its sample j) against the passes if every lane shaded its
visible samples in turn (the busiest lane's count).  Prints one JSON object."""
import ctypes
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from cpp_volume_rendering_amd import _native as N  # noqa: E402
from cpp_volume_rendering_amd import datasets as D  # noqa: E402
from cpp_volume_rendering_amd.renderer import (Camera, DataManager, RayCasting1Pass,  # noqa: E402
                                               RenderingParameters, build_tf_rgbt, make_frame)


def main():
    n, W = 512, 1024
    dm = DataManager()
    dm.SetVolume(D.marschner_lobb_u8(n), D.voxel_scale(n))
    dm.SetTransferFunction(build_tf_rgbt(D.BONSAI_TF_RGB, D.BONSAI_TF_ALPHA))
    dm.SetGradientType(N.GRADIENT_FINITE_DIFFERENCES)
    r = RayCasting1Pass(0)
    r.m_apply_gradient_shading = True
    r.SetExternalResources(dm, RenderingParameters(W, W, light_position=D.LIGHT_LIST0_POSITION))
    assert r.Init(W, W)
    cam = Camera(**D.INITIAL_STATE_CAMERA)
    r.PrepareRender(cam)
    L = N.lib()
    h = r.device.handle
    N.check(L.cvr_set_option(h, b"shade_counters", 1), "opt", h)
    img = torch.zeros((W, W, 4), dtype=torch.float16, device="cuda")
    total = torch.zeros((1,), dtype=torch.int64, device="cuda")
    out = N.Output(img.data_ptr(), None, total.data_ptr(), 1, N.FORMAT_RGBA16F)
    res = []
    for _ in range(3):   # the first frame runs unordered, later ones the learned order
        total.zero_()
        r.render_to(make_frame(cam, W, W), out)
        torch.cuda.synchronize()
        sh = (ctypes.c_uint64 * 3)()
        N.check(L.cvr_read_shade_counters(h, sh), "shade", h)
        res.append({"samples": int(total.item()), "shaded": int(sh[0]),
                    "passes_merged": int(sh[1]), "passes_today": int(sh[2])})
    last = res[-1]
    print(json.dumps({"frames": res, "lanes_per_pass_today": last["shaded"] / max(last["passes_today"], 1),
                      "lanes_per_pass_merged": last["shaded"] / max(last["passes_merged"], 1),
                      "pass_ratio": last["passes_merged"] / max(last["passes_today"], 1)}))
    r.Clean()


if __name__ == "__main__":
    main()
