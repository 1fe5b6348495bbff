#!/usr/bin/env python3
"""Config 5's parity claim, stated where it can be: CVR-SPEC (what the
HIP kernels reproduce bit for bit) against the literal GLSL reading
(oracle/glsl_literal.cpp) of ebs_ray_bbox_marching.comp on the 1024^3 EBS workload, on
row bands of the 1024^2 frame, CPU only.

At 1024^3 most of the frame is inf/NaN in BOTH readings (the float SAT's corner
differences cancel: ebsrenderer.cpp:700-716 stores BuildSAT's doubles as GL_R32F, and a
box's 8-corner sum of values ~1e9 loses every significant bit), so the comparison is
reported on the pixels finite in both readings, with the pixels finite in only one of
them counted:
  * finite_both / finite_spec_only / finite_lit_only / nonfinite_both;
  * max |dRGBA| and the share of finite-both pixels over 2e-3 (BASELINE.md's gate);
  * SSIM (eval.py's metric, tests/test_ssim.py) of the two bands with every pixel that
    is non-finite in either reading set to 0 in both.
Three cases: SAT ambient occlusion only, SAT box-chain shadow only, both (the bench's
workload).  Writes profiles/r05/ebs_literal_1024.json.

  python tests/models/ebs_literal_1024.py [--rows 0:32,496:528] [--threads 8]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import oracle as O  # noqa: E402
import test_literal as TL  # noqa: E402

from cpp_volume_rendering_amd import datasets as D  # noqa: E402
from cpp_volume_rendering_amd.ssim import ssim_rgba  # noqa: E402


def compare(a, b):
    fa, fb = np.isfinite(a).all(-1), np.isfinite(b).all(-1)
    both = fa & fb
    d = np.abs(a.astype(np.float64) - b)
    px = np.where(both, d.max(-1), 0.0)
    a0 = np.where(both[..., None], a, 0.0).astype(np.float32)
    b0 = np.where(both[..., None], b, 0.0).astype(np.float32)
    shaded = both & (a[..., 3] > 0)
    return {"pixels": int(both.size), "finite_both": int(both.sum()),
            "finite_both_shaded": int(shaded.sum()),
            "finite_spec_only": int((fa & ~fb).sum()), "finite_lit_only": int((fb & ~fa).sum()),
            "nonfinite_both": int((~fa & ~fb).sum()),
            "max_abs_diff_finite": float(px.max()),
            "frac_over_2e-3_finite": float((px[both] > 2e-3).mean()) if both.any() else None,
            "ssim_finite_zeroed": round(ssim_rgba(a0, b0), 6)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--size", type=int, default=1024)
    ap.add_argument("--res", type=int, default=1024)
    ap.add_argument("--rows", default="0:32,496:528")
    ap.add_argument("--threads", type=int, default=0)
    ap.add_argument("--out", default=os.path.join(ROOT, "profiles", "r05", "ebs_literal_1024.json"))
    a = ap.parse_args()
    n, W = a.size, a.res
    t = O.tf_table_double(D.BONSAI_TF_RGB, D.BONSAI_TF_ALPHA)
    tf = O.tf_rgbt(t)
    vol = D.marschner_lobb_u8(n)
    sc = D.voxel_scale(n)
    v16 = O.volume_r16f(vol)
    st = O.default_step(sc)
    t0 = time.time()
    sat = O.sat_build(vol, O.ext_lut(t, 1)).astype(np.float32)
    out = {"workload": f"EBS {n}^3 Marschner-Lobb u8, {W}^2, bonsai_01.tf1d, camera 'Initial State', "
                       "point light of list 0, SAT AO 15 shells + box-chain shadow (1 deg cone)",
           "what": __doc__.split("\n\n")[1].replace("\n", " "),
           "sat_build_s": round(time.time() - t0, 1), "bands": {}}
    base = dict(light=TL.LIGHT0["position"], light_forward=TL.LIGHT0["forward"], threads=a.threads)
    cases = {"occlusion_only": dict(base, apply_shadow=False),
             "shadow_only": dict(base, apply_occlusion=False),
             "occlusion_and_shadow": dict(base)}
    for band in a.rows.split(","):
        y0, y1 = (int(v) for v in band.split(":"))
        res = {}
        for name, kw in cases.items():
            t1 = time.time()
            spec = O.render_ebs(v16, sc, tf, sat, D.INITIAL_STATE_CAMERA, W, W, st, rows=(y0, y1), **kw)[0]
            lit = O.render_ebs(v16, sc, tf, sat, D.INITIAL_STATE_CAMERA, W, W, st, rows=(y0, y1),
                               literal=0, **kw)[0]
            r = compare(spec[y0:y1], lit[y0:y1])
            r["seconds"] = round(time.time() - t1, 1)
            res[name] = r
            print(band, name, json.dumps(r), flush=True)
        out["bands"][band] = res
    os.makedirs(os.path.dirname(a.out), exist_ok=True)
    with open(a.out, "w") as f:
        json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
