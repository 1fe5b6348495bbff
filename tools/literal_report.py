#!/usr/bin/env python3
"""Prints the CVR-SPEC vs literal-GLSL distances that tests/test_literal.py asserts
(BASELINE.md gate: |dRGBA| <= 2e-3 for >= 99.9 % of pixels, max 2e-2, SSIM >= 0.99)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
import oracle as O  # noqa: E402
import test_literal as T  # noqa: E402

from cpp_volume_rendering_amd import datasets as D  # noqa: E402

t = O.tf_table_double(D.BONSAI_TF_RGB, D.BONSAI_TF_ALPHA)
tables = (t, O.tf_rgbt(t), O.tf_rgbt(t, extinction_input=True))
out = {}
vol, sc, v16, st = T._vol(O, 512)
spec = O.render_rc1pass(v16, sc, tables[1], T.CAM, 1024, 1024, st)[0]
for w in (0, 8):
    lit = O.render_rc1pass(v16, sc, tables[1], T.CAM, 1024, 1024, st, literal=w)[0]
    out[f"rc1pass_512_1024_w{w}"] = T.gate(spec, lit)
vol, sc, v16, st = T._vol(O, 128)
g = O.gradient(vol, "fd")
kw = dict(grad=g, phong=True, light=D.LIGHT_LIST0_POSITION)
a = O.render_rc1pass(v16, sc, tables[1], T.CAM, 512, 512, st, **kw)[0]
b = O.render_rc1pass(v16, sc, tables[1], T.CAM, 512, 512, st, literal=0, **kw)[0]
out["phong_128_512"] = T.gate(a, b)
print(json.dumps(out, indent=1))
