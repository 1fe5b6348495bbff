"""The image metric of the reference's evaluation (eval.py: ImageMagick
`compare -metric SSIM`), restated in cpp_volume_rendering_amd/ssim.py and pinned
against the values the reference stored in ssim_comparison_results.xlsx for its
own image pairs (fixtures copied by tests/golden/make_ssim_fixtures.py)."""
import json
import os

import numpy as np
import pytest

from cpp_volume_rendering_amd.ssim import ssim_rgb8, ssim_rgba


@pytest.fixture(scope="module")
def pairs(golden_dir):
    d = os.path.join(golden_dir, "ssim")
    with open(os.path.join(d, "pairs.json")) as f:
        return d, json.load(f)["pairs"]


def _png(path):
    from PIL import Image
    return np.asarray(Image.open(path).convert("RGB"))


def test_ssim_reproduces_reference_eval(pairs):
    d, ps = pairs
    assert len(ps) == 3
    for p in ps:
        s = ssim_rgb8(_png(os.path.join(d, p["a"])), _png(os.path.join(d, p["b"])))
        assert abs(s - p["ssim"]) < 1e-6, (p, s)


def test_ssim_identity_and_order(pairs):
    d, ps = pairs
    a = _png(os.path.join(d, ps[0]["a"]))
    b = _png(os.path.join(d, ps[0]["b"]))
    assert ssim_rgb8(a, a) == pytest.approx(1.0, abs=1e-12)
    assert ssim_rgb8(a, b) == pytest.approx(ssim_rgb8(b, a), abs=1e-12)


def test_ssim_rgba_composites_over_white():
    rgba = np.zeros((32, 32, 4), np.float32)
    rgba[8:24, 8:24] = (0.2, 0.4, 0.1, 0.8)
    assert ssim_rgba(rgba, rgba) == pytest.approx(1.0, abs=1e-12)
    other = rgba.copy()
    other[8:24, 8:24, 3] = 0.2
    assert ssim_rgba(rgba, other) < 0.99
