"""Image parity metric of the reference's evaluation (eval.py:12-64).

eval.py scores renders with ImageMagick's `magick compare -metric SSIM`.  That
metric is the Gaussian-window SSIM (sigma 1.5, 11x11 window, i.e. a Gaussian
truncated at 3.5 sigma; K1 = 0.01, K2 = 0.03, L = 255) averaged over the R, G, B
channels.  This restatement reproduces the reference's own
ssim_comparison_results.xlsx to < 1e-6 (tests/test_ssim.py, fixtures in
tests/golden/ssim/).  Images are compared as the RGB8 screenshot the reference
writes: the premultiplied RGBA frame composited over the white clear colour
(renderingmanager.cpp:103-112, 476-492; renderer.composite_over_white).
"""
from __future__ import annotations

import numpy as np
from scipy.ndimage import gaussian_filter

K1, K2, L = 0.01, 0.03, 255.0
SIGMA, TRUNCATE = 1.5, 3.5


def ssim_channel(a: np.ndarray, b: np.ndarray) -> float:
    a = a.astype(np.float64)
    b = b.astype(np.float64)
    c1, c2 = (K1 * L) ** 2, (K2 * L) ** 2

    def blur(x):
        return gaussian_filter(x, SIGMA, truncate=TRUNCATE, mode="reflect")

    mu_a, mu_b = blur(a), blur(b)
    saa = blur(a * a) - mu_a * mu_a
    sbb = blur(b * b) - mu_b * mu_b
    sab = blur(a * b) - mu_a * mu_b
    m = ((2 * mu_a * mu_b + c1) * (2 * sab + c2)) / ((mu_a ** 2 + mu_b ** 2 + c1) * (saa + sbb + c2))
    return float(m.mean())


def ssim_rgb8(a: np.ndarray, b: np.ndarray) -> float:
    """SSIM of two (H, W, >=3) uint8 images, mean over R, G, B."""
    if a.shape[:2] != b.shape[:2]:
        raise ValueError("images differ in size")
    return float(np.mean([ssim_channel(a[..., c], b[..., c]) for c in range(3)]))


def ssim_rgba(a: np.ndarray, b: np.ndarray) -> float:
    """SSIM of two premultiplied float RGBA frames as their screenshots (over white)."""
    from .renderer import composite_over_white
    return ssim_rgb8(composite_over_white(a), composite_over_white(b))
