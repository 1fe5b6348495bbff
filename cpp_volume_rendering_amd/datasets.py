"""Synthetic inputs for the benchmark and parity workloads.

The reference's own volume (data/raw/Bonsai.1.256x256x256.raw) is a missing
blob, so every workload is generated: analytic fields need no seed, the blob
field uses numpy.random.default_rng(12345).  Writers emit the reference's own
file grammars (.syn: reader.cpp:283-371, .raw: reader.cpp:162-225) so the
native readers are exercised end to end.
"""
from __future__ import annotations

import numpy as np

# data/#list_camera_states entry 0 ("Initial State") and data/#list_light_sources list 0
INITIAL_STATE_CAMERA = dict(eye=(256.0, 256.0, 512.0), center=(0.0, 0.0, 0.0), up=(0.0, 1.0, 0.0))
LIGHT_LIST0_POSITION = (-206.873, -51.0699, 557.011)

# data/tf1dcp/bonsai_01.tf1d control points (r, g, b, iso) and (alpha, iso)
BONSAI_TF_RGB = ((0.00, 0.90, 0.00, 0), (0.00, 0.90, 0.00, 58), (0.00, 0.00, 0.00, 59),
                 (0.70, 0.35, 0.00, 60), (0.90, 0.55, 0.00, 255))
BONSAI_TF_ALPHA = ((0.0, 0), (0.0, 35), (0.5, 40), (0.8, 255))


def voxel_scale(n: int) -> tuple:
    """Voxel size 512/N: every config shares the +-256 world box."""
    s = 512.0 / float(n)
    return (s, s, s)


def sphere_u8(n: int = 64) -> np.ndarray:
    """C1: radial ramp v = clamp(floor(255*(1 - d/(0.45 N))), 0, 255), d = |p + 0.5 - N/2|."""
    i = np.arange(n, dtype=np.float64) + 0.5 - n / 2.0
    z, y, x = np.meshgrid(i, i, i, indexing="ij")
    d = np.sqrt(x * x + y * y + z * z)
    v = np.floor(255.0 * (1.0 - d / (0.45 * n)))
    return np.clip(v, 0, 255).astype(np.uint8)


def marschner_lobb_u8(n: int, alpha: float = 0.25, fm: float = 6.0) -> np.ndarray:
    """Marschner-Lobb test field on [-1,1]^3 sampled at voxel centres, quantised to u8.

    rho = (1 - sin(pi z / 2) + alpha (1 + cos(2 pi fm cos(pi r / 2)))) / (2 (1 + alpha)),
    r = sqrt(x^2 + y^2).  Generated slab by slab to bound host memory at 1024^3.
    """
    c = (np.arange(n, dtype=np.float64) + 0.5) / n * 2.0 - 1.0
    out = np.empty((n, n, n), dtype=np.uint8)
    yy, xx = np.meshgrid(c, c, indexing="ij")
    r = np.sqrt(xx * xx + yy * yy)
    ring = alpha * (1.0 + np.cos(2.0 * np.pi * fm * np.cos(np.pi * r / 2.0)))
    for k in range(n):
        rho = (1.0 - np.sin(np.pi * c[k] / 2.0) + ring) / (2.0 * (1.0 + alpha))
        out[k] = np.clip(np.rint(255.0 * rho), 0, 255).astype(np.uint8)
    return out


def blobs_u8(n: int, count: int = 24, seed: int = 12345) -> np.ndarray:
    """Sparse Gaussian blobs (mostly empty space) from default_rng(seed)."""
    rng = np.random.default_rng(seed)
    centres = rng.uniform(0.15, 0.85, size=(count, 3)) * n
    radii = rng.uniform(0.03, 0.09, size=count) * n
    amps = rng.uniform(120, 255, size=count)
    out = np.zeros((n, n, n), dtype=np.float32)
    c = np.arange(n, dtype=np.float32) + 0.5
    for (cx, cy, cz), rad, amp in zip(centres, radii, amps):
        lo = np.maximum(np.floor(np.array([cz, cy, cx]) - 3 * rad).astype(int), 0)
        hi = np.minimum(np.ceil(np.array([cz, cy, cx]) + 3 * rad).astype(int), n)
        z = c[lo[0]:hi[0], None, None] - cz
        y = c[None, lo[1]:hi[1], None] - cy
        x = c[None, None, lo[2]:hi[2]] - cx
        g = amp * np.exp(-(x * x + y * y + z * z) / (2.0 * rad * rad))
        out[lo[0]:hi[0], lo[1]:hi[1], lo[2]:hi[2]] += g.astype(np.float32)
    return np.clip(np.rint(out), 0, 255).astype(np.uint8)


def write_syn(path: str, vol: np.ndarray) -> None:
    """Write a u8 volume in the .syn grammar, listing every voxel (kind 0 lines)."""
    d, h, w = vol.shape
    zz, yy, xx = np.meshgrid(np.arange(d), np.arange(h), np.arange(w), indexing="ij")
    rows = np.stack([np.zeros(vol.size, dtype=np.int64), xx.ravel(), yy.ravel(), zz.ravel(),
                     vol.ravel().astype(np.int64)], axis=1)
    with open(path, "w") as f:
        f.write(f"{w} {h} {d}\n")
        np.savetxt(f, rows, fmt="%d")


def raw_name(stem: str, vol: np.ndarray) -> str:
    d, h, w = vol.shape
    return f"{stem}.{vol.dtype.itemsize}.{w}x{h}x{d}.raw"


def write_raw(path: str, vol: np.ndarray) -> None:
    np.ascontiguousarray(vol).tofile(path)
