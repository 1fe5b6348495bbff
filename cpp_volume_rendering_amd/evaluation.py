"""The evaluation sweep of cppvolrend (second half).

Mirrors ``ParameterSpace`` / ``ParameterRangeNumeric`` (cppvolrend/utils/
parameterspace.h, parameterspace.cpp) and the sweep loop of
``RenderingManager`` (renderingmanager.cpp:261-317, 805-857): every point of the
renderer's parameter space (``FillParameterSpace``) is rendered for a number of
frames, the time per frame is taken, the last frame's screenshot is saved as
``img/NNNN.png`` and one CSV row ``<values>,TimePerFrame (ms),FramesPerSecond,
"NNNN.png"`` is written to ``eval.csv``.  The reference's ``data/<n>b skipping``
folders hold sweeps of the isosurface renderers in this format; ``ssim.py``
compares such image folders as its ``eval.py`` does.

The frames render on the GPU through the renderer's own ``Redraw``; the time per
frame is wall time around ``frames`` redraws on one stream, synchronised at both
ends (the reference measures GLUT wall time over the same frames).
"""
from __future__ import annotations

import os
import struct
import time
import zlib
from typing import Callable, Optional

import numpy as np

# FillParameterSpace dimension name -> renderer attribute (the pointer each
# ParameterRangeFloat was built on: rc1prenderer.cpp:225-229,
# rc1custompisoadaptrenderer.cpp:349-355, rc1pisoadaptrenderer.cpp:191-197)
PARAMETER_ATTRIBUTES = {
    "StepSize": "m_u_step_size",
    "StepSizeSmall": "m_u_step_size_small",
    "StepSizeLarge": "m_u_step_size_large",
    "StepSizeRange": "m_u_step_size_range",
}


def std_to_string(v) -> str:
    """std::to_string of a float / double ("%f") or an int."""
    if isinstance(v, (int, np.integer)):
        return str(int(v))
    return "%f" % float(v)


class ParameterRange:
    """ParameterRangeNumeric<float>: [start, end] by incr, accumulated with += in
    float32; NumSteps = 1 + ceil((end - start) / incr) (parameterspace.h)."""

    def __init__(self, name: str, target, attr: str, start: float, end: float, incr: float,
                 dtype=np.float32):
        if start > end or incr <= 0:
            raise ValueError(f"{name}: bad range [{start}, {end}] by {incr}")
        self.name, self.target, self.attr = name, target, attr
        self.dtype = dtype
        self.start, self.end, self.incr = dtype(start), dtype(end), dtype(incr)
        self._saved = None

    @property
    def value(self):
        return self.dtype(getattr(self.target, self.attr))

    def _set(self, v):
        setattr(self.target, self.attr, float(v))

    def Start(self): self._set(self.start)
    def Incr(self): self._set(self.dtype(self.value + self.incr))
    def End(self) -> bool: return bool(self.value > self.end)

    def NumSteps(self) -> int:
        return 1 + int(np.ceil(self.dtype(self.end - self.start) / self.incr))

    def SaveCurrentValue(self): self._saved = getattr(self.target, self.attr)
    def RestoreCurrentValue(self): setattr(self.target, self.attr, self._saved)
    def GetValueStr(self) -> str: return std_to_string(self.value)


class ParameterSpace:
    """parameterspace.cpp: the last dimension varies fastest."""

    def __init__(self):
        self.dims: list[ParameterRange] = []

    @classmethod
    def from_renderer(cls, renderer) -> "ParameterSpace":
        pspace: dict = {}
        renderer.FillParameterSpace(pspace)
        ps = cls()
        for name, (lo, hi, step) in pspace.items():
            ps.AddParameterDimension(ParameterRange(name, renderer, PARAMETER_ATTRIBUTES[name],
                                                    lo, hi, step))
        return ps

    def AddParameterDimension(self, p: ParameterRange): self.dims.append(p)
    def ClearParameterDimensions(self): self.dims.clear()
    def GetNumDimensions(self) -> int: return len(self.dims)
    def GetDimensionName(self, i: int) -> str: return self.dims[i].name
    def GetDimensionValue(self, i: int) -> str: return self.dims[i].GetValueStr()

    def GetNumSamplePoints(self) -> int:
        if not self.dims:
            return 0
        n = 1
        for d in self.dims:
            n *= d.NumSteps()
        return n

    def StartEvaluation(self):
        for d in self.dims:
            d.SaveCurrentValue()
            d.Start()

    def EndEvaluation(self):
        for d in self.dims:
            d.RestoreCurrentValue()

    def IncrEvaluation(self) -> bool:
        dim = len(self.dims) - 1
        if dim < 0:
            return False
        while dim >= 0:
            self.dims[dim].Incr()
            if self.dims[dim].End():
                self.dims[dim].Start()
                dim -= 1
            else:
                break
        return dim >= 0


def write_png_rgb8(path: str, rgb_bottom_up: np.ndarray) -> None:
    """8-bit RGB PNG of a glReadPixels-order image (row 0 = bottom): the file's
    first row is the top of the screen, as the IM library writes it."""
    img = np.ascontiguousarray(rgb_bottom_up[::-1], dtype=np.uint8)
    h, w, _ = img.shape
    raw = b"".join(b"\x00" + img[y].tobytes() for y in range(h))

    def chunk(tag: bytes, data: bytes) -> bytes:
        return (struct.pack(">I", len(data)) + tag + data
                + struct.pack(">I", zlib.crc32(tag + data) & 0xFFFFFFFF))

    with open(path, "wb") as f:
        f.write(b"\x89PNG\r\n\x1a\n")
        f.write(chunk(b"IHDR", struct.pack(">IIBBBBB", w, h, 8, 2, 0, 0, 0)))
        f.write(chunk(b"IDAT", zlib.compress(raw, 6)))
        f.write(chunk(b"IEND", b""))


def run_evaluation(renderer, camera, out_dir: str, frames_per_sample: int = 100,
                   stream=None, on_sample: Optional[Callable[[int, list], None]] = None) -> str:
    """The sweep of RenderingManager (renderingmanager.cpp:805-857 start, :261-317
    per frame): returns the path of eval.csv.  The renderer must be Init()ed."""
    import torch
    ps = ParameterSpace.from_renderer(renderer)
    img_dir = os.path.join(out_dir, "img")
    os.makedirs(img_dir, exist_ok=True)
    csv_path = os.path.join(out_dir, "eval.csv")
    frames = max(1, min(int(frames_per_sample), 500))        # ImGui clamp (:813-815)
    dev_index = renderer._device_index
    s = stream if stream is not None else torch.cuda.current_stream(dev_index)
    with open(csv_path, "w", newline="") as csv:
        csv.write("".join(f"{ps.GetDimensionName(i)}," for i in range(ps.GetNumDimensions()))
                  + "TimePerFrame (ms),FramesPerSecond,ImageFile\n")
        ps.StartEvaluation()
        sample = 0
        try:
            while True:
                values = [ps.GetDimensionValue(i) for i in range(ps.GetNumDimensions())]
                torch.cuda.synchronize(dev_index)
                t0 = time.perf_counter()
                for _ in range(frames):
                    renderer.SetOutdated()                  # always redraw (:177-180)
                    renderer.PrepareRender(camera)
                    renderer.Redraw(s, count_samples=False)
                torch.cuda.synchronize(dev_index)
                tpf = (time.perf_counter() - t0) * 1e3 / frames
                name = "%04d.png" % sample
                write_png_rgb8(os.path.join(img_dir, name), renderer.Screenshot())
                csv.write("".join(f"{v}," for v in values)
                          + f"{std_to_string(tpf)},{std_to_string(1000.0 / tpf)},\"{name}\"\n")
                if on_sample:
                    on_sample(sample, values)
                if not ps.IncrEvaluation():
                    break
                sample += 1
        finally:
            ps.EndEvaluation()
    return csv_path
