"""The kernels normalise vectors with a short exact sequence instead of the IEEE
division and square-root operators (cvr_device.h: rcp_cr = hardware reciprocal +
one fma Newton step, sqrt_cr_normal = the compiler's own correctly rounded sqrt
without its tiny-input scaling) and take pow without branches (cvr_powf_nb).
cvr_selftest_arith checks both against the IEEE
operators for EVERY float of the ranges the kernels use them on (every
significand of every exponent), on the device, bit for bit — so the shortcut
cannot change a pixel; the renderers' GPU == oracle tests check it end to end."""
import ctypes

import numpy as np
import pytest

from cpp_volume_rendering_amd import _native as N
from cpp_volume_rendering_amd.renderer import Device

pytestmark = pytest.mark.gpu


def test_rcp_and_sqrt_shortcuts_exact_everywhere():
    import torch
    assert torch.cuda.is_available(), "GPU tests need a HIP device"
    dev = Device(0)
    try:
        out = np.full(3, 99, np.uint64)
        N.check(N.lib().cvr_selftest_arith(dev.handle, out.ctypes.data_as(
            ctypes.POINTER(ctypes.c_uint64))), "cvr_selftest_arith", dev.handle)
    finally:
        dev.close()
    assert int(out[0]) == 0, f"rcp_cr differs from 1/b on {int(out[0])} floats"
    assert int(out[1]) == 0, f"sqrt_cr_normal differs from sqrtf on {int(out[1])} floats"
    assert int(out[2]) == 0, f"cvr_powf_nb differs from cvr_powf on {int(out[2])} arguments"
