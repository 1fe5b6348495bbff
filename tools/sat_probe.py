"""Time the EBS SAT build (cvr_set_extinction_sat) for several z-chunk sizes."""
import ctypes, os, sys, time
import numpy as np
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from cpp_volume_rendering_amd import _native as N
from cpp_volume_rendering_amd import datasets as D
from cpp_volume_rendering_amd.renderer import Device, build_ext_lut

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
chunks = [int(v) for v in (sys.argv[2] if len(sys.argv) > 2 else "16,32,64").split(",")]
dev = Device(0)
dev.set_volume(D.marschner_lobb_u8(n), D.voxel_scale(n))
lut = build_ext_lut(D.BONSAI_TF_RGB, D.BONSAI_TF_ALPHA)
ref = None
for c in chunks + chunks:
    N.check(N.lib().cvr_set_option(dev.handle, b"sat_chunk", c), "opt")
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    dev.set_extinction_sat(lut)
    ms = (time.perf_counter() - t0) * 1e3
    # compare a slab of the float SAT across chunk sizes (must be identical)
    dims = (ctypes.c_int * 3)()
    sat = dev.extinction_sat() if n <= 512 else None
    same = None
    if sat is not None:
        if ref is None:
            ref = sat
        same = bool(np.array_equal(sat.view(np.uint32), ref.view(np.uint32)))
    print(f"N={n} chunk={c}: {ms:.1f} ms  identical={same}", flush=True)
dev.close()
