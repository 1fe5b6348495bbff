"""Time the EBS frame (cvr_render_extbsd, kernel time via kernel_timing) at one size for
several shader settings, to see where the time goes.  Usage: python tools/ebs_probe.py [N]"""
import ctypes, os, sys
import numpy as np
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from cpp_volume_rendering_amd import _native as N
from cpp_volume_rendering_amd import datasets as D
from cpp_volume_rendering_amd.renderer import Camera, Device, build_ext_lut, build_tf_rgbt, make_frame

n = int(sys.argv[1]) if len(sys.argv) > 1 else 512
W = int(sys.argv[2]) if len(sys.argv) > 2 else 1024
dev = Device(0)
dev.set_volume(D.marschner_lobb_u8(n), D.voxel_scale(n))
dev.set_transfer_function(build_tf_rgbt(D.BONSAI_TF_RGB, D.BONSAI_TF_ALPHA))
dev.set_extinction_sat(build_ext_lut(D.BONSAI_TF_RGB, D.BONSAI_TF_ALPHA))
L = N.lib()
frame = make_frame(Camera(**D.INITIAL_STATE_CAMERA), W, W)
img = torch.zeros((W, W, 4), dtype=torch.float32, device="cuda")
tot = torch.zeros(1, dtype=torch.int64, device="cuda")
s = torch.cuda.current_stream()
dev.set_stream(s.cuda_stream)


def params(**kw):
    p = N.EbsParams()
    p.ka, p.kd, p.ks, p.shininess = 0.5, 0.5, 0.8, 30.0
    p.ispecular[:] = [1, 1, 1]
    p.light_pos[:] = list(D.LIGHT_LIST0_POSITION)
    p.light_forward[:] = [-0.346883, -0.0856335, 0.933991]
    p.apply_occlusion, p.occlusion_shells, p.occlusion_radius = 1, 15, 1.0
    p.apply_shadow, p.shadow_type = 1, 0
    p.shadow_cone_angle_deg, p.shadow_sample_interval = 1.0, 2.0
    p.shadow_initial_step, p.shadow_ui_weight, p.shadow_max_distance = 2.0, 1.0, 0.0
    for k, v in kw.items():
        setattr(p, k, v)
    return p


cases = {"default": {}, "ao_only": dict(apply_shadow=0), "shadow_only": dict(apply_occlusion=0),
         "ao_3shells": dict(apply_shadow=0, occlusion_shells=3),
         "shadow_short": dict(apply_occlusion=0, shadow_max_distance=40.0)}
res = {}
for name, kw in cases.items():
    p = params(**kw)
    N.check(L.cvr_set_option(dev.handle, b"shade_counters", 1), "opt")
    tot.zero_()
    out = N.Output(img.data_ptr(), None, tot.data_ptr(), 1)
    N.check(L.cvr_render_extbsd(dev.handle, ctypes.byref(frame), ctypes.byref(p), ctypes.byref(out)), "r", dev.handle)
    sh = (ctypes.c_uint64 * 3)()
    N.check(L.cvr_read_shade_counters(dev.handle, sh), "sh", dev.handle)
    N.check(L.cvr_set_option(dev.handle, b"shade_counters", 0), "opt")
    N.check(L.cvr_set_option(dev.handle, b"kernel_timing", 3), "opt")
    for _ in range(3):
        N.check(L.cvr_render_extbsd(dev.handle, ctypes.byref(frame), ctypes.byref(p), ctypes.byref(N.Output(img.data_ptr(), None, None, 1))), "r", dev.handle)
    torch.cuda.synchronize()
    kt = (ctypes.c_float * 3)(); nk = ctypes.c_int()
    N.check(L.cvr_read_kernel_times(dev.handle, kt, 3, ctypes.byref(nk)), "kt", dev.handle)
    N.check(L.cvr_set_option(dev.handle, b"kernel_timing", 0), "opt")
    ms = float(np.median(kt[:nk.value]))
    res[name] = {"ms": round(ms, 3), "samples": int(tot.item()), "shaded": sh[0], "fetches": sh[2],
                 "Gfetch_s": round(sh[2] / ms / 1e6, 1)}
    print(name, res[name], flush=True)
