"""Locate non-finite pixels of the EBS frame (diagnostics)."""
import ctypes, sys, os
import numpy as np
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from cpp_volume_rendering_amd import _native as N
from cpp_volume_rendering_amd import datasets as D
from cpp_volume_rendering_amd.renderer import Camera, Device, make_frame, build_ext_lut, build_tf_rgbt

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
W = int(sys.argv[2]) if len(sys.argv) > 2 else 1024
dev = Device(0)
vol = D.marschner_lobb_u8(n)
dev.set_volume(vol, D.voxel_scale(n))
dev.set_transfer_function(build_tf_rgbt(D.BONSAI_TF_RGB, D.BONSAI_TF_ALPHA))
dev.set_extinction_sat(build_ext_lut(D.BONSAI_TF_RGB, D.BONSAI_TF_ALPHA))
for occ, sh in [(1, 1), (1, 0), (0, 1)]:
    p = N.EbsParams()
    p.ka, p.kd, p.ks, p.shininess = 0.5, 0.5, 0.8, 30.0
    p.ispecular[:] = [1, 1, 1]
    p.light_pos[:] = list(D.LIGHT_LIST0_POSITION)
    p.light_forward[:] = [-0.346883, -0.0856335, 0.933991]
    p.apply_occlusion, p.occlusion_shells, p.occlusion_radius = occ, 15, 1.0
    p.apply_shadow, p.shadow_type = sh, 0
    p.shadow_cone_angle_deg, p.shadow_sample_interval, p.shadow_initial_step = 1.0, 2.0, 2.0
    p.shadow_ui_weight = 1.0
    img = np.zeros((W, W, 4), np.float32)
    out = N.Output(img.ctypes.data, None, None, 0)
    fr = make_frame(Camera(**D.INITIAL_STATE_CAMERA), W, W)
    N.check(N.lib().cvr_render_extbsd(dev.handle, ctypes.byref(fr), ctypes.byref(p), ctypes.byref(out)), "ebs", dev.handle)
    bad = np.argwhere(~np.isfinite(img).all(-1))
    print(f"occ {occ} shadow {sh}: {len(bad)} non-finite pixels; first {bad[:5].tolist()}",
          img[tuple(bad[0])] if len(bad) else "")
dev.close()
