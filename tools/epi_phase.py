"""Time the LPT-order epilogue truncated after each phase (diagnostics)."""
import ctypes, os, sys, subprocess
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from cpp_volume_rendering_amd import _native as N, datasets as D
from cpp_volume_rendering_amd.renderer import Camera, Device, build_tf_rgbt, make_frame
stop = int(sys.argv[1])
dev = Device(0)
L = N.lib()
dev.set_volume(D.marschner_lobb_u8(512), D.voxel_scale(512))
dev.set_transfer_function(build_tf_rgbt(D.BONSAI_TF_RGB, D.BONSAI_TF_ALPHA))
frame = make_frame(Camera(**D.INITIAL_STATE_CAMERA), 1024, 1024)
p = N.Rc1passParams()
img = torch.zeros((1024, 1024, 4), dtype=torch.float32, device="cuda")
out = N.Output(img.data_ptr(), None, None, 1)
for i in range(30):
    if i == 0:
        L.cvr_set_option(dev.handle, b"async_order", 0)   # serial: durations are not contended
    if i == 6:
        L.cvr_set_option(dev.handle, b"debug_epi_stop", stop)
    N.check(L.cvr_render_rc1pass(dev.handle, ctypes.byref(frame), ctypes.byref(p), ctypes.byref(out)), "r", dev.handle)
torch.cuda.synchronize()
