import ctypes, sys
sys.path.insert(0, '.')
import torch
from cpp_volume_rendering_amd import _native as N, datasets as D
from cpp_volume_rendering_amd.renderer import Camera, Device, build_tf_rgbt, make_frame
for field in ("ml", "blobs"):
    for sh in (2, 3, 4, 5):
        dev = Device(0)
        L = N.lib()
        L.cvr_set_option(dev.handle, b"macro", sh)
        vol = D.marschner_lobb_u8(512) if field == "ml" else D.blobs_u8(512)
        dev.set_volume(vol, D.voxel_scale(512))
        dev.set_transfer_function(build_tf_rgbt(D.BONSAI_TF_RGB, D.BONSAI_TF_ALPHA))
        frame = make_frame(Camera(**D.INITIAL_STATE_CAMERA), 64, 64)
        p = N.Rc1passParams()
        img = torch.zeros((64, 64, 4), dtype=torch.float32, device="cuda")
        out = N.Output(img.data_ptr(), None, None, 1)
        N.check(L.cvr_render_rc1pass(dev.handle, ctypes.byref(frame), ctypes.byref(p), ctypes.byref(out)), "r", dev.handle)
        torch.cuda.synchronize()
        print(field, sh, L.cvr_get_option(dev.handle, b"occ_empty_permille"))
        dev.close()
