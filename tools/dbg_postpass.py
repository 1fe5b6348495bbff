import sys, os
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "."))
import numpy as np, torch, ctypes
import oracle as O
from cpp_volume_rendering_amd import _native as N
from cpp_volume_rendering_amd.renderer import Device
dev = Device(0)
rng = np.random.default_rng(24)
for (sw, sh) in [(72, 56), (16, 16), (40, 16)]:
    frame = (rng.random((sh*2, sw*2, 4)) * 1.5 - 0.25).astype(np.float16)
    f = torch.from_numpy(frame.copy()).cuda()
    out = torch.zeros((sh, sw, 4), dtype=torch.float16, device="cuda")
    dev.set_stream(torch.cuda.current_stream().cuda_stream)
    N.check(N.lib().cvr_multiscale_filter(dev.handle, 2, 4, f.data_ptr(), sw*2, sh*2, out.data_ptr(), sw, sh), "f", dev.handle)
    torch.cuda.synchronize()
    got = out.cpu().numpy()
    want = O.multiscale_filter(2, 4, frame.copy(), sw, sh)
    # also mode-2 hat (no digital filter) to check the downscale itself
    d = np.argwhere(got.view(np.uint16) != want.view(np.uint16))
    print(sw, sh, "ndiff", len(d), d[:8].tolist())
    for (y, x, c) in d[:4].tolist():
        print(y, x, c, float(got[y, x, c]), float(want[y, x, c]))
