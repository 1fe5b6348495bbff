"""Host-side mirror of cppvolrend's renderer-plugin API over the C-ABI.

The classes follow the reference names and call sequence so that code (and
tests) read like the reference:

    RenderingManager::InitData  -> DataManager.read_* / RenderingParameters
    BaseVolumeRenderer          -> BaseVolumeRenderer   (cppvolrend/volrenderbase.h:25-96)
    RayCasting1Pass             -> RayCasting1Pass      (cppvolrend/structured/rc1pass/rc1prenderer.*)
    RC1PConeTracingDirOcclusionShading
                                -> RC1PConeTracingDirOcclusionShading
                                                        (cppvolrend/structured/rc1pdosct/dosrcrenderer.*)
    RC1PExtinctionBasedShading  -> RC1PExtinctionBasedShading
                                                        (cppvolrend/structured/rc1pextbsd/ebsrenderer.*)

Per frame: ``PrepareRender(camera)`` (calls ``Update`` when outdated) then
``Redraw()``, exactly as RenderingManager::Display does
(cppvolrend/renderingmanager.cpp:199-208).  Every call goes to libcvr.so; the
image lives in device memory (a torch tensor on the renderer's device).
"""
from __future__ import annotations

import ctypes
import math
from dataclasses import dataclass, field
from typing import Optional

import numpy as np
import torch

from . import _native as N

STRUCTURED = "STRUCTURED"   # vis::GRID_VOLUME_DATA_TYPE::STRUCTURED


@dataclass
class Camera:
    """vis::CameraData subset used by the ray generator (libs/vis_utils/camera.cpp)."""
    eye: tuple = (256.0, 256.0, 512.0)       # data/#list_camera_states "Initial State"
    center: tuple = (0.0, 0.0, 0.0)
    up: tuple = (0.0, 1.0, 0.0)
    fovy_deg: float = 45.0                   # camera.cpp:25
    aspect: float = 0.0                      # 0: width / height (Camera::UpdateAspectRatio)

    def to_c(self) -> N.Camera:
        c = N.Camera()
        c.eye[:] = [float(v) for v in self.eye]
        c.center[:] = [float(v) for v in self.center]
        c.up[:] = [float(v) for v in self.up]
        c.fovy_deg = float(self.fovy_deg)
        c.aspect = float(self.aspect)
        return c

    def GetEye(self):
        return self.eye


@dataclass
class RenderingParameters:
    """vis::RenderingParameters defaults (libs/volvis_utils/renderingparameters.cpp:17-32)."""
    screen_width: int = 768
    screen_height: int = 768
    blinnphong_ka: float = 0.5
    blinnphong_kd: float = 0.5
    blinnphong_ks: float = 0.8
    blinnphong_shininess: float = 30.0
    light_position: tuple = (-206.873, -51.0699, 557.011)   # data/#list_light_sources list 0
    light_specular: tuple = (1.0, 1.0, 1.0)                 # lightsourcelist.cpp:24
    # the same light's camera frame and spot angle (LightSourceData, lightsourcelist.cpp:107-133)
    light_forward: tuple = (-0.346883, -0.0856335, 0.933991)
    light_up: tuple = (-0.0298143, 0.996327, 0.0802758)
    light_right: tuple = (0.937434, -0.0, 0.348162)
    spot_light_angle: float = 20.0
    camera: Camera = field(default_factory=Camera)

    def GetScreenWidth(self): return self.screen_width
    def GetScreenHeight(self): return self.screen_height
    def GetCamera(self): return self.camera
    def GetBlinnPhongLightingPosition(self): return self.light_position
    def GetLightSourceSpecular(self): return self.light_specular
    def GetBlinnPhongLightSourceCameraForward(self): return self.light_forward
    def GetBlinnPhongLightSourceCameraUp(self): return self.light_up
    def GetBlinnPhongLightSourceCameraRight(self): return self.light_right
    def GetSpotLightMaxAngle(self): return self.spot_light_angle

    def SetLight(self, light: "N.Light"):
        self.light_position = tuple(light.position)
        self.light_forward = tuple(light.forward)
        self.light_up = tuple(light.up)
        self.light_right = tuple(light.right)
        self.spot_light_angle = float(light.spot_angle_deg)


class DataManager:
    """vis::DataManager subset: the current structured volume, its TF and gradient type."""

    def __init__(self):
        self.volume: Optional[np.ndarray] = None    # (D, H, W) u8/u16, x fastest
        self.scale = (1.0, 1.0, 1.0)
        self.tf_rgbt: Optional[np.ndarray] = None  # (n, 4) float32: r, g, b, extinction
        self.tf_rgba: Optional[np.ndarray] = None  # (n, 4) float32: r, g, b, opacity
        self.ext_lut: Optional[np.ndarray] = None  # GetExtN per voxel value (EBS SAT cells)
        self.gradient_type = N.GRADIENT_NONE        # datamanager.cpp:27 (NONE by default)
        self.name = ""

    # -- inputs --------------------------------------------------------------
    def SetVolume(self, voxels: np.ndarray, scale=(1.0, 1.0, 1.0), name: str = ""):
        if voxels.ndim != 3 or voxels.dtype not in (np.uint8, np.uint16):
            raise ValueError("volume must be a (D, H, W) uint8/uint16 array")
        self.volume = np.ascontiguousarray(voxels)
        self.scale = tuple(float(s) for s in scale)
        self.name = name

    def SetTransferFunction(self, rgbt: np.ndarray, rgba: Optional[np.ndarray] = None):
        """rgbt: GenerateTexture_1D_RGBt (alpha as extinction, what the march samples);
        rgba: GenerateTexture_1D_RGBA (alpha as opacity, what the extinction volume of
        the occlusion renderer filters; transferfunction1d.cpp:58-87)."""
        rgbt = np.ascontiguousarray(rgbt, dtype=np.float32)
        if rgbt.ndim != 2 or rgbt.shape[1] != 4:
            raise ValueError("transfer function must be (n, 4) r, g, b, extinction")
        self.tf_rgbt = rgbt
        if rgba is not None:
            rgba = np.ascontiguousarray(rgba, dtype=np.float32)
            if rgba.shape != rgbt.shape:
                raise ValueError("RGBA transfer function must match the RGBt one")
        self.tf_rgba = rgba

    def ReadVolume(self, path: str, scale=None):
        """.raw (name.<bytes>.<W>x<H>x<D>.raw), .syn or .pvm, like
        VolumeReader::ReadStructuredVolume (reader.cpp:24-60)."""
        L = N.lib()
        w, h, d, b = ctypes.c_int(), ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
        bp = path.encode()
        if path.endswith(".raw"):
            N.check(L.cvr_read_raw(bp, None, 0, w, h, d, b), "cvr_read_raw")
            dt = np.uint8 if b.value == 1 else np.uint16
            vox = np.empty((d.value, h.value, w.value), dtype=dt)
            N.check(L.cvr_read_raw(bp, vox.ctypes.data, vox.nbytes, w, h, d, b), "cvr_read_raw")
        elif path.endswith(".syn"):
            N.check(L.cvr_read_syn(bp, None, 0, w, h, d), "cvr_read_syn")
            vox = np.empty((d.value, h.value, w.value), dtype=np.uint8)
            N.check(L.cvr_read_syn(bp, vox.ctypes.data, vox.nbytes, w, h, d), "cvr_read_syn")
        elif path.endswith(".pvm"):
            # VolumeReader::readpvm (reader.cpp:100-159): the PVM2/3 spacing is the scale
            sc = (ctypes.c_float * 3)()
            N.check(L.cvr_read_pvm(bp, None, 0, w, h, d, b, sc), "cvr_read_pvm")
            dt = np.uint8 if b.value == 1 else np.uint16
            vox = np.empty((d.value, h.value, w.value), dtype=dt)
            N.check(L.cvr_read_pvm(bp, vox.ctypes.data, vox.nbytes, w, h, d, b, sc),
                    "cvr_read_pvm")
            scale = scale or tuple(float(v) for v in sc)
        else:
            raise ValueError(f"unsupported volume format: {path}")
        self.SetVolume(vox, scale or (1.0, 1.0, 1.0), name=path)

    def SetExtinctionTable(self, ext_lut: np.ndarray):
        """GetExtN(v / (2^bits - 1)) for every voxel value (build_ext_lut)."""
        self.ext_lut = np.ascontiguousarray(ext_lut, dtype=np.float32)

    def ReadTransferFunction(self, path: str):
        self.SetTransferFunction(read_tf1d(path))

    # -- accessors (reference names) -----------------------------------------
    def GetCurrentStructuredVolume(self): return self.volume
    def GetCurrentTransferFunction(self): return self.tf_rgbt

    def SetGradientType(self, gtype: int):
        self.gradient_type = int(gtype)


def read_tf1d(path: str) -> np.ndarray:
    L = N.lib()
    n = ctypes.c_int()
    N.check(L.cvr_read_tf1d(path.encode(), None, n), "cvr_read_tf1d")
    out = np.empty((n.value, 4), dtype=np.float32)
    N.check(L.cvr_read_tf1d(path.encode(), N.fptr(out), n), "cvr_read_tf1d")
    return out


def build_ext_lut(rgb_cp, alpha_cp, bytes_per_voxel: int = 1, max_density: int = 255,
                  extinction_input: bool = False) -> np.ndarray:
    """TransferFunction1D::GetExtN of every voxel value: the EBS SAT cell values."""
    rgb = np.ascontiguousarray(np.asarray(rgb_cp, dtype=np.float64).reshape(-1, 4))
    a = np.ascontiguousarray(np.asarray(alpha_cp, dtype=np.float64).reshape(-1, 2))
    out = np.empty(256 if bytes_per_voxel == 1 else 65536, dtype=np.float32)
    N.check(N.lib().cvr_tf1d_ext_lut(N.dptr(rgb), rgb.shape[0], N.dptr(a), a.shape[0],
                                     max_density, int(extinction_input), int(bytes_per_voxel),
                                     N.fptr(out)), "cvr_tf1d_ext_lut")
    return out


def build_tf_rgbt(rgb_cp, alpha_cp, max_density: int = 255, extinction_input: bool = False):
    """TransferFunction1D control points -> GenerateTexture_1D_RGBt data (float, pre-fp16)."""
    rgb = np.ascontiguousarray(np.asarray(rgb_cp, dtype=np.float64).reshape(-1, 4))
    a = np.ascontiguousarray(np.asarray(alpha_cp, dtype=np.float64).reshape(-1, 2))
    out = np.empty((max_density + 1, 4), dtype=np.float32)
    N.check(N.lib().cvr_tf1d_build_rgbt(N.dptr(rgb), rgb.shape[0], N.dptr(a), a.shape[0],
                                        max_density, int(extinction_input), N.fptr(out)),
            "cvr_tf1d_build_rgbt")
    return out


def read_camera_state(path: str, index: int = 0) -> Camera:
    c = N.Camera()
    name = ctypes.create_string_buffer(256)
    cnt = ctypes.c_int()
    N.check(N.lib().cvr_read_camera_state(path.encode(), index, c, name, 256, cnt),
            "cvr_read_camera_state")
    return Camera(tuple(c.eye), tuple(c.center), tuple(c.up), c.fovy_deg, 0.0)


def read_light(path: str, list_index: int = 0, light: int = 0) -> N.Light:
    out = N.Light()
    cnt = ctypes.c_int()
    N.check(N.lib().cvr_read_light(path.encode(), list_index, light, ctypes.byref(out), cnt),
            "cvr_read_light")
    return out


def read_light_position(path: str, list_index: int = 0, light: int = 0):
    pos = (ctypes.c_float * 3)()
    cnt = ctypes.c_int()
    N.check(N.lib().cvr_read_light_position(path.encode(), list_index, light, pos, cnt),
            "cvr_read_light_position")
    return tuple(pos)


class Device:
    """One libcvr context (cvr_ctx) bound to a HIP device; owns all device data."""

    def __init__(self, device: int = 0, devices=None):
        """devices (a list of device indices): one context over all of them in this
        process (cvr_create_group: every frame split over the devices and gathered
        on devices[0], which is also `device`)."""
        self._h = ctypes.c_void_p()
        if devices is not None:
            devs = [int(d) for d in devices]
            self.device = devs[0]
            arr = (ctypes.c_int * len(devs))(*devs)
            N.check(N.lib().cvr_create_group(arr, len(devs), ctypes.byref(self._h)),
                    "cvr_create_group")
        else:
            self.device = device
            N.check(N.lib().cvr_create(device, ctypes.byref(self._h)), "cvr_create")

    @property
    def group_size(self) -> int:
        return int(N.lib().cvr_group_size(self.handle))

    @property
    def handle(self):
        if not self._h:
            raise N.CvrError(N.CVR_ERR_STATE, "Device", "context destroyed")
        return self._h

    def close(self):
        if self._h:
            N.lib().cvr_destroy(self._h)
            self._h = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def set_stream(self, stream: Optional[int]):
        N.check(N.lib().cvr_set_stream(self.handle, stream), "cvr_set_stream", self.handle)

    def synchronize(self):
        N.check(N.lib().cvr_synchronize(self.handle), "cvr_synchronize", self.handle)

    def set_volume(self, voxels: np.ndarray, scale):
        vox = np.ascontiguousarray(voxels)
        d, h, w = vox.shape
        sc = np.asarray(scale, dtype=np.float32)
        N.check(N.lib().cvr_set_volume(self.handle, vox.ctypes.data, vox.dtype.itemsize, w, h, d,
                                       N.fptr(sc)), "cvr_set_volume", self.handle)

    def set_volume_device(self, voxels: torch.Tensor, scale):
        if not voxels.is_cuda or not voxels.is_contiguous():
            raise ValueError("expected a contiguous device tensor")
        d, h, w = voxels.shape
        sc = np.asarray(scale, dtype=np.float32)
        N.check(N.lib().cvr_set_volume_device(self.handle, voxels.data_ptr(),
                                              voxels.element_size(), w, h, d, N.fptr(sc)),
                "cvr_set_volume_device", self.handle)

    def set_transfer_function(self, rgbt: np.ndarray):
        t = np.ascontiguousarray(rgbt, dtype=np.float32)
        N.check(N.lib().cvr_set_transfer_function(self.handle, N.fptr(t), t.shape[0]),
                "cvr_set_transfer_function", self.handle)

    def set_gradient(self, mode: int):
        N.check(N.lib().cvr_set_gradient(self.handle, int(mode)), "cvr_set_gradient", self.handle)

    def set_extinction_volume(self, tf_rgba: np.ndarray, res=(128, 128, 128), sigma0: float = 1.0):
        t = np.ascontiguousarray(tf_rgba, dtype=np.float32)
        r = (ctypes.c_int * 3)(*[int(v) for v in res])
        N.check(N.lib().cvr_set_extinction_volume(self.handle, N.fptr(t), t.shape[0], r,
                                                  float(sigma0)),
                "cvr_set_extinction_volume", self.handle)

    def set_extinction_sat(self, ext_lut: np.ndarray):
        t = np.ascontiguousarray(ext_lut, dtype=np.float32)
        N.check(N.lib().cvr_set_extinction_sat(self.handle, N.fptr(t), t.shape[0]),
                "cvr_set_extinction_sat", self.handle)

    def extinction_sat(self) -> np.ndarray:
        """The float SAT as a (D+2, H+2, W+2) array."""
        L = N.lib()
        dims = (ctypes.c_int * 3)()
        N.check(L.cvr_copy_extinction_sat(self.handle, None, 0, dims), "cvr_copy_extinction_sat",
                self.handle)
        a = np.zeros((dims[2], dims[1], dims[0]), np.float32)
        N.check(L.cvr_copy_extinction_sat(self.handle, N.fptr(a), a.size, dims),
                "cvr_copy_extinction_sat", self.handle)
        return a

    def extinction_levels(self) -> list:
        """Every level of the extinction pyramid as (d, h, w) float32 arrays."""
        L = N.lib()
        nl = ctypes.c_int()
        dims = (ctypes.c_int * 3)()
        N.check(L.cvr_copy_extinction_level(self.handle, 0, None, dims, nl),
                "cvr_copy_extinction_level", self.handle)
        out = []
        for lv in range(nl.value):
            N.check(L.cvr_copy_extinction_level(self.handle, lv, None, dims, None),
                    "cvr_copy_extinction_level", self.handle)
            a = np.zeros((dims[2], dims[1], dims[0]), np.float32)
            N.check(L.cvr_copy_extinction_level(self.handle, lv, N.fptr(a), dims, None),
                    "cvr_copy_extinction_level", self.handle)
            out.append(a)
        return out

    def device_bytes(self) -> int:
        return int(N.lib().cvr_device_bytes(self.handle))


def make_frame(camera: Camera, width: int, height: int, tile_size: int = 0, rank: int = 0,
               nranks: int = 1) -> N.Frame:
    f = N.Frame()
    f.camera = camera.to_c()
    f.width, f.height = int(width), int(height)
    f.tile_size, f.rank, f.nranks = int(tile_size), int(rank), int(nranks)
    return f


def tiles_for_rank(frame: N.Frame, rank: int) -> int:
    return int(N.lib().cvr_tiles_for_rank(ctypes.byref(frame), rank))


class BaseVolumeRenderer:
    """cppvolrend/volrenderbase.h:25-96 (GL-free)."""

    # volrenderbase.h:28-33
    SINGLE_RAY_PER_PIXEL, MULTIPLE_RAYS_PER_PIXEL, DOWN_SCALING_RENDER, UP_SCALING_RENDER = range(4)

    def __init__(self):
        self.vr_built = False
        self.vr_outdated = True
        self.vr_pixel_multiscaling_support = False
        self.vr_pixel_multiscaling_mode = 0
        self.m_ext_data_manager: Optional[DataManager] = None
        self.m_ext_rendering_parameters: Optional[RenderingParameters] = None

    # non-virtual API
    def SetExternalResources(self, data_mgr: DataManager, rdr_prm: RenderingParameters):
        self.m_ext_data_manager = data_mgr
        self.m_ext_rendering_parameters = rdr_prm

    def PrepareRender(self, camera: Camera):
        if self.IsOutdated():
            self.Update(camera)
            self.vr_outdated = False

    def SetOutdated(self): self.vr_outdated = True
    def IsOutdated(self): return self.vr_outdated
    def IsBuilt(self): return self.vr_built
    def SetBuilt(self, b: bool): self.vr_built = bool(b)
    def IsPixelMultiScalingSupported(self): return self.vr_pixel_multiscaling_support

    def GetCurrentMultiScalingMode(self):      # volrenderbase.cpp:106-109
        return self.vr_pixel_multiscaling_mode if self.IsPixelMultiScalingSupported() else 0

    def SetCurrentMultiScalingMode(self, f: int):
        self.vr_pixel_multiscaling_mode = int(f)

    # multiscaling entry points (volrenderbase.h:50-52); RenderingManager::Display
    # dispatches on GetCurrentMultiScalingMode (renderingmanager.cpp:199-208, 1200-1217)
    def MultiSampleRedraw(self): pass
    def DownScalingRedraw(self): pass
    def UpScalingRedraw(self): pass

    # virtual API
    def GetName(self) -> str: raise NotImplementedError
    def GetAbbreviationName(self) -> str: raise NotImplementedError
    def GetDataTypeSupport(self) -> str: raise NotImplementedError
    def Init(self, swidth: int, sheight: int) -> bool: raise NotImplementedError
    def Update(self, camera: Camera) -> bool: raise NotImplementedError
    def Redraw(self): pass
    def ReloadShaders(self): pass
    def FillParameterSpace(self, pspace: dict): pspace.clear()

    def Reshape(self, w: int, h: int):
        self.SetOutdated()

    def Clean(self):
        self.SetBuilt(False)


class RayCasting1Pass(BaseVolumeRenderer):
    """HIP implementation of RayCasting1Pass (cppvolrend/structured/rc1pass/rc1prenderer.cpp).

    ``devices`` (a list of GPU indices): the renderer runs on all of them from this one
    process (cvr_create_group: each frame split into screen tiles over the devices and
    gathered on devices[0]; same pixels as one GPU)."""

    def __init__(self, device: int = 0, devices=None):
        super().__init__()
        self._devices = list(devices) if devices is not None else None
        if self._devices:
            device = self._devices[0]
        self.m_u_step_size = 0.5                    # rc1prenderer.cpp:21
        self.m_apply_gradient_shading = False       # :22
        self._device_index = device
        self._dev: Optional[Device] = None
        self._frame: Optional[N.Frame] = None
        self._params = N.Rc1passParams()
        self.width = self.height = 0
        self.rgba: Optional[torch.Tensor] = None    # (H, W, 4) float32 (float16 when multiscaling)
        self.screen: Optional[torch.Tensor] = None  # the screen image (rgba, or the filtered frame)
        self.screen_width = self.screen_height = 0
        self.m_kernel_filter = N.FILTER_HAT         # renderoutputframe.cpp:34
        self.vr_pixel_multiscaling_support = True   # rc1prenderer.cpp:25
        self.samples: Optional[torch.Tensor] = None  # (H, W) int32 iteration counts
        self.total: Optional[torch.Tensor] = None   # (1,) int64 sum of samples

    def GetName(self): return "1-Pass - Ray Casting"
    def GetAbbreviationName(self): return "s_1rc"
    def GetDataTypeSupport(self): return STRUCTURED

    @property
    def device(self) -> Device:
        if self._dev is None:
            raise N.CvrError(N.CVR_ERR_STATE, "RayCasting1Pass", "Init() not called")
        return self._dev

    def Init(self, swidth: int, sheight: int) -> bool:
        if self.IsBuilt():
            self.Clean()
        dm = self.m_ext_data_manager
        if dm is None or dm.volume is None or dm.tf_rgbt is None:
            return False                            # rc1prenderer.cpp:54
        self._dev = Device(self._device_index, devices=self._devices)
        self._dev.set_volume(dm.volume, dm.scale)
        self._dev.set_transfer_function(dm.tf_rgbt)
        if dm.gradient_type != N.GRADIENT_NONE:
            self._dev.set_gradient(dm.gradient_type)
        sc = np.asarray(dm.scale, dtype=np.float32)
        self.m_u_step_size = float(N.lib().cvr_default_step(N.fptr(sc)))   # :62-63
        self.Reshape(swidth, sheight)
        self.SetBuilt(True)
        self.SetOutdated()
        return True

    def Reshape(self, w: int, h: int):
        """Screen size (w, h).  The frame is rendered at the multiscaling mode's resolution
        (BaseVolumeRenderer::Reshape, volrenderbase.cpp:42-66): float32 RGBA for a single
        ray per pixel, else the RGBA16F render target the post-pass filters into
        ``screen`` (RGBA16F, w x h)."""
        self.screen_width, self.screen_height = int(w), int(h)
        mode = self.GetCurrentMultiScalingMode()
        rw, rh = ctypes.c_int(), ctypes.c_int()
        N.check(N.lib().cvr_multiscale_resolution(mode, int(w), int(h), ctypes.byref(rw),
                                                  ctypes.byref(rh)), "cvr_multiscale_resolution")
        self.width, self.height = rw.value, rh.value
        dev = torch.device("cuda", self._device_index)
        self.rgba = torch.zeros((self.height, self.width, 4),
                                dtype=torch.float16 if mode else torch.float32, device=dev)
        self.samples = torch.zeros((self.height, self.width), dtype=torch.int32, device=dev)
        self.total = torch.zeros((1,), dtype=torch.int64, device=dev)
        self.screen = (torch.zeros((h, w, 4), dtype=torch.float16, device=dev) if mode
                       else self.rgba)
        super().Reshape(w, h)

    def SetCurrentMultiScalingMode(self, f: int):
        """Switch the multiscaling mode (AddImGuiMultiSampleOptions, volrenderbase.cpp:
        119-171): the render target is resized for it."""
        super().SetCurrentMultiScalingMode(f)
        if self.rgba is not None:
            self.Reshape(self.screen_width, self.screen_height)

    def SetImageKernelFilter(self, k: int):
        """RenderFrameToScreen::SetImageKernelFilter (vis::IMAGE_FILTER_KERNEL, default
        K2_HAT, renderoutputframe.cpp:34, 541-545)."""
        self.m_kernel_filter = int(k)

    def _camera_frame(self, camera: Camera) -> N.Frame:
        """The frame at the render resolution; the aspect stays the screen's
        (Camera::GetAspectRatio, passed as a uniform, rc1prenderer.cpp:100-101)."""
        if camera.aspect == 0 and self.GetCurrentMultiScalingMode():
            camera = Camera(camera.eye, camera.center, camera.up, camera.fovy_deg,
                            self.screen_width / self.screen_height)
        return make_frame(camera, self.width, self.height)

    def Update(self, camera: Camera) -> bool:
        rp = self.m_ext_rendering_parameters or RenderingParameters()
        self._frame = self._camera_frame(camera)
        p = self._params
        p.step = float(self.m_u_step_size)
        p.apply_gradient_shading = int(bool(self.m_apply_gradient_shading) and
                                       self.m_ext_data_manager.gradient_type != N.GRADIENT_NONE)
        p.ka, p.kd = rp.blinnphong_ka, rp.blinnphong_kd
        p.ks, p.shininess = rp.blinnphong_ks, rp.blinnphong_shininess
        p.ispecular[:] = [float(v) for v in rp.light_specular]
        p.light_pos[:] = [float(v) for v in rp.light_position]
        return True

    def Redraw(self, stream: Optional[torch.cuda.Stream] = None, count_samples: bool = True):
        """Dispatch the ray-march into self.rgba (asynchronous on `stream`)."""
        if self._frame is None:
            raise N.CvrError(N.CVR_ERR_STATE, f"{type(self).__name__}.Redraw", "Update() not called")
        s = stream if stream is not None else torch.cuda.current_stream(self._device_index)
        self.device.set_stream(s.cuda_stream)
        if count_samples:
            with torch.cuda.stream(s):
                self.total.zero_()                  # the kernel accumulates into it
        mode = self.GetCurrentMultiScalingMode()
        out = N.Output(self.rgba.data_ptr(),
                       self.samples.data_ptr() if count_samples else None,
                       self.total.data_ptr() if count_samples else None, 1,
                       N.FORMAT_RGBA16F if mode else N.FORMAT_RGBA32F)
        self.render_to(self._frame, out)
        if mode:    # the post-pass of RenderFrameToScreen, same stream
            N.check(N.lib().cvr_multiscale_filter(self.device.handle, mode, self.m_kernel_filter,
                                                  self.rgba.data_ptr(), self.width, self.height,
                                                  self.screen.data_ptr(), self.screen_width,
                                                  self.screen_height),
                    "cvr_multiscale_filter", self.device.handle)

    # rc1prenderer.cpp:153-190: the same dispatch, then the mode's filter (Redraw does both)
    def MultiSampleRedraw(self, stream=None, count_samples: bool = True):
        assert self.GetCurrentMultiScalingMode() == self.MULTIPLE_RAYS_PER_PIXEL
        self.Redraw(stream, count_samples)

    def DownScalingRedraw(self, stream=None, count_samples: bool = True):
        assert self.GetCurrentMultiScalingMode() == self.DOWN_SCALING_RENDER
        self.Redraw(stream, count_samples)

    def UpScalingRedraw(self, stream=None, count_samples: bool = True):
        assert self.GetCurrentMultiScalingMode() == self.UP_SCALING_RENDER
        self.Redraw(stream, count_samples)

    def Screenshot(self) -> np.ndarray:
        """RenderingManager::SaveScreenshot's pixels: the screen image blended over white,
        RGB8, row 0 = bottom (renderingmanager.cpp:103-112, 476-492).  Synchronises."""
        w, h = self.screen_width, self.screen_height
        rgb = torch.empty((h, w, 3), dtype=torch.uint8, device=self.screen.device)
        s = torch.cuda.current_stream(self._device_index)
        self.device.set_stream(s.cuda_stream)
        N.check(N.lib().cvr_screenshot_rgb8(self.device.handle, self.screen.data_ptr(),
                                            N.FORMAT_RGBA16F if self.screen.dtype == torch.float16
                                            else N.FORMAT_RGBA32F, w, h, rgb.data_ptr()),
                "cvr_screenshot_rgb8", self.device.handle)
        return rgb.cpu().numpy()

    # C entry of this renderer's frame (cvr_render_rc1pass / _dosct / _extbsd)
    _ENTRY = "cvr_render_rc1pass"

    def render_to(self, frame: N.Frame, out: N.Output):
        """One frame (or this rank's screen tiles of it) into `out`, with the parameters
        of the last Update(), asynchronous on the device's current stream."""
        N.check(getattr(N.lib(), self._ENTRY)(self.device.handle, ctypes.byref(frame),
                                              ctypes.byref(self._params), ctypes.byref(out)),
                self._ENTRY, self.device.handle)

    def render_frames_to(self, frames, outs):
        """Several frames in ONE launch (cvr_render_rc1pass_frames): frames[i] into
        outs[i] (device outputs; outs[0].total gets the samples of all of them), the
        same pixels as len(frames) render_to calls."""
        if self._ENTRY != "cvr_render_rc1pass":
            raise NotImplementedError(f"{type(self).__name__}: one frame per call")
        n = len(frames)
        fa = (N.Frame * n)(*frames)
        oa = (N.Output * n)(*outs)
        N.check(N.lib().cvr_render_rc1pass_frames(self.device.handle, fa, n,
                                                  ctypes.byref(self._params), oa),
                "cvr_render_rc1pass_frames", self.device.handle)

    def FillParameterSpace(self, pspace: dict):
        pspace.clear()
        pspace["StepSize"] = (0.2, 2.0, 0.1)        # rc1prenderer.cpp:225-229

    def Clean(self):
        if self._dev is not None:
            self._dev.close()
            self._dev = None
        super().Clean()


def default_cone_params(occlusion: bool) -> N.ConeParams:
    """sampler_occlusion / sampler_shadow defaults (dosrcrenderer.cpp:47-58); the covered
    distance is left 0 so the library applies diagonal * 0.50 / 0.75 (:112-113)."""
    c = N.ConeParams()
    if occlusion:
        c.half_angle_deg, c.max_packing, c.ui_weight = 20.0, 1, 0.35
    else:
        c.half_angle_deg, c.max_packing, c.ui_weight = 0.5, 0, 1.0
    c.covered_distance = 0.0
    c.initial_step = 3.0      # 3 * sigma0 (:366-367)
    return c


class RC1PConeTracingDirOcclusionShading(RayCasting1Pass):
    """HIP implementation of RC1PConeTracingDirOcclusionShading
    (cppvolrend/structured/rc1pdosct/dosrcrenderer.cpp): the single-pass march with
    cone-traced directional ambient occlusion and cone shadows per sample."""

    POINT_LIGHT, SPOT_LIGHT, DIRECTIONAL_LIGHT = 0, 1, 2   # type_of_shadow combo (:543)

    def __init__(self, device: int = 0, devices=None):
        super().__init__(device, devices)
        self.glsl_apply_occlusion = True            # dosrcrenderer.cpp:44
        self.glsl_apply_shadow = False              # :53
        self.type_of_shadow = self.POINT_LIGHT      # :59
        self.sampler_occlusion = default_cone_params(True)
        self.sampler_shadow = default_cone_params(False)
        self.ext_res = (128, 128, 128)              # extcoefvolumegenerator.cpp:10-15
        self.base_level_sigma0 = 1.0
        self._params = N.DosParams()

    def GetName(self): return "1-Pass - Ray Casting - Dir. Occlusion Shading"
    def GetAbbreviationName(self): return "s_1rc_dos"

    def Init(self, swidth: int, sheight: int) -> bool:
        dm = self.m_ext_data_manager
        if dm is None or dm.tf_rgba is None:
            return False
        if not super().Init(swidth, sheight):
            return False
        self.GenerateExtCoefVolume()
        return True

    def GenerateExtCoefVolume(self):
        """dosrcrenderer.cpp:745-764: the pyramid from the volume and the RGBA TF."""
        self.device.set_extinction_volume(self.m_ext_data_manager.tf_rgba, self.ext_res,
                                          self.base_level_sigma0)
        self.SetOutdated()

    def Update(self, camera: Camera) -> bool:
        rp = self.m_ext_rendering_parameters or RenderingParameters()
        self._frame = self._camera_frame(camera)
        p = self._params
        p.step = float(self.m_u_step_size)
        p.apply_gradient_shading = int(bool(self.m_apply_gradient_shading) and
                                       self.m_ext_data_manager.gradient_type != N.GRADIENT_NONE)
        p.ka, p.kd = rp.blinnphong_ka, rp.blinnphong_kd
        p.ks, p.shininess = rp.blinnphong_ks, rp.blinnphong_shininess
        p.ispecular[:] = [float(v) for v in rp.light_specular]
        p.light.position[:] = [float(v) for v in rp.light_position]
        p.light.forward[:] = [float(v) for v in rp.light_forward]
        p.light.up[:] = [float(v) for v in rp.light_up]
        p.light.right[:] = [float(v) for v in rp.light_right]
        p.light.spot_angle_deg = float(rp.spot_light_angle)
        p.apply_occlusion = int(bool(self.glsl_apply_occlusion))
        p.apply_shadow = int(bool(self.glsl_apply_shadow))
        p.shadow_type = int(self.type_of_shadow)
        p.occlusion = self.sampler_occlusion
        p.shadow = self.sampler_shadow
        return True

    _ENTRY = "cvr_render_dosct"


class RC1PExtinctionBasedShading(RayCasting1Pass):
    """HIP implementation of RC1PExtinctionBasedShading
    (cppvolrend/structured/rc1pextbsd/ebsrenderer.cpp): the single-pass march with a
    summed-area-table ambient occlusion and a SAT box-chain shadow per sample."""

    POINT_LIGHT, DIRECTIONAL_LIGHT = 0, 1

    def __init__(self, device: int = 0, devices=None):
        super().__init__(device, devices)
        self.apply_ambient_occlusion = True          # ebsrenderer.cpp:27-31
        self.ambient_occlusion_shells = 15
        self.ambient_occlusion_radius = 1.0
        self.apply_directional_shadows = True        # :33-42
        self.dir_shadow_cone_angle = 1.0
        self.dir_shadow_sample_interval = 2.0
        self.dir_shadow_initial_step = 2.0
        self.dir_shadow_user_interface_weight = 1.0
        self.dir_cone_max_distance = 0.0             # 0: 0.75 * diagonal, set at Init (:98-105)
        self.type_of_shadow = self.POINT_LIGHT
        self._params = N.EbsParams()

    def GetName(self): return "1-Pass - Ray Casting - Extinction Based Shading"
    def GetAbbreviationName(self): return "s_1rc_ebs"

    def Init(self, swidth: int, sheight: int) -> bool:
        dm = self.m_ext_data_manager
        if dm is None or dm.ext_lut is None:
            return False
        if not super().Init(swidth, sheight):
            return False
        self.device.set_extinction_sat(dm.ext_lut)   # GenerateExtinctionSAT3DTex (:88-90)
        return True

    def Update(self, camera: Camera) -> bool:
        rp = self.m_ext_rendering_parameters or RenderingParameters()
        self._frame = self._camera_frame(camera)
        p = self._params
        p.step = float(self.m_u_step_size)
        p.apply_gradient_shading = int(bool(self.m_apply_gradient_shading) and
                                       self.m_ext_data_manager.gradient_type != N.GRADIENT_NONE)
        p.ka, p.kd = rp.blinnphong_ka, rp.blinnphong_kd
        p.ks, p.shininess = rp.blinnphong_ks, rp.blinnphong_shininess
        p.ispecular[:] = [float(v) for v in rp.light_specular]
        p.light_pos[:] = [float(v) for v in rp.light_position]
        p.light_forward[:] = [float(v) for v in rp.light_forward]
        p.apply_occlusion = int(bool(self.apply_ambient_occlusion))
        p.occlusion_shells = int(self.ambient_occlusion_shells)
        p.occlusion_radius = float(self.ambient_occlusion_radius)
        p.apply_shadow = int(bool(self.apply_directional_shadows))
        p.shadow_type = int(self.type_of_shadow)
        p.shadow_cone_angle_deg = float(self.dir_shadow_cone_angle)
        p.shadow_sample_interval = float(self.dir_shadow_sample_interval)
        p.shadow_initial_step = float(self.dir_shadow_initial_step)
        p.shadow_ui_weight = float(self.dir_shadow_user_interface_weight)
        p.shadow_max_distance = float(self.dir_cone_max_distance)
        return True

    _ENTRY = "cvr_render_extbsd"


class RayCasting1PassIsoAdapt(RayCasting1Pass):
    """HIP implementation of RayCasting1PassIsoAdapt
    (cppvolrend/structured/rc1pisoadapt/rc1pisoadaptrenderer.cpp): first-hit
    isosurfaces with adaptive steps (small within StepSizeRange of the isovalue),
    composited front to back with one colour.  No transfer function."""

    VARIANT = 2

    def __init__(self, device: int = 0, devices=None):
        super().__init__(device, devices)
        self._params = N.IsoParams()
        N.lib().cvr_iso_params_default(self.VARIANT, ctypes.byref(self._params))
        d = self._params
        self.m_u_isovalue = d.isovalue              # rc1pisoadaptrenderer.cpp:15-20
        self.m_u_step_size_small = d.step_small
        self.m_u_step_size_large = d.step_large
        self.m_u_step_size_range = d.step_range
        self.m_u_color = tuple(d.color)
        self.num_blocks = tuple(d.num_blocks)
        self.vr_pixel_multiscaling_support = False  # BaseVolumeRenderer default

    def GetName(self): return "1-Pass - Isosurface Raycaster Adaptive"
    def GetAbbreviationName(self): return "iso"

    def Init(self, swidth: int, sheight: int) -> bool:
        if self.IsBuilt():
            self.Clean()
        dm = self.m_ext_data_manager
        if dm is None or dm.volume is None:
            return False                            # GetCurrentVolumeTexture() == nullptr
        self._dev = Device(self._device_index, devices=self._devices)
        self._dev.set_volume(dm.volume, dm.scale)
        if dm.gradient_type != N.GRADIENT_NONE:
            self._dev.set_gradient(dm.gradient_type)
        self.Reshape(swidth, sheight)
        self.SetBuilt(True)
        self.SetOutdated()
        return True

    def Update(self, camera: Camera) -> bool:
        rp = self.m_ext_rendering_parameters or RenderingParameters()
        self._frame = self._camera_frame(camera)
        p = self._params
        p.variant = self.VARIANT
        p.num_blocks[:] = [int(b) for b in self.num_blocks]
        p.isovalue = float(self.m_u_isovalue)
        p.step_small = float(self.m_u_step_size_small)
        p.step_large = float(self.m_u_step_size_large)
        p.step_range = float(self.m_u_step_size_range)
        p.color[:] = [float(c) for c in self.m_u_color]
        p.apply_gradient_shading = int(bool(self.m_apply_gradient_shading) and
                                       self.m_ext_data_manager.gradient_type != N.GRADIENT_NONE)
        p.ka, p.kd = rp.blinnphong_ka, rp.blinnphong_kd
        p.ks, p.shininess = rp.blinnphong_ks, rp.blinnphong_shininess
        p.ispecular[:] = [float(v) for v in rp.light_specular]
        p.light_pos[:] = [float(v) for v in rp.light_position]
        return True

    def FillParameterSpace(self, pspace: dict):
        pspace.clear()                              # rc1pisoadaptrenderer.cpp:191-197
        pspace["StepSizeSmall"] = (0.01, 0.25, 0.05)
        pspace["StepSizeLarge"] = (0.25, 2.0, 0.25)
        pspace["StepSizeRange"] = (0.05, 0.26, 0.05)

    _ENTRY = "cvr_render_iso"


class CustomRayCasting1PassIsoAdapt(RayCasting1PassIsoAdapt):
    """HIP implementation of CustomRayCasting1PassIsoAdapt
    (cppvolrend/structured/rc1pisocustom/rc1custompisoadaptrenderer.cpp): the adaptive
    isosurface march with empty-space skipping over a 4^3 min/max block grid
    (ComputeBlocksFromVolume, built on the GPU)."""

    VARIANT = 0

    def GetName(self): return "1-Pass - Custom Isosurface Raycaster Adaptive"

    def BlockRanges(self):
        """The (min, max) block tables the shader reads, float32 (nz, ny, nx)."""
        nb = (ctypes.c_int * 3)(*[int(b) for b in self.num_blocks])
        shape = (nb[2], nb[1], nb[0])
        lo = np.empty(shape, np.float32)
        hi = np.empty(shape, np.float32)
        N.check(N.lib().cvr_iso_block_ranges(self.device.handle, nb, N.fptr(lo), N.fptr(hi)),
                "cvr_iso_block_ranges", self.device.handle)
        return lo, hi


class CustomRayCasting1PassIsodfsAdapt(CustomRayCasting1PassIsoAdapt):
    """HIP implementation of CustomRayCasting1PassIsodfsAdapt ("Empty Sapce Skipping V2",
    cppvolrend/structured/rc1pisodfscustom/rc1custompisoadaptdfsrenderer.cpp): 32^3
    blocks, the block exit distance as the skip, a 0.001 skip tolerance and steps
    capped at half a block diagonal."""

    VARIANT = 1

    def GetName(self): return "Empty Sapce Skipping V2"


def composite_over_white(rgba: np.ndarray) -> np.ndarray:
    """Screen image as RenderFrameToScreen::Draw blends it over the white clear colour
    with SRC_ALPHA / ONE_MINUS_SRC_ALPHA (renderingmanager.cpp:103-112), as RGB8."""
    rgb = rgba[..., :3] * rgba[..., 3:4] + (1.0 - rgba[..., 3:4])
    return np.clip(np.floor(rgb * 255.0 + 0.5), 0, 255).astype(np.uint8)


def default_step(scale) -> float:
    sx, sy, sz = (float(s) for s in scale)
    return float(np.float32((0.5 / math.sqrt(3.0)) * math.sqrt(sx * sx + sy * sy + sz * sz)))
