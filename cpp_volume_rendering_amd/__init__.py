"""MI355X-native structured volume ray-caster (cppvolrend rc1pass hot path).

The product is ``lib/libcvr.so`` (HIP kernels for gfx950 + the C-ABI of
include/cvr.h); this package is the host-side mirror of the reference's
renderer-plugin API over that ABI.
"""
from . import _native
from .renderer import (BaseVolumeRenderer, Camera, DataManager, Device, RayCasting1Pass,
                       RenderingParameters, build_tf_rgbt, composite_over_white, make_frame,
                       read_camera_state, read_light_position, read_tf1d, tiles_for_rank)

__all__ = ["BaseVolumeRenderer", "Camera", "DataManager", "Device", "RayCasting1Pass",
           "RenderingParameters", "build_tf_rgbt", "composite_over_white", "make_frame",
           "read_camera_state", "read_light_position", "read_tf1d", "tiles_for_rank", "_native"]
