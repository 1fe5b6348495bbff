"""ctypes wrapper of oracle/build/liboracle.so — the CPU restatement of the
reference's rc1pass path (see cvr_oracle.cpp for the file:line map).
TEST INFRASTRUCTURE ONLY."""
from __future__ import annotations

import ctypes
import math
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "build", "liboracle.so")

_lib = None


class OracleRc1pass(ctypes.Structure):
    _fields_ = [("vol", ctypes.c_void_p), ("N", ctypes.c_int * 3), ("scale", ctypes.c_float * 3),
                ("tf", ctypes.c_void_p), ("tf_n", ctypes.c_int), ("grad", ctypes.c_void_p),
                ("eye", ctypes.c_float * 3), ("center", ctypes.c_float * 3),
                ("up", ctypes.c_float * 3), ("fovy_deg", ctypes.c_float),
                ("aspect", ctypes.c_float), ("W", ctypes.c_int), ("H", ctypes.c_int),
                ("step", ctypes.c_float), ("phong", ctypes.c_int), ("ka", ctypes.c_float),
                ("kd", ctypes.c_float), ("ks", ctypes.c_float), ("shininess", ctypes.c_float),
                ("ispec", ctypes.c_float * 3), ("light", ctypes.c_float * 3),
                ("filter_bits", ctypes.c_int)]


class OracleExtVol(ctypes.Structure):
    _fields_ = [("vol", ctypes.c_void_p), ("N", ctypes.c_int * 3), ("scale", ctypes.c_float * 3),
                ("tf_rgba", ctypes.c_void_p), ("tf_n", ctypes.c_int), ("res", ctypes.c_int * 3),
                ("sigma0", ctypes.c_float)]


class OracleDosCone(ctypes.Structure):
    _fields_ = [("sections", ctypes.c_void_p), ("counts", ctypes.c_int * 3),
                ("axes", ctypes.c_float * 30), ("initial_step", ctypes.c_float),
                ("ray7w", ctypes.c_float), ("ui_weight", ctypes.c_float)]


class OracleDos(ctypes.Structure):
    _fields_ = [("base", OracleRc1pass), ("ext", ctypes.c_void_p), ("ext_res", ctypes.c_int * 3),
                ("ext_levels", ctypes.c_int), ("apply_occlusion", ctypes.c_int),
                ("apply_shadow", ctypes.c_int), ("shadow_type", ctypes.c_int),
                ("light_forward", ctypes.c_float * 3), ("light_up", ctypes.c_float * 3),
                ("light_right", ctypes.c_float * 3), ("spot_angle_deg", ctypes.c_float),
                ("occ", OracleDosCone), ("sdw", OracleDosCone)]


class OracleEbs(ctypes.Structure):
    _fields_ = [("base", OracleRc1pass), ("sat", ctypes.c_void_p), ("sat_dims", ctypes.c_int * 3),
                ("apply_occlusion", ctypes.c_int), ("occ_shells", ctypes.c_int),
                ("occ_radius", ctypes.c_float), ("apply_shadow", ctypes.c_int),
                ("shadow_type", ctypes.c_int), ("cone_angle", ctypes.c_float),
                ("interval", ctypes.c_float), ("initial_step", ctypes.c_float),
                ("ui_weight", ctypes.c_float), ("max_distance", ctypes.c_float),
                ("light_forward", ctypes.c_float * 3)]


class OracleIso(ctypes.Structure):
    _fields_ = [("base", OracleRc1pass), ("variant", ctypes.c_int), ("nb", ctypes.c_int * 3),
                ("bmin", ctypes.c_void_p), ("bmax", ctypes.c_void_p), ("iso", ctypes.c_float),
                ("step_small", ctypes.c_float), ("step_large", ctypes.c_float),
                ("step_range", ctypes.c_float), ("color", ctypes.c_float * 4)]


def build() -> None:
    subprocess.run(["make", "-C", HERE, "-s"], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = ctypes.CDLL(LIB_PATH)
        F, P, I = ctypes.c_float, ctypes.c_void_p, ctypes.c_int
        L.oracle_q16.argtypes, L.oracle_q16.restype = [F], F
        L.oracle_expf.argtypes, L.oracle_expf.restype = [F], F
        L.oracle_powf.argtypes, L.oracle_powf.restype = [F, F], F
        L.oracle_lookat.argtypes = [P, P, P, F, P, P]
        L.oracle_default_step.argtypes, L.oracle_default_step.restype = [P], F
        L.oracle_tf_build_double.argtypes = [P, I, P, I, I, P]
        L.oracle_tf_rgbt.argtypes = [P, I, I, I, P]
        L.oracle_tf_get.argtypes = [P, I, ctypes.c_double, ctypes.c_double, P]
        L.oracle_volume_r16f.argtypes = [P, I, ctypes.c_int64, P]
        L.oracle_gradient_fd.argtypes = [P, I, I, I, I, P]
        L.oracle_gradient_sobel.argtypes = [P, I, I, I, I, P]
        L.oracle_render_rc1pass.argtypes = [ctypes.POINTER(OracleRc1pass), P, P, I]
        L.oracle_render_rc1pass.restype = ctypes.c_uint64
        L.oracle_render_rc1pass_rows.argtypes = [ctypes.POINTER(OracleRc1pass), I, I, P, P, I]
        L.oracle_render_rc1pass_rows.restype = ctypes.c_uint64
        L.oracle_num_threads.restype = I
        L.oracle_logf.argtypes, L.oracle_logf.restype = [F], F
        L.oracle_ext_levels.argtypes, L.oracle_ext_levels.restype = [P], I
        L.oracle_ext_volume.argtypes = [ctypes.POINTER(OracleExtVol), P, I]
        L.oracle_ext_volume.restype = I
        L.oracle_render_dos.argtypes = [ctypes.POINTER(OracleDos), P, P, I]
        L.oracle_render_dos.restype = ctypes.c_uint64
        L.oracle_render_dos_rows.argtypes = [ctypes.POINTER(OracleDos), I, I, P, P, I]
        L.oracle_render_dos_rows.restype = ctypes.c_uint64
        L.oracle_ext_lut.argtypes = [P, I, I, I, P]
        L.oracle_ext_lut.restype = None
        L.oracle_sat_build.argtypes = [P, I, I, I, I, P, P]
        L.oracle_sat_build.restype = None
        L.oracle_sat_planes.argtypes = [P, I, I, I, I, P, P, I, P]
        L.oracle_sat_planes.restype = None
        L.oracle_check_div_by_recip.argtypes = [ctypes.c_uint64, ctypes.c_uint64, I, I]
        L.oracle_check_div_by_recip.restype = ctypes.c_uint64
        L.oracle_render_rc1pass_literal.argtypes = [ctypes.POINTER(OracleRc1pass), I, I, P, P, I, I]
        L.oracle_render_rc1pass_literal.restype = ctypes.c_uint64
        L.oracle_render_dos_literal.argtypes = [ctypes.POINTER(OracleDos), I, I, P, P, I, I]
        L.oracle_render_dos_literal.restype = ctypes.c_uint64
        L.oracle_render_ebs_literal.argtypes = [ctypes.POINTER(OracleEbs), I, I, P, P, I, I]
        L.oracle_render_ebs_literal.restype = ctypes.c_uint64
        L.oracle_render_ebs_rows.argtypes = [ctypes.POINTER(OracleEbs), I, I, P, P, I]
        L.oracle_render_ebs_rows.restype = ctypes.c_uint64
        L.oracle_multiscale_filter.argtypes = [I, I, P, I, I, P, I, I]
        L.oracle_multiscale_filter.restype = I
        L.oracle_screenshot_rgb8.argtypes = [P, I, I, I, P]
        L.oracle_iso_blocks.argtypes = [P, I, I, I, I, P, P, P]
        L.oracle_render_iso_rows.argtypes = [ctypes.POINTER(OracleIso), I, I, P, P, I]
        L.oracle_render_iso_rows.restype = ctypes.c_uint64
        L.oracle_screenshot_rgb8.restype = None
        _lib = L
    return _lib


def _p(a):
    return a.ctypes.data


def q16(x: float) -> float:
    return lib().oracle_q16(x)


def expf(x: float) -> float:
    return lib().oracle_expf(x)


def powf(x: float, y: float) -> float:
    return lib().oracle_powf(x, y)


def lookat(eye, center, up, fovy_deg=45.0):
    e = np.asarray(eye, np.float32); c = np.asarray(center, np.float32)
    u = np.asarray(up, np.float32)
    out = np.zeros(16, np.float32); t = np.zeros(1, np.float32)
    lib().oracle_lookat(_p(e), _p(c), _p(u), fovy_deg, _p(out), _p(t))
    return out, float(t[0])


def default_step(scale) -> float:
    s = np.asarray(scale, np.float32)
    return float(lib().oracle_default_step(_p(s)))


def tf_table_double(rgb_cp, alpha_cp, max_density=255) -> np.ndarray:
    rgb = np.ascontiguousarray(np.asarray(rgb_cp, np.float64).reshape(-1, 4))
    a = np.ascontiguousarray(np.asarray(alpha_cp, np.float64).reshape(-1, 2))
    out = np.zeros((max_density + 1, 4), np.float64)
    lib().oracle_tf_build_double(_p(rgb), rgb.shape[0], _p(a), a.shape[0], max_density, _p(out))
    return out


def tf_rgbt(table: np.ndarray, extinction_input=False, round16=True) -> np.ndarray:
    t = np.ascontiguousarray(table, np.float64)
    out = np.zeros((t.shape[0], 4), np.float32)
    lib().oracle_tf_rgbt(_p(t), t.shape[0], int(extinction_input), int(round16), _p(out))
    return out


def tf_get(table: np.ndarray, value: float, max_data_value: float = -1.0) -> np.ndarray:
    t = np.ascontiguousarray(table, np.float64)
    out = np.zeros(4, np.float32)
    lib().oracle_tf_get(_p(t), t.shape[0] - 1, value, max_data_value, _p(out))
    return out


def volume_r16f(vox: np.ndarray) -> np.ndarray:
    v = np.ascontiguousarray(vox)
    out = np.empty(v.shape, np.float32)
    lib().oracle_volume_r16f(_p(v), v.dtype.itemsize, v.size, _p(out))
    return out


def gradient(vox: np.ndarray, mode: str = "fd") -> np.ndarray:
    v = np.ascontiguousarray(vox)
    d, h, w = v.shape
    out = np.empty((d, h, w, 3), np.float32)
    fn = lib().oracle_gradient_fd if mode == "fd" else lib().oracle_gradient_sobel
    fn(_p(v), v.dtype.itemsize, w, h, d, _p(out))
    return out


def _params(vol16, scale, tf, grad, camera, W, H, step, phong, ka, kd, ks, shininess, ispec,
            light, aspect=0.0):
    P = OracleRc1pass()
    d, h, w = vol16.shape
    P.vol = _p(vol16)
    P.N[:] = [w, h, d]
    P.scale[:] = [float(s) for s in scale]
    P.tf = _p(tf)
    P.tf_n = tf.shape[0]
    P.grad = _p(grad) if grad is not None else None
    P.eye[:] = [float(v) for v in camera["eye"]]
    P.center[:] = [float(v) for v in camera["center"]]
    P.up[:] = [float(v) for v in camera["up"]]
    P.fovy_deg = float(camera.get("fovy_deg", 45.0))
    P.aspect = float(aspect)
    P.W, P.H = int(W), int(H)
    P.step = float(step)
    P.phong = int(phong)
    P.ka, P.kd, P.ks, P.shininess = ka, kd, ks, shininess
    P.ispec[:] = [float(v) for v in ispec]
    P.light[:] = [float(v) for v in light]
    return P


def render_rc1pass(vol16: np.ndarray, scale, tf: np.ndarray, camera: dict, W: int, H: int,
                   step: float, grad: np.ndarray | None = None, phong: bool = False,
                   ka=0.5, kd=0.5, ks=0.8, shininess=30.0, ispec=(1.0, 1.0, 1.0),
                   light=(0.0, 0.0, 0.0), threads: int = 0, rows=None, literal=None,
                   filter_bits: int = 0):
    """Full frame (or rows=(y0,y1)) of ray_marching_1p.comp. Returns (rgba HxWx4, counts HxW, S).
    literal=None: CVR-SPEC (what the HIP kernels reproduce bit for bit), with every GL_LINEAR
    weight rounded to `filter_bits` fraction bits (0 = exact: CVR-SPEC; 8 = CVR-SPEC-8, the
    library's filter_bits option); literal=b: the literal GLSL reading (glsl_literal.cpp)
    with GL filter weights quantised to b fraction bits (0 = exact float weights)."""
    vol16 = np.ascontiguousarray(vol16, np.float32)
    # the TF texture is GL_RGBA16F (GenerateTexture_1D_RGBt): entries round to half (RNE)
    tf = np.ascontiguousarray(np.asarray(tf, np.float32).astype(np.float16), np.float32)
    if grad is not None:
        grad = np.ascontiguousarray(grad, np.float32)
    P = _params(vol16, scale, tf, grad, camera, W, H, step, phong, ka, kd, ks, shininess, ispec,
                light, aspect=camera.get("aspect", 0.0))
    P.filter_bits = int(filter_bits)
    rgba = np.zeros((H, W, 4), np.float32)
    cnt = np.zeros((H, W), np.uint32)
    if literal is not None:
        y0, y1 = rows if rows is not None else (0, H)
        S = lib().oracle_render_rc1pass_literal(ctypes.byref(P), int(y0), int(y1), _p(rgba),
                                                _p(cnt), int(threads), int(literal))
    elif rows is None:
        S = lib().oracle_render_rc1pass(ctypes.byref(P), _p(rgba), _p(cnt), int(threads))
    else:
        S = lib().oracle_render_rc1pass_rows(ctypes.byref(P), int(rows[0]), int(rows[1]),
                                             _p(rgba), _p(cnt), int(threads))
    return rgba, cnt, int(S)


def num_threads() -> int:
    return int(lib().oracle_num_threads())


def logf(x: float) -> float:
    return lib().oracle_logf(x)


def _q16_array(a) -> np.ndarray:
    return np.ascontiguousarray(np.asarray(a, np.float32).astype(np.float16), np.float32)


def ext_level_dims(res, L):
    return [max(1, int(r) >> L) for r in res]


def ext_volume(vol16: np.ndarray, scale, tf_rgba: np.ndarray, res=(128, 128, 128),
               sigma0: float = 1.0, threads: int = 0):
    """Extinction-coefficient mip volume (extcoefvolumegenerator.cpp:230-408).
    Returns a list of levels, each (d, h, w) float32 of half-rounded extinctions."""
    vol16 = np.ascontiguousarray(vol16, np.float32)
    tf_rgba = _q16_array(tf_rgba)
    P = OracleExtVol()
    d, h, w = vol16.shape
    P.vol = _p(vol16)
    P.N[:] = [w, h, d]
    P.scale[:] = [float(s) for s in scale]
    P.tf_rgba = _p(tf_rgba)
    P.tf_n = tf_rgba.shape[0]
    P.res[:] = [int(r) for r in res]
    P.sigma0 = float(sigma0)
    nl = lib().oracle_ext_levels((ctypes.c_int * 3)(*P.res))
    sizes = [int(np.prod(ext_level_dims(res, L))) for L in range(nl)]
    flat = np.zeros(sum(sizes), np.float32)
    lib().oracle_ext_volume(ctypes.byref(P), _p(flat), int(threads))
    out, o = [], 0
    for L in range(nl):
        dx, dy, dz = ext_level_dims(res, L)
        out.append(flat[o:o + sizes[L]].reshape(dz, dy, dx))
        o += sizes[L]
    return out


def _cone(tables, keep):
    """OracleDosCone from a cvr_cone_tables (sections RGBA16F-rounded as uploaded)."""
    C = OracleDosCone()
    n = tables.n_sections
    sec = _q16_array([list(tables.sections[i]) for i in range(max(n, 1))])
    keep.append(sec)
    C.sections = _p(sec)
    C.counts[:] = list(tables.counts)
    C.axes[:] = [tables.axes[i][j] for i in range(10) for j in range(3)]
    C.initial_step = tables.initial_step
    C.ray7w = tables.ray7_adj_weight
    C.ui_weight = tables.ui_weight
    return C


def render_dos(vol16, scale, tf_rgbt, ext_levels, camera, W, H, step, occ_tables, sdw_tables,
               apply_occlusion=True, apply_shadow=False, shadow_type=0, light=None,
               grad=None, phong=False, ka=0.5, kd=0.5, ks=0.8, shininess=30.0,
               ispec=(1.0, 1.0, 1.0), threads: int = 0, rows=None, literal=None,
               filter_bits: int = 0):
    """Directional-occlusion shading frame (ray_bbox_marching.comp), or rows=(y0, y1) of
    it.  light = dict with position/forward/up/right/spot_angle_deg.  literal,
    filter_bits: as render_rc1pass (filter_bits rounds the weights of the volume, TF,
    gradient and extinction-pyramid fetches).
    Returns (rgba, counts, S)."""
    vol16 = np.ascontiguousarray(vol16, np.float32)
    tf = _q16_array(tf_rgbt)
    if grad is not None:
        grad = np.ascontiguousarray(grad, np.float32)
    light = light or {}
    pos = light.get("position", (0.0, 0.0, 0.0))
    Q = OracleDos()
    Q.base = _params(vol16, scale, tf, grad, camera, W, H, step, phong, ka, kd, ks, shininess,
                     ispec, pos)
    Q.base.filter_bits = int(filter_bits)
    res = list(ext_levels[0].shape[::-1])
    flat = np.ascontiguousarray(np.concatenate([l.ravel() for l in ext_levels]), np.float32)
    Q.ext = _p(flat)
    Q.ext_res[:] = res
    Q.ext_levels = len(ext_levels)
    Q.apply_occlusion, Q.apply_shadow, Q.shadow_type = int(apply_occlusion), int(apply_shadow), int(shadow_type)
    Q.light_forward[:] = [float(v) for v in light.get("forward", (0.0, 0.0, -1.0))]
    Q.light_up[:] = [float(v) for v in light.get("up", (0.0, 1.0, 0.0))]
    Q.light_right[:] = [float(v) for v in light.get("right", (1.0, 0.0, 0.0))]
    Q.spot_angle_deg = float(light.get("spot_angle_deg", 4.0))
    keep = []
    Q.occ = _cone(occ_tables, keep)
    Q.sdw = _cone(sdw_tables, keep)
    rgba = np.zeros((H, W, 4), np.float32)
    cnt = np.zeros((H, W), np.uint32)
    y0, y1 = rows if rows is not None else (0, H)
    if literal is not None:
        S = lib().oracle_render_dos_literal(ctypes.byref(Q), int(y0), int(y1), _p(rgba), _p(cnt),
                                            int(threads), int(literal))
    else:
        S = lib().oracle_render_dos_rows(ctypes.byref(Q), int(y0), int(y1), _p(rgba), _p(cnt),
                                         int(threads))
    return rgba, cnt, int(S)


def ext_lut(table: np.ndarray, bpv: int = 1, extinction_input: bool = False) -> np.ndarray:
    """GetExtN(v / (2^bits - 1)) for every voxel value (the EBS SAT cell values)."""
    t = np.ascontiguousarray(table, np.float64)
    out = np.zeros(256 if bpv == 1 else 65536, np.float32)
    lib().oracle_ext_lut(_p(t), t.shape[0] - 1, int(bpv), int(extinction_input), _p(out))
    return out


def sat_build(vox: np.ndarray, lut: np.ndarray) -> np.ndarray:
    """GenerateExtinctionSAT3DTex + SummedAreaTable3D<double>::BuildSAT, literally.
    Returns the (D+2, H+2, W+2) double SAT."""
    v = np.ascontiguousarray(vox)
    d, h, w = v.shape
    lut = np.ascontiguousarray(lut, np.float32)
    out = np.zeros((d + 2, h + 2, w + 2), np.float64)
    lib().oracle_sat_build(_p(v), v.dtype.itemsize, w, h, d, _p(lut), _p(out))
    return out


def sat_planes(vox: np.ndarray, lut: np.ndarray, zs) -> np.ndarray:
    """Planes zs of the float SAT of sat_build, by the same recurrence streamed over z
    (two double planes of memory): for full-size (1024^3) checks."""
    v = np.ascontiguousarray(vox)
    d, h, w = v.shape
    zs = np.ascontiguousarray(sorted(int(z) for z in zs), np.int32)
    assert zs.size and 0 <= zs[0] and zs[-1] < d + 2
    lut = np.ascontiguousarray(lut, np.float32)
    out = np.zeros((zs.size, h + 2, w + 2), np.float32)
    lib().oracle_sat_planes(_p(v), v.dtype.itemsize, w, h, d, _p(lut), _p(zs), int(zs.size),
                            _p(out))
    return out


def ebs_max_distance(n_xyz, scale) -> float:
    """dir_cone_max_distance = 0.75f * Dv (ebsrenderer.cpp:98-105), float arithmetic."""
    f = np.float32
    vw = f(n_xyz[0] * float(scale[0])); vh = f(n_xyz[1] * float(scale[1])); vd = f(n_xyz[2] * float(scale[2]))
    dv = np.sqrt(f(f(vw * vw + vh * vh) + vd * vd), dtype=np.float32)
    return float(f(f(0.75) * dv))


def render_ebs(vol16, scale, tf_rgbt, sat_f32, camera, W, H, step, apply_occlusion=True,
               occ_shells=15, occ_radius=1.0, apply_shadow=True, shadow_type=0,
               cone_angle_deg=1.0, interval=2.0, initial_step=2.0, ui_weight=1.0,
               max_distance=None, light=(0.0, 0.0, 0.0), light_forward=(0.0, 0.0, -1.0),
               grad=None, phong=False, ka=0.5, kd=0.5, ks=0.8, shininess=30.0,
               ispec=(1.0, 1.0, 1.0), threads: int = 0, rows=None, literal=None,
               filter_bits: int = 0):
    """Extinction-based shading frame (ebs_ray_bbox_marching.comp).  Returns (rgba, counts, S).
    literal, filter_bits: as render_rc1pass (filter_bits rounds the weights of the volume,
    TF, gradient and every SAT fetch)."""
    vol16 = np.ascontiguousarray(vol16, np.float32)
    tf = _q16_array(tf_rgbt)
    sat = np.ascontiguousarray(sat_f32, np.float32)
    if grad is not None:
        grad = np.ascontiguousarray(grad, np.float32)
    Q = OracleEbs()
    Q.base = _params(vol16, scale, tf, grad, camera, W, H, step, phong, ka, kd, ks, shininess,
                     ispec, light)
    Q.base.filter_bits = int(filter_bits)
    Q.sat = _p(sat)
    Q.sat_dims[:] = list(sat.shape[::-1])
    Q.apply_occlusion, Q.occ_shells, Q.occ_radius = int(apply_occlusion), int(occ_shells), float(occ_radius)
    Q.apply_shadow, Q.shadow_type = int(apply_shadow), int(shadow_type)
    # DirSdwConeAngle uniform: (float)(angle * glm::pi<double>() / 180.0) (ebsrenderer.cpp:161)
    Q.cone_angle = float(np.float32(cone_angle_deg * math.pi / 180.0))
    Q.interval, Q.initial_step, Q.ui_weight = float(interval), float(initial_step), float(ui_weight)
    d, h, w = vol16.shape
    Q.max_distance = ebs_max_distance((w, h, d), scale) if max_distance is None else float(max_distance)
    Q.light_forward[:] = [float(v) for v in light_forward]
    rgba = np.zeros((H, W, 4), np.float32)
    cnt = np.zeros((H, W), np.uint32)
    y0, y1 = rows if rows is not None else (0, H)
    if literal is not None:
        S = lib().oracle_render_ebs_literal(ctypes.byref(Q), int(y0), int(y1), _p(rgba), _p(cnt),
                                            int(threads), int(literal))
    else:
        S = lib().oracle_render_ebs_rows(ctypes.byref(Q), int(y0), int(y1), _p(rgba), _p(cnt),
                                         int(threads))
    return rgba, cnt, int(S)


def multiscale_filter(mode: int, kernel: int, frame_f16: np.ndarray, screen_w: int,
                      screen_h: int) -> np.ndarray:
    """RenderFrameToScreen's multiscaling post-pass on an RGBA16F frame (h, w, 4) float16.
    Returns the (screen_h, screen_w, 4) float16 screen image.  Mode 3 with a cardinal
    kernel prefilters `frame_f16` in place, as the reference does."""
    assert frame_f16.dtype == np.float16 and frame_f16.flags.c_contiguous
    fh, fw = frame_f16.shape[:2]
    out = np.zeros((screen_h, screen_w, 4), np.float16)
    st = lib().oracle_multiscale_filter(mode, kernel, _p(frame_f16), fw, fh, _p(out), screen_w,
                                        screen_h)
    assert st == 0
    return out


def screenshot_rgb8(frame: np.ndarray) -> np.ndarray:
    """The frame blended over white (SRC_ALPHA, ONE_MINUS_SRC_ALPHA) as RGB8."""
    frame = np.ascontiguousarray(frame)
    h, w = frame.shape[:2]
    out = np.zeros((h, w, 3), np.uint8)
    lib().oracle_screenshot_rgb8(_p(frame), int(frame.dtype == np.float16), w, h, _p(out))
    return out


# Block counts of the two isosurface renderers (rc1custompisoadaptrenderer.cpp:190,
# rc1custompisoadaptdfsrenderer.cpp:190)
ISO_BLOCKS = {0: (4, 4, 4), 1: (32, 32, 32), 2: (1, 1, 1)}   # variant 2 has none


def iso_blocks(vox: np.ndarray, nb) -> tuple[np.ndarray, np.ndarray]:
    """ComputeBlocksFromVolume: per-block (min, max) of v / (2^bits - 1), float32 (nz, ny, nx)."""
    vox = np.ascontiguousarray(vox)
    d, h, w = vox.shape
    nb = [int(x) for x in nb]
    bmin = np.empty((nb[2], nb[1], nb[0]), np.float32)
    bmax = np.empty_like(bmin)
    nba = (ctypes.c_int * 3)(*nb)
    lib().oracle_iso_blocks(_p(vox), vox.dtype.itemsize, w, h, d, nba, _p(bmin), _p(bmax))
    return bmin, bmax


def render_iso(vol16: np.ndarray, vox: np.ndarray, scale, camera: dict, W: int, H: int,
               variant: int = 0, nb=None, isovalue=0.5, step_small=0.05, step_large=1.0,
               step_range=0.1, color=(0.66, 0.6, 0.05, 1.0), grad: np.ndarray | None = None,
               phong: bool = False, ka=0.5, kd=0.5, ks=0.8, shininess=30.0,
               ispec=(1.0, 1.0, 1.0), light=(0.0, 0.0, 0.0), threads: int = 0, rows=None):
    """One frame of an isosurface ray-caster (variant 0: custom adaptive with 4^3
    blocks, 1: "Empty Space Skipping V2", 2: RayCasting1PassIsoAdapt, no blocks).  vol16: the R16F volume as float; vox: the raw voxels (block
    table).  Returns (rgba HxWx4, counts HxW, S, (bmin, bmax))."""
    vol16 = np.ascontiguousarray(vol16, np.float32)
    nb = ISO_BLOCKS[variant] if nb is None else tuple(int(x) for x in nb)
    bmin, bmax = iso_blocks(vox, nb)
    if grad is not None:
        grad = np.ascontiguousarray(grad, np.float32)
    dummy_tf = np.zeros((2, 4), np.float32)
    Q = OracleIso()
    Q.base = _params(vol16, scale, dummy_tf, grad, camera, W, H, 1.0, phong, ka, kd, ks,
                     shininess, ispec, light, aspect=camera.get("aspect", 0.0))
    Q.variant = int(variant)
    Q.nb[:] = list(nb)
    Q.bmin, Q.bmax = _p(bmin), _p(bmax)
    Q.iso, Q.step_small, Q.step_large, Q.step_range = isovalue, step_small, step_large, step_range
    Q.color[:] = [float(c) for c in color]
    rgba = np.zeros((H, W, 4), np.float32)
    cnt = np.zeros((H, W), np.uint32)
    y0, y1 = (0, H) if rows is None else (int(rows[0]), int(rows[1]))
    S = lib().oracle_render_iso_rows(ctypes.byref(Q), y0, y1, _p(rgba), _p(cnt), int(threads))
    return rgba, cnt, int(S), (bmin, bmax)


def check_div_by_recip(n: int, seed: int = 1, lo: int = -20, hi: int = 20) -> int:
    """Mismatches of the reciprocal-corrected division (cvr_device.h div_by_recip) against
    IEEE a / b over n random pairs (a = +-m * 2^-e, e in [lo, hi]; b = +-m * 2^[-8, 8])."""
    return int(lib().oracle_check_div_by_recip(n, seed, lo, hi))


def finite_shaded_bands(rgba: np.ndarray, band: int, need: int, max_bands: int = 4):
    """Row bands of a frame where the parity check compares real shading: up to
    `max_bands` non-overlapping `band`-row windows, richest first in pixels that are
    shaded (alpha > 0) and finite in every channel, until `need` such pixels are covered.
    (The EBS frame at 1024^3 is mostly inf/NaN -- the float-SAT cancellation of
    ebsrenderer.cpp:700-716 -- so a centre band would compare NaN with NaN.)
    Returns [(y0, y1), ...] and the count of finite shaded pixels they hold."""
    ok = np.isfinite(rgba).all(-1) & (rgba[..., 3] > 0)
    per_row = ok.sum(1).astype(np.int64)
    win = np.convolve(per_row, np.ones(band, np.int64), mode="valid")   # win[y] = rows y..y+band-1
    taken = np.zeros(per_row.shape[0], bool)
    bands, got = [], 0
    for y in np.argsort(-win, kind="stable"):
        if len(bands) == max_bands or got >= need or win[y] == 0:
            break
        if taken[y:y + band].any():
            continue
        taken[y:y + band] = True
        bands.append((int(y), int(y) + band))
        got += int(win[y])
    return sorted(bands), got
