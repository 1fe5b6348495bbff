// cvr_api.cpp — C-ABI implementation (include/cvr.h): context, device
// resources, render dispatch, and the host-side camera / TF helpers.
//
// Compiled with -ffp-contract=off: the camera and TF arithmetic below feed the
// kernels and must be bit-reproducible (CVR-SPEC).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <new>
#include <vector>

#include "cvr_internal.h"

using cvr::Ctx;

namespace {

cvr_status fail(Ctx* c, cvr_status st, const char* fmt, ...) {
  if (c) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof(buf), fmt, ap);
    va_end(ap);
    c->err = buf;
  }
  return st;
}

#define HIP_TRY(ctx, expr)                                                                    \
  do {                                                                                        \
    hipError_t _e = (expr);                                                                   \
    if (_e != hipSuccess)                                                                     \
      return fail(ctx, _e == hipErrorOutOfMemory ? CVR_ERR_OOM : CVR_ERR_HIP, "%s: %s (%s:%d)", \
                  #expr, hipGetErrorString(_e), __FILE__, __LINE__);                         \
  } while (0)

void free_dev(void*& p) {
  if (p) (void)hipFree(p);
  p = nullptr;
}

// Before a state change writes or frees device state that frames read (volume
// cells, TF, gradient, occupancy, cone tables, extinction pyramid, SAT): frames
// may be in flight on any render stream the caller rotates (non-blocking
// streams do not wait for the null-stream copies below), so the whole device
// drains first.  The reference's equivalent is the GL pipeline's implicit
// ordering on Init after a TF change (renderingmanager.cpp:1050-1127).
#define QUIESCE(c)                             \
  do {                                         \
    HIP_TRY(c, hipSetDevice((c)->device));     \
    HIP_TRY(c, hipDeviceSynchronize());        \
  } while (0)

// float -> binary16 bits, round to nearest even (the GL driver's conversion of
// GL_FLOAT client data to a 16F internal format).
uint16_t to_half_bits(float f) {
  _Float16 h = (_Float16)f;
  uint16_t b;
  std::memcpy(&b, &h, 2);
  return b;
}
float half_round(float f) {
  _Float16 h = (_Float16)f;
  return (float)h;
}
float half_to_float_host(uint16_t b) {
  _Float16 h;
  std::memcpy(&h, &b, 2);
  return (float)h;
}

struct V3 { float x, y, z; };
inline V3 sub(V3 a, V3 b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
inline V3 cross(V3 x, V3 y) {
  return {x.y * y.z - y.y * x.z, x.z * y.x - y.z * x.x, x.x * y.y - y.x * x.y};
}
inline float gdot(V3 a, V3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
inline V3 gnormalize(V3 v) {
  float inv = 1.0f / std::sqrt(v.x * v.x + v.y * v.y + v.z * v.z);
  return {v.x * inv, v.y * inv, v.z * inv};
}

}  // namespace

extern "C" {
#pragma GCC visibility push(default)

int cvr_abi_version(void) { return CVR_ABI_VERSION; }

const char* cvr_status_string(cvr_status s) {
  switch (s) {
    case CVR_OK: return "CVR_OK";
    case CVR_ERR_ARG: return "CVR_ERR_ARG";
    case CVR_ERR_HIP: return "CVR_ERR_HIP";
    case CVR_ERR_OOM: return "CVR_ERR_OOM";
    case CVR_ERR_STATE: return "CVR_ERR_STATE";
    case CVR_ERR_IO: return "CVR_ERR_IO";
  }
  return "CVR_ERR_UNKNOWN";
}

// glm::lookAt (glm 0.9.5, include/glm/gtc/matrix_transform.inl:403-428), float.
cvr_status cvr_camera_lookat(const cvr_camera* cam, float out_view[16], float* out_tan) {
  if (!cam || !out_view || !out_tan) return CVR_ERR_ARG;
  V3 eye{cam->eye[0], cam->eye[1], cam->eye[2]};
  V3 center{cam->center[0], cam->center[1], cam->center[2]};
  V3 up{cam->up[0], cam->up[1], cam->up[2]};
  V3 f = gnormalize(sub(center, eye));
  V3 s = gnormalize(cross(f, up));
  V3 u = cross(s, f);
  float* R = out_view;
  for (int i = 0; i < 16; i++) R[i] = (i % 5 == 0) ? 1.0f : 0.0f;
  R[0] = s.x; R[4] = s.y; R[8] = s.z;
  R[1] = u.x; R[5] = u.y; R[9] = u.z;
  R[2] = -f.x; R[6] = -f.y; R[10] = -f.z;
  R[12] = -gdot(s, eye);
  R[13] = -gdot(u, eye);
  R[14] = gdot(f, eye);
  // (float)tan(DEGREE_TO_RADIANS(fovy) / 2.0): rc1prenderer.cpp:97, math_utils/utils.h:13
  double rad = (double)cam->fovy_deg * (3.14159265358979323846 / 180.0);
  *out_tan = (float)std::tan(rad / 2.0);
  return CVR_OK;
}

// rc1prenderer.cpp:62-63
float cvr_default_step(const float scale[3]) {
  double sx = scale[0], sy = scale[1], sz = scale[2];
  return (float)((0.5f / std::sqrt(3.0f)) * std::sqrt(sx * sx + sy * sy + sz * sz));
}

// TransferFunction1D::BuildLinear + GenerateTexture_1D_RGBt
// (transferfunction1d.cpp:319-358, 89-118; transferfunction.h:79-82).
// TransferFunction1D::BuildLinear (transferfunction1d.cpp:319-358): the double
// table m_transferfunction of max_density + 1 entries.
static cvr_status build_tf_table(const double* rgb_cp, int n_rgb, const double* a_cp, int n_a,
                                 int max_density, std::vector<double>& tab) {
  if (max_density < 1 || n_rgb < 0 || n_a < 0) return CVR_ERR_ARG;
  if ((n_rgb > 0 && !rgb_cp) || (n_a > 0 && !a_cp)) return CVR_ERR_ARG;
  const int n = max_density + 1;
  tab.assign((size_t)n * 4, 0.0);   // glm 0.9.5 dvec4 zero-init
  for (int i = 0; i + 1 < n_rgb; i++) {
    // TransferControlPoint keeps its colour in a glm::vec4 (float)
    float c0[3], c1[3];
    for (int k = 0; k < 3; k++) {
      c0[k] = (float)rgb_cp[i * 4 + k];
      c1[k] = (float)rgb_cp[(i + 1) * 4 + k];
    }
    int i0 = (int)rgb_cp[i * 4 + 3], i1 = (int)rgb_cp[(i + 1) * 4 + 3];
    double diff[3] = {(double)(c1[0] - c0[0]), (double)(c1[1] - c0[1]), (double)(c1[2] - c0[2])};
    for (int x = i0; x <= i1; x++) {
      if (x < 0 || x >= n) return CVR_ERR_ARG;
      double k = (double)(x - i0) / (double)(i1 - i0);
      for (int ch = 0; ch < 3; ch++) tab[(size_t)x * 4 + ch] = (double)c0[ch] + diff[ch] * k;
    }
  }
  for (int i = 0; i + 1 < n_a; i++) {
    float a0 = (float)a_cp[i * 2], a1 = (float)a_cp[(i + 1) * 2];
    int i0 = (int)a_cp[i * 2 + 1], i1 = (int)a_cp[(i + 1) * 2 + 1];
    double diff = (double)(a1 - a0);
    for (int x = i0; x <= i1; x++) {
      if (x < 0 || x >= n) return CVR_ERR_ARG;
      double k = (double)(x - i0) / (double)(i1 - i0);
      tab[(size_t)x * 4 + 3] = (double)a0 + diff * k;
    }
  }
  return CVR_OK;
}

// TransferFunction1D::BuildLinear + GenerateTexture_1D_RGBt
// (transferfunction1d.cpp:319-358, 89-118; transferfunction.h:79-82).
cvr_status cvr_tf1d_build_rgbt(const double* rgb_cp, int n_rgb, const double* a_cp, int n_a,
                               int max_density, int extinction_input, float* out_rgbt) {
  if (!out_rgbt) return CVR_ERR_ARG;
  std::vector<double> tab;
  cvr_status st = build_tf_table(rgb_cp, n_rgb, a_cp, n_a, max_density, tab);
  if (st != CVR_OK) return st;
  const int n = max_density + 1;
  for (int i = 0; i < n; i++) {
    out_rgbt[i * 4 + 0] = (float)tab[(size_t)i * 4 + 0];
    out_rgbt[i * 4 + 1] = (float)tab[(size_t)i * 4 + 1];
    out_rgbt[i * 4 + 2] = (float)tab[(size_t)i * 4 + 2];
    float v4 = (float)tab[(size_t)i * 4 + 3];
    if (!extinction_input) v4 = (float)std::log(1.0 / (1.0 - (double)v4));
    out_rgbt[i * 4 + 3] = v4;
  }
  return CVR_OK;
}

// TransferFunction1D::GetExtN(StructuredGridVolume::GetNormalizedSample) for every
// voxel value: Get(v / (2^bits - 1), 1.0).a (transferfunction1d.cpp:132-157) as
// float, then MaterialOpacityToExtinction in double (:189-197), as float.
cvr_status cvr_tf1d_ext_lut(const double* rgb_cp, int n_rgb, const double* a_cp, int n_a,
                            int max_density, int extinction_input, int bytes_per_voxel,
                            float* out_lut) {
  if (!out_lut || (bytes_per_voxel != 1 && bytes_per_voxel != 2)) return CVR_ERR_ARG;
  std::vector<double> tab;
  cvr_status st = build_tf_table(rgb_cp, n_rgb, a_cp, n_a, max_density, tab);
  if (st != CVR_OK) return st;
  const int nv = bytes_per_voxel == 1 ? 256 : 65536;
  const double den = bytes_per_voxel == 1 ? (256.0 - 1.0) : (65536.0 - 1.0);
  for (int v = 0; v < nv; v++) {
    double value = ((double)v / den) * ((double)max_density / 1.0);
    float a;
    if (value < 0.0f || value > (float)max_density) {
      a = 0.0f;
    } else if (std::fabs(value - (float)max_density) < 0.000001) {
      a = (float)tab[(size_t)max_density * 4 + 3];
    } else {
      const int iv = (int)value;
      const double t = value - iv;
      a = (float)((1.0 - t) * tab[(size_t)iv * 4 + 3] + t * tab[(size_t)(iv + 1) * 4 + 3]);
    }
    out_lut[v] = extinction_input ? a : (float)std::log(1.0 / (1.0 - (double)a));
  }
  return CVR_OK;
}

cvr_status cvr_create(int device, cvr_ctx** out_ctx) {
  if (!out_ctx) return CVR_ERR_ARG;
  *out_ctx = nullptr;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) return CVR_ERR_HIP;
  if (device < 0 || device >= ndev) return CVR_ERR_ARG;
  Ctx* c = new (std::nothrow) Ctx();
  if (!c) return CVR_ERR_OOM;
  c->device = device;
  if (hipSetDevice(device) != hipSuccess ||
      hipStreamCreateWithFlags(&c->own_stream, hipStreamNonBlocking) != hipSuccess ||
      hipMalloc(&c->d_total, sizeof(unsigned long long)) != hipSuccess) {
    if (c->own_stream) (void)hipStreamDestroy(c->own_stream);
    delete c;
    return CVR_ERR_HIP;
  }
  c->stream = c->own_stream;
  {
    hipDeviceProp_t prop;
    c->num_cus = hipGetDeviceProperties(&prop, device) == hipSuccess ? prop.multiProcessorCount : 256;
  }
  *out_ctx = reinterpret_cast<cvr_ctx*>(c);
  return CVR_OK;
}

void cvr_destroy(cvr_ctx* ctx) {
  Ctx* c = reinterpret_cast<Ctx*>(ctx);
  if (!c) return;
  cvr::group_release(c);
  (void)hipSetDevice(c->device);
  (void)hipStreamSynchronize(c->stream);
  cvr::comm_release(c);
  free_dev(c->d_vox);
  free_dev(c->d_cells);
  void* p = c->d_tf; free_dev(p); c->d_tf = nullptr;
  free_dev(c->d_grad);
  p = c->d_iso_mm; free_dev(p); c->d_iso_mm = nullptr;
  p = c->d_lut; free_dev(p); c->d_lut = nullptr;
  p = c->d_macro_minmax; free_dev(p); c->d_macro_minmax = nullptr;
  p = c->d_occ; free_dev(p); c->d_occ = nullptr;
  p = c->d_tf_prefix; free_dev(p); c->d_tf_prefix = nullptr;
  p = c->d_ext; free_dev(p); c->d_ext = nullptr;
  p = c->d_ext_cells; free_dev(p); c->d_ext_cells = nullptr;
  p = c->d_ext_levels; free_dev(p); c->d_ext_levels = nullptr;
  p = c->d_sat; free_dev(p); c->d_sat = nullptr;
  p = c->d_sat_cells; free_dev(p); c->d_sat_cells = nullptr;
  p = c->d_sat_scratch; free_dev(p); c->d_sat_scratch = nullptr;
  p = c->d_shade; free_dev(p); c->d_shade = nullptr;
  for (auto& J : c->flat) cvr::flat_release(J);
  p = c->d_cones; free_dev(p); c->d_cones = nullptr;
  delete[] c->cone_tab;
  p = c->d_total; free_dev(p); c->d_total = nullptr;
  free_dev(c->d_scratch);
  if (c->side) (void)hipStreamSynchronize(c->side);
  for (auto& o : c->oslot) {
    p = o.d_order; free_dev(p); o.d_order = nullptr;
    p = o.d_cost; free_dev(p); o.d_cost = nullptr;
    if (o.done) (void)hipEventDestroy(o.done);
  }
  if (c->ev_frame) (void)hipEventDestroy(c->ev_frame);
  if (c->ev_counters) (void)hipEventDestroy(c->ev_counters);
  c->ev_counters = nullptr;
  c->counters_stream = nullptr;
  if (c->side) (void)hipStreamDestroy(c->side);
  p = c->d_tile_stats; free_dev(p); c->d_tile_stats = nullptr;
  p = c->d_tile_samples; free_dev(p); c->d_tile_samples = nullptr;
  for (hipEvent_t e : c->ev_start) (void)hipEventDestroy(e);
  for (hipEvent_t e : c->ev_stop) (void)hipEventDestroy(e);
  if (c->own_stream) (void)hipStreamDestroy(c->own_stream);
  delete c;
}

const char* cvr_last_error(const cvr_ctx* ctx) {
  const Ctx* c = reinterpret_cast<const Ctx*>(ctx);
  return c ? c->err.c_str() : "null context";
}

cvr_status cvr_set_stream(cvr_ctx* ctx, void* stream) {
  Ctx* c = reinterpret_cast<Ctx*>(ctx);
  if (!c) return CVR_ERR_ARG;
  c->stream = (hipStream_t)stream;     // NULL = the legacy default stream
  return CVR_OK;
}

cvr_status cvr_set_option(cvr_ctx* ctx, const char* key, int value) {
  Ctx* c = reinterpret_cast<Ctx*>(ctx);
  if (!c || !key) return CVR_ERR_ARG;
  if (c->group) {
    for (const char* k : {"split_streams", "gather_sets", "gather_root_idle", "exchange_lag"})
      if (!std::strcmp(key, k))
        return fail(c, CVR_ERR_ARG, "option '%s' belongs to the group's own exchange", key);
    return cvr::group_each(c, [&](cvr_ctx* _m) { return cvr_set_option(_m, key, value); });
  }
  if (!std::strcmp(key, "batch")) {
    if (value != 0 && value != 2 && value != 4)
      return fail(c, CVR_ERR_ARG, "batch must be 0 (auto), 2 or 4");
    c->batch = value;
    return CVR_OK;
  }
  if (!std::strcmp(key, "tile_order")) {
    if (value < 0 || value > 2) return fail(c, CVR_ERR_ARG, "tile_order must be 0, 1 or 2");
    c->use_order = value;
    for (auto& o : c->oslot) o.valid = 0;
    return CVR_OK;
  }
  if (!std::strcmp(key, "stale_deg")) {
    if (value < 0 || value > 180) return fail(c, CVR_ERR_ARG, "stale_deg must be 0..180");
    c->stale_deg = value;
    return CVR_OK;
  }
  if (!std::strcmp(key, "quad")) {
    if (value < 0 || value > 100) return fail(c, CVR_ERR_ARG, "quad must be a percentage");
    c->quad_pct = value;
    for (auto& o : c->oslot) o.valid = 0;
    return CVR_OK;
  }
  if (!std::strcmp(key, "filter_bits")) {
    if (value != 0 && value != 8)
      return fail(c, CVR_ERR_ARG, "filter_bits must be 0 (exact weights) or 8 (texture-unit weights)");
    c->filter_bits = value;
    for (auto& o : c->oslot) o.valid = 0;
    return CVR_OK;
  }
  if (!std::strcmp(key, "sat_chunk")) {
    if (value < 1 || value > 64) return fail(c, CVR_ERR_ARG, "sat_chunk must be 1..64");
    c->sat_chunk = value;
    return CVR_OK;
  }
  if (!std::strcmp(key, "sat_layout")) {
    if (value < 0 || value > 1)
      return fail(c, CVR_ERR_ARG, "sat_layout must be 0 (cell4 copy) or 1 (the plain float SAT)");
    if (value == 1 && c->d_sat_cells) {   // the copy is not needed any more (17 GiB at 1024^3)
      HIP_TRY(c, hipSetDevice(c->device));
      HIP_TRY(c, hipDeviceSynchronize());
      void* p = c->d_sat_cells; free_dev(p); c->d_sat_cells = nullptr;
    }
    c->sat_layout = value;
    return CVR_OK;
  }
  if (!std::strcmp(key, "sat_keep_scratch")) {
    if (value < 0 || value > 1) return fail(c, CVR_ERR_ARG, "sat_keep_scratch must be 0 or 1");
    c->sat_keep_scratch = value;
    if (!value && c->d_sat_scratch) {
      HIP_TRY(c, hipSetDevice(c->device));
      HIP_TRY(c, hipDeviceSynchronize());
      void* p = c->d_sat_scratch; free_dev(p); c->d_sat_scratch = nullptr;
    }
    return CVR_OK;
  }
  if (!std::strcmp(key, "shade_flat")) {
    if (value < 0 || value > 1) return fail(c, CVR_ERR_ARG, "shade_flat must be 0 or 1");
    c->shade_flat = value;
    return CVR_OK;
  }
  if (!std::strcmp(key, "flat_group")) {
    if (value < 1 || value > 4096) return fail(c, CVR_ERR_ARG, "flat_group must be in [1, 4096]");
    c->flat_group = value;
    return CVR_OK;
  }
  if (!std::strcmp(key, "debug_flat_limit")) {   // tests: force the flat pipeline's fallback
    if (value < 0) return fail(c, CVR_ERR_ARG, "debug_flat_limit must be >= 0");
    c->debug_flat_limit = value;
    return CVR_OK;
  }
  if (!std::strcmp(key, "shade_counters")) {
    c->shade_counters = value ? 1 : 0;
    return CVR_OK;
  }
  if (!std::strcmp(key, "tile_stats")) {
    c->tile_stats = value != 0;
    return CVR_OK;
  }
  if (!std::strcmp(key, "kernel_timing")) {
    if (value < 0 || value > 4096) return fail(c, CVR_ERR_ARG, "kernel_timing must be 0..4096 frames");
    HIP_TRY(c, hipSetDevice(c->device));
    HIP_TRY(c, hipStreamSynchronize(c->stream));
    for (hipEvent_t e : c->ev_start) (void)hipEventDestroy(e);
    for (hipEvent_t e : c->ev_stop) (void)hipEventDestroy(e);
    c->ev_start.clear();
    c->ev_stop.clear();
    c->timed_frames = 0;
    for (int i = 0; i < value; i++) {
      hipEvent_t a, b;
      HIP_TRY(c, hipEventCreate(&a));
      c->ev_start.push_back(a);
      HIP_TRY(c, hipEventCreate(&b));
      c->ev_stop.push_back(b);
    }
    return CVR_OK;
  }
  if (!std::strcmp(key, "macro")) {
    if (value != 0 && (value < 2 || value > 6))
      return fail(c, CVR_ERR_ARG, "macro must be 0 (no empty-space skipping) or 2..6");
    c->macro_shift = value;
    c->occ_valid = 0;
    return CVR_OK;
  }
  if (!std::strcmp(key, "cell_skip")) {
    if (value < 0 || value > 4)
      return fail(c, CVR_ERR_ARG, "cell_skip must be 0 (off), 1 (empty-sample flags), 2 (+ distance "
                                  "skip per lane), 3 (+ distance skip when every lane can) or 4 (+ "
                                  "distance skip, equal for the lanes that can)");
    c->cell_skip = value;
    return CVR_OK;
  }
  if (!std::strcmp(key, "skip_min_pct")) {
    if (value < 0 || value > 101) return fail(c, CVR_ERR_ARG, "skip_min_pct must be 0..101");
    c->skip_min_pct = value;
    return CVR_OK;
  }
  if (!std::strcmp(key, "tile_cost")) {
    if (value < 0 || value > 1) return fail(c, CVR_ERR_ARG, "tile_cost must be 0 (longest ray) or 1 (time)");
    c->cost_time = value;
    return CVR_OK;
  }
  if (!std::strcmp(key, "max_waves_cu")) {
    if (value < 0 || value > 32) return fail(c, CVR_ERR_ARG, "max_waves_cu must be 0..32");
    c->max_waves_cu = value;
    return CVR_OK;
  }
  if (!std::strcmp(key, "launch_interleave")) {
    if (value < 0 || value > 1) return fail(c, CVR_ERR_ARG, "launch_interleave must be 0 or 1");
    c->launch_interleave = value;
    return CVR_OK;
  }
  if (!std::strcmp(key, "gather_root_idle")) {
    if (value < 0 || value > 1) return fail(c, CVR_ERR_ARG, "gather_root_idle must be 0 or 1");
    c->gather_root_idle = value;
    return CVR_OK;
  }
  if (!std::strcmp(key, "gather_sets")) {
    // exchange g waits for exchange g + D - B, which the 64-event ring still holds
    // while B - D < 64 (cvr_comm.cpp): any B <= 64 with D >= 1 render streams
    if (value < 0 || value > CVR_MAX_GATHER_SETS)
      return fail(c, CVR_ERR_ARG, "gather_sets must be 0..%d", CVR_MAX_GATHER_SETS);
    c->gather_sets = value;
    return CVR_OK;
  }
  if (!std::strcmp(key, "exchange_code")) {
    if (value < 0 || value > 1) return fail(c, CVR_ERR_ARG, "exchange_code must be 0 or 1");
    c->exchange_code = value;
    return CVR_OK;
  }
  if (!std::strcmp(key, "native_exp")) {
    // tolerance mode: NOT bit-exact with the oracle (DESIGN §5‴)
    if (value < 0 || value > 1) return fail(c, CVR_ERR_ARG, "native_exp must be 0 or 1");
    c->native_exp = value;
    return CVR_OK;
  }
  if (!std::strcmp(key, "encode_onepass")) {
    if (value < 0 || value > 1) return fail(c, CVR_ERR_ARG, "encode_onepass must be 0 or 1");
    c->encode_onepass = value;
    return CVR_OK;
  }
  if (!std::strcmp(key, "exchange_lag")) {
    if (value < -1 || value >= CVR_MAX_GATHER_SETS)
      return fail(c, CVR_ERR_ARG, "exchange_lag must be -1 (auto) .. %d", CVR_MAX_GATHER_SETS - 1);
    c->exchange_lag = value;
    return CVR_OK;
  }
  if (!std::strcmp(key, "split_streams")) {
    if (value < 1 || value > 32) return fail(c, CVR_ERR_ARG, "split_streams must be 1..32");
    c->split_streams = value;
    return CVR_OK;
  }
  if (!std::strcmp(key, "async_order")) {
    if (value < 0 || value > 1) return fail(c, CVR_ERR_ARG, "async_order must be 0 or 1");
    if (c->side) HIP_TRY(c, hipStreamSynchronize(c->side));
    c->async_order = value;
    for (auto& o : c->oslot) { o.valid = 0; o.pending = false; }
    return CVR_OK;
  }
  if (!std::strcmp(key, "order_interval")) {
    if (value < 1 || value > 1000000) return fail(c, CVR_ERR_ARG, "order_interval must be >= 1");
    c->order_interval = value;
    return CVR_OK;
  }
  if (!std::strcmp(key, "debug_epi_stop")) {   // diagnostics: truncated order builds
    c->epi_stop = value;
    return CVR_OK;
  }
  if (!std::strcmp(key, "debug_cell_flags_oom")) {   // tests: the skip flags' scratch "fails"
    if (value < 0 || value > 1) return fail(c, CVR_ERR_ARG, "debug_cell_flags_oom must be 0 or 1");
    c->debug_flags_oom = value;
    return CVR_OK;
  }
  if (!std::strcmp(key, "debug_keep")) {   // diagnostics only: the image is incomplete
    if (value < 0) return fail(c, CVR_ERR_ARG, "debug_keep must be >= 0");
    c->debug_keep = value;
    return CVR_OK;
  }
  if (!std::strcmp(key, "boost")) {
    if (value < 0 || value > 100) return fail(c, CVR_ERR_ARG, "boost must be a percentage");
    c->boost_pct = value;
    return CVR_OK;
  }
  if (!std::strcmp(key, "band_cap")) {
    if (value < 100 || value > 200) return fail(c, CVR_ERR_ARG, "band_cap must be 100..200");
    if (value != c->band_cap_pct)
      for (auto& o : c->oslot) o.valid = 0;   // the learned orders are laid out for the old cap
    c->band_cap_pct = value;
    return CVR_OK;
  }
  return fail(c, CVR_ERR_ARG, "unknown option '%s'", key);
}

int cvr_get_option(const cvr_ctx* ctx, const char* key) {
  const Ctx* c = reinterpret_cast<const Ctx*>(ctx);
  if (!c || !key) return -1;
  if (c->group) return cvr_get_option(cvr_group_member(const_cast<cvr_ctx*>(ctx), 0), key);
  if (!std::strcmp(key, "batch")) return c->batch;
  if (!std::strcmp(key, "tile_order")) return c->use_order;
  if (!std::strcmp(key, "stale_deg")) return c->stale_deg;
  if (!std::strcmp(key, "boost")) return c->boost_pct;
  if (!std::strcmp(key, "band_cap")) return c->band_cap_pct;
  if (!std::strcmp(key, "tile_cost")) return c->cost_time;
  if (!std::strcmp(key, "macro")) return c->macro_shift;
  if (!std::strcmp(key, "max_waves_cu")) return c->max_waves_cu;
  if (!std::strcmp(key, "debug_keep")) return c->debug_keep;
  if (!std::strcmp(key, "debug_cell_flags_oom")) return c->debug_flags_oom;
  if (!std::strcmp(key, "cell_flags_active")) return c->cell_flags_valid && !c->cell_flags_oom;   // read-only
  if (!std::strcmp(key, "debug_epi_stop")) return c->epi_stop;
  if (!std::strcmp(key, "async_order")) return c->async_order;
  if (!std::strcmp(key, "split_streams")) return c->split_streams;
  if (!std::strcmp(key, "gather_sets")) return c->gather_sets;
  if (!std::strcmp(key, "gather_root_idle")) return c->gather_root_idle;
  if (!std::strcmp(key, "exchange_code")) return c->exchange_code;
  if (!std::strcmp(key, "exchange_lag")) return c->exchange_lag;
  if (!std::strcmp(key, "encode_onepass")) return c->encode_onepass;
  if (!std::strcmp(key, "native_exp")) return c->native_exp;
  if (!std::strcmp(key, "launch_interleave")) return c->launch_interleave;
  if (!std::strcmp(key, "sat_build_us")) return c->sat_build_us;   // read-only
  if (!std::strcmp(key, "order_interval")) return c->order_interval;
  if (!std::strcmp(key, "skip_min_pct")) return c->skip_min_pct;
  if (!std::strcmp(key, "cell_skip")) return c->cell_skip;
  if (!std::strcmp(key, "cell_flags_valid")) return c->cell_flags_valid;   // read-only
  if (!std::strcmp(key, "occ_empty_permille"))   // read-only: empty macro cells (after a render)
    return c->occ_valid ? (int)(c->occ_empty * 1000.0f + 0.5f) : -1;
  if (!std::strcmp(key, "tile_stats")) return c->tile_stats;
  if (!std::strcmp(key, "shade_counters")) return c->shade_counters;
  if (!std::strcmp(key, "shade_flat")) return c->shade_flat;
  if (!std::strcmp(key, "flat_group")) return c->flat_group;
  if (!std::strcmp(key, "debug_flat_limit")) return c->debug_flat_limit;
  if (!std::strcmp(key, "flat_cap_kjobs")) {   // read-only: the context stream's job-list capacity
    for (const auto& J : c->flat)
      if (J.owned && J.stream == c->stream) return (int)(J.cap / 1000);
    return 0;
  }
  if (!std::strcmp(key, "sat_chunk")) return c->sat_chunk;
  if (!std::strcmp(key, "sat_layout")) return c->sat_layout;
  if (!std::strcmp(key, "sat_keep_scratch")) return c->sat_keep_scratch;
  if (!std::strcmp(key, "quad")) return c->quad_pct;
  if (!std::strcmp(key, "filter_bits")) return c->filter_bits;
  if (!std::strcmp(key, "kernel_timing")) return (int)c->ev_start.size();
  return -1;
}

cvr_status cvr_synchronize(cvr_ctx* ctx) {
  Ctx* c = reinterpret_cast<Ctx*>(ctx);
  if (!c) return CVR_ERR_ARG;
  if (c->group) {
    cvr_status st = cvr::group_each(c, [&](cvr_ctx* _m) { return cvr_synchronize(_m); });
    if (st != CVR_OK) return st;
  }
  HIP_TRY(c, hipSetDevice(c->device));
  HIP_TRY(c, hipStreamSynchronize(c->stream));
  if (c->side) HIP_TRY(c, hipStreamSynchronize(c->side));
  return CVR_OK;
}

size_t cvr_device_bytes(const cvr_ctx* ctx) {
  const Ctx* c = reinterpret_cast<const Ctx*>(ctx);
  if (!c) return 0;
  if (c->group) {
    size_t b = 0;
    for (int i = 0; i < cvr_group_size(ctx); i++)
      b += cvr_device_bytes(cvr_group_member(const_cast<cvr_ctx*>(ctx), i));
    return b;
  }
  return c->vox_bytes + c->cells_bytes + c->grad_bytes + (size_t)c->tf_n * 16 + c->scratch_bytes;
}

cvr_status cvr_copy_cells(cvr_ctx* ctx, void* out, size_t capacity) {
  Ctx* c = reinterpret_cast<Ctx*>(ctx);
  if (c && c->group) return cvr::group_call_root(c, [&](cvr_ctx* _m) { return cvr_copy_cells(_m, out, capacity); });
  if (!c || !out) return CVR_ERR_ARG;
  if (!c->d_cells) return fail(c, CVR_ERR_STATE, "cvr_copy_cells: no volume set");
  if (capacity < c->cells_bytes)
    return fail(c, CVR_ERR_ARG, "cvr_copy_cells: need %zu bytes", c->cells_bytes);
  HIP_TRY(c, hipSetDevice(c->device));
  HIP_TRY(c, hipDeviceSynchronize());
  HIP_TRY(c, hipMemcpy(out, c->d_cells, c->cells_bytes, hipMemcpyDeviceToHost));
  return CVR_OK;
}

static cvr_status set_volume_common(Ctx* c, const void* src, bool src_device, int bpv, int w,
                                    int h, int d, const float scale[3]) {
  if (!src || (bpv != 1 && bpv != 2) || w < 1 || h < 1 || d < 1 || !scale)
    return fail(c, CVR_ERR_ARG, "cvr_set_volume: bad arguments");
  if (!(scale[0] > 0 && scale[1] > 0 && scale[2] > 0))
    return fail(c, CVR_ERR_ARG, "cvr_set_volume: scale must be positive");
  if ((size_t)(w + 4) * (h + 4) * (d + 4) >= (size_t)1 << 32)
    return fail(c, CVR_ERR_ARG, "cvr_set_volume: volume too large for 32-bit cell indexing");
  if ((size_t)(w + 1) * (h + 1) >= (size_t)1 << 23)
    return fail(c, CVR_ERR_ARG, "cvr_set_volume: slice too large for 24-bit cell addressing");
  QUIESCE(c);   // frames in flight on any stream read the state replaced below
  free_dev(c->d_vox); c->vox_bytes = 0;
  free_dev(c->d_cells); c->cells_bytes = 0;
  free_dev(c->d_grad); c->grad_bytes = 0; c->grad_mode = 0;
  c->iso_valid = 0;
  c->N[0] = w; c->N[1] = h; c->N[2] = d;
  for (int i = 0; i < 3; i++) c->scale[i] = scale[i];
  c->bpv = bpv;
  c->vox_bytes = (size_t)w * h * d * bpv;
  HIP_TRY(c, hipMalloc(&c->d_vox, c->vox_bytes));
  HIP_TRY(c, hipMemcpyAsync(c->d_vox, src, c->vox_bytes,
                            src_device ? hipMemcpyDeviceToDevice : hipMemcpyHostToDevice, c->stream));
  // GetNormalizedSample -> (GLfloat) -> GL_R16F, as a per-value table
  const int nv = bpv == 1 ? 256 : 65536;
  std::vector<uint16_t> lut(nv);
  for (int v = 0; v < nv; v++)
    lut[v] = to_half_bits((float)((double)v / (bpv == 1 ? (256.0 - 1.0) : (65536.0 - 1.0))));
  { void* p = c->d_lut; free_dev(p); c->d_lut = nullptr; }
  { void* p = c->d_macro_minmax; free_dev(p); c->d_macro_minmax = nullptr; }
  { void* p = c->d_occ; free_dev(p); c->d_occ = nullptr; }
  c->mm_shift = -1;
  c->occ_valid = 0;
  c->cell_flags_valid = 0;   // the cells are rebuilt without flags
  c->cell_flags_set = 0;
  c->cell_flags_oom = 0;
  { void* p = c->d_ext; free_dev(p); c->d_ext = nullptr; c->ext_levels = 0; }
  { void* p = c->d_ext_cells; free_dev(p); c->d_ext_cells = nullptr; }
  { void* p = c->d_sat; free_dev(p); c->d_sat = nullptr; }
  { void* p = c->d_sat_cells; free_dev(p); c->d_sat_cells = nullptr; }
  { void* p = c->d_sat_scratch; free_dev(p); c->d_sat_scratch = nullptr; }
  c->sat_dims[0] = c->sat_dims[1] = c->sat_dims[2] = 0;
  c->cone_valid = 0;
  HIP_TRY(c, hipMalloc((void**)&c->d_lut, nv * sizeof(uint16_t)));
  uint16_t* d_lut = c->d_lut;
  hipError_t e = hipMemcpyAsync(d_lut, lut.data(), nv * sizeof(uint16_t), hipMemcpyHostToDevice,
                                c->stream);
  c->cells = cvr::make_cell_grid(c->N);
  c->cells_bytes = cvr::cell_count(c->cells) * 16;
  if (e == hipSuccess) e = hipMalloc(&c->d_cells, c->cells_bytes);
  if (e == hipSuccess)
    e = cvr::launch_build_cells_impl(c->d_vox, bpv, d_lut, c->N, c->cells, c->d_cells, c->stream);
  if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
  if (e != hipSuccess) {
    free_dev(c->d_cells); c->cells_bytes = 0;
    return fail(c, e == hipErrorOutOfMemory ? CVR_ERR_OOM : CVR_ERR_HIP,
                "cvr_set_volume: %s", hipGetErrorString(e));
  }
  return CVR_OK;
}

cvr_status cvr_set_volume(cvr_ctx* ctx, const void* voxels, int bpv, int w, int h, int d,
                          const float scale[3]) {
  Ctx* c = reinterpret_cast<Ctx*>(ctx);
  if (c && c->group) return cvr::group_each(c, [&](cvr_ctx* _m) { return cvr_set_volume(_m, voxels, bpv, w, h, d, scale); });
  if (!c) return CVR_ERR_ARG;
  return set_volume_common(c, voxels, false, bpv, w, h, d, scale);
}

cvr_status cvr_set_volume_device(cvr_ctx* ctx, const void* d_voxels, int bpv, int w, int h,
                                 int d, const float scale[3]) {
  Ctx* c = reinterpret_cast<Ctx*>(ctx);
  if (c && c->group) return cvr::group_each(c, [&](cvr_ctx* _m) { return cvr_set_volume_device(_m, d_voxels, bpv, w, h, d, scale); });
  if (!c) return CVR_ERR_ARG;
  return set_volume_common(c, d_voxels, true, bpv, w, h, d, scale);
}

cvr_status cvr_set_transfer_function(cvr_ctx* ctx, const float* rgbt, int n) {
  Ctx* c = reinterpret_cast<Ctx*>(ctx);
  if (c && c->group) return cvr::group_each(c, [&](cvr_ctx* _m) { return cvr_set_transfer_function(_m, rgbt, n); });
  if (!c) return CVR_ERR_ARG;
  if (!rgbt || n < 2 || n > 4096)
    return fail(c, CVR_ERR_ARG, "cvr_set_transfer_function: need 2 <= n <= 4096 entries");
  std::vector<float> q((size_t)n * 4);
  float amax = 0.0f;
  for (size_t i = 0; i < q.size(); i++) {
    q[i] = half_round(rgbt[i]);   // GL_RGBA16F
    if (i % 4 == 3) amax = std::isfinite(q[i]) ? std::max(amax, q[i]) : NAN;
  }
  QUIESCE(c);   // frames in flight on any stream read the state replaced below
  if (n != c->tf_n) {
    void* p = c->d_tf; free_dev(p); c->d_tf = nullptr;
    HIP_TRY(c, hipMalloc((void**)&c->d_tf, (size_t)n * 16));
    c->tf_n = n;
  }
  HIP_TRY(c, hipMemcpy(c->d_tf, q.data(), (size_t)n * 16, hipMemcpyHostToDevice));
  c->tf_max_alpha = amax;
  // occupancy support: prefix[k] = #{padded entries j < k with alpha > 0}, where
  // padded entry j is T[clamp(j - 1, 0, n - 1)] (j = 0 .. n + 1)
  std::vector<int> prefix((size_t)n + 3, 0);
  for (int j = 0; j < n + 2; j++) {
    const float a = q[(size_t)std::min(std::max(j - 1, 0), n - 1) * 4 + 3];
    prefix[(size_t)j + 1] = prefix[(size_t)j] + (a > 0.0f || a != a ? 1 : 0);
  }
  { void* p = c->d_tf_prefix; free_dev(p); c->d_tf_prefix = nullptr; }
  HIP_TRY(c, hipMalloc((void**)&c->d_tf_prefix, prefix.size() * sizeof(int)));
  HIP_TRY(c, hipMemcpy(c->d_tf_prefix, prefix.data(), prefix.size() * sizeof(int),
                       hipMemcpyHostToDevice));
  c->occ_valid = 0;
  c->cell_flags_valid = 0;
  c->cell_flags_oom = 0;
  return CVR_OK;
}

cvr_status cvr_set_gradient(cvr_ctx* ctx, int mode) {
  Ctx* c = reinterpret_cast<Ctx*>(ctx);
  if (c && c->group) return cvr::group_each(c, [&](cvr_ctx* _m) { return cvr_set_gradient(_m, mode); });
  if (!c) return CVR_ERR_ARG;
  if (mode < 0 || mode > 2) return fail(c, CVR_ERR_ARG, "cvr_set_gradient: bad mode %d", mode);
  if (mode != 0 && !c->d_vox) return fail(c, CVR_ERR_STATE, "cvr_set_gradient: no volume");
  QUIESCE(c);   // frames in flight on any stream read the state replaced below
  free_dev(c->d_grad); c->grad_bytes = 0; c->grad_mode = 0;
  if (mode == 0) return CVR_OK;
  c->grad_bytes = cvr::cell_count(c->cells) * 48;
  HIP_TRY(c, hipMalloc(&c->d_grad, c->grad_bytes));
  uint2* tmp = nullptr;
  hipError_t e = hipMalloc((void**)&tmp, (size_t)c->N[0] * c->N[1] * c->N[2] * 8);
  if (e == hipSuccess) e = cvr::launch_gradient(*c, mode, tmp, c->stream);
  if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
  (void)hipFree(tmp);
  if (e != hipSuccess) {
    free_dev(c->d_grad); c->grad_bytes = 0;
    return fail(c, e == hipErrorOutOfMemory ? CVR_ERR_OOM : CVR_ERR_HIP, "cvr_set_gradient: %s",
                hipGetErrorString(e));
  }
  c->grad_mode = mode;
  return CVR_OK;
}

int cvr_tiles_for_rank(const cvr_frame* f, int rank) {
  if (!f || f->width < 1 || f->height < 1) return 0;
  if (f->nranks <= 1) return 1;
  if (f->tile_size < 16 || f->tile_size % 16 != 0 || rank < 0 || rank >= f->nranks) return 0;
  int ntx = (f->width + f->tile_size - 1) / f->tile_size;
  int nty = (f->height + f->tile_size - 1) / f->tile_size;
  int nt = ntx * nty;
  return nt > rank ? (nt - rank + f->nranks - 1) / f->nranks : 0;
}

// The per-tile sample counts and shade counters are shared by every render
// stream.  A frame that uses them on stream s first waits for the last frame
// that used them on another stream (frames in flight on rotated streams), and
// records the event after its own epilogue (counters_release).
static cvr_status counters_acquire(Ctx* c, hipStream_t s) {
  if (!c->ev_counters) HIP_TRY(c, hipEventCreateWithFlags(&c->ev_counters, hipEventDisableTiming));
  if (c->counters_stream && c->counters_stream != s)
    HIP_TRY(c, hipStreamWaitEvent(s, c->ev_counters, 0));
  return CVR_OK;
}

static cvr_status counters_release(Ctx* c, hipStream_t s) {
  HIP_TRY(c, hipEventRecord(c->ev_counters, s));
  c->counters_stream = s;
  return CVR_OK;
}

static cvr_status ensure_scratch(Ctx* c, size_t bytes) {
  if (c->scratch_bytes >= bytes) return CVR_OK;
  free_dev(c->d_scratch);
  c->scratch_bytes = 0;
  HIP_TRY(c, hipMalloc(&c->d_scratch, bytes));
  c->scratch_bytes = bytes;
  return CVR_OK;
}

// Occupancy of the macro cells for the current volume, TF and macro size
// (rebuilt lazily after any of them changes; on the context stream).
static cvr_status ensure_occupancy(Ctx* c) {
  if (c->occ_valid) return CVR_OK;
  if (!c->d_lut || !c->d_tf_prefix) return fail(c, CVR_ERR_STATE, "occupancy: no volume or TF");
  QUIESCE(c);   // frames in flight on other streams may still read d_occ
  const int sh = c->macro_shift;
  if (c->mm_shift != sh) {
    for (int i = 0; i < 3; i++) c->mdim[i] = ((c->N[i] - 1) >> sh) + 1;
    const size_t nm = (size_t)c->mdim[0] * c->mdim[1] * c->mdim[2];
    { void* p = c->d_macro_minmax; free_dev(p); c->d_macro_minmax = nullptr; }
    { void* p = c->d_occ; free_dev(p); c->d_occ = nullptr; }
    HIP_TRY(c, hipMalloc((void**)&c->d_macro_minmax, nm * sizeof(uint32_t)));
    HIP_TRY(c, hipMalloc((void**)&c->d_occ, nm));
    HIP_TRY(c, cvr::launch_macro_minmax(*c, sh, c->mdim, c->d_macro_minmax, c->stream));
    c->mm_shift = sh;
  }
  const int nm = c->mdim[0] * c->mdim[1] * c->mdim[2];
  if (!c->d_total) HIP_TRY(c, hipMalloc((void**)&c->d_total, sizeof(unsigned long long)));
  unsigned int* d_n = reinterpret_cast<unsigned int*>(c->d_total);
  HIP_TRY(c, hipMemsetAsync(d_n, 0, sizeof(unsigned int), c->stream));
  HIP_TRY(c, cvr::launch_occupancy(c->d_macro_minmax, nm, c->d_lut, c->d_tf_prefix, c->tf_n,
                                   c->d_occ, d_n, c->stream));
  unsigned int n_empty = 0;
  HIP_TRY(c, hipMemcpyAsync(&n_empty, d_n, sizeof(n_empty), hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(c, hipStreamSynchronize(c->stream));
  c->occ_empty = (float)n_empty / (float)nm;
  c->occ_valid = 1;
  return CVR_OK;
}

// Skip flags of the density cells for the current volume and TF (rebuilt lazily
// after either changes; on the context stream).  Frames in flight on other
// streams may still read the cells' old flags, so the device drains first (a
// TF change is rare); the two scratch bytes per cell are freed after the build.
static cvr_status ensure_cell_flags(Ctx* c) {
  if (c->cell_flags_valid) return CVR_OK;
  if (!c->d_cells || !c->d_tf_prefix) return fail(c, CVR_ERR_STATE, "cell flags: no volume or TF");
  HIP_TRY(c, hipSetDevice(c->device));
  HIP_TRY(c, hipDeviceSynchronize());
  const size_t n = cvr::cell_count(c->cells);
  if (c->debug_flags_oom)   // tests: the scratch allocation fails
    return fail(c, CVR_ERR_OOM, "cell flags: scratch allocation failed (debug_cell_flags_oom)");
  uint8_t* t = nullptr;
  HIP_TRY(c, hipMalloc((void**)&t, 2 * n));
  hipError_t e = cvr::launch_cell_flags(*c, false, t, t + n, c->stream);
  if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
  (void)hipFree(t);
  if (e != hipSuccess)
    return fail(c, e == hipErrorOutOfMemory ? CVR_ERR_OOM : CVR_ERR_HIP, "cell flags: %s",
                hipGetErrorString(e));
  c->cell_flags_valid = 1;
  c->cell_flags_set = 1;
  return CVR_OK;
}

// The per-cell skip is a bit-exact optimisation, so a frame must not fail for
// want of its 2 bytes of scratch per cell (2.1 GB at 1024^3, next to the EBS
// SAT): on OOM the frame renders without it (every density read takes |corner|,
// so stale flags in the sign bits are ignored) until the next volume or TF
// change, which clears cell_flags_oom and retries the build.  The frame itself
// succeeds, so the OOM message is not left in cvr_last_error.  Any other error is
// returned.
static cvr_status cell_flags_or_off(Ctx* c) {
  if (c->cell_flags_oom && !c->cell_flags_valid) return CVR_ERR_OOM;
  const cvr_status st = ensure_cell_flags(c);
  if (st == CVR_ERR_OOM) {
    (void)hipGetLastError();   // clear the failed allocation's error
    c->cell_flags_oom = 1;
    c->err.clear();
  }
  return st;
}

// Camera, volume and tiling constants of one frame (shared by every renderer):
// ray generation (glm lookAt + tan(fovy/2)), VolumeGridSize, step, TF size, and
// the 8x8 wave tiles of the whole image or of this rank's packed tiles.
static void fill_frame_args(Ctx* c, const cvr_frame* f, float step, cvr::Rc1passArgs& A,
                            int& ntiles, size_t& npix) {
  float V[16], tanh;
  cvr_camera_lookat(&f->camera, V, &tanh);
  if (f->use_view)
    for (int i = 0; i < 16; i++) V[i] = f->view[i];
  for (int i = 0; i < 3; i++) {
    A.eye[i] = f->camera.eye[i];
    A.col0[i] = V[0 * 4 + i];
    A.col1[i] = V[1 * 4 + i];
    A.col2[i] = V[2 * 4 + i];
  }
  A.tan_half_fovy = tanh;
  A.aspect = f->camera.aspect > 0 ? f->camera.aspect : (float)f->width / (float)f->height;
  A.W = f->width;
  A.H = f->height;
  for (int i = 0; i < 3; i++) {
    float G = (float)c->N[i] * c->scale[i];     // VolumeGridSize, rc1prenderer.cpp:241
    A.half_grid[i] = G * 0.5f;
    A.n_over_g[i] = (float)c->N[i] / G;
    A.nm1[i] = (float)(c->N[i] - 1);
    A.N[i] = c->N[i];
  }
  A.cells = c->cells;
  A.step = step > 0 ? step : cvr_default_step(c->scale);
  A.tf_n = c->tf_n;
  // Sample opacity: a TF lerp lies within [0, max alpha] up to an ulp, and h <= step.
  const double ext = (double)c->tf_max_alpha * (double)A.step * (1.0 + 1.0 / 1024.0);
  A.exp_fast = (ext >= 0.0 && ext <= 86.0) ? 1 : 0;
  A.exp_native = c->native_exp;
  if (f->nranks <= 1) {
    A.packed = 0;
    ntiles = ((f->width + 7) / 8) * ((f->height + 7) / 8);
    npix = (size_t)f->width * f->height;
  } else {
    A.packed = 1;
    A.tile = f->tile_size; A.rank = f->rank; A.nranks = f->nranks;
    A.ntx = (f->width + f->tile_size - 1) / f->tile_size;
    A.my_tiles = cvr_tiles_for_rank(f, f->rank);
    const int s8 = f->tile_size / 8;
    ntiles = A.my_tiles * s8 * s8;
    npix = (size_t)A.my_tiles * f->tile_size * f->tile_size;
  }
  A.ntiles = ntiles;
}

// The view a launch order was learned on: eye, unit forward direction (the
// centre pixel's ray, -(row 2 of mat3(View))), tan(fovy/2).
static void view_signature(const cvr::Rc1passArgs& A, float v[7]) {
  const float fx = -A.col0[2], fy = -A.col1[2], fz = -A.col2[2];
  const float n = std::sqrt(fx * fx + fy * fy + fz * fz);
  const float inv = n > 0.0f ? 1.0f / n : 0.0f;
  v[0] = A.eye[0]; v[1] = A.eye[1]; v[2] = A.eye[2];
  v[3] = fx * inv; v[4] = fy * inv; v[5] = fz * inv;
  v[6] = A.tan_half_fovy;
}

// Tile costs shift with the view: an order learned on a view more than `deg`
// degrees (direction, or an eye displacement of the matching chord of the eye's
// distance to the volume centre, or a zoom of that fraction) away is stale.
static bool view_close(const float a[7], const float b[7], int deg) {
  if (deg <= 0) return true;
  const double rad = deg * 3.14159265358979 / 180.0;
  const double c = (double)a[3] * b[3] + (double)a[4] * b[4] + (double)a[5] * b[5];
  if (c < std::cos(rad)) return false;
  const double dx = a[0] - b[0], dy = a[1] - b[1], dz = a[2] - b[2];
  const double r = std::sqrt((double)b[0] * b[0] + (double)b[1] * b[1] + (double)b[2] * b[2]);
  if (std::sqrt(dx * dx + dy * dy + dz * dz) > rad * std::max(r, 1e-6)) return false;
  return std::fabs((double)a[6] - b[6]) <= rad * std::fabs((double)b[6]);
}

// nf frames (1..kMaxLaunchFrames) in one ray-march launch; nf = 1 is cvr_render_rc1pass.
static cvr_status render_rc1pass_frames(Ctx* c, const cvr_frame* frames, int nf,
                                        const cvr_rc1pass_params* p, const cvr_output* outs) {
  const cvr_frame* f = frames;
  const cvr_output* o = outs;
  if (!f || !p || !o || !o->rgba) return fail(c, CVR_ERR_ARG, "cvr_render_rc1pass: null argument");
  if (nf < 1 || nf > cvr::kMaxLaunchFrames)
    return fail(c, CVR_ERR_ARG, "cvr_render_rc1pass_frames: nframes %d not in 1..%d", nf,
                cvr::kMaxLaunchFrames);
  for (int i = 1; i < nf; i++) {
    const cvr_frame& g = frames[i];
    if (g.width != f->width || g.height != f->height || g.tile_size != f->tile_size ||
        g.rank != f->rank || g.nranks != f->nranks)
      return fail(c, CVR_ERR_ARG, "cvr_render_rc1pass_frames: frame %d differs from frame 0 in "
                                  "viewport or screen split", i);
    if (!outs[i].rgba || !outs[i].on_device || outs[i].format != o->format || outs[i].total)
      return fail(c, CVR_ERR_ARG, "cvr_render_rc1pass_frames: output %d must be a device buffer of "
                                  "frame 0's format, without a total", i);
  }
  if (nf > 1 && !o->on_device)
    return fail(c, CVR_ERR_ARG, "cvr_render_rc1pass_frames: the outputs must be device buffers");
  if (o->format != CVR_FORMAT_RGBA32F && o->format != CVR_FORMAT_RGBA16F)
    return fail(c, CVR_ERR_ARG, "cvr_render_rc1pass: unknown output format %d", o->format);
  if (f->width < 1 || f->height < 1 || f->width > 32768 || f->height > 32768)
    return fail(c, CVR_ERR_ARG, "cvr_render_rc1pass: bad viewport %dx%d", f->width, f->height);
  if (!c->d_cells) return fail(c, CVR_ERR_STATE, "cvr_render_rc1pass: no volume set");
  if (!c->d_tf) return fail(c, CVR_ERR_STATE, "cvr_render_rc1pass: no transfer function set");
  const bool phong = p->apply_gradient_shading != 0;
  if (phong && !c->d_grad)
    return fail(c, CVR_ERR_STATE, "cvr_render_rc1pass: gradient shading needs cvr_set_gradient");
  const bool packed = f->nranks > 1;
  if (packed && (f->tile_size < 16 || f->tile_size % 16 != 0 || f->rank < 0 || f->rank >= f->nranks))
    return fail(c, CVR_ERR_ARG, "cvr_render_rc1pass: bad tiling (tile %d, rank %d/%d)",
                f->tile_size, f->rank, f->nranks);

  cvr::Rc1passArgs A{};
  cvr::RenderPlan plan{};
  size_t npix;
  fill_frame_args(c, f, p->step, A, plan.ntiles, npix);
  A.ka = p->ka; A.kd = p->kd; A.ks = p->ks; A.shininess = p->shininess;
  for (int i = 0; i < 3; i++) { A.ispec[i] = p->ispecular[i]; A.light[i] = p->light_pos[i]; }
  A.filter_bits = c->filter_bits;
  A.tile_stats = nullptr;
  A.cost_time = c->cost_time;
  A.occ = nullptr;
  A.cell_skip = 0;
  if (c->cell_skip > 0) {   // (the quad march ignores it)
    const cvr_status st = cell_flags_or_off(c);
    if (st == CVR_OK) {
      A.cell_skip = c->cell_skip;
      A.inv_step = 1.0f / A.step;
    } else if (st != CVR_ERR_OOM) {
      return st;
    }
  }
  if (c->macro_shift > 0 && A.cell_skip == 0) {
    cvr_status st = ensure_occupancy(c);
    if (st != CVR_OK) return st;
    // the skip path costs the march registers and a probe: worth it only
    // with enough empty space (the Marschner-Lobb headline field has ~4 %)
    if (c->occ_empty * 100.0f >= (float)c->skip_min_pct) {
      A.occ = c->d_occ;
      for (int i = 0; i < 3; i++) A.mdim[i] = c->mdim[i];
      A.mshift = c->macro_shift;
    }
  }
  if (c->tile_stats) {
    if (c->tile_stats_n < plan.ntiles) {
      void* p = c->d_tile_stats; free_dev(p); c->d_tile_stats = nullptr; c->tile_stats_n = 0;
      HIP_TRY(c, hipMalloc((void**)&c->d_tile_stats, (size_t)plan.ntiles * 32));
      c->tile_stats_n = plan.ntiles;
    }
    A.tile_stats = c->d_tile_stats;
  }
  A.shade_ctr = nullptr;
  const bool use_counters = c->shade_counters || o->total;
  if (use_counters) {
    cvr_status st = counters_acquire(c, c->stream);
    if (st != CVR_OK) return st;
  }
  if (c->shade_counters) {   // measurement: shaded samples (gradient fetches), skipped samples
    if (!c->d_shade) HIP_TRY(c, hipMalloc((void**)&c->d_shade, 3 * sizeof(unsigned long long)));
    HIP_TRY(c, hipMemsetAsync(c->d_shade, 0, 3 * sizeof(unsigned long long), c->stream));
    A.shade_ctr = c->d_shade;
  }
  plan.quad_pct = c->filter_bits ? 0 : c->quad_pct;   // the quad march has no filter_bits variant
  {
    // Bands are cut by predicted work, so one may hold more than 1/8 of the
    // tiles: up to band_cap % of the even share (default 130;
    // tile_epilogue_kernel moves the band boundaries the least that fits the
    // cap); every band gets that many slots (+3 per quad-split tile), and the
    // slots past a band's entries are empty workgroups.
    const int seg_avg = (plan.ntiles + 7) / 8;
    const int cap = (int)(((long long)seg_avg * c->band_cap_pct + 99) / 100);
    plan.max_seg = std::min(std::min(plan.ntiles, cap), cvr::kMaxBandTiles);
    if (plan.max_seg < seg_avg) plan.max_seg = seg_avg;   // (too large to order; see can_order)
    int per_band = plan.max_seg + 3 * (int)(((long long)plan.max_seg * plan.quad_pct) / 100);
    per_band = (per_band + 3) & ~3;   // whole groups of 4 waves per workgroup (raymarch.hip)
    plan.order_slots = 8 * per_band;
    plan.boost = (int)(((long long)seg_avg * c->boost_pct) / 100);
    plan.keep = c->debug_keep;
    plan.epi_stop = c->epi_stop;
  }

  HIP_TRY(c, hipSetDevice(c->device));
  hipStream_t s = c->stream;
  float4* d_out;
  uint32_t* d_samples;
  unsigned long long* d_total;
  A.out_half = o->format == CVR_FORMAT_RGBA16F;
  size_t rgba_bytes = npix * (A.out_half ? 8 : 16), smp_bytes = npix * 4;
  if (o->on_device) {
    d_out = (float4*)o->rgba;
    d_samples = (uint32_t*)o->samples;
    d_total = (unsigned long long*)o->total;
  } else {
    cvr_status st = ensure_scratch(c, rgba_bytes + (o->samples ? smp_bytes : 0));
    if (st != CVR_OK) return st;
    d_out = (float4*)c->d_scratch;
    d_samples = o->samples ? (uint32_t*)((char*)c->d_scratch + rgba_bytes) : nullptr;
    d_total = o->total ? c->d_total : nullptr;
  }
  // device outputs: the kernel ADDS to *total (the caller zeroes it); host
  // outputs: the context's own counter is reset here.
  if (d_total && !o->on_device) HIP_TRY(c, hipMemsetAsync(d_total, 0, sizeof(unsigned long long), s));

  // Longest-first (LPT) order learned three frames back (same plan): the kernel
  // records each wave tile's critical path into this frame's slot, and the
  // slot's order is rebuilt from it on the side stream while the next frame
  // renders (tile_epilogue_kernel: work-balanced XCD bands + bucket LPT).
  const bool can_order = c->use_order == 1 && (plan.ntiles + 7) / 8 <= cvr::kMaxBandTiles;
  A.interleave = c->use_order == 2;
  float vsig[7];
  view_signature(A, vsig);
  // frames 1.. of a multi-frame launch: their views (the rest of A is frame 0's)
  cvr::LaunchFrames lf;
  lf.n = nf;
  lf.grid = 0;
  bool views_close = true;   // every frame of the launch near frame 0's view (one launch order)
  for (int i = 0; i < nf; i++) {
    cvr::Rc1passArgs Ai = A;
    if (i > 0) {
      int nti;
      size_t npi;
      fill_frame_args(c, &frames[i], p->step, Ai, nti, npi);
      float vi[7];
      view_signature(Ai, vi);
      if (!view_close(vi, vsig, c->stale_deg)) views_close = false;
    }
    cvr::FrameView& v = lf.view[i];
    for (int k = 0; k < 3; k++) {
      v.eye[k] = Ai.eye[k];
      v.col0[k] = Ai.col0[k];
      v.col1[k] = Ai.col1[k];
      v.col2[k] = Ai.col2[k];
    }
    v.tan_half_fovy = Ai.tan_half_fovy;
    v.aspect = Ai.aspect;
    lf.out[i] = (float4*)outs[i].rgba;
    lf.samples[i] = (uint32_t*)outs[i].samples;
  }
  if (nf > 1) plan.frames = &lf;
  const int key = (plan.ntiles << 2) ^ (plan.quad_pct << 24) ^
                  (packed ? (f->rank << 8) ^ (f->nranks << 12) ^ 1 : 0);
  const int* order = nullptr;
  uint32_t* tile_cost = nullptr;
  // One slot per render stream: frames issued on different streams may overlap
  // on the device (the screen-tile split alternates two), and a slot's order,
  // costs and rebuilds stay in its stream's order.  async_order: slots rotate.
  int si = -1;
  if (c->async_order) {
    si = (int)(c->frame_no % 3);
  } else {
    for (int i = 0; i < Ctx::kOrderSlots; i++)
      if (c->oslot[i].owned && c->oslot[i].stream == s) si = i;
    if (si < 0) {
      si = c->slot_rr++ % Ctx::kOrderSlots;
      Ctx::OrderSlot& o = c->oslot[si];
      if (o.owned) HIP_TRY(c, hipDeviceSynchronize());   // the slot's last frame is done
      o.stream = s;
      o.owned = true;
      o.valid = 0;
      o.frames = 0;
    }
  }
  Ctx::OrderSlot& os = c->oslot[si];
  if (can_order) {
    if (c->async_order && !c->side) {   // side stream + events only for side-stream sorts
      int lo = 0, hi = 0;
      HIP_TRY(c, hipDeviceGetStreamPriorityRange(&lo, &hi));
      HIP_TRY(c, hipStreamCreateWithPriority(&c->side, hipStreamNonBlocking, hi));
      HIP_TRY(c, hipEventCreateWithFlags(&c->ev_frame, hipEventDisableTiming));
      for (auto& o : c->oslot) HIP_TRY(c, hipEventCreateWithFlags(&o.done, hipEventDisableTiming));
    }
    // the slot's previous sort must be done before this frame reads its order
    // and overwrites its costs (it ran alongside the previous frame)
    if (os.pending) HIP_TRY(c, hipStreamWaitEvent(s, os.done, 0));
    if (os.units < plan.order_slots || os.ntiles < plan.ntiles) {
      if (c->side) HIP_TRY(c, hipStreamSynchronize(c->side));
      void* p = os.d_order; free_dev(p); os.d_order = nullptr;
      p = os.d_cost; free_dev(p); os.d_cost = nullptr;
      os.units = os.ntiles = 0;
      os.valid = 0;
      HIP_TRY(c, hipMalloc((void**)&os.d_order, (size_t)plan.order_slots * sizeof(int)));
      HIP_TRY(c, hipMalloc((void**)&os.d_cost, (size_t)plan.ntiles * sizeof(uint32_t) + 64));
      HIP_TRY(c, hipMemsetAsync(os.d_cost, 0, (size_t)plan.ntiles * sizeof(uint32_t) + 64, s));
      os.units = plan.order_slots;
      os.ntiles = plan.ntiles;
    }
    order = (os.valid && os.key == key) ? os.d_order : nullptr;
    // an order learned on a distant view costs more than none (interleaved
    // screen order): measured +18 % mean over the 24 reference views
    if (order && os.has_view && !view_close(vsig, os.view, c->stale_deg)) order = nullptr;
    if (!views_close) order = nullptr;   // frames far apart in one launch: no shared order
    tile_cost = os.d_cost;
  }
  // without an order, tiles go to the XCDs interleaved (tile t on XCD t mod 8):
  // it balances any view, where contiguous bands need the learned costs
  if (!order && c->use_order == 1) A.interleave = 1;
  // Sample total: every wave tile stores its count, a sum epilogue adds them up
  // (one atomic per band; a per-wave atomic on one word serialises the frame).
  unsigned long long* tile_samples = nullptr;
  if (d_total) {
    if (c->tile_samples_n < plan.ntiles) {
      void* p = c->d_tile_samples; free_dev(p); c->d_tile_samples = nullptr; c->tile_samples_n = 0;
      HIP_TRY(c, hipMalloc((void**)&c->d_tile_samples, (size_t)plan.ntiles * 8));
      HIP_TRY(c, hipMemsetAsync(c->d_tile_samples, 0, (size_t)plan.ntiles * 8, s));
      c->tile_samples_n = plan.ntiles;
    }
    tile_samples = c->d_tile_samples;
  }
  const size_t nev = c->ev_start.size();
  const size_t slot = nev ? (size_t)(c->timed_frames % (long long)nev) : 0;
  if (nev) HIP_TRY(c, hipEventRecord(c->ev_start[slot], s));
  HIP_TRY(c, cvr::launch_rc1pass(*c, A, phong, d_out, d_samples, tile_samples, order, tile_cost,
                                 plan, s));
  if (nev) {
    HIP_TRY(c, hipEventRecord(c->ev_stop[slot], s));
    c->timed_frames++;
  }
  // The order is rebuilt every order_interval-th frame (and whenever it is
  // missing or stale for this plan): costs shift slowly between frames, and
  // the rebuild (~15 us on the frame's stream) would otherwise cost ~10 %.
  // ... and only while the camera holds still (or moves little) from frame to
  // frame: when every frame jumps to a distant view, a new order would never be
  // used and its rebuild (~15 us on the frame's stream) is skipped
  const bool steady = views_close && (!os.has_last || view_close(vsig, os.last_view, c->stale_deg));
  std::memcpy(os.last_view, vsig, sizeof(vsig));
  os.has_last = true;
  const bool rebuild = tile_cost && !c->async_order && steady &&
                       (!order || os.frames % std::max(1, c->order_interval) == 0);
  os.frames++;
  if (rebuild) {
    // one epilogue on the frame's stream: sum + order for the next frame
    HIP_TRY(c, cvr::launch_tile_epilogue(tile_cost, tile_samples, d_total, plan, os.d_order, s));
    os.pending = false;
    os.valid = 1;
    os.key = key;
    std::memcpy(os.view, vsig, sizeof(vsig));
    os.has_view = true;
  } else if (tile_samples) {
    HIP_TRY(c, cvr::launch_tile_epilogue(nullptr, tile_samples, d_total, plan, nullptr, s));
  }
  if (tile_cost && c->async_order) {
    HIP_TRY(c, hipEventRecord(c->ev_frame, s));
    HIP_TRY(c, hipStreamWaitEvent(c->side, c->ev_frame, 0));
    HIP_TRY(c, cvr::launch_tile_epilogue(tile_cost, nullptr, nullptr, plan, os.d_order, c->side));
    HIP_TRY(c, hipEventRecord(os.done, c->side));
    os.pending = true;
    os.valid = 1;
    os.key = key;
    std::memcpy(os.view, vsig, sizeof(vsig));
    os.has_view = true;
  }
  c->frame_no++;
  if (use_counters) {
    cvr_status st = counters_release(c, s);
    if (st != CVR_OK) return st;
  }
  if (!o->on_device) {
    HIP_TRY(c, hipMemcpyAsync(o->rgba, d_out, rgba_bytes, hipMemcpyDeviceToHost, s));
    if (o->samples) HIP_TRY(c, hipMemcpyAsync(o->samples, d_samples, smp_bytes, hipMemcpyDeviceToHost, s));
    if (o->total) HIP_TRY(c, hipMemcpyAsync(o->total, d_total, 8, hipMemcpyDeviceToHost, s));
    HIP_TRY(c, hipStreamSynchronize(s));
  }
  return CVR_OK;
}

cvr_status cvr_render_rc1pass(cvr_ctx* ctx, const cvr_frame* f, const cvr_rc1pass_params* p,
                              const cvr_output* o) {
  Ctx* c = reinterpret_cast<Ctx*>(ctx);
  if (c && c->group)
    return cvr::group_render(c, f, 1, o, [&](cvr_ctx* _m, const cvr_frame* mf, int, const cvr_output* mo) {
      return cvr_render_rc1pass(_m, mf, p, mo);
    });
  if (!c) return CVR_ERR_ARG;
  return render_rc1pass_frames(c, f, 1, p, o);
}

cvr_status cvr_render_rc1pass_frames(cvr_ctx* ctx, const cvr_frame* frames, int nframes,
                                     const cvr_rc1pass_params* p, const cvr_output* outs) {
  Ctx* c = reinterpret_cast<Ctx*>(ctx);
  if (c && c->group)
    return cvr::group_render(c, frames, nframes, outs, [&](cvr_ctx* _m, const cvr_frame* mf, int nf, const cvr_output* mo) {
      return cvr_render_rc1pass_frames(_m, mf, nf, p, mo);
    });
  if (!c) return CVR_ERR_ARG;
  return render_rc1pass_frames(c, frames, nframes, p, outs);
}

cvr_status cvr_copy_tile_stats(cvr_ctx* ctx, uint64_t* out, int max_tiles, int* out_tiles) {
  Ctx* c = reinterpret_cast<Ctx*>(ctx);
  if (c && c->group) return cvr::group_call_root(c, [&](cvr_ctx* _m) { return cvr_copy_tile_stats(_m, out, max_tiles, out_tiles); });
  if (!c || !out_tiles) return CVR_ERR_ARG;
  *out_tiles = c->tile_stats_n;
  if (!out) return CVR_OK;
  if (!c->d_tile_stats) return fail(c, CVR_ERR_STATE, "tile_stats option was not enabled");
  int n = max_tiles < c->tile_stats_n ? max_tiles : c->tile_stats_n;
  HIP_TRY(c, hipSetDevice(c->device));
  HIP_TRY(c, hipStreamSynchronize(c->stream));
  HIP_TRY(c, hipMemcpy(out, c->d_tile_stats, (size_t)n * 32, hipMemcpyDeviceToHost));
  return CVR_OK;
}

cvr_status cvr_selftest_arith(cvr_ctx* ctx, uint64_t out[3]) {
  Ctx* c = reinterpret_cast<Ctx*>(ctx);
  if (c && c->group) return cvr::group_call_root(c, [&](cvr_ctx* _m) { return cvr_selftest_arith(_m, out); });
  if (!c || !out) return CVR_ERR_ARG;
  HIP_TRY(c, hipSetDevice(c->device));
  unsigned long long* d = nullptr;
  HIP_TRY(c, hipMalloc((void**)&d, 3 * sizeof(unsigned long long)));
  hipError_t e = hipMemsetAsync(d, 0, 3 * sizeof(unsigned long long), c->stream);
  if (e == hipSuccess) e = cvr::launch_selftest_arith(-100, 200, -96, 222, d, c->stream);
  if (e == hipSuccess) e = hipMemcpyAsync(out, d, 3 * sizeof(uint64_t), hipMemcpyDeviceToHost, c->stream);
  if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
  (void)hipFree(d);
  HIP_TRY(c, e);
  return CVR_OK;
}

cvr_status cvr_read_shade_counters(cvr_ctx* ctx, uint64_t out[3]) {
  Ctx* c = reinterpret_cast<Ctx*>(ctx);
  if (!c || !out) return CVR_ERR_ARG;
  if (c->group) {
    uint64_t sum[3] = {0, 0, 0};
    cvr_status st = cvr::group_each(c, [&](cvr_ctx* _m) {
      uint64_t v[3];
      cvr_status e = cvr_read_shade_counters(_m, v);
      for (int i = 0; i < 3; i++) sum[i] += v[i];
      return e;
    });
    for (int i = 0; i < 3; i++) out[i] = sum[i];
    return st;
  }
  if (!c->d_shade) return fail(c, CVR_ERR_STATE, "shade_counters option was not enabled");
  HIP_TRY(c, hipSetDevice(c->device));
  HIP_TRY(c, hipStreamSynchronize(c->stream));
  HIP_TRY(c, hipMemcpy(out, c->d_shade, 3 * sizeof(uint64_t), hipMemcpyDeviceToHost));
  return CVR_OK;
}

cvr_status cvr_read_kernel_times(cvr_ctx* ctx, float* ms, int max_frames, int* out_frames) {
  Ctx* c = reinterpret_cast<Ctx*>(ctx);
  if (c && c->group) return cvr::group_call_root(c, [&](cvr_ctx* _m) { return cvr_read_kernel_times(_m, ms, max_frames, out_frames); });
  if (!c || !out_frames || max_frames < 0 || (max_frames > 0 && !ms)) return CVR_ERR_ARG;
  const long long nev = (long long)c->ev_start.size();
  if (!nev) return fail(c, CVR_ERR_STATE, "kernel_timing option was not enabled");
  const long long have = c->timed_frames < nev ? c->timed_frames : nev;
  const int n = (int)(have < max_frames ? have : max_frames);
  HIP_TRY(c, hipSetDevice(c->device));
  // the most recent n frames, oldest first
  for (int i = 0; i < n; i++) {
    const size_t slot = (size_t)((c->timed_frames - n + i) % nev);
    HIP_TRY(c, hipEventSynchronize(c->ev_stop[slot]));
    HIP_TRY(c, hipEventElapsedTime(&ms[i], c->ev_start[slot], c->ev_stop[slot]));
  }
  *out_frames = n;
  c->timed_frames = 0;
  return CVR_OK;
}

cvr_status cvr_multiscale_resolution(int mode, int sw, int sh, int* rw, int* rh) {
  if (!rw || !rh || sw < 1 || sh < 1 || mode < 0 || mode > 3) return CVR_ERR_ARG;
  // UpdateScreenResolutionMultiScaling, multiplier (2, 2) or (-2, -2)
  if (mode == CVR_SINGLE_RAY_PER_PIXEL) { *rw = sw; *rh = sh; }
  else if (mode == CVR_UP_SCALING_RENDER) { *rw = sw / 2; *rh = sh / 2; }
  else { *rw = sw * 2; *rh = sh * 2; }
  return (*rw >= 1 && *rh >= 1) ? CVR_OK : CVR_ERR_ARG;
}

cvr_status cvr_multiscale_filter(cvr_ctx* ctx, int mode, int kernel, void* d_frame, int fw, int fh,
                                 void* d_screen, int sw, int sh) {
  Ctx* c = reinterpret_cast<Ctx*>(ctx);
  if (c && c->group) return cvr::group_call_root(c, [&](cvr_ctx* _m) { return cvr_multiscale_filter(_m, mode, kernel, d_frame, fw, fh, d_screen, sw, sh); });
  if (!c) return CVR_ERR_ARG;
  if (!d_frame || !d_screen || mode < 1 || mode > 3 || kernel < 0 || kernel > 5 || fw < 1 ||
      fh < 1 || sw < 1 || sh < 1 || d_frame == d_screen)
    return fail(c, CVR_ERR_ARG, "cvr_multiscale_filter: bad arguments");
  const bool cardinal = kernel == CVR_FILTER_CARDINAL_BSPLINE_3 || kernel == CVR_FILTER_CARDINAL_OMOMS3;
  // the digital filter's pre-factored LU needs lines longer than its 8/9 factors
  if (cardinal && mode != CVR_MULTIPLE_RAYS_PER_PIXEL &&
      (mode == CVR_DOWN_SCALING_RENDER ? (sw < 16 || sh < 16) : (fw < 16 || fh < 16)))
    return fail(c, CVR_ERR_ARG, "cvr_multiscale_filter: cardinal kernels need >= 16 px lines");
  HIP_TRY(c, hipSetDevice(c->device));
  HIP_TRY(c, cvr::launch_multiscale(mode, kernel, d_frame, fw, fh, d_screen, sw, sh, c->stream));
  return CVR_OK;
}

cvr_status cvr_screenshot_rgb8(cvr_ctx* ctx, const void* d_frame, int format, int w, int h,
                               void* d_rgb) {
  Ctx* c = reinterpret_cast<Ctx*>(ctx);
  if (c && c->group) return cvr::group_call_root(c, [&](cvr_ctx* _m) { return cvr_screenshot_rgb8(_m, d_frame, format, w, h, d_rgb); });
  if (!c) return CVR_ERR_ARG;
  if (!d_frame || !d_rgb || w < 1 || h < 1 ||
      (format != CVR_FORMAT_RGBA32F && format != CVR_FORMAT_RGBA16F))
    return fail(c, CVR_ERR_ARG, "cvr_screenshot_rgb8: bad arguments");
  HIP_TRY(c, hipSetDevice(c->device));
  HIP_TRY(c, cvr::launch_screenshot(d_frame, format == CVR_FORMAT_RGBA16F, w, h, (uint8_t*)d_rgb,
                                    c->stream));
  return CVR_OK;
}

cvr_status cvr_unpack_tiles_device_n(cvr_ctx* ctx, const cvr_frame* f, const void* d_gathered,
                                     int tpr_max, int nframes, int frame_index, int format,
                                     void* d_rgba) {
  Ctx* c = reinterpret_cast<Ctx*>(ctx);
  if (c && c->group) return cvr::group_call_root(c, [&](cvr_ctx* _m) { return cvr_unpack_tiles_device_n(_m, f, d_gathered, tpr_max, nframes, frame_index, format, d_rgba); });
  if (!c) return CVR_ERR_ARG;
  if (!f || !d_gathered || !d_rgba || f->nranks < 1 || f->tile_size < 16 || tpr_max < 0 ||
      nframes < 1 || frame_index < 0 || frame_index >= nframes ||
      (format != CVR_FORMAT_RGBA32F && format != CVR_FORMAT_RGBA16F))
    return fail(c, CVR_ERR_ARG, "cvr_unpack_tiles_device: bad arguments");
  HIP_TRY(c, hipSetDevice(c->device));
  const size_t px = format == CVR_FORMAT_RGBA16F ? 8 : 16;
  const char* src = static_cast<const char*>(d_gathered) +
                    (size_t)frame_index * tpr_max * f->tile_size * f->tile_size * px;
  HIP_TRY(c, cvr::launch_unpack_tiles(src, d_rgba, format == CVR_FORMAT_RGBA16F, f->width,
                                      f->height, f->tile_size, f->nranks, tpr_max, c->stream,
                                      (size_t)nframes * tpr_max));
  return CVR_OK;
}

cvr_status cvr_unpack_tiles_device(cvr_ctx* ctx, const cvr_frame* f, const void* d_packed,
                                   int tpr_max, int format, void* d_rgba) {
  return cvr_unpack_tiles_device_n(ctx, f, d_packed, tpr_max, 1, 0, format, d_rgba);
}

size_t cvr_tile_code_bound(int tile, int ntiles) {
  if (tile < 16 || tile % 16 != 0 || tile > 64 || ntiles < 0) return 0;
  return cvr::tile_code_bound_bytes(tile, ntiles);
}

cvr_status cvr_encode_tiles(cvr_ctx* ctx, const void* d_tiles, int tile, int ntiles, void* d_stream,
                            unsigned long long* d_bytes) {
  Ctx* c = reinterpret_cast<Ctx*>(ctx);
  if (c && c->group) return cvr::group_call_root(c, [&](cvr_ctx* _m) { return cvr_encode_tiles(_m, d_tiles, tile, ntiles, d_stream, d_bytes); });
  if (!c) return CVR_ERR_ARG;
  if ((!d_tiles && ntiles > 0) || !d_stream || !d_bytes || !cvr_tile_code_bound(tile, ntiles))
    return fail(c, CVR_ERR_ARG, "cvr_encode_tiles: bad arguments");
  HIP_TRY(c, hipSetDevice(c->device));
  if (c->encode_onepass && tile <= 32) {   // (8 tiles staged in LDS per workgroup)
    // the exchange's one-launch form: tiles in claim order (the start table says where).
    // Its counter is the caller's own length word, zeroed first, so encodes on several
    // streams never share one.
    HIP_TRY(c, hipMemsetAsync(d_bytes, 0, sizeof(unsigned long long), c->stream));
    HIP_TRY(c, cvr::launch_exchange_encode(d_tiles, tile, ntiles, ntiles, 1, d_stream, d_bytes, d_bytes,
                                           nullptr, c->stream));
    return CVR_OK;
  }
  HIP_TRY(c, cvr::launch_tile_encode(d_tiles, tile, ntiles, d_stream, d_bytes, c->stream));
  return CVR_OK;
}

cvr_status cvr_decode_tiles(cvr_ctx* ctx, const void* d_stream, int tile, int ntiles, void* d_tiles) {
  Ctx* c = reinterpret_cast<Ctx*>(ctx);
  if (c && c->group) return cvr::group_call_root(c, [&](cvr_ctx* _m) { return cvr_decode_tiles(_m, d_stream, tile, ntiles, d_tiles); });
  if (!c) return CVR_ERR_ARG;
  if (!d_stream || (!d_tiles && ntiles > 0) || !cvr_tile_code_bound(tile, ntiles))
    return fail(c, CVR_ERR_ARG, "cvr_decode_tiles: bad arguments");
  HIP_TRY(c, hipSetDevice(c->device));
  HIP_TRY(c, cvr::launch_tile_decode(d_stream, tile, ntiles, d_tiles, c->stream));
  return CVR_OK;
}



// Output handling shared by the shaded renderers (device or host buffers, the
// sample total through per-tile counts + the sum epilogue, kernel timing events,
// shade counters).  launch(out, samples, shade, tile_samples, stream).
extern "C++" {
template <class Launch>
static cvr_status render_shaded(Ctx* c, const cvr_output* o, int ntiles, size_t npix,
                                const Launch& launch, bool flat_jobs = false) {
  hipStream_t s = c->stream;
  float4* d_out;
  uint32_t* d_samples;
  unsigned long long* d_total;
  const size_t rgba_bytes = npix * (o->format == CVR_FORMAT_RGBA16F ? 8 : 16), smp_bytes = npix * 4;
  if (o->on_device) {
    d_out = (float4*)o->rgba;
    d_samples = (uint32_t*)o->samples;
    d_total = (unsigned long long*)o->total;
  } else {
    cvr_status st = ensure_scratch(c, rgba_bytes + (o->samples ? smp_bytes : 0));
    if (st != CVR_OK) return st;
    d_out = (float4*)c->d_scratch;
    d_samples = o->samples ? (uint32_t*)((char*)c->d_scratch + rgba_bytes) : nullptr;
    d_total = o->total ? c->d_total : nullptr;
  }
  // (flat shading keeps one job-list set per render stream: no wait for it here)
  (void)flat_jobs;
  const bool use_counters = d_total || c->shade_counters;
  if (use_counters) {
    cvr_status st = counters_acquire(c, s);
    if (st != CVR_OK) return st;
  }
  if (d_total && !o->on_device) HIP_TRY(c, hipMemsetAsync(d_total, 0, sizeof(unsigned long long), s));
  unsigned long long* tile_samples = nullptr;
  if (d_total) {
    if (c->tile_samples_n < ntiles) {
      void* q = c->d_tile_samples; free_dev(q); c->d_tile_samples = nullptr; c->tile_samples_n = 0;
      HIP_TRY(c, hipMalloc((void**)&c->d_tile_samples, (size_t)ntiles * 8));
      HIP_TRY(c, hipMemsetAsync(c->d_tile_samples, 0, (size_t)ntiles * 8, s));
      c->tile_samples_n = ntiles;
    }
    tile_samples = c->d_tile_samples;
  }
  unsigned long long* shade = nullptr;
  if (c->shade_counters) {
    if (!c->d_shade) HIP_TRY(c, hipMalloc((void**)&c->d_shade, 3 * sizeof(unsigned long long)));
    HIP_TRY(c, hipMemsetAsync(c->d_shade, 0, 3 * sizeof(unsigned long long), s));
    shade = c->d_shade;
  }
  const size_t nev = c->ev_start.size();
  const size_t slot = nev ? (size_t)(c->timed_frames % (long long)nev) : 0;
  if (nev) HIP_TRY(c, hipEventRecord(c->ev_start[slot], s));
  HIP_TRY(c, launch(d_out, d_samples, shade, tile_samples, s));
  if (nev) {
    HIP_TRY(c, hipEventRecord(c->ev_stop[slot], s));
    c->timed_frames++;
  }
  if (tile_samples) {
    cvr::RenderPlan plan{};
    plan.ntiles = ntiles;
    HIP_TRY(c, cvr::launch_tile_epilogue(nullptr, tile_samples, d_total, plan, nullptr, s));
  }
  if (use_counters) {
    cvr_status st = counters_release(c, s);
    if (st != CVR_OK) return st;
  }
  if (!o->on_device) {
    HIP_TRY(c, hipMemcpyAsync(o->rgba, d_out, rgba_bytes, hipMemcpyDeviceToHost, s));
    if (o->samples) HIP_TRY(c, hipMemcpyAsync(o->samples, d_samples, smp_bytes, hipMemcpyDeviceToHost, s));
    if (o->total) HIP_TRY(c, hipMemcpyAsync(o->total, d_total, 8, hipMemcpyDeviceToHost, s));
    HIP_TRY(c, hipStreamSynchronize(s));
  }
  return CVR_OK;
}
}  // extern "C++"

// ---------------------------------------------------------------------------
// Directional-occlusion shading (rc1pdosct)
// ---------------------------------------------------------------------------

cvr_status cvr_set_extinction_volume(cvr_ctx* ctx, const float* tf_rgba, int n, const int res_in[3],
                                     float sigma0) {
  Ctx* c = reinterpret_cast<Ctx*>(ctx);
  if (c && c->group) return cvr::group_each(c, [&](cvr_ctx* _m) { return cvr_set_extinction_volume(_m, tf_rgba, n, res_in, sigma0); });
  if (!c) return CVR_ERR_ARG;
  if (!tf_rgba || n < 2 || n > cvr::kMaxTfLds)
    return fail(c, CVR_ERR_ARG, "cvr_set_extinction_volume: need 2 <= n <= 4096 TF entries");
  if (!c->d_cells) return fail(c, CVR_ERR_STATE, "cvr_set_extinction_volume: no volume set");
  int res[3] = {128, 128, 128};   // ExtinctionCoefficientVolume defaults (:10-15)
  if (res_in)
    for (int i = 0; i < 3; i++) res[i] = res_in[i];
  for (int i = 0; i < 3; i++)
    if (res[i] < 1 || res[i] > 4096) return fail(c, CVR_ERR_ARG, "cvr_set_extinction_volume: bad resolution");
  if (!(sigma0 > 0.0f)) sigma0 = 1.0f;
  int nl = 1;
  for (int m = std::max(res[0], std::max(res[1], res[2])); m > 1; m >>= 1) nl++;
  if (nl > cvr::kMaxExtLevels) return fail(c, CVR_ERR_ARG, "cvr_set_extinction_volume: too many levels");
  long long off[cvr::kMaxExtLevels + 1] = {0};
  for (int L = 0; L < nl; L++) {
    long long v = 1;
    for (int i = 0; i < 3; i++) v *= std::max(1, res[i] >> L);
    off[L + 1] = off[L] + v;
  }
  // the RGBA16F opacity TF (GenerateTexture_1D_RGBA, transferfunction1d.cpp:58-87)
  std::vector<float> q((size_t)n * 4);
  for (size_t i = 0; i < q.size(); i++) q[i] = half_round(tf_rgba[i]);
  QUIESCE(c);   // frames in flight on any stream read the state replaced below
  { void* p = c->d_ext; free_dev(p); c->d_ext = nullptr; c->ext_levels = 0; }
  { void* p = c->d_ext_cells; free_dev(p); c->d_ext_cells = nullptr; }
  // cell8 texels are addressed with 32-bit byte offsets (16 B each)
  if (off[nl] > (1LL << 28)) return fail(c, CVR_ERR_ARG, "cvr_set_extinction_volume: resolution too large");
  float4* d_tf = nullptr;
  HIP_TRY(c, hipMalloc((void**)&d_tf, (size_t)n * 16));
  hipError_t e = hipMemcpy(d_tf, q.data(), (size_t)n * 16, hipMemcpyHostToDevice);
  if (e == hipSuccess) e = hipMalloc((void**)&c->d_ext, (size_t)off[nl] * sizeof(uint16_t));
  if (e == hipSuccess) e = hipMalloc((void**)&c->d_ext_cells, (size_t)off[nl] * sizeof(uint4));
  if (e == hipSuccess)
    e = cvr::launch_ext_volume(*c, d_tf, n, res, sigma0, nl, off, c->d_ext, c->d_ext_cells, c->stream);
  if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
  (void)hipFree(d_tf);
  if (e != hipSuccess) {
    void* p = c->d_ext; free_dev(p); c->d_ext = nullptr;
    p = c->d_ext_cells; free_dev(p); c->d_ext_cells = nullptr;
    return fail(c, e == hipErrorOutOfMemory ? CVR_ERR_OOM : CVR_ERR_HIP,
                "cvr_set_extinction_volume: %s", hipGetErrorString(e));
  }
  {
    cvr::ExtLevel lv[cvr::kMaxExtLevels] = {};
    for (int L = 0; L < nl; L++) {
      int d[3];
      for (int i = 0; i < 3; i++) d[i] = std::max(1, res[i] >> L);
      lv[L].off = (int)off[L];
      lv[L].dx = d[0]; lv[L].dy = d[1]; lv[L].dz = d[2];
      const float G[3] = {(float)c->N[0] * c->scale[0], (float)c->N[1] * c->scale[1],
                          (float)c->N[2] * c->scale[2]};
      lv[L].sx = (float)d[0] / G[0];   // d / G, rounded once
      lv[L].sy = (float)d[1] / G[1];
      lv[L].sz = (float)d[2] / G[2];
      lv[L].mx = (float)(d[0] - 1);
      lv[L].my = (float)(d[1] - 1);
      lv[L].mz = (float)(d[2] - 1);
    }
    if (!c->d_ext_levels) HIP_TRY(c, hipMalloc((void**)&c->d_ext_levels, sizeof(lv)));
    HIP_TRY(c, hipMemcpy(c->d_ext_levels, lv, sizeof(lv), hipMemcpyHostToDevice));
  }
  for (int i = 0; i < 3; i++) c->ext_res[i] = res[i];
  c->ext_levels = nl;
  {   // level values are Gaussian averages of these opacities: all < 1 -> finite tau
    bool fin = true;
    for (size_t i = 3; i < q.size(); i += 4) fin = fin && q[i] >= 0.0f && q[i] < 1.0f;
    c->ext_finite = fin ? 1 : 0;
  }
  for (int L = 0; L <= nl; L++) c->ext_off[L] = off[L];
  c->ext_sigma0 = sigma0;
  c->cone_valid = 0;
  return CVR_OK;
}

cvr_status cvr_copy_extinction_level(cvr_ctx* ctx, int level, float* out, int dims[3],
                                     int* n_levels) {
  Ctx* c = reinterpret_cast<Ctx*>(ctx);
  if (c && c->group) return cvr::group_call_root(c, [&](cvr_ctx* _m) { return cvr_copy_extinction_level(_m, level, out, dims, n_levels); });
  if (!c) return CVR_ERR_ARG;
  if (n_levels) *n_levels = c->ext_levels;
  if (!c->d_ext) return fail(c, CVR_ERR_STATE, "cvr_copy_extinction_level: no extinction volume");
  if (level < 0 || level >= c->ext_levels) return fail(c, CVR_ERR_ARG, "cvr_copy_extinction_level: bad level");
  int d[3];
  for (int i = 0; i < 3; i++) d[i] = std::max(1, c->ext_res[i] >> level);
  if (dims) for (int i = 0; i < 3; i++) dims[i] = d[i];
  if (!out) return CVR_OK;
  const size_t nv = (size_t)d[0] * d[1] * d[2];
  std::vector<uint16_t> h(nv);
  HIP_TRY(c, hipSetDevice(c->device));
  HIP_TRY(c, hipStreamSynchronize(c->stream));
  HIP_TRY(c, hipMemcpy(h.data(), c->d_ext + c->ext_off[level], nv * 2, hipMemcpyDeviceToHost));
  for (size_t i = 0; i < nv; i++) out[i] = half_to_float_host(h[i]);
  return CVR_OK;
}

static bool same_cone(const cvr_cone_params& a, const cvr_cone_params& b) {
  return std::memcmp(&a, &b, sizeof(a)) == 0;
}

cvr_status cvr_render_dosct(cvr_ctx* ctx, const cvr_frame* f, const cvr_dos_params* p,
                            const cvr_output* o) {
  Ctx* c = reinterpret_cast<Ctx*>(ctx);
  if (c && c->group)
    return cvr::group_render(c, f, 1, o, [&](cvr_ctx* _m, const cvr_frame* mf, int, const cvr_output* mo) {
      return cvr_render_dosct(_m, mf, p, mo);
    });
  if (!c) return CVR_ERR_ARG;
  if (!f || !p || !o || !o->rgba) return fail(c, CVR_ERR_ARG, "cvr_render_dosct: null argument");

  if (o->format != CVR_FORMAT_RGBA32F && o->format != CVR_FORMAT_RGBA16F)
    return fail(c, CVR_ERR_ARG, "cvr_render_dosct: unknown output format %d", o->format);
  if (f->width < 1 || f->height < 1 || f->width > 32768 || f->height > 32768)
    return fail(c, CVR_ERR_ARG, "cvr_render_dosct: bad viewport %dx%d", f->width, f->height);
  if (!c->d_cells || !c->d_tf) return fail(c, CVR_ERR_STATE, "cvr_render_dosct: no volume or TF");
  if (!c->d_ext) return fail(c, CVR_ERR_STATE, "cvr_render_dosct: needs cvr_set_extinction_volume");
  const bool phong = p->apply_gradient_shading != 0;
  if (phong && !c->d_grad) return fail(c, CVR_ERR_STATE, "cvr_render_dosct: Phong needs cvr_set_gradient");
  if (p->shadow_type < 0 || p->shadow_type > 2) return fail(c, CVR_ERR_ARG, "cvr_render_dosct: bad shadow type");
  if (f->nranks > 1 && (f->tile_size < 16 || f->tile_size % 16 != 0 || f->rank < 0 || f->rank >= f->nranks))
    return fail(c, CVR_ERR_ARG, "cvr_render_dosct: bad tiling");
  HIP_TRY(c, hipSetDevice(c->device));

  // cone tables: covered distance <= 0 -> the volume diagonal * 0.50 / 0.75
  // (GetDiagonal in double, dosrcrenderer.cpp:112-113)
  cvr_cone_params cp[2] = {p->occlusion, p->shadow};
  {
    double vw = c->N[0] * (double)c->scale[0], vh = c->N[1] * (double)c->scale[1],
           vd = c->N[2] * (double)c->scale[2];
    const double diag = std::sqrt(vw * vw + vh * vh + vd * vd);
    if (!(cp[0].covered_distance > 0.0f)) cp[0].covered_distance = (float)(diag * 0.50f);
    if (!(cp[1].covered_distance > 0.0f)) cp[1].covered_distance = (float)(diag * 0.75f);
  }
  if (!c->cone_valid || !same_cone(cp[0], c->cone_key[0]) || !same_cone(cp[1], c->cone_key[1])) {
    if (!c->cone_tab) c->cone_tab = new cvr_cone_tables[2];
    for (int k = 0; k < 2; k++) {
      cvr_status st = cvr_build_cone_tables(&cp[k], c->ext_sigma0, &c->cone_tab[k]);
      if (st != CVR_OK) return fail(c, st, "cvr_render_dosct: cone tables (%s)", k ? "shadow" : "occlusion");
    }
    std::vector<float> up(2 * CVR_MAX_CONE_SECTIONS * 4, 0.0f);
    for (int k = 0; k < 2; k++)
      for (int i = 0; i < c->cone_tab[k].n_sections; i++)
        for (int j = 0; j < 4; j++)   // GetConeSectionsInfoTex uploads RGBA16F
          up[((size_t)k * CVR_MAX_CONE_SECTIONS + i) * 4 + j] = half_round(c->cone_tab[k].sections[i][j]);
    if (!c->d_cones) HIP_TRY(c, hipMalloc((void**)&c->d_cones, up.size() * sizeof(float)));
    QUIESCE(c);   // DOS frames in flight on other streams read d_cones
    HIP_TRY(c, hipMemcpy(c->d_cones, up.data(), up.size() * sizeof(float), hipMemcpyHostToDevice));
    c->cone_key[0] = cp[0];
    c->cone_key[1] = cp[1];
    c->cone_valid = 1;
  }

  cvr::DosArgs Q{};
  int ntiles = 0;
  size_t npix = 0;
  fill_frame_args(c, f, p->step, Q.a, ntiles, npix);
  Q.a.filter_bits = c->filter_bits;   // GL_LINEAR weights of every fetch (CVR-SPEC-8 at 8)
  if (c->cell_skip > 0) {   // the per-cell skip flags in the count / emit march
    const cvr_status st = cell_flags_or_off(c);
    if (st == CVR_OK) {
      Q.a.cell_skip = 1;
      Q.a.inv_step = 1.0f / Q.a.step;
    } else if (st != CVR_ERR_OOM) {
      return st;
    }
  }
  Q.a.out_half = o->format == CVR_FORMAT_RGBA16F;
  Q.a.ka = p->ka;   // Phong ambient/diffuse/specular weights of the surface term
  Q.a.kd = p->kd;
  Q.a.ks = p->ks;
  Q.a.shininess = p->shininess;
  for (int i = 0; i < 3; i++) { Q.a.ispec[i] = p->ispecular[i]; Q.a.light[i] = p->light.position[i]; }
  for (int i = 0; i < 3; i++) Q.G[i] = (float)c->N[i] * c->scale[i];
  Q.ext_levels = c->ext_levels;
  Q.levels = c->d_ext_levels;
  Q.apply_occlusion = p->apply_occlusion != 0;
  Q.apply_shadow = p->apply_shadow != 0;
  Q.shadow_type = p->shadow_type;
  Q.phong = phong;
  // ShadeSample (:607-656): ka only with occlusion, kd/ks only with shadows
  Q.ka = Q.apply_occlusion ? p->ka : 0.0f;
  Q.kd = Q.apply_shadow ? p->kd : 0.0f;
  Q.ks = Q.apply_shadow ? p->ks : 0.0f;
  for (int i = 0; i < 3; i++) {
    Q.lfwd[i] = p->light.forward[i];
    Q.lup[i] = p->light.up[i];
    Q.lright[i] = p->light.right[i];
  }
  // SpotLightMaxAngle: glm::cos(glm::pi<float>() * angle / 180.f) (dosrcrenderer.cpp:158)
  Q.spot_cos = std::cos(3.14159265358979323846f * p->light.spot_angle_deg / 180.0f);
  Q.zero_skip = c->ext_finite;
  Q.count_taps = c->shade_counters ? 1 : 0;
  for (int k = 0; k < 2; k++) {
    cvr::DosCone& C = k ? Q.sdw : Q.occ;
    const cvr_cone_tables& T = c->cone_tab[k];
    for (int i = 0; i < 3; i++) C.counts[i] = T.counts[i];
    C.initial_step = T.initial_step;
    C.ray7w = T.ray7_adj_weight;
    C.ui_weight = T.ui_weight;
    for (int i = 0; i < 10; i++)
      for (int j = 0; j < 3; j++) C.axes[3 * i + j] = T.axes[i][j];
    C.sections = c->d_cones + (size_t)k * CVR_MAX_CONE_SECTIONS;
    // exit tables: the sections' track and border scale, replaying the kernel's
    // float recurrence (track += interval) on the RGBA16F-rounded table
    float track = T.initial_step;
    int s0 = 0;
    for (int st = 0; st < 3; st++) {
      cvr::ConeStageExit& X = C.exit[st];
      X.nruns = 0;
      bool ok = Q.zero_skip != 0;
      for (int i = s0; i < s0 + T.counts[st]; i++) {
        const float mip = half_round(T.sections[i][1]);
        const float inv = std::ldexp(1.0f, -(2 * (int)mip + 1));
        if (!(mip >= 0.0f)) ok = false;
        if (X.nruns == 0 || inv != X.run_inv[X.nruns - 1]) {
          if (X.nruns == cvr::kMaxConeRuns) ok = false;
          else {
            X.run_first[X.nruns] = i;
            X.run_t[X.nruns] = track;
            X.run_inv[X.nruns] = inv;
            X.nruns++;
          }
        }
        track = track + half_round(T.sections[i][0]);
      }
      s0 += T.counts[st];
      X.end_s = s0;
      X.end_track = track;
      if (!ok) X.nruns = 0;
    }
  }

  return render_shaded(c, o, ntiles, npix, [&](float4* out, uint32_t* smp, unsigned long long* shade,
                                                unsigned long long* ts, hipStream_t st) {
    return cvr::launch_dos(*c, Q, out, smp, shade, ts, st);
  }, c->shade_flat != 0);
}


// ---------------------------------------------------------------------------
// Extinction-based shading (rc1pextbsd)
// ---------------------------------------------------------------------------

cvr_status cvr_set_extinction_sat(cvr_ctx* ctx, const float* ext_lut, int lut_n) {
  Ctx* c = reinterpret_cast<Ctx*>(ctx);
  if (c && c->group) return cvr::group_each(c, [&](cvr_ctx* _m) { return cvr_set_extinction_sat(_m, ext_lut, lut_n); });
  if (!c) return CVR_ERR_ARG;
  if (!c->d_vox) return fail(c, CVR_ERR_STATE, "cvr_set_extinction_sat: no volume set");
  const int nv = c->bpv == 1 ? 256 : 65536;
  if (!ext_lut || lut_n != nv)
    return fail(c, CVR_ERR_ARG, "cvr_set_extinction_sat: need one extinction per voxel value (%d)", nv);
  const int w = c->N[0] + 2, h = c->N[1] + 2, d = c->N[2] + 2;
  const size_t cells = (size_t)w * h * d;
  // the shader indexes texels (plus one cell4 plane) with 32-bit / 24-bit products
  if (w > 4096 || h > 4096 || d > 4096 || cells >= ((size_t)1 << 31))
    return fail(c, CVR_ERR_ARG, "cvr_set_extinction_sat: volume too large for the SAT");
  QUIESCE(c);   // frames in flight on any stream read the state replaced below
  // Same grid as the last build (a TF change): rebuild into the existing buffers.
  // Freeing and re-allocating the ~30 GB of a 1024^3 SAT costs seconds.
  const bool same = c->d_sat && c->sat_dims[0] == w && c->sat_dims[1] == h && c->sat_dims[2] == d;
  if (!same) {
    void* p = c->d_sat; free_dev(p); c->d_sat = nullptr;
    p = c->d_sat_cells; free_dev(p); c->d_sat_cells = nullptr;
    p = c->d_sat_scratch; free_dev(p); c->d_sat_scratch = nullptr;
    c->sat_dims[0] = c->sat_dims[1] = c->sat_dims[2] = 0;
  }
  float* d_lut = nullptr;
  hipError_t e = hipMalloc((void**)&d_lut, (size_t)nv * sizeof(float));
  if (e == hipSuccess) e = hipMemcpy(d_lut, ext_lut, (size_t)nv * sizeof(float), hipMemcpyHostToDevice);
  // the double recurrence's grid: kept with the SAT for rebuilds (sat_keep_scratch,
  // 8.6 GB at 1024^3) or allocated for this build only
  if (e == hipSuccess && !c->d_sat_scratch) e = hipMalloc(&c->d_sat_scratch, cells * sizeof(double));
  double* d_sd = (double*)c->d_sat_scratch;
  // the float SAT plus kSatPlainPadPlanes zero planes (the plain layout's clamped
  // +1 neighbours: cvr_sat_layout_check)
  const size_t pad_floats = cvr::sat_plain_floats(w, h, d) - cells;
  if (e == hipSuccess && !same) e = hipMalloc((void**)&c->d_sat, cvr::sat_plain_floats(w, h, d) * sizeof(float));
  if (e == hipSuccess && !same) e = hipMemsetAsync(c->d_sat + cells, 0, pad_floats * sizeof(float), c->stream);
  // GPU time of the two compute phases (option "sat_build_us"): the wall time of
  // this call also holds the allocations of ~50 GB at 1024^3
  hipEvent_t ev[4] = {};
  for (hipEvent_t& x : ev)
    if (e == hipSuccess) e = hipEventCreate(&x);
  if (e == hipSuccess) e = hipEventRecord(ev[0], c->stream);
  if (e == hipSuccess) e = cvr::launch_sat_build(*c, d_lut, d_sd, c->d_sat, c->stream);
  if (e == hipSuccess) e = hipEventRecord(ev[1], c->stream);
  if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
  (void)hipFree(d_lut);
  if (!c->sat_keep_scratch) { void* p = c->d_sat_scratch; free_dev(p); c->d_sat_scratch = nullptr; }
  // the cell4 copy only for the layout that reads it
  if (e == hipSuccess && c->sat_layout == 0 && !c->d_sat_cells)
    e = hipMalloc((void**)&c->d_sat_cells, cvr::sat_cells_float4s(w, h, d) * sizeof(float4));
  if (e == hipSuccess) e = hipEventRecord(ev[2], c->stream);
  if (e == hipSuccess && c->sat_layout == 0) e = cvr::launch_sat_cells(*c, c->d_sat, c->d_sat_cells, c->stream);
  if (e == hipSuccess) e = hipEventRecord(ev[3], c->stream);
  if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
  if (e == hipSuccess) {
    float a = 0.f, b = 0.f;
    if (hipEventElapsedTime(&a, ev[0], ev[1]) == hipSuccess &&
        hipEventElapsedTime(&b, ev[2], ev[3]) == hipSuccess)
      c->sat_build_us = (int)((a + b) * 1000.0f);
  }
  if (e == hipSuccess && c->sat_layout == 1) {   // a copy from an earlier layout is stale now
    void* p = c->d_sat_cells; free_dev(p); c->d_sat_cells = nullptr;
  }
  for (hipEvent_t x : ev)
    if (x) (void)hipEventDestroy(x);
  if (e != hipSuccess) {
    void* p = c->d_sat; free_dev(p); c->d_sat = nullptr;
    p = c->d_sat_cells; free_dev(p); c->d_sat_cells = nullptr;
    p = c->d_sat_scratch; free_dev(p); c->d_sat_scratch = nullptr;
    c->sat_dims[0] = c->sat_dims[1] = c->sat_dims[2] = 0;
    return fail(c, e == hipErrorOutOfMemory ? CVR_ERR_OOM : CVR_ERR_HIP,
                "cvr_set_extinction_sat: %s", hipGetErrorString(e));
  }
  c->sat_dims[0] = w; c->sat_dims[1] = h; c->sat_dims[2] = d;
  return CVR_OK;
}

cvr_status cvr_sat_layout_check(const int dims[3], int layout, int pad_planes, unsigned long long out[4]) {
  if (!dims || !out || (layout != 0 && layout != 1)) return CVR_ERR_ARG;
  const long long w = dims[0], h = dims[1], d = dims[2];
  if (w < 1 || h < 1 || d < 1) return CVR_ERR_ARG;
  const int pad = pad_planes >= 0 ? pad_planes : cvr::kSatPlainPadPlanes;
  // bytes allocated: cell4 = float4 per texel of d + 1 planes (sat_cells_float4s);
  // plain = floats of d + pad planes (sat_plain_floats)
  const unsigned long long alloc = layout == 0 ? (unsigned long long)cvr::sat_cells_float4s((int)w, (int)h, (int)d) * 16ull
                                               : (unsigned long long)(w * h * (d + pad)) * 4ull;
  bool wrap = (w * h) >= (1ll << 24) || h >= (1ll << 24) || w >= (1ll << 24) || (d - 1) * h + (h - 1) >= (1ll << 24);
  unsigned long long end = 0;
  const uint32_t pz = (uint32_t)(w * h);
  for (int c = 0; c < 8; c++) {   // the clamped extremes of every axis
    const uint32_t tx = (c & 1) ? (uint32_t)(w - 1) : 0u, ty = (c & 2) ? (uint32_t)(h - 1) : 0u,
                   tz = (c & 4) ? (uint32_t)(d - 1) : 0u;
    const uint32_t idx = cvr::sat_texel_index(tx, ty, tz, (uint32_t)w, (uint32_t)h);
    const unsigned long long exact = ((unsigned long long)tz * h + ty) * w + tx;
    if (idx != exact) wrap = true;
    if (layout == 0) {
      for (unsigned long long e : {exact, exact + pz}) {
        if (e + 1 > 0xffffffffull) wrap = true;
        end = std::max(end, (e + 1) * 16ull);
      }
    } else {
      for (unsigned long long e : {exact, exact + w, exact + pz, exact + pz + w}) {
        if (e + 2 > 0xffffffffull) wrap = true;   // the 32-bit element index of the pair
        end = std::max(end, (e + 2) * 4ull);      // a float pair: elements e, e + 1
      }
    }
  }
  out[0] = end;
  out[1] = alloc;
  out[2] = wrap ? 1ull : 0ull;
  out[3] = (!wrap && end <= alloc) ? 1ull : 0ull;
  return CVR_OK;
}

cvr_status cvr_copy_extinction_sat(cvr_ctx* ctx, float* out, size_t capacity, int dims[3]) {
  Ctx* c = reinterpret_cast<Ctx*>(ctx);
  if (c && c->group) return cvr::group_call_root(c, [&](cvr_ctx* _m) { return cvr_copy_extinction_sat(_m, out, capacity, dims); });
  if (!c) return CVR_ERR_ARG;
  if (!c->d_sat) return fail(c, CVR_ERR_STATE, "cvr_copy_extinction_sat: no SAT built");
  if (dims) for (int i = 0; i < 3; i++) dims[i] = c->sat_dims[i];
  if (!out) return CVR_OK;
  const size_t n = (size_t)c->sat_dims[0] * c->sat_dims[1] * c->sat_dims[2];
  if (capacity < n) return fail(c, CVR_ERR_ARG, "cvr_copy_extinction_sat: buffer too small");
  HIP_TRY(c, hipSetDevice(c->device));
  HIP_TRY(c, hipStreamSynchronize(c->stream));
  HIP_TRY(c, hipMemcpy(out, c->d_sat, n * sizeof(float), hipMemcpyDeviceToHost));
  return CVR_OK;
}

cvr_status cvr_render_extbsd(cvr_ctx* ctx, const cvr_frame* f, const cvr_ebs_params* p,
                             const cvr_output* o) {
  Ctx* c = reinterpret_cast<Ctx*>(ctx);
  if (c && c->group)
    return cvr::group_render(c, f, 1, o, [&](cvr_ctx* _m, const cvr_frame* mf, int, const cvr_output* mo) {
      return cvr_render_extbsd(_m, mf, p, mo);
    });
  if (!c) return CVR_ERR_ARG;
  if (!f || !p || !o || !o->rgba) return fail(c, CVR_ERR_ARG, "cvr_render_extbsd: null argument");
  if (c->filter_bits && c->sat_layout != 0)
    return fail(c, CVR_ERR_ARG, "cvr_render_extbsd: filter_bits %d needs sat_layout 0 (the cell4 copy)",
                c->filter_bits);
  if (o->format != CVR_FORMAT_RGBA32F && o->format != CVR_FORMAT_RGBA16F)
    return fail(c, CVR_ERR_ARG, "cvr_render_extbsd: unknown output format %d", o->format);
  if (f->width < 1 || f->height < 1 || f->width > 32768 || f->height > 32768)
    return fail(c, CVR_ERR_ARG, "cvr_render_extbsd: bad viewport %dx%d", f->width, f->height);
  if (!c->d_cells || !c->d_tf) return fail(c, CVR_ERR_STATE, "cvr_render_extbsd: no volume or TF");
  if (!c->d_sat) return fail(c, CVR_ERR_STATE, "cvr_render_extbsd: needs cvr_set_extinction_sat");
  if (c->sat_layout == 0 && !c->d_sat_cells) {   // switched back to the cell4 copy: build it
    const int w = c->sat_dims[0], h = c->sat_dims[1], d = c->sat_dims[2];
    HIP_TRY(c, hipSetDevice(c->device));
    HIP_TRY(c, hipMalloc((void**)&c->d_sat_cells, cvr::sat_cells_float4s(w, h, d) * sizeof(float4)));
    const hipError_t e = cvr::launch_sat_cells(*c, c->d_sat, c->d_sat_cells, c->stream);
    if (e != hipSuccess) {   // never leave an unbuilt copy behind for the next frame to read
      void* q = c->d_sat_cells; free_dev(q); c->d_sat_cells = nullptr;
      return fail(c, CVR_ERR_HIP, "cvr_render_extbsd: cell4 SAT build: %s", hipGetErrorString(e));
    }
  }
  const bool phong = p->apply_gradient_shading != 0;
  if (phong && !c->d_grad) return fail(c, CVR_ERR_STATE, "cvr_render_extbsd: Phong needs cvr_set_gradient");
  if (p->shadow_type < 0 || p->shadow_type > 1) return fail(c, CVR_ERR_ARG, "cvr_render_extbsd: bad shadow type");
  if (p->apply_occlusion && p->occlusion_shells < 1)
    return fail(c, CVR_ERR_ARG, "cvr_render_extbsd: need >= 1 occlusion shell");
  if (p->apply_shadow && !(p->shadow_sample_interval > 0.0f))
    return fail(c, CVR_ERR_ARG, "cvr_render_extbsd: shadow sample interval must be positive");
  if (f->nranks > 1 && (f->tile_size < 16 || f->tile_size % 16 != 0 || f->rank < 0 || f->rank >= f->nranks))
    return fail(c, CVR_ERR_ARG, "cvr_render_extbsd: bad tiling");
  HIP_TRY(c, hipSetDevice(c->device));

  cvr::EbsArgs Q{};
  int ntiles = 0;
  size_t npix = 0;
  fill_frame_args(c, f, p->step, Q.a, ntiles, npix);
  Q.a.filter_bits = c->filter_bits;   // GL_LINEAR weights of every fetch (CVR-SPEC-8 at 8)
  if (c->cell_skip > 0) {   // the per-cell skip flags in the count / emit march
    const cvr_status st = cell_flags_or_off(c);
    if (st == CVR_OK) {
      Q.a.cell_skip = 1;
      Q.a.inv_step = 1.0f / Q.a.step;
    } else if (st != CVR_ERR_OOM) {
      return st;
    }
  }
  Q.a.out_half = o->format == CVR_FORMAT_RGBA16F;
  Q.a.ka = p->ka; Q.a.kd = p->kd; Q.a.ks = p->ks;
  Q.a.shininess = p->shininess;
  for (int i = 0; i < 3; i++) { Q.a.ispec[i] = p->ispecular[i]; Q.a.light[i] = p->light_pos[i]; }
  for (int i = 0; i < 3; i++) {
    Q.S[i] = c->scale[i];
    Q.G[i] = (float)c->N[i] * c->scale[i];
    Q.inv_vs[i] = 1.0f / (Q.G[i] + Q.S[i] * 2.0f);        // inv_vol_scaled (:75)
    Q.sat_dims[i] = c->sat_dims[i];
    Q.sat_pz = (uint32_t)c->sat_dims[0] * (uint32_t)c->sat_dims[1];
    Q.nsat[i] = (float)c->sat_dims[i];
    Q.nsat_m1[i] = (float)(c->sat_dims[i] - 1);
    Q.min_sat[i] = Q.S[i] * 0.5f;                        // MinSATPosition (:66)
    Q.max_sat[i] = Q.G[i] + Q.S[i] * 1.5f;               // MaxSATPosition (:67)
    Q.lfwd[i] = p->light_forward[i];
  }
  Q.apply_occlusion = p->apply_occlusion != 0;
  Q.occ_shells = p->occlusion_shells;
  Q.occ_radius = p->occlusion_radius;
  {   // ExtinctionAmbientOcclusion's per-shell weights (:117-144), float as the shader
    const float R = Q.occ_radius;
    for (int i = 0; i < cvr::EbsArgs::kMaxAoShells; i++) {
      const float r1 = i == 0 ? R : R * (float)(i + 1);
      Q.ao_w[i] = 1.0f / (r1 * r1);
    }
    const float rshi = R * (float)Q.occ_shells;
    Q.ao_wa = 1.0f / (rshi * rshi);
  }
  Q.apply_shadow = p->apply_shadow != 0;
  Q.shadow_type = p->shadow_type;
  Q.phong = phong;
  // DirSdwConeAngle = (float)(angle * pi / 180.0) (ebsrenderer.cpp:161); its cos / sin
  const float ang = (float)(p->shadow_cone_angle_deg * 3.14159265358979323846 / 180.0);
  Q.p_cs = std::cos(ang); Q.p_sn = std::sin(ang);
  Q.n_cs = std::cos(-ang); Q.n_sn = std::sin(-ang);
  Q.recip_cone = std::fabs(p->shadow_cone_angle_deg) <= 44.0f;
  Q.interval = p->shadow_sample_interval;
  Q.initial_step = p->shadow_initial_step;
  Q.ui_weight = p->shadow_ui_weight;
  if (p->shadow_max_distance > 0.0f) {
    Q.max_distance = p->shadow_max_distance;
  } else {
    // dir_cone_max_distance = 0.75f * Dv (ebsrenderer.cpp:98-105, float arithmetic)
    const float vw = (float)((double)c->N[0] * (double)c->scale[0]);
    const float vh = (float)((double)c->N[1] * (double)c->scale[1]);
    const float vd = (float)((double)c->N[2] * (double)c->scale[2]);
    Q.max_distance = 0.75f * std::sqrt((vw * vw + vh * vh) + vd * vd);
  }
  // ShadeSample (:502-518): ka only with occlusion, kd/ks only with shadows
  Q.ka = Q.apply_occlusion ? p->ka : 0.0f;
  Q.kd = Q.apply_shadow ? p->kd : 0.0f;
  Q.ks = Q.apply_shadow ? p->ks : 0.0f;
  return render_shaded(c, o, ntiles, npix, [&](float4* out, uint32_t* smp, unsigned long long* shade,
                                                unsigned long long* ts, hipStream_t st) {
    return cvr::launch_ebs(*c, Q, out, smp, shade, ts, st);
  }, c->shade_flat != 0);
}



// ---------------------------------------------------------------------------
// Isosurface ray-casters with block skipping (rc1pisocustom, rc1pisodfscustom)
// ---------------------------------------------------------------------------

void cvr_iso_params_default(int variant, cvr_iso_params* p) {
  if (!p) return;
  std::memset(p, 0, sizeof(*p));
  p->variant = variant;
  const int nb = variant == 1 ? 32 : 4;          // :190 of either renderer
  for (int i = 0; i < 3; i++) p->num_blocks[i] = nb;
  p->isovalue = 0.5f;                           // constructor defaults (:119-127)
  p->step_small = 0.05f;
  p->step_large = 1.0f;
  p->step_range = 0.1f;
  p->color[0] = 0.66f; p->color[1] = 0.6f; p->color[2] = 0.05f; p->color[3] = 1.0f;
  p->ka = 0.5f; p->kd = 0.5f; p->ks = 0.8f; p->shininess = 30.0f;
  for (int i = 0; i < 3; i++) p->ispecular[i] = 1.0f;
}

// The block table for nb: raw extremes on the GPU, normalised here exactly as
// ComputeBlocksFromVolume stores them (v / 255 or v / 65535 in double, pushed
// into a float vector; empty blocks keep numeric_limits<float>::max / lowest).
static cvr_status ensure_iso_blocks(Ctx* c, const int nb[3]) {
  if (c->iso_valid && c->d_iso_mm && c->iso_nb[0] == nb[0] && c->iso_nb[1] == nb[1] &&
      c->iso_nb[2] == nb[2])
    return CVR_OK;
  const size_t n = (size_t)nb[0] * nb[1] * nb[2];
  HIP_TRY(c, hipSetDevice(c->device));
  uint2* d_raw = nullptr;
  HIP_TRY(c, hipMalloc((void**)&d_raw, n * sizeof(uint2)));
  std::vector<uint2> raw(n);
  hipError_t e = cvr::launch_block_minmax(c->d_vox, c->bpv, c->N, nb, d_raw, c->stream);
  if (e == hipSuccess) e = hipMemcpyAsync(raw.data(), d_raw, n * sizeof(uint2), hipMemcpyDeviceToHost, c->stream);
  if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
  (void)hipFree(d_raw);
  if (e != hipSuccess) return fail(c, CVR_ERR_HIP, "cvr_render_iso: block table: %s", hipGetErrorString(e));
  const double mx = c->bpv == 1 ? 255.0 : 65535.0;
  std::vector<float2> mm(n);
  for (size_t i = 0; i < n; i++) {
    if (raw[i].x > raw[i].y) {
      mm[i] = make_float2(3.40282347e38f, -3.40282347e38f);
    } else {
      mm[i] = make_float2((float)((double)raw[i].x / mx), (float)((double)raw[i].y / mx));
    }
  }
  // frames still running on any render stream may read the old table
  HIP_TRY(c, hipDeviceSynchronize());
  if (c->d_iso_mm && (c->iso_nb[0] * c->iso_nb[1] * c->iso_nb[2]) != (int)n) {
    void* p = c->d_iso_mm; free_dev(p); c->d_iso_mm = nullptr;
  }
  if (!c->d_iso_mm) HIP_TRY(c, hipMalloc((void**)&c->d_iso_mm, n * sizeof(float2)));
  HIP_TRY(c, hipMemcpy(c->d_iso_mm, mm.data(), n * sizeof(float2), hipMemcpyHostToDevice));
  for (int i = 0; i < 3; i++) c->iso_nb[i] = nb[i];
  c->iso_valid = 1;
  return CVR_OK;
}

static void iso_blocks_of(const cvr_iso_params* p, int nb[3]) {
  for (int i = 0; i < 3; i++)
    nb[i] = p->num_blocks[i] > 0 ? p->num_blocks[i] : (p->variant == 1 ? 32 : 4);
}

cvr_status cvr_iso_block_ranges(cvr_ctx* ctx, const int num_blocks[3], float* out_min, float* out_max) {
  Ctx* c = reinterpret_cast<Ctx*>(ctx);
  if (c && c->group) return cvr::group_call_root(c, [&](cvr_ctx* _m) { return cvr_iso_block_ranges(_m, num_blocks, out_min, out_max); });
  if (!c) return CVR_ERR_ARG;
  if (!num_blocks || !out_min || !out_max) return fail(c, CVR_ERR_ARG, "cvr_iso_block_ranges: null argument");
  if (!c->d_vox) return fail(c, CVR_ERR_STATE, "cvr_iso_block_ranges: no volume set");
  for (int i = 0; i < 3; i++)
    if (num_blocks[i] < 1 || num_blocks[i] > 1024)
      return fail(c, CVR_ERR_ARG, "cvr_iso_block_ranges: bad block count %d", num_blocks[i]);
  HIP_TRY(c, hipSetDevice(c->device));
  HIP_TRY(c, hipStreamSynchronize(c->stream));
  cvr_status st = ensure_iso_blocks(c, num_blocks);
  if (st != CVR_OK) return st;
  const size_t n = (size_t)num_blocks[0] * num_blocks[1] * num_blocks[2];
  std::vector<float2> mm(n);
  HIP_TRY(c, hipMemcpy(mm.data(), c->d_iso_mm, n * sizeof(float2), hipMemcpyDeviceToHost));
  for (size_t i = 0; i < n; i++) { out_min[i] = mm[i].x; out_max[i] = mm[i].y; }
  return CVR_OK;
}

cvr_status cvr_render_iso(cvr_ctx* ctx, const cvr_frame* f, const cvr_iso_params* p,
                          const cvr_output* o) {
  Ctx* c = reinterpret_cast<Ctx*>(ctx);
  if (c && c->group)
    return cvr::group_render(c, f, 1, o, [&](cvr_ctx* _m, const cvr_frame* mf, int, const cvr_output* mo) {
      return cvr_render_iso(_m, mf, p, mo);
    });
  if (!c) return CVR_ERR_ARG;
  if (!f || !p || !o || !o->rgba) return fail(c, CVR_ERR_ARG, "cvr_render_iso: null argument");
  if (c->filter_bits)
    return fail(c, CVR_ERR_ARG, "cvr_render_iso: filter_bits %d is implemented for cvr_render_rc1pass only", c->filter_bits);
  if (o->format != CVR_FORMAT_RGBA32F && o->format != CVR_FORMAT_RGBA16F)
    return fail(c, CVR_ERR_ARG, "cvr_render_iso: unknown output format %d", o->format);
  if (f->width < 1 || f->height < 1 || f->width > 32768 || f->height > 32768)
    return fail(c, CVR_ERR_ARG, "cvr_render_iso: bad viewport %dx%d", f->width, f->height);
  if (!c->d_cells || !c->d_vox) return fail(c, CVR_ERR_STATE, "cvr_render_iso: no volume set");
  if (p->variant < 0 || p->variant > 2) return fail(c, CVR_ERR_ARG, "cvr_render_iso: bad variant %d", p->variant);
  const bool phong = p->apply_gradient_shading != 0;
  if (phong && !c->d_grad) return fail(c, CVR_ERR_STATE, "cvr_render_iso: Phong needs cvr_set_gradient");
  if (f->nranks > 1 && (f->tile_size < 16 || f->tile_size % 16 != 0 || f->rank < 0 || f->rank >= f->nranks))
    return fail(c, CVR_ERR_ARG, "cvr_render_iso: bad tiling");
  int nb[3];
  iso_blocks_of(p, nb);
  for (int i = 0; i < 3; i++)
    if (nb[i] > 1024) return fail(c, CVR_ERR_ARG, "cvr_render_iso: bad block count %d", nb[i]);
  HIP_TRY(c, hipSetDevice(c->device));
  if (p->variant != 2) {   // RayCasting1PassIsoAdapt has no blocks
    cvr_status st = ensure_iso_blocks(c, nb);
    if (st != CVR_OK) return st;
  }

  cvr::IsoArgs Q{};
  int ntiles = 0;
  size_t npix = 0;
  fill_frame_args(c, f, 1.0f, Q.a, ntiles, npix);
  Q.a.out_half = o->format == CVR_FORMAT_RGBA16F;
  Q.a.ka = p->ka; Q.a.kd = p->kd; Q.a.ks = p->ks; Q.a.shininess = p->shininess;
  for (int i = 0; i < 3; i++) { Q.a.ispec[i] = p->ispecular[i]; Q.a.light[i] = p->light_pos[i]; }
  for (int i = 0; i < 3; i++) {
    Q.G[i] = (float)c->N[i] * c->scale[i];
    Q.nb[i] = (float)nb[i];
    Q.nbi[i] = nb[i];
  }
  Q.iso = p->isovalue;
  Q.step_small = p->step_small;
  Q.step_large = p->step_large;
  Q.step_range = p->step_range;
  {   // length(VolumeGridSize / numBlocks) * 0.5 (rc1pisodfscustom ...iso_adapt.comp:222-223)
    const float b0 = Q.G[0] / Q.nb[0], b1 = Q.G[1] / Q.nb[1], b2 = Q.G[2] / Q.nb[2];
    Q.half_block_len = std::sqrt(std::fmaf(b2, b2, std::fmaf(b1, b1, b0 * b0))) * 0.5f;
  }
  for (int i = 0; i < 3; i++) {
    Q.bs[i] = Q.G[i] / Q.nb[i];
    Q.nhg[i] = -Q.G[i] * 0.5f;
    Q.inv_g[i] = 1.0f / Q.G[i];
  }
  for (int i = 0; i < 4; i++) Q.color[i] = p->color[i];
  const float2* mm = p->variant != 2 ? c->d_iso_mm : nullptr;
  const int variant = p->variant;
  return render_shaded(c, o, ntiles, npix, [&](float4* out, uint32_t* smp, unsigned long long*,
                                                unsigned long long* ts, hipStream_t st2) {
    return cvr::launch_iso(*c, Q, variant, phong, mm, out, smp, ts, st2);
  });
}

#pragma GCC visibility pop
}  // extern "C"
