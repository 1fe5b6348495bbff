/*
 * cvr_oracle.cpp — CPU restatement of cppvolrend's structured single-pass
 * ray-march (rc1pass) and its inputs.  TEST INFRASTRUCTURE ONLY.
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load
 * this library, and only as the checker / the timed CPU baseline.  The product
 * (cpp_volume_rendering_amd, libcvr.so) never links or calls it.
 *
 * Reference (paths relative to the reference root, read-only):
 *   ray generation .............. cppvolrend/structured/rc1pass/ray_marching_1p.comp:87-99
 *   ray/AABB slab test .......... cppvolrend/structured/_common_shaders/ray_bbox_intersection.comp:18-52
 *   march + FTB composite + ERT . ray_marching_1p.comp:106-176
 *   Blinn-Phong ................. ray_marching_1p.comp:48-81 (applied at :145-146)
 *   step size ................... cppvolrend/structured/rc1pass/rc1prenderer.cpp:62-63
 *   volume texture (R16F) ....... libs/volvis_utils/utils.cpp:20-56, structuredgridvolume.cpp:121-151
 *   TF table (RGBA16F, a->tau) .. libs/volvis_utils/transferfunction1d.cpp:89-130, 319-358;
 *                                 transferfunction.h:74-82
 *   TF CPU lookup (Get) ......... transferfunction1d.cpp:132-157
 *   FD gradient (RGB16F) ........ libs/volvis_utils/utils.cpp:146-284
 *   Sobel-Feldman gradient ...... libs/volvis_utils/utils.cpp:287-350
 *   camera ...................... libs/vis_utils/camera.cpp:281-284 (glm 0.9.5 lookAt,
 *                                 include/glm/gtc/matrix_transform.inl:403-428)
 *
 * Parity status: the GLSL shaders cannot execute in this image (Windows/GL-only
 * app, no headless GL), so this restatement follows them by reading.  Its CPU
 * table builders are pinned against golden vectors emitted by the reference's own
 * C++ compiled under oracle/ref (TransferFunction1D, SummedAreaTable3D); the
 * shader arithmetic itself (GL hardware texture filtering) is "parity unpinned"
 * at the level of the vendor's fixed-point filter weights — see DESIGN.md §Parity.
 *
 * Arithmetic contract ("CVR-SPEC", shared with the HIP kernels):
 *   - compiled with -ffp-contract=off; every fused multiply-add is an explicit fmaf;
 *   - division and sqrt are IEEE correctly rounded;
 *   - exp/pow use the polynomial cvr_expf/cvr_powf below (fma/rint/ldexp only);
 *   - fp16 storage is emulated with round-to-nearest-even float->half.
 * With that contract the GPU kernels reproduce this file bit for bit.
 */
#include <cmath>
#include <cstdint>
#include <cstring>
#include <cstdio>
#include <vector>
#include <algorithm>
#ifdef _OPENMP
#include <omp.h>
#endif

#define ORACLE_API extern "C" __attribute__((visibility("default")))

#include "oracle_types.h"

namespace {

// ---------------------------------------------------------------------------
// fp16 emulation (GL_R16F / GL_RGBA16F / GL_RGB16F internal formats)
// ---------------------------------------------------------------------------
inline uint32_t f2u(float f) { uint32_t u; std::memcpy(&u, &f, 4); return u; }
inline float u2f(uint32_t u) { float f; std::memcpy(&f, &u, 4); return f; }

// float -> IEEE binary16, round to nearest even (what a GL driver does when it
// converts GL_FLOAT client data to a 16F internal format).
uint16_t float_to_half(float f) {
  uint32_t x = f2u(f);
  uint32_t sign = (x >> 16) & 0x8000u;
  uint32_t absx = x & 0x7fffffffu;
  if (absx >= 0x7f800000u) {                 // inf / nan
    return (uint16_t)(sign | 0x7c00u | (absx > 0x7f800000u ? 0x200u : 0u));
  }
  if (absx >= 0x477ff000u) return (uint16_t)(sign | 0x7c00u);  // rounds to inf
  if (absx < 0x38800000u) {                  // half subnormal or zero
    if (absx < 0x33000000u) return (uint16_t)sign;             // < 2^-25 -> 0
    uint32_t mant = (absx & 0x7fffffu) | 0x800000u;
    int e = (int)(absx >> 23);               // 102..112
    int shift = 126 - e;                     // 14..24
    uint32_t hm = mant >> shift;
    uint32_t rem = mant & ((1u << shift) - 1u);
    uint32_t halfway = 1u << (shift - 1);
    if (rem > halfway || (rem == halfway && (hm & 1u))) hm++;
    return (uint16_t)(sign | hm);
  }
  uint32_t e = (absx >> 23) - 112u;          // rebias 127 -> 15
  uint32_t m = absx & 0x7fffffu;
  uint32_t h = (e << 10) | (m >> 13);
  uint32_t rem = m & 0x1fffu;
  if (rem > 0x1000u || (rem == 0x1000u && (h & 1u))) h++;
  return (uint16_t)(sign | h);
}

float half_to_float(uint16_t h) {
  uint32_t sign = ((uint32_t)h & 0x8000u) << 16;
  uint32_t e = (h >> 10) & 0x1fu;
  uint32_t m = h & 0x3ffu;
  if (e == 0) {
    if (m == 0) return u2f(sign);
    float v = (float)m * 5.9604644775390625e-8f;   // m * 2^-24, exact
    return sign ? -v : v;
  }
  if (e == 31) return u2f(sign | 0x7f800000u | (m << 13));
  return u2f(sign | ((e + 112u) << 23) | (m << 13));
}

inline float q16(float f) { return half_to_float(float_to_half(f)); }

// ---------------------------------------------------------------------------
// CVR-SPEC math helpers
// ---------------------------------------------------------------------------
struct v3 { float x, y, z; };
inline v3 mk(float x, float y, float z) { return v3{x, y, z}; }
inline float dot3(v3 a, v3 b) { return std::fmaf(a.z, b.z, std::fmaf(a.y, b.y, a.x * b.x)); }
inline v3 normalize3(v3 v) {
  float inv = 1.0f / std::sqrt(dot3(v, v));
  return mk(v.x * inv, v.y * inv, v.z * inv);
}
inline float lerpf(float a, float b, float t) { return std::fmaf(t, b - a, a); }

// exp(x): Cody-Waite reduction + degree-6 polynomial (Cephes expf coefficients).
float cvr_expf(float x) {
  if (x != x) return x;
  if (x < -86.0f) return 0.0f;
  if (x > 88.5f) return INFINITY;
  float n = std::rint(x * 1.44269504088896341f);
  float r = std::fmaf(n, -0.693359375f, x);
  r = std::fmaf(n, 2.12194440e-4f, r);
  float p = 1.9875691500e-4f;
  p = std::fmaf(p, r, 1.3981999507e-3f);
  p = std::fmaf(p, r, 8.3334519073e-3f);
  p = std::fmaf(p, r, 4.1665795894e-2f);
  p = std::fmaf(p, r, 1.6666665459e-1f);
  p = std::fmaf(p, r, 5.0000001201e-1f);
  float r2 = r * r;
  float y = std::fmaf(p, r2, r) + 1.0f;
  return std::ldexp(y, (int)n);
}

// ln(x): Cephes logf polynomial (x in [sqrt(1/2), sqrt(2)) * 2^e).
// 0 and subnormals -> -inf, negatives -> NaN.
float cvr_logf(float x) {
  if (x != x) return x;
  if (x < 0.0f) return NAN;
  if (x < 1.17549435e-38f) return -INFINITY;
  if (x == INFINITY) return INFINITY;
  uint32_t bits = f2u(x);
  int e = (int)((bits >> 23) & 0xffu) - 126;
  float m = u2f((bits & 0x007fffffu) | 0x3f000000u);       // [0.5, 1)
  if (m < 0.70710678118654752f) { m = m + m; e = e - 1; }
  float f = m - 1.0f;
  float z = f * f;
  float p = 7.0376836292e-2f;
  p = std::fmaf(p, f, -1.1514610310e-1f);
  p = std::fmaf(p, f, 1.1676998740e-1f);
  p = std::fmaf(p, f, -1.2420140846e-1f);
  p = std::fmaf(p, f, 1.4249322787e-1f);
  p = std::fmaf(p, f, -1.6668057665e-1f);
  p = std::fmaf(p, f, 2.0000714765e-1f);
  p = std::fmaf(p, f, -2.4999993993e-1f);
  p = std::fmaf(p, f, 3.3333331174e-1f);
  float r = (p * f) * z;
  float fe = (float)e;
  r = std::fmaf(fe, -2.12194440e-4f, r);
  r = std::fmaf(-0.5f, z, r);
  float lnx = f + r;
  return std::fmaf(fe, 0.693359375f, lnx);
}

// pow(x, y) for x >= 0: exp(y * ln x).
float cvr_powf(float x, float y) {
  if (x != x || y != y) return x + y;
  if (!(x > 0.0f) || x < 1.17549435e-38f) {
    if (y > 0.0f) return 0.0f;
    if (y == 0.0f) return 1.0f;
    return INFINITY;
  }
  if (x == INFINITY) return y > 0.0f ? INFINITY : (y == 0.0f ? 1.0f : 0.0f);
  return cvr_expf(y * cvr_logf(x));
}

// ---------------------------------------------------------------------------
// Camera: glm 0.9.5 lookAt (float), tan(fovy/2) via DEGREE_TO_RADIANS in double
// ---------------------------------------------------------------------------
inline v3 cross3(v3 x, v3 y) {   // glm::cross: x.y*y.z - y.y*x.z, ...
  return mk(x.y * y.z - y.y * x.z, x.z * y.x - y.z * x.x, x.x * y.y - y.x * x.y);
}
inline float glm_dot(v3 a, v3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
inline v3 glm_normalize(v3 v) {
  float sqr = v.x * v.x + v.y * v.y + v.z * v.z;
  float inv = 1.0f / std::sqrt(sqr);
  return mk(v.x * inv, v.y * inv, v.z * inv);
}

}  // namespace

// ===========================================================================
// Exported oracle API
// ===========================================================================

ORACLE_API float oracle_q16(float f) { return q16(f); }
ORACLE_API uint16_t oracle_float_to_half(float f) { return float_to_half(f); }
ORACLE_API float oracle_half_to_float(uint16_t h) { return half_to_float(h); }
ORACLE_API float oracle_expf(float x) { return cvr_expf(x); }
ORACLE_API float oracle_powf(float x, float y) { return cvr_powf(x, y); }
ORACLE_API float oracle_logf(float x) { return cvr_logf(x); }

// glm::lookAt (column-major, out[col*4+row]) and tan(fovy/2).
ORACLE_API void oracle_lookat(const float eye_[3], const float center_[3], const float up_[3],
                              float fovy_deg, float out_view[16], float* out_tan) {
  v3 eye = mk(eye_[0], eye_[1], eye_[2]);
  v3 center = mk(center_[0], center_[1], center_[2]);
  v3 up = mk(up_[0], up_[1], up_[2]);
  v3 f = glm_normalize(mk(center.x - eye.x, center.y - eye.y, center.z - eye.z));
  v3 s = glm_normalize(cross3(f, up));
  v3 u = cross3(s, f);
  float R[16] = {1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1};
  R[0 * 4 + 0] = s.x; R[1 * 4 + 0] = s.y; R[2 * 4 + 0] = s.z;
  R[0 * 4 + 1] = u.x; R[1 * 4 + 1] = u.y; R[2 * 4 + 1] = u.z;
  R[0 * 4 + 2] = -f.x; R[1 * 4 + 2] = -f.y; R[2 * 4 + 2] = -f.z;
  R[3 * 4 + 0] = -glm_dot(s, eye);
  R[3 * 4 + 1] = -glm_dot(u, eye);
  R[3 * 4 + 2] = glm_dot(f, eye);
  std::memcpy(out_view, R, sizeof(R));
  // (float)tan(DEGREE_TO_RADIANS(fovy) / 2.0), rc1prenderer.cpp:97, math_utils/utils.h:13
  double rad = (double)fovy_deg * (3.14159265358979323846264338327950288 / 180.0);
  *out_tan = (float)std::tan(rad / 2.0);
}

// Default integration step (rc1prenderer.cpp:62-63).
ORACLE_API float oracle_default_step(const float scale[3]) {
  double sx = scale[0], sy = scale[1], sz = scale[2];
  return (float)((0.5f / std::sqrt(3.0f)) * std::sqrt(sx * sx + sy * sy + sz * sz));
}

// TransferFunction1D::BuildLinear (transferfunction1d.cpp:319-358) into a
// double table of (max_density+1) x 4, zero where no control segment covers
// an isovalue (glm 0.9.5 zero-initialises dvec4).
ORACLE_API void oracle_tf_build_double(const double* rgb_cp, int n_rgb, const double* a_cp,
                                       int n_a, int max_density, double* out_table) {
  int n = max_density + 1;
  for (int i = 0; i < 4 * n; i++) out_table[i] = 0.0;
  for (int i = 0; i < n_rgb - 1; i++) {
    // TransferControlPoint stores its colour as glm::vec4 (float)
    int i0 = (int)rgb_cp[i * 4 + 3], i1 = (int)rgb_cp[(i + 1) * 4 + 3];
    float c0[3], c1[3];
    for (int c = 0; c < 3; c++) { c0[c] = (float)rgb_cp[i * 4 + c]; c1[c] = (float)rgb_cp[(i + 1) * 4 + c]; }
    double diff[3];
    for (int c = 0; c < 3; c++) diff[c] = (double)(c1[c] - c0[c]);
    for (int x = i0; x <= i1; x++) {
      double k = (double)(x - i0) / (double)(i1 - i0);
      if (x < 0 || x >= n) continue;
      for (int c = 0; c < 3; c++) out_table[x * 4 + c] = (double)c0[c] + diff[c] * k;
    }
  }
  for (int i = 0; i < n_a - 1; i++) {
    int i0 = (int)a_cp[i * 2 + 1], i1 = (int)a_cp[(i + 1) * 2 + 1];
    float a0 = (float)a_cp[i * 2], a1 = (float)a_cp[(i + 1) * 2];
    double diff = (double)(a1 - a0);
    for (int x = i0; x <= i1; x++) {
      double k = (double)(x - i0) / (double)(i1 - i0);
      if (x < 0 || x >= n) continue;
      out_table[x * 4 + 3] = (double)a0 + diff * k;
    }
  }
}

// GenerateTexture_1D_RGBt (transferfunction1d.cpp:89-118): rgb as float,
// alpha -> extinction tau = log(1/(1-a)) (transferfunction.h:79-82) unless the
// TF already holds extinction; the GL upload rounds to RGBA16F.
ORACLE_API void oracle_tf_rgbt(const double* table, int n, int extinction_input, int round16,
                               float* out_rgbt) {
  for (int i = 0; i < n; i++) {
    float r = (float)table[i * 4 + 0], g = (float)table[i * 4 + 1], b = (float)table[i * 4 + 2];
    float v4 = (float)table[i * 4 + 3];
    if (!extinction_input) v4 = (float)std::log(1.0 / (1.0 - (double)v4));
    float o[4] = {r, g, b, v4};
    for (int c = 0; c < 4; c++) out_rgbt[i * 4 + c] = round16 ? q16(o[c]) : o[c];
  }
}

// TransferFunction1D::Get(value, max) (transferfunction1d.cpp:132-157): the
// CPU mapping used by the EBS SAT build (no half-texel skew).
ORACLE_API void oracle_tf_get(const double* table, int max_density, double value,
                              double max_data_value, float out[4]) {
  if (max_data_value >= 0) value = value * ((double)max_density / max_data_value);
  if (value < 0.0f || value > (float)max_density) { out[0] = out[1] = out[2] = out[3] = 0; return; }
  if (std::fabs(value - (float)max_density) < 0.000001) {
    for (int c = 0; c < 4; c++) out[c] = (float)table[max_density * 4 + c];
    return;
  }
  int iv = (int)value;
  double t = value - iv;
  for (int c = 0; c < 4; c++) out[c] = (float)((1.0 - t) * table[iv * 4 + c] + t * table[(iv + 1) * 4 + c]);
}

// GetNormalizedSample (structuredgridvolume.cpp:121-151) -> (GLfloat) ->
// GL_R16F (utils.cpp:20-56).  out[i] = float value of the stored half.
ORACLE_API void oracle_volume_r16f(const void* voxels, int bytes_per_voxel, int64_t count,
                                   float* out) {
  if (bytes_per_voxel == 1) {
    const uint8_t* v = (const uint8_t*)voxels;
    for (int64_t i = 0; i < count; i++) out[i] = q16((float)((double)v[i] / (256.0 - 1.0)));
  } else {
    const uint16_t* v = (const uint16_t*)voxels;
    for (int64_t i = 0; i < count; i++) out[i] = q16((float)((double)v[i] / (65536.0 - 1.0)));
  }
}

namespace {
inline double norm_sample(const void* vox, int bpv, int w, int h, int d, int x, int y, int z) {
  if (x < 0 || y < 0 || z < 0 || x >= w || y >= h || z >= d) return 0.0;
  int64_t i = (int64_t)x + (int64_t)y * w + (int64_t)z * w * h;
  if (bpv == 1) return (double)((const uint8_t*)vox)[i] / (256.0 - 1.0);
  return (double)((const uint16_t*)vox)[i] / (65536.0 - 1.0);
}
}  // namespace

// GenerateGradientTexture with its defaults (gradient_sample_size 1, no filter,
// normalised; utils.cpp:146-190, 245-284): xyz per voxel, RGB16F-rounded.
ORACLE_API void oracle_gradient_fd(const void* vox, int bpv, int w, int h, int d, float* out_xyz) {
#pragma omp parallel for schedule(static)
  for (int z = 0; z < d; z++)
    for (int y = 0; y < h; y++)
      for (int x = 0; x < w; x++) {
        double gx = norm_sample(vox, bpv, w, h, d, x + 1, y, z) - norm_sample(vox, bpv, w, h, d, x - 1, y, z);
        double gy = norm_sample(vox, bpv, w, h, d, x, y + 1, z) - norm_sample(vox, bpv, w, h, d, x, y - 1, z);
        double gz = norm_sample(vox, bpv, w, h, d, x, y, z + 1) - norm_sample(vox, bpv, w, h, d, x, y, z - 1);
        // glm::normalize<double>: v * inversesqrt(dot(v,v)), inversesqrt = 1/sqrt
        double sqr = gx * gx + gy * gy + gz * gz;
        double inv = 1.0 / std::sqrt(sqr);
        gx *= inv; gy *= inv; gz *= inv;
        if (gx != gx) { gx = gy = gz = 0.0; }
        int64_t i = ((int64_t)z * h + y) * w + x;
        out_xyz[i * 3 + 0] = q16((float)gx);
        out_xyz[i * 3 + 1] = q16((float)gy);
        out_xyz[i * 3 + 2] = q16((float)gz);
      }
}

// GenerateSobelFeldmanGradientTexture (utils.cpp:287-350), unnormalised, RGB16F.
ORACLE_API void oracle_gradient_sobel(const void* vox, int bpv, int w, int h, int d, float* out_xyz) {
#pragma omp parallel for schedule(static)
  for (int z = 0; z < d; z++)
    for (int y = 0; y < h; y++)
      for (int x = 0; x < w; x++) {
        double sx = 0, sy = 0, sz = 0;
        for (int v1 = -1; v1 <= 1; v1++)
          for (int v2 = -1; v2 <= 1; v2++) {
            double wgt = std::pow(2.0, std::abs(v1) + std::abs(v2));
            sz += norm_sample(vox, bpv, w, h, d, x + v1, y + v2, z - 1) * (4.0 / wgt)
                + norm_sample(vox, bpv, w, h, d, x + v1, y + v2, z + 1) * (-4.0 / wgt);
            sy += norm_sample(vox, bpv, w, h, d, x + v1, y - 1, z + v2) * (4.0 / wgt)
                + norm_sample(vox, bpv, w, h, d, x + v1, y + 1, z + v2) * (-4.0 / wgt);
            sx += norm_sample(vox, bpv, w, h, d, x - 1, y + v2, z + v1) * (4.0 / wgt)
                + norm_sample(vox, bpv, w, h, d, x + 1, y + v2, z + v1) * (-4.0 / wgt);
          }
        int64_t i = ((int64_t)z * h + y) * w + x;
        out_xyz[i * 3 + 0] = q16((float)sx);
        out_xyz[i * 3 + 1] = q16((float)sy);
        out_xyz[i * 3 + 2] = q16((float)sz);
      }
}

// ---------------------------------------------------------------------------
// rc1pass ray-march
// ---------------------------------------------------------------------------


namespace {

// A GL_LINEAR weight at `bits` fraction bits (0: exact): the fixed-point filter
// weights of GPU texture units, rounded to nearest even (CVR-SPEC-8, the
// library's filter_bits option; glsl_literal.cpp weight() rounds the same way).
inline float filter_weight(float a, int bits) {
  if (bits <= 0) return a;
  const float s = std::ldexp(1.0f, bits);
  return std::nearbyint(a * s) * (1.0f / s);
}

struct Tex {
  const float* v; int N[3]; int comps;
  int wbits = 0;   // filter_weight fraction bits
  // trilinear, clamp-to-edge, texel-centre convention; x,y,z already in texel space
  inline void sample(float x, float y, float z, float* out) const {
    float cx = std::fmin(std::fmax(x, -1.0f), (float)(N[0] - 1));
    float cy = std::fmin(std::fmax(y, -1.0f), (float)(N[1] - 1));
    float cz = std::fmin(std::fmax(z, -1.0f), (float)(N[2] - 1));
    float flx = std::floor(cx), fly = std::floor(cy), flz = std::floor(cz);
    float ax = filter_weight(cx - flx, wbits), ay = filter_weight(cy - fly, wbits),
          az = filter_weight(cz - flz, wbits);
    int ix = (int)flx, iy = (int)fly, iz = (int)flz;
    int x0 = std::max(ix, 0), x1 = std::min(ix + 1, N[0] - 1);
    int y0 = std::max(iy, 0), y1 = std::min(iy + 1, N[1] - 1);
    int z0 = std::max(iz, 0), z1 = std::min(iz + 1, N[2] - 1);
    auto at = [&](int i, int j, int k, int c) {
      return v[(((int64_t)k * N[1] + j) * N[0] + i) * comps + c];
    };
    for (int c = 0; c < comps; c++) {
      float c00 = lerpf(at(x0, y0, z0, c), at(x1, y0, z0, c), ax);
      float c10 = lerpf(at(x0, y1, z0, c), at(x1, y1, z0, c), ax);
      float c01 = lerpf(at(x0, y0, z1, c), at(x1, y0, z1, c), ax);
      float c11 = lerpf(at(x0, y1, z1, c), at(x1, y1, z1, c), ax);
      float c0 = lerpf(c00, c10, ay);
      float c1 = lerpf(c01, c11, ay);
      out[c] = lerpf(c0, c1, az);
    }
  }
};

// texture(TexTransferFunc, density): 1D linear, clamp-to-edge, x = u*n - 0.5
inline void tf_lookup(const float* tf, int n, float density, float out[4], int wbits = 0) {
  float x = std::fmaf(density, (float)n, -0.5f);
  x = std::fmin(std::fmax(x, -1.0f), (float)(n - 1));
  float fl = std::floor(x);
  float a = filter_weight(x - fl, wbits);
  int i = (int)fl;
  int i0 = std::max(i, 0), i1 = std::min(i + 1, n - 1);
  for (int c = 0; c < 4; c++) out[c] = lerpf(tf[i0 * 4 + c], tf[i1 * 4 + c], a);
}

}  // namespace

// Renders rows [y0, y1) of the full frame.  out: W*H*4 floats, counts: W*H.
static void rc1pass_rows(const OracleRc1pass& P, int y0, int y1, float* out, uint32_t* counts,
                         int nthreads) {
  float V[16], tanf;
  oracle_lookat(P.eye, P.center, P.up, P.fovy_deg, V, &tanf);
  const float aspect = P.aspect > 0 ? P.aspect : (float)P.W / (float)P.H;
  const v3 eye = mk(P.eye[0], P.eye[1], P.eye[2]);
  // VolumeGridSize = resolution * voxel size (rc1prenderer.cpp:233-241)
  const v3 G = mk((float)P.N[0] * P.scale[0], (float)P.N[1] * P.scale[1], (float)P.N[2] * P.scale[2]);
  const v3 half = mk(G.x * 0.5f, G.y * 0.5f, G.z * 0.5f);
  const v3 NoG = mk((float)P.N[0] / G.x, (float)P.N[1] / G.y, (float)P.N[2] / G.z);
  const v3 light = mk(P.light[0], P.light[1], P.light[2]);
  Tex vol{P.vol, {P.N[0], P.N[1], P.N[2]}, 1, P.filter_bits};
  Tex grd{P.grad, {P.N[0], P.N[1], P.N[2]}, 3, P.filter_bits};
  const float step = P.step;
  const int W = P.W, H = P.H;
#ifdef _OPENMP
  if (nthreads > 0) omp_set_num_threads(nthreads);
#endif
#pragma omp parallel for schedule(dynamic, 1)
  for (int py = y0; py < y1; py++) {
    for (int px = 0; px < W; px++) {
      int64_t pix = (int64_t)py * W + px;
      float dst[4] = {0, 0, 0, 0};
      uint32_t cnt = 0;
      // ray generation (ray_marching_1p.comp:93-99)
      float fx = (float)px + 0.5f, fy = (float)py + 0.5f;
      float vx = std::fmaf(fx / (float)W, 2.0f, -1.0f);
      float vy = std::fmaf(fy / (float)H, 2.0f, -1.0f);
      v3 c = mk((vx * tanf) * aspect, vy * tanf, -1.0f);
      // vec3 * mat3(View): component j = dot(c, column j)
      v3 d = mk(dot3(c, mk(V[0], V[1], V[2])), dot3(c, mk(V[4], V[5], V[6])),
                dot3(c, mk(V[8], V[9], V[10])));
      v3 dir = normalize3(d);
      dir = normalize3(dir);   // RayAABBIntersection normalises again (:219)
      // slab test (ray_bbox_intersection.comp:18-30)
      v3 inv = mk(1.0f / dir.x, 1.0f / dir.y, 1.0f / dir.z);
      v3 ta = mk(inv.x * (-half.x - eye.x), inv.y * (-half.y - eye.y), inv.z * (-half.z - eye.z));
      v3 tb = mk(inv.x * (half.x - eye.x), inv.y * (half.y - eye.y), inv.z * (half.z - eye.z));
      float tnear = std::fmax(std::fmax(std::fmin(ta.x, tb.x), std::fmin(ta.y, tb.y)), std::fmin(ta.z, tb.z));
      float tfar = std::fmin(std::fmin(std::fmax(ta.x, tb.x), std::fmax(ta.y, tb.y)), std::fmax(ta.z, tb.z));
      bool hit = tfar > tnear;
      tnear = std::fmax(tnear, 0.0f);
      if (hit) {
        float D = std::fabs(tfar - tnear);
        v3 tpos = mk(std::fmaf(dir.x, tnear, eye.x) + half.x, std::fmaf(dir.y, tnear, eye.y) + half.y,
                     std::fmaf(dir.z, tnear, eye.z) + half.z);
        // texel-space ray: x_tex = (p / G) * N - 0.5 = p * (N/G) - 0.5
        v3 o = mk(std::fmaf(tpos.x, NoG.x, -0.5f), std::fmaf(tpos.y, NoG.y, -0.5f), std::fmaf(tpos.z, NoG.z, -0.5f));
        v3 dt = mk(dir.x * NoG.x, dir.y * NoG.y, dir.z * NoG.z);
        float s = 0.0f;
        while (s < D) {
          float h = std::fmin(step, D - s);
          float t = std::fmaf(h, 0.5f, s);
          float x = std::fmaf(dt.x, t, o.x), y = std::fmaf(dt.y, t, o.y), z = std::fmaf(dt.z, t, o.z);
          float dens;
          vol.sample(x, y, z, &dens);
          float src[4];
          tf_lookup(P.tf, P.tf_n, dens, src, P.filter_bits);
          cnt++;
          if (src[3] > 0.0f) {
            if (P.phong && P.grad) {
              float g[3];
              grd.sample(x, y, z, g);
              if (g[0] != 0.0f || g[1] != 0.0f || g[2] != 0.0f) {
                // world position of the sample: Tpos - G/2 (ray_marching_1p.comp:56)
                v3 wp = mk(std::fmaf(dir.x, t, tpos.x) - half.x, std::fmaf(dir.y, t, tpos.y) - half.y,
                           std::fmaf(dir.z, t, tpos.z) - half.z);
                v3 n = normalize3(mk(g[0], g[1], g[2]));
                v3 L = normalize3(mk(light.x - wp.x, light.y - wp.y, light.z - wp.z));
                v3 Ve = normalize3(mk(eye.x - wp.x, eye.y - wp.y, eye.z - wp.z));
                v3 Hv = normalize3(mk(Ve.x + L.x, Ve.y + L.y, Ve.z + L.z));
                float dd = std::fmax(0.0f, dot3(n, L));
                float ds = std::fmax(0.0f, dot3(Hv, n));
                float pw = cvr_powf(ds, P.shininess);
                float f = std::fmaf(P.kd, dd, P.ka);
                for (int k = 0; k < 3; k++) src[k] = std::fmaf(P.ispec[k] * P.ks, pw, src[k] * f);
              }
            }
            float a = 1.0f - cvr_expf(-(src[3] * h));
            float om = 1.0f - dst[3];
            dst[0] = std::fmaf(om, src[0] * a, dst[0]);
            dst[1] = std::fmaf(om, src[1] * a, dst[1]);
            dst[2] = std::fmaf(om, src[2] * a, dst[2]);
            dst[3] = std::fmaf(om, a, dst[3]);
            if (dst[3] > 0.99f) break;
          }
          s = s + h;
        }
      }
      if (out) for (int k = 0; k < 4; k++) out[pix * 4 + k] = dst[k];
      if (counts) counts[pix] = cnt;
    }
  }
}

// Full-frame render. Returns the total iteration count S.
ORACLE_API uint64_t oracle_render_rc1pass(const OracleRc1pass* P, float* out_rgba,
                                          uint32_t* out_counts, int nthreads) {
  std::vector<uint32_t> tmp;
  uint32_t* counts = out_counts;
  if (!counts) { tmp.resize((size_t)P->W * P->H); counts = tmp.data(); }
  rc1pass_rows(*P, 0, P->H, out_rgba, counts, nthreads);
  uint64_t total = 0;
  for (int64_t i = 0; i < (int64_t)P->W * P->H; i++) total += counts[i];
  return total;
}

// Bounded-sample render for the CPU baseline: rows [y0, y1) only.
ORACLE_API uint64_t oracle_render_rc1pass_rows(const OracleRc1pass* P, int y0, int y1,
                                               float* out_rgba, uint32_t* out_counts, int nthreads) {
  rc1pass_rows(*P, y0, y1, out_rgba, out_counts, nthreads);
  uint64_t total = 0;
  for (int64_t i = (int64_t)y0 * P->W; i < (int64_t)y1 * P->W; i++) total += out_counts[i];
  return total;
}

ORACLE_API int oracle_num_threads(void) {
#ifdef _OPENMP
  return omp_get_max_threads();
#else
  return 1;
#endif
}

// ===========================================================================
// Directional-occlusion shading (rc1pdosct), SURVEY.md §8 rows A9-A13
// ===========================================================================
//
// Extinction-coefficient mip volume, ExtinctionCoefficientVolume custom-resolution
// path (extcoefvolumegenerator.cpp:230-408, glslextgen/gen_extcoefvol_anysize.comp,
// gen_extcoefvol_anysize_mmlevel.comp, backtotau.comp), CVR-SPEC:
//   level 0 voxel i: p = ((float)i + 0.5) * (G / R0); 7^3 taps f = k * S0 (k in -3..3,
//     x outer, z inner); w = (S0*S0*S0) * exp(-((fx*fx + fy*fy) + fz*fz) / ((2*S0)*S0));
//     c = 0 outside [0,1]^3 of (p+f)/G, else TF opacity (RGBA16F table, alpha) of the
//     trilinear R16F density at texel fmaf(u, N, -0.5); sums in tap order; value
//     q16(sum(w*c) / sum(w)).
//   level L >= 1: R_L = max(1, R0 >> L); the same with Si = S0 * 2^L over level L-1
//     (trilinear at fmaf(u, R_{L-1}, -0.5)), voxel size G / R_L.
//   then every level: tau = q16(-1 * log(1 - opacity)).
struct OracleExtVol {
  const float* vol; int N[3]; float scale[3];   // R16F volume values, voxel scale
  const float* tf_rgba; int tf_n;                // opacity TF (half-rounded RGBA)
  int res[3]; float sigma0;
};

namespace {

int ext_levels(const int res[3]) {
  int m = std::max(res[0], std::max(res[1], res[2])), n = 1;
  while (m > 1) { m >>= 1; n++; }
  return n;
}

void ext_level_dims(const int res[3], int L, int out[3]) {
  for (int i = 0; i < 3; i++) out[i] = std::max(1, res[i] >> L);
}

}  // namespace

ORACLE_API int oracle_ext_levels(const int res[3]) { return ext_levels(res); }

// out: all levels concatenated (level 0 first), x-fastest; returns the level count.
ORACLE_API int oracle_ext_volume(const OracleExtVol* P, float* out, int nthreads) {
  const int nl = ext_levels(P->res);
  const v3 G = mk((float)P->N[0] * P->scale[0], (float)P->N[1] * P->scale[1],
                  (float)P->N[2] * P->scale[2]);
  Tex vol{P->vol, {P->N[0], P->N[1], P->N[2]}, 1};
#ifdef _OPENMP
  if (nthreads > 0) omp_set_num_threads(nthreads);
#endif
  std::vector<int64_t> off(nl + 1, 0);
  for (int L = 0; L < nl; L++) {
    int d[3];
    ext_level_dims(P->res, L, d);
    off[L + 1] = off[L] + (int64_t)d[0] * d[1] * d[2];
  }
  for (int L = 0; L < nl; L++) {
    int d[3], pd[3];
    ext_level_dims(P->res, L, d);
    if (L > 0) ext_level_dims(P->res, L - 1, pd);
    const float S = L == 0 ? P->sigma0 : P->sigma0 * (float)(1 << L);
    const v3 vs = mk(G.x / (float)d[0], G.y / (float)d[1], G.z / (float)d[2]);
    const float S3 = (S * S) * S, den = (2.0f * S) * S;
    Tex prev{out + (L > 0 ? off[L - 1] : 0), {pd[0], pd[1], pd[2]}, 1};
    const int64_t nv = (int64_t)d[0] * d[1] * d[2];
#pragma omp parallel for schedule(static)
    for (int64_t v = 0; v < nv; v++) {
      const int i = (int)(v % d[0]), j = (int)((v / d[0]) % d[1]), k = (int)(v / ((int64_t)d[0] * d[1]));
      const v3 gp = mk(((float)i + 0.5f) * vs.x, ((float)j + 0.5f) * vs.y, ((float)k + 0.5f) * vs.z);
      float swc = 0.0f, sw = 0.0f;
      for (int tx = -3; tx <= 3; tx++)
        for (int ty = -3; ty <= 3; ty++)
          for (int tz = -3; tz <= 3; tz++) {
            const float fx = (float)tx * S, fy = (float)ty * S, fz = (float)tz * S;
            const float w = S3 * cvr_expf(-((fx * fx + fy * fy) + fz * fz) / den);
            const v3 p = mk(gp.x + fx, gp.y + fy, gp.z + fz);
            const v3 u = mk(p.x / G.x, p.y / G.y, p.z / G.z);
            float c = 0.0f;
            if (!(u.x < 0.0f || u.y < 0.0f || u.z < 0.0f || u.x > 1.0f || u.y > 1.0f || u.z > 1.0f)) {
              if (L == 0) {
                float dens, rgba[4];
                vol.sample(std::fmaf(u.x, (float)P->N[0], -0.5f), std::fmaf(u.y, (float)P->N[1], -0.5f),
                           std::fmaf(u.z, (float)P->N[2], -0.5f), &dens);
                tf_lookup(P->tf_rgba, P->tf_n, dens, rgba);
                c = rgba[3];
              } else {
                prev.sample(std::fmaf(u.x, (float)pd[0], -0.5f), std::fmaf(u.y, (float)pd[1], -0.5f),
                            std::fmaf(u.z, (float)pd[2], -0.5f), &c);
              }
            }
            swc = swc + w * c;
            sw = sw + w;
          }
      out[off[L] + v] = q16(swc / sw);
    }
  }
  for (int64_t v = 0; v < off[nl]; v++) out[v] = q16(-1.0f * cvr_logf(1.0f - out[v]));
  return nl;
}

// Cone-traced directional occlusion + shadows (ray_bbox_marching.comp), CVR-SPEC:
// the march, sampling and composite of rc1pass; for src.a > 0 ShadeSample
// (:607-656) with the cones of :116-562.  Vector forms: pos + d * t = fmaf per
// component; k*a.z + u*a.y + v*a.x = fmaf(v, a.x, fmaf(u, a.y, k * a.z));
// cross = glm order without fma; dot/normalize as rc1pass.  Cone tables arrive
// RGBA16F-rounded (GetConeSectionsInfoTex).




namespace {

struct ExtVol {
  const float* v; int res[3]; int nl; v3 G;
  std::vector<int64_t> off;
  int wbits = 0;   // GL_LINEAR weights at this many fraction bits (filter_bits)
  // GetGaussianExtinction (:92-112): textureLod at an integer level, clamp-to-edge,
  // plus the CONSIDER_BORDERS attenuation outside the box
  float gge(v3 p, float mip) const {
    int L = (int)mip;
    L = std::min(std::max(L, 0), nl - 1);
    int d[3];
    ext_level_dims(res, L, d);
    Tex t{v + off[L], {d[0], d[1], d[2]}, 1, wbits};
    // texel coordinate p/G*d - 0.5 as fma(p, d/G, -0.5) with d/G rounded once
    // (the convention of the volume fetch, n_over_g in the march)
    const v3 s = mk((float)d[0] / G.x, (float)d[1] / G.y, (float)d[2] / G.z);
    float rg;
    t.sample(std::fmaf(p.x, s.x, -0.5f), std::fmaf(p.y, s.y, -0.5f), std::fmaf(p.z, s.z, -0.5f),
             &rg);
    if (p.x < 0.0f || p.x > G.x || p.y < 0.0f || p.y > G.y || p.z < 0.0f || p.z > G.z) {
      const float sg = std::ldexp(1.0f, (int)mip);   // pow(2.0, mip) of an integer level
      const v3 c = mk(std::fmin(std::fmax(p.x, 0.0f), G.x) - p.x, std::fmin(std::fmax(p.y, 0.0f), G.y) - p.y,
                      std::fmin(std::fmax(p.z, 0.0f), G.z) - p.z);
      const float dist = (c.x * c.x + c.y * c.y) + c.z * c.z;
      rg = rg * cvr_expf(-(dist) / ((2.0f * sg) * sg));
    }
    return rg;
  }
};

inline v3 vmad(v3 d, float t, v3 p) {
  return mk(std::fmaf(d.x, t, p.x), std::fmaf(d.y, t, p.y), std::fmaf(d.z, t, p.z));
}
inline v3 cone_axis(const float* a, v3 k, v3 u, v3 v) {
  return mk(std::fmaf(v.x, a[0], std::fmaf(u.x, a[1], k.x * a[2])),
            std::fmaf(v.y, a[0], std::fmaf(u.y, a[1], k.y * a[2])),
            std::fmaf(v.z, a[0], std::fmaf(u.z, a[1], k.z * a[2])));
}

// Cone1/3/7 RayOcclusion == Cone1/3/7 RayShadow (the same accumulation); the
// 1 -> 3 -> 7 ray splits of :124-140 / :210-217.  Returns the visibility.
float cone_trace(const ExtVol& E, const OracleDosCone& C, v3 pos, v3 k, v3 u, v3 v) {
  float rays[7], last[7];
  float track = C.initial_step;
  rays[0] = 0.0f;
  last[0] = 0.0f;
  int s = 0;
  for (int i = 0; i < C.counts[0]; i++, s++) {
    const float* sec = C.sections + 4 * s;
    const float amptau = E.gge(vmad(k, track, pos), sec[1]) * sec[3];
    rays[0] += ((last[0] + amptau) * sec[2]) * C.ui_weight;
    last[0] = amptau;
    track += sec[0];
  }
  if (C.counts[1] + C.counts[2] == 0) return cvr_expf(-rays[0]);
  rays[2] = rays[0]; rays[1] = rays[0];
  last[2] = last[0]; last[1] = last[0];
  v3 vk[7];
  for (int j = 0; j < 3; j++) vk[j] = cone_axis(C.axes + 3 * j, k, u, v);
  for (int i = 0; i < C.counts[1]; i++, s++) {
    const float* sec = C.sections + 4 * s;
    for (int j = 0; j < 3; j++) {
      const float amptau = E.gge(vmad(vk[j], track, pos), sec[1]) * sec[3];
      rays[j] += ((last[j] + amptau) * sec[2]) * C.ui_weight;
      last[j] = amptau;
    }
    track += sec[0];
  }
  if (C.counts[2] == 0)
    return ((cvr_expf(-rays[0]) + cvr_expf(-rays[1])) + cvr_expf(-rays[2])) / 3.0f;
  // transform 3 to 7
  rays[6] = rays[5] = rays[2];
  rays[4] = rays[3] = rays[1];
  float avg = ((rays[2] + rays[1]) + rays[0]) / 3.0f;
  rays[2] = rays[1] = rays[0];
  rays[0] = avg;
  last[6] = last[5] = last[2];
  last[4] = last[3] = last[1];
  float avgt = ((last[2] + last[1]) + last[0]) / 3.0f;
  last[2] = last[1] = last[0];
  last[0] = avgt;
  for (int j = 0; j < 7; j++) vk[j] = cone_axis(C.axes + 3 * (3 + j), k, u, v);
  for (int i = 0; i < C.counts[2]; i++, s++) {
    const float* sec = C.sections + 4 * s;
    for (int j = 0; j < 7; j++) {
      const float amptau = E.gge(vmad(vk[j], track, pos), sec[1]) * sec[3];
      rays[j] += ((last[j] + amptau) * sec[2]) * C.ui_weight;
      last[j] = amptau;
    }
    track += sec[0];
  }
  float side = cvr_expf(-rays[1]);
  for (int j = 2; j < 7; j++) side = side + cvr_expf(-rays[j]);
  return (cvr_expf(-rays[0]) + side * C.ray7w) / (1.0f + C.ray7w * 6.0f);
}

}  // namespace

namespace {

// The single-pass march shared by the shaded renderers (ray_bbox_marching.comp
// :658-734, ebs_ray_bbox_marching.comp:552-625): rows [y0, y1) of the frame.
// For every sample with alpha > 0, shade(src, tx, wp, cam_dir, x, y, z) turns
// src.rgb into the shaded colour (tx: position in the [0, G] box, wp: world
// position, x/y/z: texel coordinates of the volume fetch).
template <class Shade>
uint64_t shaded_march_rows(const OracleRc1pass& P, int y0, int y1, float* out_rgba,
                           uint32_t* out_counts, int nthreads, const Shade& shade) {
  float V[16], tanf;
  oracle_lookat(P.eye, P.center, P.up, P.fovy_deg, V, &tanf);
  const float aspect = P.aspect > 0 ? P.aspect : (float)P.W / (float)P.H;
  const v3 eye = mk(P.eye[0], P.eye[1], P.eye[2]);
  const v3 G = mk((float)P.N[0] * P.scale[0], (float)P.N[1] * P.scale[1], (float)P.N[2] * P.scale[2]);
  const v3 half = mk(G.x * 0.5f, G.y * 0.5f, G.z * 0.5f);
  const v3 NoG = mk((float)P.N[0] / G.x, (float)P.N[1] / G.y, (float)P.N[2] / G.z);
  Tex vol{P.vol, {P.N[0], P.N[1], P.N[2]}, 1, P.filter_bits};
  const int W = P.W, H = P.H;
  std::vector<uint32_t> tmp;
  uint32_t* counts = out_counts;
  if (!counts) { tmp.resize((size_t)W * H); counts = tmp.data(); }
#ifdef _OPENMP
  if (nthreads > 0) omp_set_num_threads(nthreads);
#endif
  y0 = std::max(0, y0);
  y1 = std::min(H, y1);
#pragma omp parallel for schedule(dynamic, 1)
  for (int py = y0; py < y1; py++) {
    for (int px = 0; px < W; px++) {
      const int64_t pix = (int64_t)py * W + px;
      float dst[4] = {0, 0, 0, 0};
      uint32_t cnt = 0;
      float fx = (float)px + 0.5f, fy = (float)py + 0.5f;
      float vx = std::fmaf(fx / (float)W, 2.0f, -1.0f);
      float vy = std::fmaf(fy / (float)H, 2.0f, -1.0f);
      v3 c = mk((vx * tanf) * aspect, vy * tanf, -1.0f);
      v3 d = mk(dot3(c, mk(V[0], V[1], V[2])), dot3(c, mk(V[4], V[5], V[6])),
                dot3(c, mk(V[8], V[9], V[10])));
      const v3 cam_dir = normalize3(d);          // camera_dir (:668-669)
      const v3 dir = normalize3(cam_dir);        // r.Dir, RayAABBIntersection (:590)
      v3 inv = mk(1.0f / dir.x, 1.0f / dir.y, 1.0f / dir.z);
      v3 ta = mk(inv.x * (-half.x - eye.x), inv.y * (-half.y - eye.y), inv.z * (-half.z - eye.z));
      v3 tb = mk(inv.x * (half.x - eye.x), inv.y * (half.y - eye.y), inv.z * (half.z - eye.z));
      float tnear = std::fmax(std::fmax(std::fmin(ta.x, tb.x), std::fmin(ta.y, tb.y)), std::fmin(ta.z, tb.z));
      float tfar = std::fmin(std::fmin(std::fmax(ta.x, tb.x), std::fmax(ta.y, tb.y)), std::fmax(ta.z, tb.z));
      const bool hit = tfar > tnear;
      tnear = std::fmax(tnear, 0.0f);
      if (hit) {
        const float D = std::fabs(tfar - tnear);
        const v3 tpos = mk(std::fmaf(dir.x, tnear, eye.x) + half.x, std::fmaf(dir.y, tnear, eye.y) + half.y,
                           std::fmaf(dir.z, tnear, eye.z) + half.z);
        const v3 o = mk(std::fmaf(tpos.x, NoG.x, -0.5f), std::fmaf(tpos.y, NoG.y, -0.5f), std::fmaf(tpos.z, NoG.z, -0.5f));
        const v3 dt = mk(dir.x * NoG.x, dir.y * NoG.y, dir.z * NoG.z);
        float s = 0.0f;
        while (s < D) {
          const float h = std::fmin(P.step, D - s);
          const float t = std::fmaf(h, 0.5f, s);
          const float x = std::fmaf(dt.x, t, o.x), y = std::fmaf(dt.y, t, o.y), z = std::fmaf(dt.z, t, o.z);
          float dens;
          vol.sample(x, y, z, &dens);
          float src[4];
          tf_lookup(P.tf, P.tf_n, dens, src, P.filter_bits);
          cnt++;
          if (src[3] > 0.0f) {
            const v3 tx = vmad(dir, t, tpos);              // tx_pos, volume box at [0, G]
            const v3 wp = mk(tx.x - half.x, tx.y - half.y, tx.z - half.z);
            shade(src, tx, wp, cam_dir, x, y, z);
            const float a = 1.0f - cvr_expf(-(src[3] * h));
            const float om = 1.0f - dst[3];
            dst[0] = std::fmaf(om, src[0] * a, dst[0]);
            dst[1] = std::fmaf(om, src[1] * a, dst[1]);
            dst[2] = std::fmaf(om, src[2] * a, dst[2]);
            dst[3] = std::fmaf(om, a, dst[3]);
            if (dst[3] > 0.99f) break;
          }
          s = s + h;
        }
      }
      if (out_rgba) for (int q = 0; q < 4; q++) out_rgba[pix * 4 + q] = dst[q];
      counts[pix] = cnt;
    }
  }
  uint64_t total = 0;
  for (int64_t i = (int64_t)y0 * W; i < (int64_t)y1 * W; i++) total += counts[i];
  return total;
}

}  // namespace

// Rows [y0, y1) of the frame (the whole frame: 0, H).  out: W*H*4, counts: W*H.
ORACLE_API uint64_t oracle_render_dos_rows(const OracleDos* Q, int y0, int y1, float* out_rgba,
                                           uint32_t* out_counts, int nthreads) {
  const OracleRc1pass& P = Q->base;
  const v3 eye = mk(P.eye[0], P.eye[1], P.eye[2]);
  const v3 G = mk((float)P.N[0] * P.scale[0], (float)P.N[1] * P.scale[1], (float)P.N[2] * P.scale[2]);
  const v3 light = mk(P.light[0], P.light[1], P.light[2]);
  const v3 lfwd = mk(Q->light_forward[0], Q->light_forward[1], Q->light_forward[2]);
  const v3 lup = mk(Q->light_up[0], Q->light_up[1], Q->light_up[2]);
  const v3 lright = mk(Q->light_right[0], Q->light_right[1], Q->light_right[2]);
  Tex grd{P.grad, {P.N[0], P.N[1], P.N[2]}, 3, P.filter_bits};
  ExtVol E{Q->ext, {Q->ext_res[0], Q->ext_res[1], Q->ext_res[2]}, Q->ext_levels, G, {}, P.filter_bits};
  E.off.assign(E.nl + 1, 0);
  for (int L = 0; L < E.nl; L++) {
    int d[3];
    ext_level_dims(E.res, L, d);
    E.off[L + 1] = E.off[L] + (int64_t)d[0] * d[1] * d[2];
  }
  // SpotLightMaxAngle uniform: glm::cos(glm::pi<float>() * angle / 180.f) (dosrcrenderer.cpp:158)
  const float spot_cos = std::cos(3.14159265358979323846f * Q->spot_angle_deg / 180.0f);
  const float ka = Q->apply_occlusion ? P.ka : 0.0f;
  const float kd = Q->apply_shadow ? P.kd : 0.0f;
  const float ks = Q->apply_shadow ? P.ks : 0.0f;
  auto shade = [&](float* src, v3 tx, v3 wp, v3 cam_dir, float x, float y, float z) {
    // eye-space frame of the occlusion cones (:681-684)
    const v3 v_right = normalize3(cross3(cam_dir, mk(0.0f, 1.0f, 0.0f)));
    const v3 v_up = normalize3(cross3(mk(-cam_dir.x, -cam_dir.y, -cam_dir.z), v_right));
    float iocc = 0.0f, isdw = 0.0f;
    if (Q->apply_occlusion) {
      const v3 k = normalize3(mk(eye.x - wp.x, eye.y - wp.y, eye.z - wp.z));
      iocc = cone_trace(E, Q->occ, tx, k, v_up, v_right);
    }
    if (Q->apply_shadow) {
      v3 k, u, v;
      bool lit = true;
      if (Q->shadow_type == 2) {
        k = lfwd; v = lup; u = lright;
      } else {
        k = normalize3(mk(light.x - wp.x, light.y - wp.y, light.z - wp.z));
        u = normalize3(cross3(k, lright));
        v = normalize3(cross3(k, u));
        if (Q->shadow_type == 1 && dot3(k, lfwd) < spot_cos) lit = false;
      }
      // Cone1RayShadow(pos, k, v, u) is called as (pos, k, u, v): swapped (:559-561)
      isdw = lit ? cone_trace(E, Q->sdw, tx, k, v, u) : 0.0f;
    }
    const float inv_k = 1.0f / (ka + kd);
    if (P.phong && P.grad) {
      float g[3];
      grd.sample(x, y, z, g);
      if (g[0] != 0.0f || g[1] != 0.0f || g[2] != 0.0f) {
        const v3 n = normalize3(mk(g[0], g[1], g[2]));
        const v3 L = normalize3(mk(light.x - wp.x, light.y - wp.y, light.z - wp.z));
        const v3 Ve = normalize3(mk(eye.x - wp.x, eye.y - wp.y, eye.z - wp.z));
        const v3 Hv = normalize3(mk(Ve.x + L.x, Ve.y + L.y, Ve.z + L.z));
        const float dd = std::fmax(0.0f, dot3(n, L));
        const float ds = std::fmax(0.0f, dot3(Hv, n));
        const float diff = inv_k * (iocc * ka + (isdw * kd) * dd);
        const float spec = (isdw * ks) * cvr_powf(ds, P.shininess);
        for (int q = 0; q < 3; q++) src[q] = std::fmaf(P.ispec[q], spec, src[q] * diff);
      }
    } else {
      for (int q = 0; q < 3; q++) src[q] = inv_k * ((src[q] * iocc) * ka + (src[q] * isdw) * kd);
    }
  };
  return shaded_march_rows(P, y0, y1, out_rgba, out_counts, nthreads, shade);
}

ORACLE_API uint64_t oracle_render_dos(const OracleDos* Q, float* out_rgba, uint32_t* out_counts,
                                      int nthreads) {
  return oracle_render_dos_rows(Q, 0, Q->base.H, out_rgba, out_counts, nthreads);
}

// ===========================================================================
// Extinction-based shading (rc1pextbsd), SURVEY.md §8 rows A14-A15
// ===========================================================================

// GetExtN(v / (2^bits - 1)) for every voxel value v (transferfunction1d.cpp:
// 132-157, 189-197; MaterialOpacityToExtinction, transferfunction.h:79-82):
// Get(norm, 1.0).a as float, then log(1 / (1 - a)) in double, returned as float.
ORACLE_API void oracle_ext_lut(const double* table, int max_density, int bpv, int extinction_input,
                               float* out_lut) {
  const int nv = bpv == 1 ? 256 : 65536;
  const double den = bpv == 1 ? (256.0 - 1.0) : (65536.0 - 1.0);
  for (int v = 0; v < nv; v++) {
    float g[4];
    oracle_tf_get(table, max_density, (double)v / den, 1.0, g);
    const float a = g[3];
    out_lut[v] = extinction_input ? a : (float)std::log(1.0 / (1.0 - (double)a));
  }
}

// RC1PExtinctionBasedShading::GenerateExtinctionSAT3DTex (ebsrenderer.cpp:624-662) and
// SummedAreaTable3D<double>::BuildSAT (summedareatable.h:218-278), literally: a
// (W+2)(H+2)(D+2) grid with a zero border, the interior holding lut[voxel], summed in
// double in the reference's order.  out: x-fastest doubles.
ORACLE_API void oracle_sat_build(const void* vox, int bpv, int W, int H, int D, const float* lut,
                                 double* out) {
  const int w = W + 2, h = H + 2, d = D + 2;
  auto at = [&](int x, int y, int z) -> double& { return out[x + (int64_t)w * y + (int64_t)w * h * z]; };
  auto get = [&](int x, int y, int z) -> double {
    if (x < 0 || y < 0 || z < 0) return 0.0;
    if (x >= w) x = w - 1;
    if (y >= h) y = h - 1;
    if (z >= d) z = d - 1;
    return at(x, y, z);
  };
  for (int x = 0; x < w; x++)
    for (int y = 0; y < h; y++)
      for (int z = 0; z < d; z++) {
        double val;
        if (x == 0 || y == 0 || z == 0 || x == w - 1 || y == h - 1 || z == d - 1) {
          val = 0.0f;
        } else {
          const int64_t i = (int64_t)(x - 1) + (int64_t)(y - 1) * W + (int64_t)(z - 1) * W * H;
          const int v = bpv == 1 ? ((const uint8_t*)vox)[i] : ((const uint16_t*)vox)[i];
          val = lut[v];
        }
        at(x, y, z) = val;
      }
  at(0, 0, 0) = get(0, 0, 0);
  for (int x = 1; x < w; x++) at(x, 0, 0) = get(x - 1, 0, 0) + get(x, 0, 0);
  for (int y = 1; y < h; y++) at(0, y, 0) = get(0, y - 1, 0) + get(0, y, 0);
  for (int z = 1; z < d; z++) at(0, 0, z) = get(0, 0, z - 1) + get(0, 0, z);
  for (int x = 1; x < w; x++)
    for (int z = 1; z < d; z++)
      at(x, 0, z) = get(x - 1, 0, z) + get(x, 0, z - 1) - get(x - 1, 0, z - 1) + get(x, 0, z);
  for (int x = 1; x < w; x++)
    for (int y = 1; y < h; y++)
      at(x, y, 0) = get(x - 1, y, 0) + get(x, y - 1, 0) - get(x - 1, y - 1, 0) + get(x, y, 0);
  for (int y = 1; y < h; y++)
    for (int z = 1; z < d; z++)
      at(0, y, z) = get(0, y - 1, z) + get(0, y, z - 1) - get(0, y - 1, z - 1) + get(0, y, z);
  for (int x = 1; x < w; x++)
    for (int y = 1; y < h; y++)
      for (int z = 1; z < d; z++) {
        double val = get(x, y, z)
                   + get(x - 1, y - 1, z - 1)
                   + get(x, y, z - 1)
                   + get(x, y - 1, z)
                   + get(x - 1, y, z)
                   - get(x - 1, y - 1, z)
                   - get(x, y - 1, z - 1)
                   - get(x - 1, y, z - 1);
        at(x, y, z) = val;
      }
}

// The same recurrence streamed over z with two double planes ((W+2)(H+2) doubles
// each) instead of the whole (W+2)(H+2)(D+2) grid: every BuildSAT cell is a
// function of its seven lower neighbours only (summedareatable.h:218-278), so any
// order that visits a cell after them reproduces the reference's doubles exactly.
// Emits, as float, the planes listed in zs[0..nz) (ascending), for full-size
// checks (1026^3 would need 8.6 GB as one double grid).
ORACLE_API void oracle_sat_planes(const void* vox, int bpv, int W, int H, int D, const float* lut,
                                  const int* zs, int nz, float* out) {
  const int w = W + 2, h = H + 2, d = D + 2;
  const size_t plane = (size_t)w * h;
  std::vector<double> prev(plane, 0.0), cur(plane, 0.0);
  auto raw = [&](int x, int y, int z) -> double {
    if (x == 0 || y == 0 || z == 0 || x == w - 1 || y == h - 1 || z == d - 1) return 0.0f;
    const int64_t i = (int64_t)(x - 1) + (int64_t)(y - 1) * W + (int64_t)(z - 1) * W * H;
    const int v = bpv == 1 ? ((const uint8_t*)vox)[i] : ((const uint16_t*)vox)[i];
    return lut[v];
  };
  int k = 0;
  for (int z = 0; z < d && k < nz; z++) {
    auto C = [&](int x, int y) -> double& { return cur[(size_t)x + (size_t)w * y]; };
    auto P = [&](int x, int y) -> double { return prev[(size_t)x + (size_t)w * y]; };
    if (z == 0) {
      C(0, 0) = raw(0, 0, 0);
      for (int x = 1; x < w; x++) C(x, 0) = C(x - 1, 0) + raw(x, 0, 0);
      for (int y = 1; y < h; y++) C(0, y) = C(0, y - 1) + raw(0, y, 0);
      for (int x = 1; x < w; x++)
        for (int y = 1; y < h; y++)
          C(x, y) = C(x - 1, y) + C(x, y - 1) - C(x - 1, y - 1) + raw(x, y, 0);
    } else {
      C(0, 0) = P(0, 0) + raw(0, 0, z);
      for (int x = 1; x < w; x++) C(x, 0) = C(x - 1, 0) + P(x, 0) - P(x - 1, 0) + raw(x, 0, z);
      for (int y = 1; y < h; y++) C(0, y) = C(0, y - 1) + P(0, y) - P(0, y - 1) + raw(0, y, z);
      for (int y = 1; y < h; y++)
        for (int x = 1; x < w; x++)
          C(x, y) = raw(x, y, z) + P(x - 1, y - 1) + P(x, y) + C(x, y - 1) + C(x - 1, y)
                  - C(x - 1, y - 1) - P(x, y - 1) - P(x - 1, y);
    }
    if (z == zs[k]) {
      float* o = out + (size_t)k * plane;
      for (size_t i = 0; i < plane; i++) o[i] = (float)cur[i];
      k++;
    }
    std::swap(prev, cur);
  }
}



namespace {

struct Sat {
  Tex t;            // comps = 1
  v3 S, G, inv_vs, nsat, min_sat, max_sat;
  // GetSummed3Density: texture(TexVolumeSAT3D, p * inv_vol_scaled).r
  float f(float x, float y, float z) const {
    const float ux = x * inv_vs.x, uy = y * inv_vs.y, uz = z * inv_vs.z;
    float r;
    t.sample(std::fmaf(ux, nsat.x, -0.5f), std::fmaf(uy, nsat.y, -0.5f), std::fmaf(uz, nsat.z, -0.5f), &r);
    return r;
  }
  // EvaluateSAT3D (ebs_ray_bbox_marching.comp:85-99)
  float box(v3 p1, v3 p2) const {
    const float V1 = f(p2.x, p2.y, p2.z), V2 = f(p1.x, p2.y, p2.z);
    const float V3 = f(p2.x, p2.y, p1.z), V4 = f(p1.x, p2.y, p1.z);
    const float V5 = f(p2.x, p1.y, p2.z), V6 = f(p1.x, p1.y, p2.z);
    const float V7 = f(p2.x, p1.y, p1.z), V8 = f(p1.x, p1.y, p1.z);
    return (V1 - V2 - V3 + V4 - V5 + V6 + V7 - V8);
  }
  v3 offset_clamp(v3 p) const {   // clamp(p + VolumeScales, MinSATPosition, MaxSATPosition)
    return mk(std::fmin(std::fmax(p.x + S.x, min_sat.x), max_sat.x),
              std::fmin(std::fmax(p.y + S.y, min_sat.y), max_sat.y),
              std::fmin(std::fmax(p.z + S.z, min_sat.z), max_sat.z));
  }
  float ao_box(v3 p1, v3 p2) const { return box(offset_clamp(p1), offset_clamp(p2)); }
  // EvaluateShadowSAT3D (:148-185, texture path)
  float shadow_box(v3 p1, v3 p2, float uiw) const {
    const float volquery = ((std::fabs(p1.x - p2.x) / S.x)) * ((std::fabs(p1.y - p2.y) / S.y)) *
                           ((std::fabs(p1.z - p2.z) / S.z));
    return ((box(offset_clamp(p1), offset_clamp(p2)) / volquery)) * uiw;
  }
};

// ExtinctionAmbientOcclusion (:109-146)
float ebs_occlusion(const Sat& T, v3 tx, int shells, float R) {
  const v3 r0 = mk(R * T.S.x, R * T.S.y, R * T.S.z);
  const float SAT_Sh0 = T.ao_box(mk(tx.x - r0.x, tx.y - r0.y, tx.z - r0.z),
                                 mk(tx.x + r0.x, tx.y + r0.y, tx.z + r0.z));
  const float rsh0 = R;
  const float tSh0 = SAT_Sh0 * (1.0f / (rsh0 * rsh0));
  float SAT_Shi = SAT_Sh0, tshi = tSh0;
  for (int i = 1; i < shells; i++) {
    const float r1 = R * (float)(i + 1);
    const v3 ri = mk(r1 * T.S.x, r1 * T.S.y, r1 * T.S.z);
    const float SAT_Shi_1 = T.ao_box(mk(tx.x - ri.x, tx.y - ri.y, tx.z - ri.z),
                                     mk(tx.x + ri.x, tx.y + ri.y, tx.z + ri.z));
    const float tshi_1 = tshi + (SAT_Shi_1 - SAT_Shi) * (1.0f / (r1 * r1));
    SAT_Shi = SAT_Shi_1;
    tshi = tshi_1;
  }
  const float rshi = R * (float)shells;
  const float W_A = 1.0f / (rshi * rshi);
  const float Stau = W_A * tshi;
  return cvr_expf(-(Stau));
}

struct ConeCS { float p_cs, p_sn, n_cs, n_sn; };

// One box chain along the dominant axis a (ConeZAxis :187-275, ConeYAxis :277-364,
// ConeXAxis :366-453).  The three are written out as the reference has them.
float cone_z(const Sat& T, const OracleEbs& Q, const ConeCS& c, v3 pos, v3 cv) {
  float Stau = 0.0f;
  float signal = 1.0f;
  if (cv.z < 0) signal = -1.0f;
  const v3 proj_y = normalize3(mk(0.0f, cv.y, cv.z));
  const v3 proj_x = normalize3(mk(cv.x, 0.0f, cv.z));
  const v3 pj_x1 = normalize3(mk(proj_x.x * c.n_cs - proj_x.z * c.n_sn, 0.0f, proj_x.x * c.n_sn + proj_x.z * c.n_cs));
  const v3 pj_x2 = normalize3(mk(proj_x.x * c.p_cs - proj_x.z * c.p_sn, 0.0f, proj_x.x * c.p_sn + proj_x.z * c.p_cs));
  const v3 pj_y1 = normalize3(mk(0.0f, proj_y.y * c.n_cs - proj_y.z * c.n_sn, proj_y.y * c.n_sn + proj_y.z * c.n_cs));
  const v3 pj_y2 = normalize3(mk(0.0f, proj_y.y * c.p_cs - proj_y.z * c.p_sn, proj_y.y * c.p_sn + proj_y.z * c.p_cs));
  const float si = Q.interval * signal * T.S.z;
  float z_pos = Q.initial_step * signal * T.S.z;
  const float vmin = T.S.z * 0.5f, vmax = T.G.z - T.S.z * 0.5f;
  while ((z_pos / cv.z) < Q.max_distance &&
         (pos.z + (z_pos + si) > vmin && pos.z + (z_pos + si) < vmax)) {
    const float z_mean = std::fabs(z_pos + si * 0.5f);
    const float p_x1 = pj_x1.x * (z_mean / std::fabs(pj_x1.z));
    const float p_x2 = pj_x2.x * (z_mean / std::fabs(pj_x2.z));
    const float p_y1 = pj_y1.y * (z_mean / std::fabs(pj_y1.z));
    const float p_y2 = pj_y2.y * (z_mean / std::fabs(pj_y2.z));
    float x1 = std::fmin(p_x1, p_x2), x2 = std::fmax(p_x1, p_x2);
    float y1 = std::fmin(p_y1, p_y2), y2 = std::fmax(p_y1, p_y2);
    const float xdiff = std::fabs(x2 - x1), ydiff = std::fabs(y2 - y1);
    const float xs = (std::ceil(xdiff / T.S.x) - (xdiff / T.S.x)) * 0.5f;
    const float ys = (std::ceil(ydiff / T.S.y) - (ydiff / T.S.y)) * 0.5f;
    x1 = x1 - xs * T.S.x; x2 = x2 + xs * T.S.x;
    y1 = y1 - ys * T.S.y; y2 = y2 + ys * T.S.y;
    const float z1 = std::fmin(z_pos, z_pos + si), z2 = std::fmax(z_pos, z_pos + si);
    Stau += T.shadow_box(mk(pos.x + x1, pos.y + y1, pos.z + z1), mk(pos.x + x2, pos.y + y2, pos.z + z2),
                         Q.ui_weight);
    z_pos = z_pos + si;
  }
  return Stau;
}

float cone_y(const Sat& T, const OracleEbs& Q, const ConeCS& c, v3 pos, v3 cv) {
  float Stau = 0.0f;
  float signal = 1.0f;
  if (cv.y < 0) signal = -1.0f;
  const v3 proj_x = normalize3(mk(cv.x, cv.y, 0.0f));
  const v3 proj_z = normalize3(mk(0.0f, cv.y, cv.z));
  const v3 pj_x1 = normalize3(mk(proj_x.x * c.n_cs - proj_x.y * c.n_sn, proj_x.x * c.n_sn + proj_x.y * c.n_cs, 0.0f));
  const v3 pj_x2 = normalize3(mk(proj_x.x * c.p_cs - proj_x.y * c.p_sn, proj_x.x * c.p_sn + proj_x.y * c.p_cs, 0.0f));
  const v3 pj_z1 = normalize3(mk(0.0f, proj_z.z * c.n_sn + proj_z.y * c.n_cs, proj_z.z * c.n_cs - proj_z.y * c.n_sn));
  const v3 pj_z2 = normalize3(mk(0.0f, proj_z.z * c.p_sn + proj_z.y * c.p_cs, proj_z.z * c.p_cs - proj_z.y * c.p_sn));
  const float si = Q.interval * signal * T.S.y;
  float y_pos = Q.initial_step * signal * T.S.y;
  const float vmin = T.S.y * 0.5f, vmax = T.G.y - T.S.y * 0.5f;
  while ((y_pos / cv.y) < Q.max_distance &&
         (pos.y + (y_pos + si) > vmin && pos.y + (y_pos + si) < vmax)) {
    const float y_mean = std::fabs(y_pos + si * 0.5f);
    const float p_x1 = pj_x1.x * (y_mean / std::fabs(pj_x1.y));
    const float p_x2 = pj_x2.x * (y_mean / std::fabs(pj_x2.y));
    const float p_z1 = pj_z1.z * (y_mean / std::fabs(pj_z1.y));
    const float p_z2 = pj_z2.z * (y_mean / std::fabs(pj_z2.y));
    float x1 = std::fmin(p_x1, p_x2), x2 = std::fmax(p_x1, p_x2);
    float z1 = std::fmin(p_z1, p_z2), z2 = std::fmax(p_z1, p_z2);
    const float xdiff = std::fabs(x2 - x1), zdiff = std::fabs(z2 - z1);
    const float xs = (std::ceil(xdiff / T.S.x) - (xdiff / T.S.x)) * 0.5f;
    const float zs = (std::ceil(zdiff / T.S.z) - (zdiff / T.S.z)) * 0.5f;
    x1 = x1 - xs * T.S.x; x2 = x2 + xs * T.S.x;
    z1 = z1 - zs * T.S.z; z2 = z2 + zs * T.S.z;
    const float y1 = std::fmin(y_pos, y_pos + si), y2 = std::fmax(y_pos, y_pos + si);
    Stau += T.shadow_box(mk(pos.x + x1, pos.y + y1, pos.z + z1), mk(pos.x + x2, pos.y + y2, pos.z + z2),
                         Q.ui_weight);
    y_pos = y_pos + si;
  }
  return Stau;
}

float cone_x(const Sat& T, const OracleEbs& Q, const ConeCS& c, v3 pos, v3 cv) {
  float Stau = 0.0f;
  float signal = 1.0f;
  if (cv.x < 0) signal = -1.0f;
  const v3 proj_y = normalize3(mk(cv.x, cv.y, 0.0f));
  const v3 proj_z = normalize3(mk(cv.x, 0.0f, cv.z));
  const v3 pj_y1 = normalize3(mk(proj_y.y * c.n_sn + proj_y.x * c.n_cs, proj_y.y * c.n_cs - proj_y.x * c.n_sn, 0.0f));
  const v3 pj_y2 = normalize3(mk(proj_y.y * c.p_sn + proj_y.x * c.p_cs, proj_y.y * c.p_cs - proj_y.x * c.p_sn, 0.0f));
  const v3 pj_z1 = normalize3(mk(proj_z.z * c.n_sn + proj_z.x * c.n_cs, 0.0f, proj_z.z * c.n_cs - proj_z.x * c.n_sn));
  const v3 pj_z2 = normalize3(mk(proj_z.z * c.p_sn + proj_z.x * c.p_cs, 0.0f, proj_z.z * c.p_cs - proj_z.x * c.p_sn));
  const float si = Q.interval * signal * T.S.x;
  float x_pos = Q.initial_step * signal * T.S.x;
  const float vmin = T.S.x * 0.5f, vmax = T.G.x - T.S.x * 0.5f;
  while ((x_pos / cv.x) < Q.max_distance &&
         (pos.x + (x_pos + si) > vmin && pos.x + (x_pos + si) < vmax)) {
    const float x_mean = std::fabs(x_pos + si * 0.5f);
    const float p_y1 = pj_y1.y * (x_mean / std::fabs(pj_y1.x));
    const float p_y2 = pj_y2.y * (x_mean / std::fabs(pj_y2.x));
    const float p_z1 = pj_z1.z * (x_mean / std::fabs(pj_z1.x));
    const float p_z2 = pj_z2.z * (x_mean / std::fabs(pj_z2.x));
    float y1 = std::fmin(p_y1, p_y2), y2 = std::fmax(p_y1, p_y2);
    float z1 = std::fmin(p_z1, p_z2), z2 = std::fmax(p_z1, p_z2);
    const float ydiff = std::fabs(y2 - y1), zdiff = std::fabs(z2 - z1);
    const float ys = (std::ceil(ydiff / T.S.y) - (ydiff / T.S.y)) * 0.5f;
    const float zs = (std::ceil(zdiff / T.S.z) - (zdiff / T.S.z)) * 0.5f;
    y1 = y1 - ys * T.S.y; y2 = y2 + ys * T.S.y;
    z1 = z1 - zs * T.S.z; z2 = z2 + zs * T.S.z;
    const float x1 = std::fmin(x_pos, x_pos + si), x2 = std::fmax(x_pos, x_pos + si);
    Stau += T.shadow_box(mk(pos.x + x1, pos.y + y1, pos.z + z1), mk(pos.x + x2, pos.y + y2, pos.z + z2),
                         Q.ui_weight);
    x_pos = x_pos + si;
  }
  return Stau;
}

}  // namespace

ORACLE_API uint64_t oracle_render_ebs_rows(const OracleEbs* Q, int y0, int y1, float* out_rgba,
                                           uint32_t* out_counts, int nthreads) {
  const OracleRc1pass& P = Q->base;
  const v3 eye = mk(P.eye[0], P.eye[1], P.eye[2]);
  const v3 light = mk(P.light[0], P.light[1], P.light[2]);
  Sat T;
  T.t = Tex{Q->sat, {Q->sat_dims[0], Q->sat_dims[1], Q->sat_dims[2]}, 1, P.filter_bits};
  T.S = mk(P.scale[0], P.scale[1], P.scale[2]);
  T.G = mk((float)P.N[0] * P.scale[0], (float)P.N[1] * P.scale[1], (float)P.N[2] * P.scale[2]);
  // inv_vol_scaled = 1.0f / (VolumeScaledSizes + VolumeScales * 2.0) (:75)
  T.inv_vs = mk(1.0f / (T.G.x + T.S.x * 2.0f), 1.0f / (T.G.y + T.S.y * 2.0f), 1.0f / (T.G.z + T.S.z * 2.0f));
  T.nsat = mk((float)Q->sat_dims[0], (float)Q->sat_dims[1], (float)Q->sat_dims[2]);
  T.min_sat = mk(T.S.x * 0.5f, T.S.y * 0.5f, T.S.z * 0.5f);
  T.max_sat = mk(T.G.x + T.S.x * 1.5f, T.G.y + T.S.y * 1.5f, T.G.z + T.S.z * 1.5f);
  ConeCS cs{std::cos(Q->cone_angle), std::sin(Q->cone_angle), std::cos(-Q->cone_angle),
            std::sin(-Q->cone_angle)};
  const v3 lfwd = mk(Q->light_forward[0], Q->light_forward[1], Q->light_forward[2]);
  Tex grd{P.grad, {P.N[0], P.N[1], P.N[2]}, 3, P.filter_bits};
  const float ka = Q->apply_occlusion ? P.ka : 0.0f;
  const float kd = Q->apply_shadow ? P.kd : 0.0f;
  const float ks = Q->apply_shadow ? P.ks : 0.0f;
  auto shade = [&](float* src, v3 tx, v3 wp, v3, float x, float y, float z) {
    float iocc = 0.0f, isdw = 0.0f;
    if (Q->apply_occlusion) iocc = ebs_occlusion(T, tx, Q->occ_shells, Q->occ_radius);
    if (Q->apply_shadow) {
      // ExtinctionDirectionalShadows (:455-481)
      const v3 cv = Q->shadow_type == 0 ? normalize3(mk(light.x - wp.x, light.y - wp.y, light.z - wp.z))
                                        : normalize3(lfwd);
      const v3 ac = mk(std::fabs(cv.x), std::fabs(cv.y), std::fabs(cv.z));
      float Stau;
      if (ac.z > ac.x && ac.z > ac.y) Stau = cone_z(T, *Q, cs, tx, cv);
      else if (ac.y > ac.x) Stau = cone_y(T, *Q, cs, tx, cv);
      else Stau = cone_x(T, *Q, cs, tx, cv);
      isdw = cvr_expf(-Stau);
    }
    const float inv_k = 1.0f / (ka + kd);
    if (P.phong && P.grad) {
      float g[3];
      grd.sample(x, y, z, g);
      if (g[0] != 0.0f || g[1] != 0.0f || g[2] != 0.0f) {
        const v3 n = normalize3(mk(g[0], g[1], g[2]));
        const v3 L = normalize3(mk(light.x - wp.x, light.y - wp.y, light.z - wp.z));
        const v3 Ve = normalize3(mk(eye.x - wp.x, eye.y - wp.y, eye.z - wp.z));
        const v3 Hv = normalize3(mk(Ve.x + L.x, Ve.y + L.y, Ve.z + L.z));
        const float dd = std::fmax(0.0f, dot3(n, L));
        const float ds = std::fmax(0.0f, dot3(Hv, n));
        const float pw = cvr_powf(ds, P.shininess);
        // (1/(ka+kd)) * (L*IOcc*ka + IShadow*(L*kd*dot_diff)) + IShadow*(ks*Ispecular*pow) (:528-530)
        for (int q = 0; q < 3; q++)
          src[q] = inv_k * ((src[q] * iocc) * ka + isdw * ((src[q] * kd) * dd)) +
                   isdw * ((ks * P.ispec[q]) * pw);
      }
    } else {
      for (int q = 0; q < 3; q++) src[q] = inv_k * ((src[q] * iocc) * ka + (src[q] * isdw) * kd);
    }
  };
  return shaded_march_rows(P, y0, y1, out_rgba, out_counts, nthreads, shade);
}

// ===========================================================================
// Post-pass: pixel multiscaling filters and the screenshot composite
//   RenderFrameToScreen::DrawMultiSampleHigherResolutionMode / ...WithDownScale /
//   ...WithUpScale ........... libs/vis_utils/renderoutputframe.cpp:265-539
//   multisample_filter.comp, downscaling_filter.comp, upscaling_filter.comp,
//   box/hat/catmullrom/mitchellnetravali/cardinalbspline/cardinalomoms_filter.comp,
//   cbs/comoms_digital_filter.comp .. libs/vis_utils/shader/renderoutputframe/
//   blend over white + glReadPixels .. cppvolrend/renderingmanager.cpp:103-112, 476-492
// Images are RGBA16F (uint16 x 4 per pixel, row 0 = bottom); every imageStore
// rounds to binary16; texelFetch outside the image reads 0; texture() is
// bilinear with clamp-to-edge (CVR-SPEC lerp).
// ===========================================================================
namespace post {

struct Px { float c[4]; };

inline Px load(const uint16_t* img, int w, int x, int y) {
  Px p;
  for (int k = 0; k < 4; k++) p.c[k] = half_to_float(img[((size_t)y * w + x) * 4 + k]);
  return p;
}
inline void store(uint16_t* img, int w, int x, int y, const Px& p) {
  for (int k = 0; k < 4; k++) img[((size_t)y * w + x) * 4 + k] = float_to_half(p.c[k]);
}
inline Px fetch(const uint16_t* img, int w, int h, int x, int y) {
  if (x < 0 || y < 0 || x >= w || y >= h) return Px{{0.f, 0.f, 0.f, 0.f}};
  return load(img, w, x, y);
}

// kernel_support / kernel_weight of <name>_filter.comp
float support(int k) { return k == 0 ? 1.0f : (k == 1 ? 2.0f : 4.0f); }
float cubic(int k, float x) {
  x = std::fabs(x);
  if (x > 2.0f) return 0.0f;
  const bool far = x > 1.0f;
  const float u = far ? 2.0f - x : 1.0f - x;
  switch (k) {
    case 2: return far ? ((0.5f * u - 0.5f) * u) * u : ((-1.5f * u + 2.0f) * u + 0.5f) * u;
    case 3: return far ? (((7 / 18.0f) * u - 1 / 3.0f) * u) * u
                       : (((-7 / 6.0f) * u + 1.5f) * u + 0.5f) * u + 1 / 18.0f;
    case 4: return far ? ((u)*u) * u : ((-3.0f * u + 3.0f) * u + 3.0f) * u + 1.0f;
    default: return far ? ((0.875f * u) * u + 0.125f) * u
                        : ((-2.625f * u + 2.625f) * u + 2.25f) * u + 1.0f;
  }
}
float weight(int k, float x) {
  if (k == 0) return x <= -0.5f || x > 0.5f ? 0.0f : 1.0f;
  if (k == 1) { x = std::fabs(x); return x > 1.0f ? 0.0f : 1.0f - x; }
  return cubic(k, x);
}

void multisample(const uint16_t* src, int sw, int sh, uint16_t* dst, int tw, int th) {
  for (int y = 0; y < th; y++)
    for (int x = 0; x < tw; x++) {
      const float u = ((float)x + 0.5f) / (float)tw, v = ((float)y + 0.5f) / (float)th;
      const float fx = u * (float)sw - 0.5f, fy = v * (float)sh - 0.5f;
      const float flx = std::floor(fx), fly = std::floor(fy);
      const float ax = fx - flx, ay = fy - fly;
      auto cl = [](int i, int n) { return i < 0 ? 0 : (i > n - 1 ? n - 1 : i); };
      const int x0 = cl((int)flx, sw), x1 = cl((int)flx + 1, sw);
      const int y0 = cl((int)fly, sh), y1 = cl((int)fly + 1, sh);
      const Px a = load(src, sw, x0, y0), b = load(src, sw, x1, y0);
      const Px c = load(src, sw, x0, y1), d = load(src, sw, x1, y1);
      Px r;
      for (int k = 0; k < 4; k++) {
        const float top = std::fma(ax, b.c[k] - a.c[k], a.c[k]);
        const float bot = std::fma(ax, d.c[k] - c.c[k], c.c[k]);
        r.c[k] = std::fma(ay, bot - top, top);
      }
      store(dst, tw, x, y, r);
    }
}

void downscale(int K, const uint16_t* src, int sw, int sh, uint16_t* dst, int tw, int th) {
  const float s_r = (float)th / (float)sh, s_c = (float)tw / (float)sw;
  const float kr = 0.5f * support(K);
  for (int jr = 0; jr < th; jr++)
    for (int jc = 0; jc < tw; jc++) {
      const float x_r = ((float)jr + 0.5f) / (float)th;
      const int il_r = (int)std::ceil((x_r - kr / (float)th) * (float)sh - 0.5f);
      const int ir_r = (int)std::floor((x_r + kr / (float)th) * (float)sh - 0.5f);
      const float x_c = ((float)jc + 0.5f) / (float)tw;
      const int il_c = (int)std::ceil((x_c - kr / (float)tw) * (float)sw - 0.5f);
      const int ir_c = (int)std::floor((x_c + kr / (float)tw) * (float)sw - 0.5f);
      Px f{{0.f, 0.f, 0.f, 0.f}};
      for (int ir = il_r; ir <= ir_r; ir++)
        for (int ic = il_c; ic <= ir_c; ic++) {
          const float wgt = weight(K, (x_r - ((float)ir + 0.5f) / (float)sh) * (float)th) *
                            weight(K, (x_c - ((float)ic + 0.5f) / (float)sw) * (float)tw);
          const Px t = fetch(src, sw, sh, ic, ir);
          for (int k = 0; k < 4; k++) f.c[k] = f.c[k] + wgt * t.c[k];
        }
      const float s = s_r * s_c;
      for (int k = 0; k < 4; k++) f.c[k] = f.c[k] * s;
      store(dst, tw, jc, jr, f);
    }
}

void upscale(int K, const uint16_t* src, int sw, int sh, uint16_t* dst, int tw, int th) {
  const float kr = 0.5f * support(K);
  for (int jr = 0; jr < th; jr++)
    for (int jc = 0; jc < tw; jc++) {
      const float x_r = ((float)jr + 0.5f) / (float)th;
      const float xi_r = x_r * (float)sh - 0.5f;
      const int il_r = (int)std::ceil(xi_r - kr), ir_r = (int)std::floor(xi_r + kr);
      const float x_c = ((float)jc + 0.5f) / (float)tw;
      const float xi_c = x_c * (float)sw - 0.5f;
      const int il_c = (int)std::ceil(xi_c - kr), ir_c = (int)std::floor(xi_c + kr);
      Px f{{0.f, 0.f, 0.f, 0.f}};
      for (int ir = il_r; ir <= ir_r; ir++)
        for (int ic = il_c; ic <= ir_c; ic++) {
          const float wgt = weight(K, xi_r - (float)ir) * weight(K, xi_c - (float)ic);
          const Px t = fetch(src, sw, sh, ic, ir);
          for (int k = 0; k < 4; k++) f.c[k] = f.c[k] + wgt * t.c[k];
        }
      store(dst, tw, jc, jr, f);
    }
}

// cbs/comoms_digital_filter.comp: direction 0 (rows), then direction 1 (columns),
// in place; imageLoad re-reads the rounded stores.
void digital(int K, uint16_t* img, int w, int h) {
  static const float Lc[8] = {.2f, .26315789f, .26760563f, .26792453f,
                              .26794742f, .26794907f, .26794918f, .26794919f};
  static const float Lo[9] = {.23529412f, .33170732f, .34266611f, .34395774f, .34411062f,
                              .34412872f, .34413087f, .34413112f, .34413115f};
  const float* L = K == 4 ? Lc : Lo;
  const int m = K == 4 ? 8 : 9;
  const float p_inv = 1.0f;
  const float L_inf = L[m - 1], v_inv = L_inf / (1.f + L_inf);
  for (int dir = 0; dir < 2; dir++) {
    const int lines = dir == 0 ? h : w, nn = dir == 0 ? w : h;
    for (int t = 0; t < lines; t++) {
      auto X = [&](int i) { return dir == 0 ? i : t; };
      auto Y = [&](int i) { return dir == 0 ? t : i; };
      auto ld = [&](int i) { return load(img, w, X(i), Y(i)); };
      auto st = [&](int i, const Px& p) { store(img, w, X(i), Y(i), p); };
      for (int i = 1; i < nn; i++) {
        const float l = i < m ? L[i - 1] : L_inf;
        const Px c = ld(i), p = ld(i - 1);
        Px r;
        for (int k = 0; k < 4; k++) r.c[k] = c.c[k] - l * p.c[k];
        st(i, r);
      }
      {
        Px c = ld(nn - 1);
        for (int k = 0; k < 4; k++) c.c[k] = c.c[k] * p_inv * v_inv;
        st(nn - 1, c);
      }
      for (int i = nn - 2; i >= 0; i--) {
        const float l = i >= m - 1 ? L_inf : L[i];
        const Px c = ld(i), n1 = ld(i + 1);
        Px r;
        for (int k = 0; k < 4; k++) r.c[k] = l * (p_inv * c.c[k] - n1.c[k]);
        st(i, r);
      }
    }
  }
}

}  // namespace post

// mode 1 multisample, 2 downscale, 3 upscale; kernel = vis::IMAGE_FILTER_KERNEL.
// `frame` is modified in place by mode 3 with a cardinal kernel (as the reference).
ORACLE_API int oracle_multiscale_filter(int mode, int kernel, uint16_t* frame, int fw, int fh,
                                        uint16_t* screen, int sw, int sh) {
  const bool cardinal = kernel == 4 || kernel == 5;
  if (mode == 1) {
    post::multisample(frame, fw, fh, screen, sw, sh);
  } else if (mode == 2) {
    post::downscale(kernel, frame, fw, fh, screen, sw, sh);
    if (cardinal) post::digital(kernel, screen, sw, sh);
  } else if (mode == 3) {
    if (cardinal) post::digital(kernel, frame, fw, fh);
    post::upscale(kernel, frame, fw, fh, screen, sw, sh);
  } else {
    return 1;
  }
  return 0;
}

// RGBA (float, or binary16 when `half`) over white -> RGB8 (glReadPixels order)
ORACLE_API void oracle_screenshot_rgb8(const void* frame, int half, int w, int h, uint8_t* rgb) {
  for (size_t i = 0; i < (size_t)w * h; i++) {
    float p[4];
    for (int k = 0; k < 4; k++)
      p[k] = half ? half_to_float(((const uint16_t*)frame)[i * 4 + k]) : ((const float*)frame)[i * 4 + k];
    for (int k = 0; k < 3; k++) {
      const float v = p[k] * p[3] + (1.0f - p[3]);
      const float q = std::floor(v * 255.0f + 0.5f);
      rgb[i * 3 + k] = (uint8_t)(q < 0.0f ? 0.0f : (q > 255.0f ? 255.0f : q));
    }
  }
}

// ===========================================================================
// Isosurface ray-casters with block empty-space skipping
// ===========================================================================
//
//   variant 0: cppvolrend/structured/rc1pisocustom/custom_ray_marching_1p_iso_adapt.comp
//              :93-130 (block index / bounds / chord), :155-246 (march), 4^3 blocks
//   variant 1: cppvolrend/structured/rc1pisodfscustom/custom_ray_marching_1p_iso_adapt.comp
//              :94-156 (block index / bounds / exit distance), :181-260 (march), 32^3 blocks
//   variant 2: cppvolrend/structured/rc1pisoadapt/ray_marching_1p_iso_adapt.comp:113-172
//              (RayCasting1PassIsoAdapt, no blocks)
//   blocks:    ComputeBlocksFromVolume, rc1custompisoadaptrenderer.cpp:20-117
//              (R32F textures, NEAREST, default REPEAT wrap)
// CVR-SPEC: r.Origin + r.Dir * t is fmaf(dir, t, eye) (as in the rc1pass ray
// entry), the composite is the rc1pass fmaf form, Blinn-Phong the rc1pass one;
// every other expression in the shader's order, unfused.  `counts` = volume
// fetches the shader issues (the skip branch's dead re-fetch of variant 1 too).
struct OracleIso {
  OracleRc1pass base;                  // volume, gradient, camera, Blinn-Phong (tf unused)
  int variant;
  int nb[3];
  const float* bmin; const float* bmax;   // nb[0]*nb[1]*nb[2] each, x-fastest
  float iso, step_small, step_large, step_range;
  float color[4];
};

ORACLE_API void oracle_iso_blocks(const void* vox, int bpv, int w, int h, int d, const int nb[3],
                                  float* out_min, float* out_max) {
  // (N + nb - 1) / nb in float, truncated (:37-39), equals the integer ceiling here
  const int bs[3] = {(w + nb[0] - 1) / nb[0], (h + nb[1] - 1) / nb[1], (d + nb[2] - 1) / nb[2]};
  const double mx = bpv == 1 ? 255.0 : 65535.0;
  size_t k = 0;
  for (int bz = 0; bz < nb[2]; bz++)
    for (int by = 0; by < nb[1]; by++)
      for (int bx = 0; bx < nb[0]; bx++, k++) {
        const int x0 = bx * bs[0], y0 = by * bs[1], z0 = bz * bs[2];
        const int x1 = std::min(x0 + bs[0], w), y1 = std::min(y0 + bs[1], h), z1 = std::min(z0 + bs[2], d);
        double lo = 3.4028234663852886e38, hi = -3.4028234663852886e38;
        for (int z = z0; z < z1; z++)
          for (int y = y0; y < y1; y++)
            for (int x = x0; x < x1; x++) {
              const size_t i = ((size_t)z * h + y) * w + x;
              const double v = (bpv == 1 ? (double)((const uint8_t*)vox)[i]
                                         : (double)((const uint16_t*)vox)[i]) / mx;
              lo = std::min(lo, v);
              hi = std::max(hi, v);
            }
        out_min[k] = (float)lo;
        out_max[k] = (float)hi;
      }
}

namespace {

constexpr uint32_t kIsoMaxIter = 1u << 22;   // the kernel's iteration bound (iso.hip)

inline v3 iso_pos(v3 eye, v3 dir, float t) {
  return mk(std::fmaf(dir.x, t, eye.x), std::fmaf(dir.y, t, eye.y), std::fmaf(dir.z, t, eye.z));
}

}  // namespace

ORACLE_API uint64_t oracle_render_iso_rows(const OracleIso* Q, int y0, int y1, float* out,
                                           uint32_t* counts, int nthreads) {
  const OracleRc1pass& P = Q->base;
  float V[16], tanf;
  oracle_lookat(P.eye, P.center, P.up, P.fovy_deg, V, &tanf);
  const float aspect = P.aspect > 0 ? P.aspect : (float)P.W / (float)P.H;
  const v3 eye = mk(P.eye[0], P.eye[1], P.eye[2]);
  const float G[3] = {(float)P.N[0] * P.scale[0], (float)P.N[1] * P.scale[1], (float)P.N[2] * P.scale[2]};
  const v3 half = mk(G[0] * 0.5f, G[1] * 0.5f, G[2] * 0.5f);
  const float NoG[3] = {(float)P.N[0] / G[0], (float)P.N[1] / G[1], (float)P.N[2] / G[2]};
  const float nbf[3] = {(float)Q->nb[0], (float)Q->nb[1], (float)Q->nb[2]};
  // length(VolumeGridSize / numBlocks) * 0.5 (variant 1, :222-223)
  const float bl[3] = {G[0] / nbf[0], G[1] / nbf[1], G[2] / nbf[2]};
  const float half_block = std::sqrt(std::fmaf(bl[2], bl[2], std::fmaf(bl[1], bl[1], bl[0] * bl[0]))) * 0.5f;
  const v3 light = mk(P.light[0], P.light[1], P.light[2]);
  Tex vol{P.vol, {P.N[0], P.N[1], P.N[2]}, 1};
  Tex grd{P.grad, {P.N[0], P.N[1], P.N[2]}, 3};
  const float iso = Q->iso;
  const int W = P.W, H = P.H;
#ifdef _OPENMP
  if (nthreads > 0) omp_set_num_threads(nthreads);
#endif
  uint64_t total = 0;
#pragma omp parallel for schedule(dynamic, 1) reduction(+ : total)
  for (int py = y0; py < y1; py++) {
    for (int px = 0; px < W; px++) {
      const int64_t pix = (int64_t)py * W + px;
      float dst[4] = {0, 0, 0, 0};
      uint32_t cnt = 0;
      float fx = (float)px + 0.5f, fy = (float)py + 0.5f;
      float vx = std::fmaf(fx / (float)W, 2.0f, -1.0f);
      float vy = std::fmaf(fy / (float)H, 2.0f, -1.0f);
      v3 c = mk((vx * tanf) * aspect, vy * tanf, -1.0f);
      v3 dv = mk(dot3(c, mk(V[0], V[1], V[2])), dot3(c, mk(V[4], V[5], V[6])), dot3(c, mk(V[8], V[9], V[10])));
      v3 dir = normalize3(normalize3(dv));
      v3 inv = mk(1.0f / dir.x, 1.0f / dir.y, 1.0f / dir.z);
      v3 ta = mk(inv.x * (-half.x - eye.x), inv.y * (-half.y - eye.y), inv.z * (-half.z - eye.z));
      v3 tb = mk(inv.x * (half.x - eye.x), inv.y * (half.y - eye.y), inv.z * (half.z - eye.z));
      float tnear = std::fmax(std::fmax(std::fmin(ta.x, tb.x), std::fmin(ta.y, tb.y)), std::fmin(ta.z, tb.z));
      const float tfar = std::fmin(std::fmin(std::fmax(ta.x, tb.x), std::fmax(ta.y, tb.y)), std::fmax(ta.z, tb.z));
      const bool hit = tfar > tnear;
      tnear = std::fmax(tnear, 0.0f);
      if (hit) {
        // texture(TexVolume, (r.Origin + r.Dir * t + G/2) / G).r
        auto density = [&](float t) {
          const v3 p = iso_pos(eye, dir, t);
          float s;
          vol.sample(std::fmaf(p.x + half.x, NoG[0], -0.5f), std::fmaf(p.y + half.y, NoG[1], -0.5f),
                     std::fmaf(p.z + half.z, NoG[2], -0.5f), &s);
          return s;
        };
        auto hit_colour_at = [&](v3 st, float rgb[3]) {   // st: s_tex_pos
          for (int k = 0; k < 3; k++) rgb[k] = Q->color[k];
          if (!(P.phong && P.grad)) return;
          float g[3];
          grd.sample(std::fmaf(st.x, NoG[0], -0.5f), std::fmaf(st.y, NoG[1], -0.5f),
                     std::fmaf(st.z, NoG[2], -0.5f), g);
          if (g[0] == 0.0f && g[1] == 0.0f && g[2] == 0.0f) return;
          const v3 wp = mk(st.x - half.x, st.y - half.y, st.z - half.z);   // ShadeBlinnPhong :58
          const v3 L = normalize3(mk(light.x - wp.x, light.y - wp.y, light.z - wp.z));
          const v3 E = normalize3(mk(eye.x - wp.x, eye.y - wp.y, eye.z - wp.z));
          const v3 Hv = normalize3(mk(E.x + L.x, E.y + L.y, E.z + L.z));
          const v3 n = normalize3(mk(g[0], g[1], g[2]));
          const float dd = std::fmax(0.0f, dot3(n, L));
          const float ds = std::fmax(0.0f, dot3(Hv, n));
          const float pw = cvr_powf(ds, P.shininess);
          const float f = std::fmaf(P.kd, dd, P.ka);
          for (int k = 0; k < 3; k++) rgb[k] = std::fmaf(P.ispec[k] * P.ks, pw, rgb[k] * f);
        };
        auto hit_colour = [&](float t, float rgb[3]) {
          const v3 p = iso_pos(eye, dir, t);
          hit_colour_at(mk(p.x + half.x, p.y + half.y, p.z + half.z), rgb);
        };
        auto composite = [&](const float rgb[3]) {   // src.rgb *= src.a; dst += (1 - dst.a) * src
          const float a = Q->color[3], om = 1.0f - dst[3];
          for (int k = 0; k < 3; k++) dst[k] = std::fmaf(om, rgb[k] * a, dst[k]);
          dst[3] = std::fmaf(om, a, dst[3]);
        };
        if (Q->variant == 2) {
          // rc1pisoadapt/ray_marching_1p_iso_adapt.comp:113-172: s in [0, D) from
          // tex_pos = r.Origin + r.Dir * tnear + G/2, no blocks
          const float D = std::fabs(tfar - tnear);
          const v3 p0 = iso_pos(eye, dir, tnear);
          const v3 tp = mk(p0.x + half.x, p0.y + half.y, p0.z + half.z);
          auto dens_at = [&](float s) {
            float v;
            vol.sample(std::fmaf(std::fmaf(dir.x, s, tp.x), NoG[0], -0.5f),
                       std::fmaf(std::fmaf(dir.y, s, tp.y), NoG[1], -0.5f),
                       std::fmaf(std::fmaf(dir.z, s, tp.z), NoG[2], -0.5f), &v);
            return v;
          };
          float prev = dens_at(0.0f);
          cnt++;
          float s = 0.0f;
          uint32_t iters = 0;
          while (s < D && iters < kIsoMaxIter) {
            iters++;
            const float step = std::fabs(prev - iso) < Q->step_range ? Q->step_small : Q->step_large;
            const float h = std::fmin(step, D - s);
            const float dens = dens_at(s + h);
            cnt++;
            if ((prev <= iso && iso < dens) || (prev >= iso && iso > dens)) {
              const float tt = (iso - prev) / (dens - prev);
              // s_tex_pos = tex_pos + r.Dir * (s + t * h); hit_colour takes t along the
              // eye ray, so restate the position directly
              const float st = std::fmaf(tt, h, s);
              float rgb[3];
              hit_colour_at(mk(std::fmaf(dir.x, st, tp.x), std::fmaf(dir.y, st, tp.y),
                               std::fmaf(dir.z, st, tp.z)), rgb);
              composite(rgb);
              if (dst[3] > 0.99f) break;
            }
            prev = dens;
            s = s + h;
          }
        } else {
        float t = tnear;
        float prev = density(t);   // prevDensity (:157-158)
        cnt++;
        uint32_t iters = 0;
        while (t < tfar && iters < kIsoMaxIter) {
          iters++;
          // getBlockIndex (:93-96) and the REPEAT-wrapped NEAREST fetch of the tables
          const v3 p = iso_pos(eye, dir, t);
          const float pp[3] = {p.x, p.y, p.z}, dd[3] = {dir.x, dir.y, dir.z};
          int b[3], wr[3];
          for (int i = 0; i < 3; i++) {
            b[i] = (int)std::floor(((pp[i] + (G[i] * 0.5f)) / G[i]) * nbf[i]);
            wr[i] = ((b[i] % Q->nb[i]) + Q->nb[i]) % Q->nb[i];
          }
          const size_t bi = ((size_t)wr[2] * Q->nb[1] + wr[1]) * Q->nb[0] + wr[0];
          const float bmin_v = Q->bmin[bi], bmax_v = Q->bmax[bi];
          // getBlockBounds (:99-103)
          float lo[3], hi[3];
          for (int i = 0; i < 3; i++) {
            const float bs = G[i] / nbf[i];
            lo[i] = -G[i] * 0.5f + bs * (float)b[i];
            hi[i] = lo[i] + bs;
          }
          if (Q->variant == 0) {
            bool tilted = false;
            if (iso < bmin_v || iso > bmax_v) {
              float dt;
              if (std::fabs(dd[0]) < 0.01f || std::fabs(dd[1]) < 0.01f || std::fabs(dd[2]) < 0.01f) {
                dt = -1.0f;
              } else {
                float tmn[3], tmx[3];
                for (int i = 0; i < 3; i++) {
                  const float t1 = (lo[i] - pp[i]) / dd[i], t2 = (hi[i] - pp[i]) / dd[i];
                  tmn[i] = std::fmin(t1, t2);
                  tmx[i] = std::fmax(t1, t2);
                }
                dt = std::fmin(std::fmin(tmx[0], tmx[1]), tmx[2]) -
                     std::fmax(std::fmax(tmn[0], tmn[1]), tmn[2]);
              }
              if (dt == -1.0f) tilted = true;
              if (dt <= Q->step_small) dt = Q->step_small;
              t += dt;
              if (!tilted) continue;
            }
            const float step = std::fabs(prev - iso) < Q->step_range ? Q->step_small : Q->step_large;
            prev = density(t);
            cnt++;
            const float h = std::fmin(step, tfar - t);
            t += h;
            const float dens = density(t);
            cnt++;
            if ((prev <= iso && iso < dens) || (prev >= iso && iso > dens)) {
              const float tt = (dens - iso) / (dens - prev);
              t -= tt;
              float rgb[3];
              hit_colour(t, rgb);
              composite(rgb);
              if (dst[3] > 0.99f) break;
            }
          } else {
            if (iso < bmin_v - 0.001f || iso > bmax_v + 0.001f) {   // isBlockSkippable
              float tmx[3];
              for (int i = 0; i < 3; i++) {
                const float rc = std::fabs(dd[i]) > 1e-6f ? 1.0f / dd[i]
                                 : (dd[i] > 0.0f ? 1e6f : (dd[i] < 0.0f ? -1e6f : 0.0f));
                tmx[i] = std::fmax((lo[i] - pp[i]) * rc, (hi[i] - pp[i]) * rc);
              }
              float exitT = std::fmin(std::fmin(tmx[0], tmx[1]), tmx[2]);
              for (int i = 0; i < 3; i++)
                if (std::fabs(exitT - tmx[i]) < 1e-5f) exitT += 1e-4f;
              t += std::fmax(Q->step_small, exitT);
              prev = density(t);   // overwritten before use
              cnt++;
              continue;
            }
            const float cur = density(t);
            cnt++;
            const float step = std::fabs(cur - iso) < Q->step_range ? Q->step_small
                                                                    : std::fmin(Q->step_large, half_block);
            const float h = std::fmin(step, tfar - t);
            prev = cur;
            t += h;
            const float dens = density(t);
            cnt++;
            if ((prev <= iso && iso < dens) || (prev >= iso && iso > dens)) {
              const float tt = (iso - prev) / (dens - prev);
              t = t - h * (1.0f - tt);
              float rgb[3];
              hit_colour(t, rgb);
              composite(rgb);
              if (dst[3] > 0.99f) break;
            }
          }
        }
        }   // variants 0, 1
      }
      if (out) for (int k = 0; k < 4; k++) out[pix * 4 + k] = dst[k];
      if (counts) counts[pix] = cnt;
      total += cnt;
    }
  }
  return total;
}

ORACLE_API uint64_t oracle_render_iso(const OracleIso* Q, float* out_rgba, uint32_t* out_counts,
                                      int nthreads) {
  return oracle_render_iso_rows(Q, 0, Q->base.H, out_rgba, out_counts, nthreads);
}

// ---------------------------------------------------------------------------
// Check of the library's division by a precomputed reciprocal (cvr_device.h
// div_by_recip: q = RN(a*y), r = fma(-b, q, a), RN(q + r*y) with y = RN(1/b))
// against IEEE division, on n log-uniform random pairs (a in [2^-lo, 2^hi],
// b in [2^-8, 2^8], both signs).  Returns the number of mismatching quotients.
// ---------------------------------------------------------------------------
ORACLE_API uint64_t oracle_check_div_by_recip(uint64_t n, uint64_t seed, int lo, int hi) {
  uint64_t bad = 0;
#pragma omp parallel for reduction(+ : bad) schedule(static)
  for (int64_t t = 0; t < (int64_t)n; t++) {
    uint64_t x = (seed + (uint64_t)t) * 0x9E3779B97F4A7C15ull;
    auto next = [&]() {
      x ^= x >> 30; x *= 0xBF58476D1CE4E5B9ull; x ^= x >> 27; x *= 0x94D049BB133111EBull;
      x ^= x >> 31;
      return x;
    };
    const uint64_t r1 = next(), r2 = next();
    // exponent uniform, mantissa uniform
    const int ea = lo + (int)((r1 >> 40) % (uint64_t)(hi - lo + 1));
    const int eb = -8 + (int)((r2 >> 40) % 17u);
    float a = std::ldexp(1.0f + (float)(r1 & 0x7fffff) / 8388608.0f, -ea);
    float b = std::ldexp(1.0f + (float)(r2 & 0x7fffff) / 8388608.0f, eb);
    if (r1 & (1ull << 63)) a = -a;
    if (r2 & (1ull << 63)) b = -b;
    const float y = 1.0f / b;
    const float q = a * y;
    const float r = std::fmaf(-b, q, a);
    const float d = std::fmaf(r, y, q);
    const float e = a / b;
    if (f2u(d) != f2u(e)) bad++;
  }
  return bad;
}
