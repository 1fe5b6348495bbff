// cvr_device.h — device helpers of the gfx950 ray-marching kernels
// (CVR-SPEC arithmetic; see DESIGN.md and oracle/cvr_oracle.cpp).
#pragma once

#include <hip/hip_runtime.h>
#include <cstdint>

#include "cvr_internal.h"

namespace cvr {


typedef _Float16 half2_t __attribute__((ext_vector_type(2)));

__device__ __forceinline__ float lerpf(float a, float b, float t) { return fmaf(t, b - a, a); }

// float -> binary16 bits, round to nearest even, as an opaque instruction: a
// plain (_Float16) cast lets the backend fold a preceding multiply or fma into
// v_fma_mixlo_f16 (one rounding straight to f16 instead of f32 then f16, which
// differs in the last f16 bit now and then, -ffp-contract=off notwithstanding).
__device__ __forceinline__ uint32_t f32_to_h16(float f) {
  uint32_t r;
  asm volatile("v_cvt_f16_f32 %0, %1" : "=v"(r) : "v"(f));
  return r & 0xffffu;
}

__device__ __forceinline__ void h2f2(uint32_t w, float& lo, float& hi) {
  half2_t p = __builtin_bit_cast(half2_t, w);
  lo = (float)p.x;
  hi = (float)p.y;
}

// exp(x), CVR-SPEC (identical to oracle cvr_expf)
__device__ __forceinline__ float cvr_expf(float x) {
  if (x != x) return x;
  if (x < -86.0f) return 0.0f;
  if (x > 88.5f) return __builtin_inff();
  float n = rintf(x * 1.44269504088896341f);
  float r = fmaf(n, -0.693359375f, x);
  r = fmaf(n, 2.12194440e-4f, r);
  float p = 1.9875691500e-4f;
  p = fmaf(p, r, 1.3981999507e-3f);
  p = fmaf(p, r, 8.3334519073e-3f);
  p = fmaf(p, r, 4.1665795894e-2f);
  p = fmaf(p, r, 1.6666665459e-1f);
  p = fmaf(p, r, 5.0000001201e-1f);
  float r2 = r * r;
  float y = fmaf(p, r2, r) + 1.0f;
  return ldexpf(y, (int)n);
}

// cvr_expf for x <= 0 (not NaN), without branches: the polynomial path on the
// argument clamped into range, then 0 below -86 -- the same value as cvr_expf.
__device__ __forceinline__ float cvr_expf_nonpos(float x) {
  const float xc = fmaxf(x, -86.0f);
  float n = rintf(xc * 1.44269504088896341f);
  float r = fmaf(n, -0.693359375f, xc);
  r = fmaf(n, 2.12194440e-4f, r);
  float p = 1.9875691500e-4f;
  p = fmaf(p, r, 1.3981999507e-3f);
  p = fmaf(p, r, 8.3334519073e-3f);
  p = fmaf(p, r, 4.1665795894e-2f);
  p = fmaf(p, r, 1.6666665459e-1f);
  p = fmaf(p, r, 5.0000001201e-1f);
  float r2 = r * r;
  float y = fmaf(p, r2, r) + 1.0f;
  return x < -86.0f ? 0.0f : ldexpf(y, (int)n);
}

// ln(x), CVR-SPEC (identical to oracle cvr_logf): Cephes logf polynomial.
__device__ __forceinline__ float cvr_logf(float x) {
  if (x != x) return x;
  if (x < 0.0f) return __builtin_nanf("");
  if (x < 1.17549435e-38f) return -__builtin_inff();
  if (x == __builtin_inff()) return x;
  uint32_t bits = __float_as_uint(x);
  int e = (int)((bits >> 23) & 0xffu) - 126;
  float m = __uint_as_float((bits & 0x007fffffu) | 0x3f000000u);
  if (m < 0.70710678118654752f) { m = m + m; e = e - 1; }
  float f = m - 1.0f;
  float z = f * f;
  float p = 7.0376836292e-2f;
  p = fmaf(p, f, -1.1514610310e-1f);
  p = fmaf(p, f, 1.1676998740e-1f);
  p = fmaf(p, f, -1.2420140846e-1f);
  p = fmaf(p, f, 1.4249322787e-1f);
  p = fmaf(p, f, -1.6668057665e-1f);
  p = fmaf(p, f, 2.0000714765e-1f);
  p = fmaf(p, f, -2.4999993993e-1f);
  p = fmaf(p, f, 3.3333331174e-1f);
  float r = (p * f) * z;
  float fe = (float)e;
  r = fmaf(fe, -2.12194440e-4f, r);
  r = fmaf(-0.5f, z, r);
  float lnx = f + r;
  return fmaf(fe, 0.693359375f, lnx);
}

// pow(x, y) for x >= 0, CVR-SPEC (identical to oracle cvr_powf)
__device__ __forceinline__ float cvr_powf(float x, float y) {
  if (x != x || y != y) return x + y;
  if (!(x > 0.0f) || x < 1.17549435e-38f) {
    if (y > 0.0f) return 0.0f;
    if (y == 0.0f) return 1.0f;
    return __builtin_inff();
  }
  if (x == __builtin_inff()) return y > 0.0f ? __builtin_inff() : (y == 0.0f ? 1.0f : 0.0f);
  return cvr_expf(y * cvr_logf(x));
}

// Branch-free CVR-SPEC exp: same values as cvr_expf (selects instead of the
// early returns, so a wave never splits on the special cases).
__device__ __forceinline__ float cvr_expf_nb(float x) {
  float xc = fminf(fmaxf(x, -86.0f), 88.5f);
  float n = rintf(xc * 1.44269504088896341f);
  float r = fmaf(n, -0.693359375f, xc);
  r = fmaf(n, 2.12194440e-4f, r);
  float p = 1.9875691500e-4f;
  p = fmaf(p, r, 1.3981999507e-3f);
  p = fmaf(p, r, 8.3334519073e-3f);
  p = fmaf(p, r, 4.1665795894e-2f);
  p = fmaf(p, r, 1.6666665459e-1f);
  p = fmaf(p, r, 5.0000001201e-1f);
  float r2 = r * r;
  float y = ldexpf(fmaf(p, r2, r) + 1.0f, (int)n);
  y = x < -86.0f ? 0.0f : y;
  y = x > 88.5f ? __builtin_inff() : y;
  return x != x ? x : y;
}

// cvr_logf's main path for a positive, normal, finite x (no special cases;
// the mantissa fold is a select): the same value as cvr_logf there.
__device__ __forceinline__ float cvr_logf_pos(float x) {
  const uint32_t bits = __float_as_uint(x);
  int e = (int)((bits >> 23) & 0xffu) - 126;
  float m = __uint_as_float((bits & 0x007fffffu) | 0x3f000000u);
  const bool fold = m < 0.70710678118654752f;
  m = fold ? m + m : m;
  e = fold ? e - 1 : e;
  float f = m - 1.0f;
  float z = f * f;
  float p = 7.0376836292e-2f;
  p = fmaf(p, f, -1.1514610310e-1f);
  p = fmaf(p, f, 1.1676998740e-1f);
  p = fmaf(p, f, -1.2420140846e-1f);
  p = fmaf(p, f, 1.4249322787e-1f);
  p = fmaf(p, f, -1.6668057665e-1f);
  p = fmaf(p, f, 2.0000714765e-1f);
  p = fmaf(p, f, -2.4999993993e-1f);
  p = fmaf(p, f, 3.3333331174e-1f);
  float r = (p * f) * z;
  float fe = (float)e;
  r = fmaf(fe, -2.12194440e-4f, r);
  r = fmaf(-0.5f, z, r);
  float lnx = f + r;
  return fmaf(fe, 0.693359375f, lnx);
}

// cvr_powf without branches: the main path on a sanitised argument, then the
// special cases selected in cvr_powf's order of precedence -- the same value as
// cvr_powf for every (x, y) (checked on the device by cvr_selftest_arith).
__device__ __forceinline__ float cvr_powf_nb(float x, float y) {
  const float inf = __builtin_inff();
  const bool tiny = !(x > 0.0f) || x < 1.17549435e-38f;     // also NaN (selected below)
  const float xs = (tiny || x == inf) ? 1.0f : x;
  float r = cvr_expf_nb(y * cvr_logf_pos(xs));
  const float r_inf = y > 0.0f ? inf : (y == 0.0f ? 1.0f : 0.0f);
  const float r_tiny = y > 0.0f ? 0.0f : (y == 0.0f ? 1.0f : inf);
  r = x == inf ? r_inf : r;
  r = tiny ? r_tiny : r;
  return (x != x || y != y) ? x + y : r;
}

struct f3 { float x, y, z; };
// a / b correctly rounded from y = 1.0f / b (itself correctly rounded), for a
// divisor reused many times: q = RN(a*y), the remainder a - b*q is exact by fma,
// and RN(q + r*y) = RN(a/b) (Markstein's correction; valid while a/b, a*y and the
// remainder stay in the normal range -- callers pass finite a of moderate size,
// either sign (RN is symmetric, so a / b and -a / b round alike), and b, 1/b in
// the normal range; a divisor that may approach 0 needs the IEEE division, see
// ebs.hip cone_div).  Checked against IEEE division in
// tests/test_exact_div.py.
__device__ __forceinline__ float div_by_recip(float a, float b, float y) {
  const float q = a * y;
  const float r = fmaf(-b, q, a);
  return fmaf(r, y, q);
}

// RN(1/b) from the hardware reciprocal (v_rcp_f32, within 1 ulp) and one
// Newton step with fma (e = 1 - b*y exact, y + e*y rounded once): 3
// instructions instead of the 11 of the IEEE division sequence.  For b and 1/b
// in the normal range; equal to 1.0f / b for EVERY such float, checked
// exhaustively on the device by cvr_selftest_arith (tests/test_selftest_gpu.py).
__device__ __forceinline__ float rcp_cr(float b) {
  const float y = __builtin_amdgcn_rcpf(b);
  const float e = fmaf(-b, y, 1.0f);
  return fmaf(e, y, y);
}

// RN(sqrt(x)) for x in [2^-96, 2^126]: the correctly rounded sqrt sequence the
// compiler emits for sqrtf (v_sqrt_f32, then the neighbours s -/+ 1 ulp tested
// by exact fma remainders) without its input scaling for tiny x and its
// zero/inf class fix-up, which are identities in this range.
__device__ __forceinline__ float sqrt_cr_normal(float x) {
  const float s = __builtin_amdgcn_sqrtf(x);
  const float sm = __uint_as_float(__float_as_uint(s) - 1u);
  const float sp = __uint_as_float(__float_as_uint(s) + 1u);
  const float rm = fmaf(-sm, s, x);
  const float rp = fmaf(-sp, s, x);
  const float r = rm <= 0.0f ? sm : s;
  return rp > 0.0f ? sp : r;
}

__device__ __forceinline__ float dot3(f3 a, f3 b) { return fmaf(a.z, b.z, fmaf(a.y, b.y, a.x * b.x)); }
// normalize(v) = v * RN(1 / RN(sqrt(dot(v, v)))) (CVR-SPEC): the short exact
// sequence when dot(v, v) lies in [2^-96, 2^126), else the IEEE operators.
__device__ __forceinline__ f3 normalize3(f3 v) {
  const float d = dot3(v, v);
  float inv;
  if (d >= 0x1p-96f && d < 0x1p126f) inv = rcp_cr(sqrt_cr_normal(d));
  else inv = 1.0f / sqrtf(d);
  return f3{v.x * inv, v.y * inv, v.z * inv};
}



// Tolerance mode only (option native_exp, NOT CVR-SPEC): the hardware exp2 of
// x * log2(e), two instructions (v_mul, v_exp_f32) against the polynomial's ~14.
// Its error against cvr_expf is ~|x| * 2^-24 relative; parity is then the
// tolerance gate of SURVEY §8(c), not bit equality (tests/test_tolerance_gpu.py).
__device__ __forceinline__ float cvr_expf_native(float x) {
  return __builtin_amdgcn_exp2f(x * 1.44269504088896341f);
}

// cvr_expf for x in [-86, 0]: the same value without the range selects (the
// host enables it only when every sample's -(alpha*h) is known to lie there).
__device__ __forceinline__ float cvr_expf_neg(float x) {
  float n = rintf(x * 1.44269504088896341f);
  float r = fmaf(n, -0.693359375f, x);
  r = fmaf(n, 2.12194440e-4f, r);
  float p = 1.9875691500e-4f;
  p = fmaf(p, r, 1.3981999507e-3f);
  p = fmaf(p, r, 8.3334519073e-3f);
  p = fmaf(p, r, 4.1665795894e-2f);
  p = fmaf(p, r, 1.6666665459e-1f);
  p = fmaf(p, r, 5.0000001201e-1f);
  float r2 = r * r;
  return ldexpf(fmaf(p, r2, r) + 1.0f, (int)n);
}


}  // namespace cvr
