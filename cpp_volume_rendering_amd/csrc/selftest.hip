// selftest.hip — exhaustive device checks of the arithmetic shortcuts the
// kernels rely on (cvr_device.h): every float b in the checked exponent range
// gives rcp_cr(b) == 1.0f / b, every x gives sqrt_cr_normal(x) == sqrtf(x), and
// the branch-free cvr_powf_nb equals cvr_powf, bit for bit.  One lane per significand, one block row per exponent.
#include <hip/hip_runtime.h>
#include <cstdint>

#include "cvr_device.h"
#include "march_common.h"

namespace cvr {

__global__ void __launch_bounds__(256)
selftest_arith_kernel(int e_rcp_lo, int e_rcp_n, int e_sqrt_lo, int e_sqrt_n,
                      unsigned long long* __restrict__ bad) {
  const uint32_t m = blockIdx.x * 256u + threadIdx.x;     // significand
  const int e = (int)blockIdx.y;
  uint32_t nbad_r = 0, nbad_s = 0;
  // reciprocal: b = +-1.m x 2^(e_rcp_lo + e)
  if (e < e_rcp_n) {
    const uint32_t ex = (uint32_t)(e_rcp_lo + e + 127);
    const float b = __uint_as_float((ex << 23) | m);
    if (__float_as_uint(rcp_cr(b)) != __float_as_uint(1.0f / b)) nbad_r++;
    if (__float_as_uint(rcp_cr(-b)) != __float_as_uint(1.0f / -b)) nbad_r++;
  }
  // square root: x = 1.m x 2^(e_sqrt_lo + e)
  if (e < e_sqrt_n) {
    const uint32_t ex = (uint32_t)(e_sqrt_lo + e + 127);
    const float x = __uint_as_float((ex << 23) | m);
    if (__float_as_uint(sqrt_cr_normal(x)) != __float_as_uint(sqrtf(x))) nbad_s++;
  }
  const unsigned long long r = wave_sum(nbad_r), s = wave_sum(nbad_s);
  if ((threadIdx.x & 63) == 0) {
    if (r) atomicAdd(&bad[0], r);
    if (s) atomicAdd(&bad[1], s);
  }
}

// cvr_powf_nb == cvr_powf: x = 1.m x 2^(e - 126) for e in [0, 128) (every
// positive normal x < 4) at several exponents y, and the special arguments.
__global__ void __launch_bounds__(256)
selftest_pow_kernel(unsigned long long* __restrict__ bad) {
  const uint32_t m = blockIdx.x * 256u + threadIdx.x;
  const int e = (int)blockIdx.y;
  const float x = __uint_as_float(((uint32_t)(e + 1) << 23) | m);
  const float ys[5] = {30.0f, 1.0f, 0.5f, 128.0f, 7.25f};
  uint32_t nbad = 0;
#pragma unroll
  for (int k = 0; k < 5; k++)
    if (__float_as_uint(cvr_powf_nb(x, ys[k])) != __float_as_uint(cvr_powf(x, ys[k]))) nbad++;
  if (blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x < 64) {   // special arguments
    const float inf = __builtin_inff(), nan = __builtin_nanf("");
    const float xs[8] = {0.0f, -0.0f, -1.0f, 1e-40f, inf, nan, 1.0f, -inf};
    const float yv[8] = {0.0f, -1.0f, 2.0f, inf, -inf, nan, 30.0f, -0.0f};
    const float xa = xs[threadIdx.x & 7], ya = yv[threadIdx.x >> 3];
    if (__float_as_uint(cvr_powf_nb(xa, ya)) != __float_as_uint(cvr_powf(xa, ya))) nbad++;
  }
  const unsigned long long v = wave_sum(nbad);
  if ((threadIdx.x & 63) == 0 && v) atomicAdd(bad, v);
}

hipError_t launch_selftest_arith(int e_rcp_lo, int e_rcp_n, int e_sqrt_lo, int e_sqrt_n,
                                 unsigned long long* bad, hipStream_t s) {
  const int n = e_rcp_n > e_sqrt_n ? e_rcp_n : e_sqrt_n;
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(selftest_arith_kernel, dim3((1u << 23) / 256, n), dim3(256), 0, s, e_rcp_lo,
                     e_rcp_n, e_sqrt_lo, e_sqrt_n, bad);
  hipLaunchKernelGGL(selftest_pow_kernel, dim3((1u << 23) / 256, 128), dim3(256), 0, s, bad + 2);
  return hipGetLastError();
}

}  // namespace cvr
