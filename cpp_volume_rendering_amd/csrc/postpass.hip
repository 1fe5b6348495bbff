// postpass.hip — the step after the ray-march: the pixel
// multiscaling filters of RenderFrameToScreen and the screenshot composite.
//
//   MULTIPLE_RAYS_PER_PIXEL  render at (2w, 2h), bilinear texture() fetch at the
//                            screen pixel centres (multisample_filter.comp)
//   DOWN_SCALING_RENDER      render at (2w, 2h), kernel-filtered decimation
//                            (downscaling_filter.comp + <kernel>_filter.comp), then
//                            for the cardinal kernels the recursive digital filter
//                            over the result (cbs/comoms_digital_filter.comp)
//   UP_SCALING_RENDER        render at (w/2, h/2), digital prefilter IN PLACE on the
//                            rendered frame for the cardinal kernels, then kernel-
//                            filtered interpolation (upscaling_filter.comp)
//   screenshot               the RGBA16F frame drawn with SRC_ALPHA /
//                            ONE_MINUS_SRC_ALPHA over the white clear colour, read
//                            back as RGB8 (renderingmanager.cpp:103-112, 476-492)
//
// Every image is RGBA16F, as the reference's textures: each imageStore rounds to
// binary16 (nearest even), and the digital filter's recursion re-reads its own
// rounded stores.  The GLSL float expressions are evaluated in the shaders' order
// without contraction (-ffp-contract=off); texelFetch outside the image reads 0
// (robust access), texture() clamps to the edge (GL_CLAMP_TO_EDGE).  These are
// small HBM-bound passes (8 B per pixel in, 8 B out, x the kernel's footprint
// served from L2).
#include <hip/hip_runtime.h>
#include <atomic>

#include <algorithm>
#include <type_traits>
#include <cstdint>

#include "cvr_device.h"
#include "cvr_internal.h"

namespace cvr {
namespace {

__device__ __forceinline__ float h2f(uint16_t h) { return (float)__builtin_bit_cast(_Float16, h); }
__device__ __forceinline__ uint16_t f2h(float f) { return (uint16_t)f32_to_h16(f); }

__device__ __forceinline__ float4 load_px(const uint2* img, int w, int x, int y) {
  const uint2 p = img[(size_t)y * w + x];
  return make_float4(h2f((uint16_t)(p.x & 0xffffu)), h2f((uint16_t)(p.x >> 16)),
                     h2f((uint16_t)(p.y & 0xffffu)), h2f((uint16_t)(p.y >> 16)));
}
__device__ __forceinline__ void store_px(uint2* img, int w, int x, int y, float4 v) {
  img[(size_t)y * w + x] = make_uint2((uint32_t)f2h(v.x) | ((uint32_t)f2h(v.y) << 16),
                                      (uint32_t)f2h(v.z) | ((uint32_t)f2h(v.w) << 16));
}
// texelFetch with robust access: 0 outside the image
__device__ __forceinline__ float4 fetch_px(const uint2* img, int w, int h, int x, int y) {
  if (x < 0 || y < 0 || x >= w || y >= h) return make_float4(0.f, 0.f, 0.f, 0.f);
  return load_px(img, w, x, y);
}

// ---- kernels of renderoutputframe/<name>_filter.comp ------------------------
struct KBox {      // box_filter.comp
  static constexpr float support = 1.0f;
  __device__ static float w(float x) { return x <= -0.5f || x > 0.5f ? 0.0f : 1.0f; }
};
struct KHat {      // hat_filter.comp
  static constexpr float support = 2.0f;
  __device__ static float w(float x) {
    x = fabsf(x);
    return x > 1.0f ? 0.0f : 1.0f - x;
  }
};
struct KCatmullRom {   // catmullrom_filter.comp
  static constexpr float support = 4.0f;
  __device__ static float k0(float u) { return ((0.5f * u - 0.5f) * u) * u; }
  __device__ static float k1(float u) { return ((-1.5f * u + 2.0f) * u + 0.5f) * u; }
  __device__ static float w(float x) {
    x = fabsf(x);
    return x > 2.0f ? 0.0f : x > 1.0f ? k0(2.0f - x) : k1(1.0f - x);
  }
};
struct KMitchell {     // mitchellnetravali_filter.comp
  static constexpr float support = 4.0f;
  __device__ static float k0(float u) { return (((7 / 18.0f) * u - 1 / 3.0f) * u) * u; }
  __device__ static float k1(float u) {
    return (((-7 / 6.0f) * u + 1.5f) * u + 0.5f) * u + 1 / 18.0f;
  }
  __device__ static float w(float x) {
    x = fabsf(x);
    return x > 2.0f ? 0.0f : x > 1.0f ? k0(2.0f - x) : k1(1.0f - x);
  }
};
struct KCardinalBSpline3 {   // cardinalbspline_filter.comp
  static constexpr float support = 4.0f;
  __device__ static float k0(float u) { return ((u)*u) * u; }
  __device__ static float k1(float u) { return ((-3.0f * u + 3.0f) * u + 3.0f) * u + 1.0f; }
  __device__ static float w(float x) {
    x = fabsf(x);
    return x > 2.0f ? 0.0f : x > 1.0f ? k0(2.0f - x) : k1(1.0f - x);
  }
};
struct KCardinalOmoms3 {     // cardinalomoms_filter.comp
  static constexpr float support = 4.0f;
  __device__ static float k0(float u) { return ((0.875f * u) * u + 0.125f) * u; }
  __device__ static float k1(float u) {
    return ((-2.625f * u + 2.625f) * u + 2.25f) * u + 1.0f;
  }
  __device__ static float w(float x) {
    x = fabsf(x);
    return x > 2.0f ? 0.0f : x > 1.0f ? k0(2.0f - x) : k1(1.0f - x);
  }
};

__device__ __forceinline__ float4 madd(float4 acc, float wgt, float4 t) {
  return make_float4(acc.x + wgt * t.x, acc.y + wgt * t.y, acc.z + wgt * t.z, acc.w + wgt * t.w);
}

// XCD-aware 2D block: the dispatcher deals workgroups to the 8 XCDs round-robin
// in linear order; remapped so that each XCD takes a contiguous run of blocks
// (row-major), whose overlapping input windows then share its L2.
__device__ __forceinline__ void xcd_block(int& bx, int& by) {
  const int nb = (int)(gridDim.x * gridDim.y), b = (int)(blockIdx.y * gridDim.x + blockIdx.x);
  const int l = (nb & 7) == 0 ? (b & 7) * (nb >> 3) + (b >> 3) : b;
  by = l / (int)gridDim.x;
  bx = l - by * (int)gridDim.x;
}

// multisample_filter.comp: texture(TexGeneratedFrame, (p + 0.5) / size), bilinear,
// clamp to edge, texel centres at (i + 0.5) / n
__global__ void multisample_kernel(const uint2* __restrict__ src, int sw, int sh,
                                   uint2* __restrict__ dst, int tw, int th) {
  const int x = blockIdx.x * 16 + (threadIdx.x & 15), y = blockIdx.y * 16 + (threadIdx.x >> 4);
  if (x >= tw || y >= th) return;
  const float u = ((float)x + 0.5f) / (float)tw, v = ((float)y + 0.5f) / (float)th;
  const float fx = u * (float)sw - 0.5f, fy = v * (float)sh - 0.5f;
  const float flx = floorf(fx), fly = floorf(fy);
  const float ax = fx - flx, ay = fy - fly;
  const int x0 = min(max((int)flx, 0), sw - 1), x1 = min(max((int)flx + 1, 0), sw - 1);
  const int y0 = min(max((int)fly, 0), sh - 1), y1 = min(max((int)fly + 1, 0), sh - 1);
  const float4 a = load_px(src, sw, x0, y0), b = load_px(src, sw, x1, y0);
  const float4 c = load_px(src, sw, x0, y1), d = load_px(src, sw, x1, y1);
  auto lerp4 = [](float4 p, float4 q, float t) {
    return make_float4(fmaf(t, q.x - p.x, p.x), fmaf(t, q.y - p.y, p.y), fmaf(t, q.z - p.z, p.z),
                       fmaf(t, q.w - p.w, p.w));
  };
  store_px(dst, tw, x, y, lerp4(lerp4(a, b, ax), lerp4(c, d, ax), ay));
}

// downscaling_filter.comp
template <class K>
__global__ void downscale_kernel(const uint2* __restrict__ src, int sw, int sh,
                                 uint2* __restrict__ dst, int tw, int th) {
  const int jc = blockIdx.x * 16 + (threadIdx.x & 15), jr = blockIdx.y * 16 + (threadIdx.x >> 4);
  if (jc >= tw || jr >= th) return;
  const float s_r = (float)th / (float)sh;
  const float s_c = (float)tw / (float)sw;
  const float kr = 0.5f * K::support;
  const float x_r = ((float)jr + 0.5f) / (float)th;
  const int il_r = (int)ceilf((x_r - kr / (float)th) * (float)sh - 0.5f);
  const int ir_r = (int)floorf((x_r + kr / (float)th) * (float)sh - 0.5f);
  const float x_c = ((float)jc + 0.5f) / (float)tw;
  const int il_c = (int)ceilf((x_c - kr / (float)tw) * (float)sw - 0.5f);
  const int ir_c = (int)floorf((x_c + kr / (float)tw) * (float)sw - 0.5f);
  float4 f = make_float4(0.f, 0.f, 0.f, 0.f);
  for (int ir = il_r; ir <= ir_r; ir++) {
    const float wr = K::w((x_r - ((float)ir + 0.5f) / (float)sh) * (float)th);
    for (int ic = il_c; ic <= ir_c; ic++) {
      const float wc = K::w((x_c - ((float)ic + 0.5f) / (float)sw) * (float)tw);
      f = madd(f, wr * wc, fetch_px(src, sw, sh, ic, ir));
    }
  }
  const float s = s_r * s_c;
  store_px(dst, tw, jc, jr, make_float4(f.x * s, f.y * s, f.z * s, f.w * s));
}

// downscaling_filter.comp with the block's input window staged in LDS.  A 16x16
// block of screen pixels reads one window of the frame (its first pixel's left /
// top tap to its last pixel's right / bottom tap: the tap range is monotone in
// the pixel index), 0 outside the frame as texelFetch's robust access.  Each
// pixel's column weights are computed once (the same expression as above) and
// reused for every row; the taps are summed in the same order with the same
// operations, so the result is bit-identical to downscale_kernel.
// wgt * (half HI ? w.hi : w.lo), one rounding (= the f32 multiply of the converted half)
template <bool HI>
__device__ __forceinline__ float mul_half(float wgt, uint32_t w) {
  float d;
  if (HI) asm("v_fma_mix_f32 %0, %1, %2, neg(0) op_sel:[0,1,0] op_sel_hi:[0,1,0]" : "=v"(d) : "v"(wgt), "v"(w));
  else asm("v_fma_mix_f32 %0, %1, %2, neg(0) op_sel_hi:[0,1,0]" : "=v"(d) : "v"(wgt), "v"(w));
  return d;
}
typedef float float2v __attribute__((ext_vector_type(2)));
constexpr int kDownMaxTaps = 12;   // taps per axis held in registers
constexpr int kUpMaxTaps = 8;

template <class K>
__global__ void __launch_bounds__(256)
downscale_lds_kernel(const uint2* __restrict__ src, int sw, int sh, uint2* __restrict__ dst, int tw,
                     int th) {
  extern __shared__ uint2 win[];
  const float kr = 0.5f * K::support;
  int bx, by;
  xcd_block(bx, by);
  bx *= 16;
  by *= 16;
  auto first_tap = [kr](int j, int t, int s) {
    const float x = ((float)j + 0.5f) / (float)t;
    return (int)ceilf((x - kr / (float)t) * (float)s - 0.5f);
  };
  auto last_tap = [kr](int j, int t, int s) {
    const float x = ((float)j + 0.5f) / (float)t;
    return (int)floorf((x + kr / (float)t) * (float)s - 0.5f);
  };
  const int r0 = first_tap(by, th, sh), r1 = last_tap(min(by + 15, th - 1), th, sh);
  const int c0 = first_tap(bx, tw, sw), c1 = last_tap(min(bx + 15, tw - 1), tw, sw);
  const int ww = c1 - c0 + 1, wp = ww | 1;   // odd pitch: rows fall on shifted banks
  const int wh = r1 - r0 + 1;
  for (int e = threadIdx.x; e < ww * wh; e += 256) {
    const int rr = e / ww, cc = e - rr * ww;
    const int r = r0 + rr, c = c0 + cc;
    win[rr * wp + cc] = (r >= 0 && r < sh && c >= 0 && c < sw) ? src[(size_t)r * sw + c] : make_uint2(0u, 0u);
  }
  // The block's 16 column and 16 row weight sets, once per block (every pixel of
  // a block column shares its column weights): the same expressions per tap.
  __shared__ float wcol[16][kDownMaxTaps], wrow[16][kDownMaxTaps];
  for (int e = threadIdx.x; e < 2 * 16 * kDownMaxTaps; e += 256) {
    const bool col = e < 16 * kDownMaxTaps;
    const int i = (col ? e : e - 16 * kDownMaxTaps) / kDownMaxTaps, q = e % kDownMaxTaps;
    const int j = (col ? bx : by) + i, t = col ? tw : th, sz = col ? sw : sh;
    const float x = ((float)j + 0.5f) / (float)t;
    const int il = (int)ceilf((x - kr / (float)t) * (float)sz - 0.5f);
    const int ir = (int)floorf((x + kr / (float)t) * (float)sz - 0.5f);
    const float wv = q <= ir - il ? K::w((x - ((float)(il + q) + 0.5f) / (float)sz) * (float)t) : 0.0f;
    if (col) wcol[i][q] = wv;
    else wrow[i][q] = wv;
  }
  __syncthreads();
  const int jc = bx + (threadIdx.x & 15), jr = by + (threadIdx.x >> 4);
  if (jc >= tw || jr >= th) return;
  const float s_r = (float)th / (float)sh;
  const float s_c = (float)tw / (float)sw;
  const float x_r = ((float)jr + 0.5f) / (float)th;
  const int il_r = (int)ceilf((x_r - kr / (float)th) * (float)sh - 0.5f);
  const int ir_r = (int)floorf((x_r + kr / (float)th) * (float)sh - 0.5f);
  const float x_c = ((float)jc + 0.5f) / (float)tw;
  const int il_c = (int)ceilf((x_c - kr / (float)tw) * (float)sw - 0.5f);
  const int ir_c = (int)floorf((x_c + kr / (float)tw) * (float)sw - 0.5f);
  const int nc = ir_c - il_c + 1;
  float wc[kDownMaxTaps];
#pragma unroll
  for (int q = 0; q < kDownMaxTaps; q++) wc[q] = wcol[threadIdx.x & 15][q];
  const float* wrj = wrow[threadIdx.x >> 4];
  // rows of taps; a tap count of 8 or 9 (every pixel at ratio 2) runs unrolled
  // without per-tap conditions; the channel sums go pairwise through v_pk_add_f32
  float2v f01 = {0.0f, 0.0f}, f23 = {0.0f, 0.0f};
  auto rows = [&](auto nct) {
    constexpr int NC = decltype(nct)::value;
    for (int ir = il_r; ir <= ir_r; ir++) {
      const float wr = wrj[ir - il_r];
      const uint2* row = win + (ir - r0) * wp + (il_c - c0);
#pragma unroll
      for (int q = 0; q < (NC > 0 ? NC : kDownMaxTaps); q++) {
        if (NC > 0 || q < nc) {
          // f += wgt * t per channel: the product of the exactly converted half in
          // one v_fma_mix (-0 addend: the rounded product, sign of zero kept), then
          // the add
          const uint2 p = row[q];
          const float wgt = wr * wc[q];
          const float2v a = {mul_half<false>(wgt, p.x), mul_half<true>(wgt, p.x)};
          const float2v b = {mul_half<false>(wgt, p.y), mul_half<true>(wgt, p.y)};
          f01 += a;
          f23 += b;
        }
      }
    }
  };
  if (nc == 8) rows(std::integral_constant<int, 8>{});
  else if (nc == 9) rows(std::integral_constant<int, 9>{});
  else rows(std::integral_constant<int, 0>{});
  const float4 f = make_float4(f01.x, f01.y, f23.x, f23.y);
  const float s = s_r * s_c;
  store_px(dst, tw, jc, jr, make_float4(f.x * s, f.y * s, f.z * s, f.w * s));
}

// upscaling_filter.comp
template <class K>
__global__ void upscale_kernel(const uint2* __restrict__ src, int sw, int sh,
                               uint2* __restrict__ dst, int tw, int th) {
  int ubx, uby;
  xcd_block(ubx, uby);
  const int jc = ubx * 16 + (threadIdx.x & 15), jr = uby * 16 + (threadIdx.x >> 4);
  if (jc >= tw || jr >= th) return;
  const float kr = 0.5f * K::support;
  const float x_r = ((float)jr + 0.5f) / (float)th;
  const float xi_r = x_r * (float)sh - 0.5f;
  const int il_r = (int)ceilf(xi_r - kr), ir_r = (int)floorf(xi_r + kr);
  const float x_c = ((float)jc + 0.5f) / (float)tw;
  const float xi_c = x_c * (float)sw - 0.5f;
  const int il_c = (int)ceilf(xi_c - kr), ir_c = (int)floorf(xi_c + kr);
  // the column weights once per pixel (the same expression for every row), the
  // taps in the same order with the same operations (products through v_fma_mix)
  const int nc = ir_c - il_c + 1;
  float4 f = make_float4(0.f, 0.f, 0.f, 0.f);
  if (nc > kUpMaxTaps) {
    for (int ir = il_r; ir <= ir_r; ir++) {
      const float wr = K::w(xi_r - (float)ir);
      for (int ic = il_c; ic <= ir_c; ic++)
        f = madd(f, wr * K::w(xi_c - (float)ic), fetch_px(src, sw, sh, ic, ir));
    }
  } else {
    float wc[kUpMaxTaps];
#pragma unroll
    for (int q = 0; q < kUpMaxTaps; q++) wc[q] = q < nc ? K::w(xi_c - (float)(il_c + q)) : 0.0f;
    for (int ir = il_r; ir <= ir_r; ir++) {
      const float wr = K::w(xi_r - (float)ir);
      const bool row_in = ir >= 0 && ir < sh;
#pragma unroll
      for (int q = 0; q < kUpMaxTaps; q++) {
        if (q < nc) {
          const int ic = il_c + q;
          const uint2 p = (row_in && ic >= 0 && ic < sw) ? src[(size_t)ir * sw + ic] : make_uint2(0u, 0u);
          const float wgt = wr * wc[q];
          f.x += mul_half<false>(wgt, p.x);
          f.y += mul_half<true>(wgt, p.x);
          f.z += mul_half<false>(wgt, p.y);
          f.w += mul_half<true>(wgt, p.y);
        }
      }
    }
  }
  store_px(dst, tw, jc, jr, f);
}

// cbs_digital_filter.comp / comoms_digital_filter.comp: the pre-factored LU
// solve of the cardinal kernel's sampled convolution, one thread per row (dir 0)
// or column (dir 1), in place, every step stored as RGBA16F.
struct LCbs {
  static constexpr int m = 8;
  __device__ static float L(int i) {
    constexpr float t[8] = {.2f, .26315789f, .26760563f, .26792453f,
                            .26794742f, .26794907f, .26794918f, .26794919f};
    return t[i];
  }
};
struct LOmoms {
  static constexpr int m = 9;
  __device__ static float L(int i) {
    constexpr float t[9] = {.23529412f, .33170732f, .34266611f, .34395774f, .34411062f,
                            .34412872f, .34413087f, .34413112f, .34413115f};
    return t[i];
  }
};

// One lane per (line, channel): the channels of a pixel are independent in the
// recursion, so a line's four channels run on four adjacent lanes.  The value a
// step stores is kept in a register as the binary16 round trip (what imageLoad
// would read back).  The recursion is sequential along a line, so the line is
// streamed through registers in batches of kDigitalBatch, software-pipelined:
// the next batch's loads are issued before the current batch's updates and
// stores (the forward pass reads values no earlier step has written; the
// reverse pass reads values this lane stored in the forward pass).
constexpr int kDigitalBatch = 32;

__device__ __forceinline__ float h16(float f) { return h2f(f2h(f)); }

// l * h and c - h for h the binary16 in the low half of `hb`, each one IEEE f32
// operation on the exactly converted half (v_fma_mix: the product or sum is
// exact before its single rounding; the -0 addend keeps the sign of a zero
// product, as a plain multiply does).
__device__ __forceinline__ float mul_h16(float l, uint32_t hb) {
  float d;
  asm("v_fma_mix_f32 %0, %1, %2, neg(0) op_sel_hi:[0,1,0]" : "=v"(d) : "v"(l), "v"(hb));
  return d;
}
__device__ __forceinline__ float sub_h16(float c, uint32_t hb) {
  float d;
  asm("v_fma_mix_f32 %0, %1, -1.0, %2 op_sel_hi:[1,0,0]" : "=v"(d) : "v"(hb), "v"(c));
  return d;
}
// (half HI ? x.hi : x.lo) - p, one rounding
template <bool HI>
__device__ __forceinline__ float half_minus(uint32_t x, float p) {
  float d;
  if (HI) asm("v_fma_mix_f32 %0, %1, 1.0, -%2 op_sel:[1,0,0] op_sel_hi:[1,0,0]" : "=v"(d) : "v"(x), "v"(p));
  else asm("v_fma_mix_f32 %0, %1, 1.0, -%2 op_sel_hi:[1,0,0]" : "=v"(d) : "v"(x), "v"(p));
  return d;
}
// (half HI ? x.hi : x.lo) - h for h the binary16 in the low half of hb, one rounding
template <bool HI>
__device__ __forceinline__ float half_minus_h16(uint32_t x, uint32_t hb) {
  float d;
  if (HI) asm("v_fma_mix_f32 %0, %1, -1.0, %2 op_sel:[0,0,1] op_sel_hi:[1,0,1]" : "=v"(d) : "v"(hb), "v"(x));
  else asm("v_fma_mix_f32 %0, %1, -1.0, %2 op_sel_hi:[1,0,1]" : "=v"(d) : "v"(hb), "v"(x));
  return d;
}

template <class LU>
__global__ void digital_filter_kernel(uint16_t* __restrict__ img, int w, int h, int dir) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  const int lines = dir == 0 ? h : w;
  if (t >= lines * 4) return;
  const int line = t >> 2, ch = t & 3;
  const int nn = dir == 0 ? w : h;
  // element i of this lane's line/channel
  const size_t base = dir == 0 ? (size_t)line * w * 4 + ch : (size_t)line * 4 + ch;
  const size_t stride = dir == 0 ? 4 : (size_t)w * 4;
  uint16_t* p = img + base;
  const int m = LU::m;
  const float p_inv = 1.0f;
  const float L_inf = LU::L(m - 1), v_inv = L_inf / (1.f + L_inf);
  constexpr int B = kDigitalBatch;
  float cur[B], nxt[B];
  // forward pass: f[i] -= L * f[i-1], i = 1 .. nn-1
  float prev = h2f(p[0]);
#pragma unroll
  for (int k = 0; k < B; k++)
    if (1 + k < nn) cur[k] = h2f(p[(size_t)(1 + k) * stride]);
  for (int i0 = 1; i0 < nn; i0 += B) {
    const bool more = i0 + B < nn;
    if (more) {
#pragma unroll
      for (int k = 0; k < B; k++)
        if (i0 + B + k < nn) nxt[k] = h2f(p[(size_t)(i0 + B + k) * stride]);
    }
#pragma unroll
    for (int k = 0; k < B; k++) {
      const int i = i0 + k;
      if (i < nn) {
        const float l = i < m ? LU::L(i - 1) : L_inf;
        const float r = cur[k] - l * prev;
        p[(size_t)i * stride] = f2h(r);
        prev = h16(r);
      }
    }
#pragma unroll
    for (int k = 0; k < B; k++) cur[k] = nxt[k];
  }
  // f[nn-1] *= p_inv * v_inv  (prev holds the stored f[nn-1])
  {
    const float r = prev * (p_inv * v_inv);
    p[(size_t)(nn - 1) * stride] = f2h(r);
    prev = h16(r);
  }
  // reverse pass: f[i] = L * (p_inv * f[i] - f[i+1]), i = nn-2 .. 0
#pragma unroll
  for (int k = 0; k < B; k++)
    if (nn - 2 - k >= 0) cur[k] = h2f(p[(size_t)(nn - 2 - k) * stride]);
  for (int i0 = nn - 2; i0 >= 0; i0 -= B) {
    const bool more = i0 - B >= 0;
    if (more) {
#pragma unroll
      for (int k = 0; k < B; k++)
        if (i0 - B - k >= 0) nxt[k] = h2f(p[(size_t)(i0 - B - k) * stride]);
    }
#pragma unroll
    for (int k = 0; k < B; k++) {
      const int i = i0 - k;
      if (i >= 0) {
        const float l = i >= m - 1 ? L_inf : LU::L(i);
        const float r = l * (p_inv * cur[k] - prev);
        p[(size_t)i * stride] = f2h(r);
        prev = h16(r);
      }
    }
#pragma unroll
    for (int k = 0; k < B; k++) cur[k] = nxt[k];
  }
}

constexpr int kDigitalUnroll = 8;   // staging loads in flight per thread

// The same recursion, parallel along the line, with the lines staged in LDS.
//
// Each step is y_i = round16(x_i - round32(l * y_(i-1))) (forward) or
// y_i = round16(round32(l * round32(x_i - y_(i+1)))) (reverse), l > 0: for fixed
// x_i a non-increasing function of the previous value (IEEE rounding is
// monotone; with -0 ordered below +0 the signed zeros too), so the composition
// of steps is monotone.  Hence if the previous value of a step lies in [-B, B],
// its result lies between the results of the two extremes, and once the two
// extreme trajectories agree bit for bit every value inside gives the same bits.
// B is a proven bound of every value of the recursion, from the largest |x| of
// the workgroup's lines M: |y| <= (M + l|y|)(1 + 2^-10) + 2^-25 covers the two
// f32 roundings and the binary16 one (subnormal: 2^-25 absolute), so
// B = ((1 + e) M + 2^-25) / (1 - l (1 + e)), e = 2^-9 (slack for the f32
// evaluation of B itself), rounded up to binary16; the reverse pass takes
// Br = (l (1 + e) B + 2^-25) / (1 - l (1 + e)).
//
// A line is cut into segments of kSeg elements, one lane each.  The lane runs
// the two extreme trajectories over the W elements before its segment (the
// warm-up reads only inputs); if they agree the result is the exact value
// entering the segment, and the lane computes its segment from it.  The
// recursion contracts by l ~ 0.27 (B-spline) / 0.34 (o-MOMS) per step, so W = 24 /
// 32 steps bring the extremes together almost always; where they do not (a
// region whose rounded recursion has a 2-cycle carries its phase from
// arbitrarily far back) the segment is left unwritten and redone after the
// parallel phase by one lane per chain, in order, from the exact value its
// predecessor ends with.  Every stored value is the one the sequential recursion
// stores.  Lines with a non-finite value, or whose bound leaves binary16, run
// sequentially (all segments redone).
constexpr int kSeg = 32;           // elements per segment
constexpr int kSegChunks = kSeg / 8;
constexpr int kSegPitch = 40;      // halves per segment in LDS (+16 B: 16 lanes' 16-B reads hit distinct banks)
constexpr int kSegMaxThreads = 512;
constexpr size_t kSegLdsMax = 64 * 1024;
#ifdef CVR_DIGITAL_PROBE   // cost probes only (tools/build_variant.sh), wrong images:
constexpr int kDigitalProbe = CVR_DIGITAL_PROBE;   // 1 staging only, 2 no redo of segments
#else
constexpr int kDigitalProbe = 0;
#endif

template <class LU> struct SegWarm;
template <> struct SegWarm<LCbs> { static constexpr int W = 24; };
template <> struct SegWarm<LOmoms> { static constexpr int W = 32; };

// v_cvt_f16_f32 without masking the upper half (only the low half is read back)
__device__ __forceinline__ uint32_t h16_raw(float f) {
  uint32_t r;
  asm("v_cvt_f16_f32 %0, %1" : "=v"(r) : "v"(f));
  return r;
}

// forward coefficient of element i >= 1 (the LU table below m), reverse of i >= 0
template <class LU>
__device__ __forceinline__ float fwd_coef(int i) {
  float c = LU::L(LU::m - 1);
#pragma unroll
  for (int j = 1; j < LU::m; j++) c = i == j ? LU::L(j - 1) : c;
  return c;
}
template <class LU>
__device__ __forceinline__ float rev_coef(int i) {
  float c = LU::L(LU::m - 1);
#pragma unroll
  for (int j = 0; j < LU::m - 1; j++) c = i == j ? LU::L(j) : c;
  return c;
}

// 8 forward steps on one 16-B chunk, elements i0 .. i0+7 (element 0 of the line is
// kept as it is).  CHECK: stop at nn.
template <class LU, bool CHECK>
__device__ __forceinline__ uint4 fwd8(uint4 v, uint32_t& prev, int i0, int nn) {
  // the table coefficients sit in chunks 0 and 1 of a line (i0 = 0, 8); with
  // compile-time k both candidates are constants: two selects per element
  float lk[8];
  const bool c0 = i0 == 0, c1 = i0 == 8;
#pragma unroll
  for (int k = 0; k < 8; k++) lk[k] = c0 ? fwd_coef<LU>(k) : (c1 ? fwd_coef<LU>(8 + k) : LU::L(LU::m - 1));
  uint32_t wd[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
  for (int k = 0; k < 8; k++) {
    if (CHECK && i0 + k >= nn) break;
    const uint32_t x = wd[k >> 1];
    const float p = mul_h16(lk[k], prev);
    uint32_t o = h16_raw((k & 1) ? half_minus<true>(x, p) : half_minus<false>(x, p));
    if (k == 0) o = i0 == 0 ? x : o;
    wd[k >> 1] = (k & 1) ? ((x & 0xffffu) | (o << 16)) : ((x & 0xffff0000u) | (o & 0xffffu));
    prev = (k & 1) ? (o & 0xffffu) : o;   // the next step reads the low half only
  }
  return make_uint4(wd[0], wd[1], wd[2], wd[3]);
}

// 8 reverse steps, elements i0+7 .. i0 (past nn-2 left alone when CHECK)
template <class LU, bool CHECK>
__device__ __forceinline__ uint4 rev8(uint4 v, uint32_t& prev, int i0, int nn) {
  float lk[8];
  const bool c0 = i0 == 0, c1 = i0 == 8;
#pragma unroll
  for (int k = 0; k < 8; k++) lk[k] = c0 ? rev_coef<LU>(k) : (c1 ? rev_coef<LU>(8 + k) : LU::L(LU::m - 1));
  uint32_t wd[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
  for (int k = 7; k >= 0; k--) {
    if (CHECK && i0 + k > nn - 2) continue;
    const uint32_t x = wd[k >> 1];
    // p_inv * f[i] = f[i] exactly (p_inv = 1)
    const uint32_t o = h16_raw(lk[k] * ((k & 1) ? half_minus_h16<true>(x, prev) : half_minus_h16<false>(x, prev)));
    wd[k >> 1] = (k & 1) ? ((x & 0xffffu) | (o << 16)) : ((x & 0xffff0000u) | (o & 0xffffu));
    prev = o;
  }
  return make_uint4(wd[0], wd[1], wd[2], wd[3]);
}

// chunk ch (elements 8ch .. 8ch+7) of a chain in the segment-padded layout
__device__ __forceinline__ uint4* seg_chunk(uint4* cb, int ch) {
  return cb + (ch / kSegChunks) * (kSegPitch / 8) + (ch % kSegChunks);
}
__device__ __forceinline__ uint32_t seg_half(const uint16_t* c, int i) {
  return c[(i / kSeg) * kSegPitch + (i % kSeg)];
}

// Forward pass over segment k of a chain from the value entering it.  TWO: also
// from a second candidate value, in lockstep (independent chains: the same
// latency), its results into `spare` (the segment's chunks).
template <class LU, bool TWO = false>
__device__ __forceinline__ void fwd_segment(uint4* cb, int k, uint32_t prev, int nn,
                                            uint32_t prev2 = 0u, uint4* spare = nullptr) {
  const int i_beg = k * kSeg, n = min(kSeg, nn - i_beg);
  const int nfull = n >> 3, nch = (n + 7) >> 3;
  uint4* base = cb + k * (kSegPitch / 8);
  uint4 v[kSegChunks], v2[kSegChunks];
#pragma unroll
  for (int q = 0; q < kSegChunks; q++) v[q] = v2[q] = base[q];   // inside the padded plane
#pragma unroll
  for (int q = 0; q < kSegChunks; q++) {
    if (q < nfull) {
      v[q] = fwd8<LU, false>(v[q], prev, i_beg + 8 * q, nn);
      if (TWO) v2[q] = fwd8<LU, false>(v2[q], prev2, i_beg + 8 * q, nn);
    } else if (q < nch) {
      v[q] = fwd8<LU, true>(v[q], prev, i_beg + 8 * q, nn);
      if (TWO) v2[q] = fwd8<LU, true>(v2[q], prev2, i_beg + 8 * q, nn);
    }
  }
#pragma unroll
  for (int q = 0; q < kSegChunks; q++)
    if (q < nch) {
      base[q] = v[q];
      if (TWO && spare) spare[q] = v2[q];
    }
}

// Reverse pass over segment k (elements min(top, nn-2) .. k*kSeg) from the value
// above it (TWO: as fwd_segment).
template <class LU, bool TWO = false>
__device__ __forceinline__ void rev_segment(uint4* cb, int k, uint32_t prev, int nn,
                                            uint32_t prev2 = 0u, uint4* spare = nullptr) {
  const int i_beg = k * kSeg;
  const int top = min(i_beg + kSeg - 1, nn - 2);
  if (top < i_beg) return;
  const int qtop = (top - i_beg) >> 3;                 // chunk of the top element
  const bool partial = ((qtop << 3) + 7) > top - i_beg;
  uint4* base = cb + k * (kSegPitch / 8);
  uint4 v[kSegChunks], v2[kSegChunks];
#pragma unroll
  for (int q = 0; q < kSegChunks; q++) v[q] = v2[q] = base[q];
#pragma unroll
  for (int q = kSegChunks - 1; q >= 0; q--) {
    if (q < qtop || (q == qtop && !partial)) {
      v[q] = rev8<LU, false>(v[q], prev, i_beg + 8 * q, nn);
      if (TWO) v2[q] = rev8<LU, false>(v2[q], prev2, i_beg + 8 * q, nn);
    } else if (q == qtop) {
      v[q] = rev8<LU, true>(v[q], prev, i_beg + 8 * q, nn);
      if (TWO) v2[q] = rev8<LU, true>(v2[q], prev2, i_beg + 8 * q, nn);
    }
  }
#pragma unroll
  for (int q = 0; q < kSegChunks; q++)
    if (q <= qtop) {
      base[q] = v[q];
      if (TWO && spare) spare[q] = v2[q];
    }
}

// The order of binary16 values with -0 below +0, as an integer key.
__device__ __forceinline__ int h16_key(uint32_t h) {
  h &= 0xffffu;
  return (h & 0x8000u) ? (int)(0x7fffu - (h & 0x7fffu)) : (int)(h + 0x8000u);
}

// Item states.  The value entering a segment is final / the two warm-up values
// are adjacent binary16 values (the entering value is one of them: both
// candidate results are computed, the first in place, the second in a spare
// slot) / unknown (recomputed once its predecessor is final).
constexpr uint8_t kSegFinal = 1, kSegTwo = 3, kSegRedo = 0, kSegTake2 = 4;
// second-candidate segments per workgroup and pass: a quarter of the segments
// (the 1024^2 frames of the bench downscaled with the B-spline kernel, values up
// to ~36, settle into 2-cycles in ~12 % of the row segments), at most 255
__host__ __device__ constexpr int spare_slots(int items) {
  return items / 4 < 16 ? 16 : (items / 4 > 255 ? 255 : items / 4);
}

// binary16 bits of a value >= b (b >= 0 finite): round to nearest, then up
__device__ __forceinline__ uint32_t h16_ceil(float b) {
  uint32_t h = f2h(b);
  if (h2f((uint16_t)h) < b) h++;
  return h;
}

template <class LU>
__global__ void __launch_bounds__(kSegMaxThreads)
digital_filter_seg_kernel(uint16_t* __restrict__ img, int w, int h, int dir, int lpw_shift, int nseg) {
  extern __shared__ uint4 lds_raw[];
  constexpr int W = SegWarm<LU>::W;
  const int S = nseg * kSegPitch;   // chain stride (halves)
  uint16_t* plane = reinterpret_cast<uint16_t*>(lds_raw);
  const int lpw = 1 << lpw_shift;
  const int lines = dir == 0 ? h : w, nn = dir == 0 ? w : h;
  // XCD-aware: workgroup b runs on XCD b % 8, so consecutive line groups go to the
  // same XCD (column groups of the column pass share 128-B lines in its L2)
  const int nblk = gridDim.x;
  const int blk = (nblk & 7) == 0 ? (int)(blockIdx.x & 7) * (nblk >> 3) + (int)(blockIdx.x >> 3)
                                  : (int)blockIdx.x;
  const int l0 = blk * lpw;
  const int nl = min(lpw, lines - l0);
  const int nchain = nl * 4, items = nchain * nseg;
  const int ni = lpw * 4 * nseg;   // item capacity
  const int nspare = spare_slots(ni);
  uint4* spare = lds_raw + (size_t)(lpw * 4) * S / 8;   // nspare x kSeg halves
  uint16_t* start_f = reinterpret_cast<uint16_t*>(spare + nspare * kSegChunks);
  uint16_t* start_r = start_f + ni;      // per item: value entering the segment (candidate 1)
  uint16_t* start2_f = start_r + ni;     // candidate 2
  uint16_t* start2_r = start2_f + ni;
  uint8_t* ok_f = reinterpret_cast<uint8_t*>(start2_r + ni);
  uint8_t* ok_r = ok_f + ni;
  uint8_t* slot_f = ok_r + ni;
  uint8_t* slot_r = slot_f + ni;
  const int nwords = (nseg + 63) >> 6;   // per chain: bit mask of unresolved segments
  unsigned long long* unres_f = reinterpret_cast<unsigned long long*>(
      (reinterpret_cast<uintptr_t>(slot_r + ni) + 7) & ~(uintptr_t)7);
  unsigned long long* unres_r = unres_f + lpw * 4 * nwords;
  for (int i = threadIdx.x; i < 2 * lpw * 4 * nwords; i += blockDim.x) unres_f[i] = 0ull;
  __shared__ uint32_t max_bits;
  __shared__ int nfail_f, nfail_r, spare_f, spare_r;
  const int tid = threadIdx.x, nthr = blockDim.x;
  if (tid == 0) { max_bits = 0u; nfail_f = 0; nfail_r = 0; spare_f = 0; spare_r = 0; }
  __syncthreads();
  uint2* px = reinterpret_cast<uint2*>(img);
  auto put = [&](int l, int i, uint2 v) {
    uint16_t* q = plane + (size_t)(l * 4) * S + (i / kSeg) * kSegPitch + (i % kSeg);
    q[0] = (uint16_t)(v.x & 0xffffu);
    q[S] = (uint16_t)(v.x >> 16);
    q[2 * S] = (uint16_t)(v.y & 0xffffu);
    q[3 * S] = (uint16_t)(v.y >> 16);
  };
  auto get = [&](int l, int i) {
    const uint16_t* q = plane + (size_t)(l * 4) * S + (i / kSeg) * kSegPitch + (i % kSeg);
    return make_uint2((uint32_t)q[0] | ((uint32_t)q[S] << 16),
                      (uint32_t)q[2 * S] | ((uint32_t)q[3 * S] << 16));
  };
  // ---- stage in (coalesced 8-B pixels), with the largest |x| (binary16 bits) ----
  const int total = dir == 0 ? nl * nn : (nn << lpw_shift);
  auto src_of = [&](int e, int& l, int& i) -> size_t {
    if (dir == 0) {
      l = e / nn;
      i = e - l * nn;
      return (size_t)(l0 + l) * w + i;
    }
    i = e >> lpw_shift;
    l = e & (lpw - 1);
    return (size_t)i * w + l0 + l;
  };
  // rows of even length from a 16-B aligned image: two pixels per 16-B load, one
  // 4-B LDS store per channel
  const bool pairs = dir == 0 && (nn & 1) == 0 && (reinterpret_cast<uintptr_t>(img) & 15) == 0;
  const int half = nn >> 1, tp = nl * half;
  uint4* p4 = reinterpret_cast<uint4*>(img);
  auto plane_word = [&](int l, int c, int i) {   // i even: channel c halves i, i+1
    return reinterpret_cast<uint32_t*>(plane + (size_t)(l * 4 + c) * S + (i / kSeg) * kSegPitch + (i % kSeg));
  };
  uint32_t mb = 0u;
  if (pairs) {
    for (int e0 = 0; e0 < tp; e0 += nthr * kDigitalUnroll) {
      uint4 v[kDigitalUnroll];
#pragma unroll
      for (int u = 0; u < kDigitalUnroll; u++) {
        const int e = e0 + u * nthr + tid;
        if (e < tp) {
          const int l = e / half, i = (e - l * half) * 2;
          v[u] = p4[((size_t)(l0 + l) * w + i) >> 1];
        }
      }
#pragma unroll
      for (int u = 0; u < kDigitalUnroll; u++) {
        const int e = e0 + u * nthr + tid;
        if (e < tp) {
          const int l = e / half, i = (e - l * half) * 2;
          const uint4 q = v[u];
          *plane_word(l, 0, i) = (q.x & 0xffffu) | (q.z << 16);
          *plane_word(l, 1, i) = (q.x >> 16) | (q.z & 0xffff0000u);
          *plane_word(l, 2, i) = (q.y & 0xffffu) | (q.w << 16);
          *plane_word(l, 3, i) = (q.y >> 16) | (q.w & 0xffff0000u);
          const uint32_t m0 = max(max(q.x & 0x7fffu, (q.x >> 16) & 0x7fffu), max(q.y & 0x7fffu, (q.y >> 16) & 0x7fffu));
          const uint32_t m1 = max(max(q.z & 0x7fffu, (q.z >> 16) & 0x7fffu), max(q.w & 0x7fffu, (q.w >> 16) & 0x7fffu));
          mb = max(mb, max(m0, m1));
        }
      }
    }
  }
  for (int e0 = 0; e0 < (pairs ? 0 : total); e0 += nthr * kDigitalUnroll) {
    uint2 v[kDigitalUnroll];
#pragma unroll
    for (int u = 0; u < kDigitalUnroll; u++) {
      const int e = e0 + u * nthr + tid;
      int l, i;
      const size_t a = src_of(e, l, i);
      if (e < total && l < nl) v[u] = px[a];
    }
#pragma unroll
    for (int u = 0; u < kDigitalUnroll; u++) {
      const int e = e0 + u * nthr + tid;
      int l, i;
      src_of(e, l, i);
      if (e < total && l < nl) {
        put(l, i, v[u]);
        mb = max(mb, max(max(v[u].x & 0x7fffu, (v[u].x >> 16) & 0x7fffu),
                         max(v[u].y & 0x7fffu, (v[u].y >> 16) & 0x7fffu)));
      }
    }
  }
  if (mb) atomicMax(&max_bits, mb);
  __syncthreads();
  if (kDigitalProbe != 1) {   // (cost probe 1: staging only)
  // ---- the bounds (every thread the same) ----
  const float L_inf = LU::L(LU::m - 1);
  const float lq = L_inf * (1.0f + 0x1p-9f);
  bool spec = max_bits < 0x7c00u && nseg > 1;   // finite inputs
  uint32_t bf = 0u, br = 0u;
  if (spec) {
    bf = h16_ceil(((1.0f + 0x1p-9f) * h2f((uint16_t)max_bits) + 0x1p-25f) / (1.0f - lq));
    br = h16_ceil((lq * h2f((uint16_t)bf) + 0x1p-25f) / (1.0f - lq));
    spec = bf < 0x7c00u && br < 0x7c00u;
  }
  // ---- forward: warm-ups (read only), then the segments ----
  for (int it = tid; it < items; it += nthr) {
    const int c = it / nseg, k = it - c * nseg;
    if (k == 0) {   // starts from the line's first element: final
      ok_f[it] = 1;
      continue;
    }
    uint32_t lo = bf | 0x8000u, hi = bf;
    bool ok = false;
    if (spec) {
      uint4* cb = reinterpret_cast<uint4*>(plane + (size_t)c * S);
      const int a = max(0, k * kSeg - W);   // from element 0 the warm-up is exact
      const int ch0 = a >> 3, nq = (k * kSeg - a) >> 3;
#pragma unroll
      for (int q = 0; q < W / 8; q++) {
        if (q < nq) {
          const uint4 v = *seg_chunk(cb, ch0 + q);
          fwd8<LU, false>(v, lo, (ch0 + q) * 8, nn);
          fwd8<LU, false>(v, hi, (ch0 + q) * 8, nn);
        }
      }
      ok = (lo & 0xffffu) == (hi & 0xffffu);
    }
    uint8_t st = ok ? kSegFinal : kSegRedo;
    if (!ok && spec && abs(h16_key(lo) - h16_key(hi)) == 1) {
      const int sl = atomicAdd(&spare_f, 1);
      if (sl < nspare) {
        st = kSegTwo;
        slot_f[it] = (uint8_t)sl;
      }
    }
    start_f[it] = (uint16_t)lo;
    start2_f[it] = (uint16_t)hi;
    ok_f[it] = st;
    if (!ok) {
      atomicAdd(&nfail_f, 1);
      atomicOr(&unres_f[c * nwords + (k >> 6)], 1ull << (k & 63));
    }
  }
  __syncthreads();
  for (int it = tid; it < items; it += nthr) {
    const int c = it / nseg, k = it - c * nseg;
    // every item runs both trajectories (a final one twice from the same value):
    // one code path for the wave, the second chain costs no latency
    uint4* cb = reinterpret_cast<uint4*>(plane + (size_t)c * S);
    const uint8_t st = k == 0 ? kSegFinal : ok_f[it];
    if (st != kSegRedo) {
      const uint32_t s1 = k ? start_f[it] : 0u;
      const bool two = st == kSegTwo;
      fwd_segment<LU, true>(cb, k, s1, nn, two ? start2_f[it] : s1,
                            two ? spare + slot_f[it] * kSegChunks : nullptr);
    }
  }
  __syncthreads();
  // resolve the segments whose warm-up did not settle, in order along each chain
  // (one lane per chain, over the chain's bit mask of such segments).  The value
  // entering one is then final: a two-candidate segment keeps the first candidate
  // or takes the second (its end value goes on to the next; the copies are made
  // afterwards, in parallel), any other is recomputed from it.
  if (nfail_f && kDigitalProbe != 2) {
    for (int c = tid; c < nchain; c += nthr) {
      uint16_t* ch = plane + (size_t)c * S;
      int kp = -2;          // the last segment resolved, and the value it ends with
      uint32_t ep = 0u;
      for (int wd = 0; wd < nwords; wd++) {
        unsigned long long m = unres_f[c * nwords + wd];
        while (m) {
          const int k = wd * 64 + __builtin_ctzll(m);
          m &= m - 1ull;
          const int it = c * nseg + k;
          const uint32_t t = kp == k - 1 ? ep : seg_half(ch, k * kSeg - 1);   // entering value
          const int last = min(nn, (k + 1) * kSeg) - 1;
          if (ok_f[it] == kSegRedo) {
            fwd_segment<LU>(reinterpret_cast<uint4*>(ch), k, t, nn);
            ep = seg_half(ch, last);
          } else if (t == start2_f[it]) {
            ok_f[it] = kSegTake2;
            ep = reinterpret_cast<const uint16_t*>(spare + slot_f[it] * kSegChunks)[last - k * kSeg];
          } else {
            ep = seg_half(ch, last);
          }
          kp = k;
        }
      }
    }
    __syncthreads();
    for (int it = tid; it < items; it += nthr) {
      if (ok_f[it] != kSegTake2) continue;
      const int c = it / nseg, k = it - c * nseg;
      uint4* base = reinterpret_cast<uint4*>(plane + (size_t)c * S) + k * (kSegPitch / 8);
      const uint4* sp = spare + slot_f[it] * kSegChunks;
      const int nch = (min(kSeg, nn - k * kSeg) + 7) >> 3;
#pragma unroll
      for (int q = 0; q < kSegChunks; q++)
        if (q < nch) base[q] = sp[q];
    }
    __syncthreads();
  }
  // f[nn-1] *= p_inv * v_inv
  const float v_inv = L_inf / (1.f + L_inf);
  for (int c = tid; c < nchain; c += nthr) {
    uint16_t* ch = plane + (size_t)c * S;
    uint16_t* last = ch + ((nn - 1) / kSeg) * kSegPitch + ((nn - 1) % kSeg);
    *last = (uint16_t)f2h(h2f(*last) * (1.0f * v_inv));
  }
  __syncthreads();
  // ---- reverse: warm-ups, then the segments ----
  for (int it = tid; it < items; it += nthr) {
    const int c = it / nseg, k = it - c * nseg;
    if (k == nseg - 1) {   // starts from the exact f[nn-1]
      ok_r[it] = 1;
      continue;
    }
    uint4* cb = reinterpret_cast<uint4*>(plane + (size_t)c * S);
    const int b0 = (k + 1) * kSeg;          // first element above the segment
    uint32_t lo = br | 0x8000u, hi = br;
    bool ok = false;
    if (b0 + W - 1 >= nn - 2) {
      // the warm-up would reach the line's end: start from the exact f[nn-1]
      lo = seg_half(reinterpret_cast<const uint16_t*>(cb), nn - 1);
      for (int ch = (nn - 2) >> 3; ch >= (b0 >> 3); ch--)
        rev8<LU, true>(*seg_chunk(cb, ch), lo, ch * 8, nn);
      ok = true;
    } else if (spec) {
#pragma unroll
      for (int q = W / 8 - 1; q >= 0; q--) {
        const uint4 v = *seg_chunk(cb, (b0 >> 3) + q);
        rev8<LU, false>(v, lo, b0 + 8 * q, nn);
        rev8<LU, false>(v, hi, b0 + 8 * q, nn);
      }
      ok = (lo & 0xffffu) == (hi & 0xffffu);
    }
    uint8_t st = ok ? kSegFinal : kSegRedo;
    if (!ok && spec && abs(h16_key(lo) - h16_key(hi)) == 1) {
      const int sl = atomicAdd(&spare_r, 1);
      if (sl < nspare) {
        st = kSegTwo;
        slot_r[it] = (uint8_t)sl;
      }
    }
    start_r[it] = (uint16_t)lo;
    start2_r[it] = (uint16_t)hi;
    ok_r[it] = st;
    if (!ok) {
      atomicAdd(&nfail_r, 1);
      atomicOr(&unres_r[c * nwords + (k >> 6)], 1ull << (k & 63));
    }
  }
  __syncthreads();
  for (int it = tid; it < items; it += nthr) {
    const int c = it / nseg, k = it - c * nseg;
    uint16_t* ch = plane + (size_t)c * S;
    uint4* cb = reinterpret_cast<uint4*>(ch);
    const uint8_t st = k == nseg - 1 ? kSegFinal : ok_r[it];
    if (st != kSegRedo) {
      const uint32_t s1 = k == nseg - 1 ? seg_half(ch, nn - 1) : start_r[it];
      const bool two = st == kSegTwo;
      rev_segment<LU, true>(cb, k, s1, nn, two ? start2_r[it] : s1,
                            two ? spare + slot_r[it] * kSegChunks : nullptr);
    }
  }
  __syncthreads();
  if (nfail_r && kDigitalProbe != 2) {
    for (int c = tid; c < nchain; c += nthr) {
      uint16_t* ch = plane + (size_t)c * S;
      int kp = -2;
      uint32_t ep = 0u;
      for (int wd = nwords - 1; wd >= 0; wd--) {
        unsigned long long m = unres_r[c * nwords + wd];
        while (m) {
          const int bit = 63 - __builtin_clzll(m);
          m &= ~(1ull << bit);
          const int k = wd * 64 + bit;
          const int it = c * nseg + k;
          const uint32_t t = kp == k + 1 ? ep : seg_half(ch, (k + 1) * kSeg);
          if (ok_r[it] == kSegRedo) {
            rev_segment<LU>(reinterpret_cast<uint4*>(ch), k, t, nn);
            ep = seg_half(ch, k * kSeg);
          } else if (t == start2_r[it]) {
            ok_r[it] = kSegTake2;
            ep = reinterpret_cast<const uint16_t*>(spare + slot_r[it] * kSegChunks)[0];
          } else {
            ep = seg_half(ch, k * kSeg);
          }
          kp = k;
        }
      }
    }
    __syncthreads();
    for (int it = tid; it < items; it += nthr) {
      if (ok_r[it] != kSegTake2) continue;
      const int c = it / nseg, k = it - c * nseg;
      uint4* base = reinterpret_cast<uint4*>(plane + (size_t)c * S) + k * (kSegPitch / 8);
      const uint4* sp = spare + slot_r[it] * kSegChunks;
      const int qtop = (min(k * kSeg + kSeg - 1, nn - 2) - k * kSeg) >> 3;
#pragma unroll
      for (int q = 0; q < kSegChunks; q++)
        if (q <= qtop) base[q] = sp[q];
    }
    __syncthreads();
  }
  }
  // ---- stage out ----
  if (pairs) {
    for (int e = tid; e < tp; e += nthr) {
      const int l = e / half, i = (e - l * half) * 2;
      const uint32_t c0 = *plane_word(l, 0, i), c1 = *plane_word(l, 1, i);
      const uint32_t c2 = *plane_word(l, 2, i), c3 = *plane_word(l, 3, i);
      p4[((size_t)(l0 + l) * w + i) >> 1] =
          make_uint4((c0 & 0xffffu) | (c1 << 16), (c2 & 0xffffu) | (c3 << 16), (c0 >> 16) | (c1 & 0xffff0000u),
                     (c2 >> 16) | (c3 & 0xffff0000u));
    }
    return;
  }
  for (int e0 = 0; e0 < total; e0 += nthr * kDigitalUnroll) {
#pragma unroll
    for (int u = 0; u < kDigitalUnroll; u++) {
      const int e = e0 + u * nthr + tid;
      int l, i;
      const size_t a = src_of(e, l, i);
      if (e < total && l < nl) px[a] = get(l, i);
    }
  }
}

// Screenshot: FragColor = texture(frame) blended SRC_ALPHA / ONE_MINUS_SRC_ALPHA over
// white, stored to an 8-bit unorm back buffer, read as RGB (row 0 = bottom).
template <bool HALF>
__global__ void screenshot_kernel(const void* __restrict__ src, int w, int h,
                                  uint8_t* __restrict__ rgb) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (size_t)w * h) return;
  float4 p;
  if (HALF) p = load_px((const uint2*)src, w, (int)(i % w), (int)(i / w));
  else p = ((const float4*)src)[i];
  const float c[3] = {p.x, p.y, p.z};
  for (int k = 0; k < 3; k++) {
    const float v = c[k] * p.w + (1.0f - p.w);
    const float q = floorf(v * 255.0f + 0.5f);
    rgb[i * 3 + k] = (uint8_t)(q < 0.0f ? 0.0f : (q > 255.0f ? 255.0f : q));
  }
}

#define CVR_KERNEL_SWITCH(KFN, kernel, g, b, s, ...)                                  \
  switch (kernel) {                                                                 \
    case 0: hipLaunchKernelGGL(KFN<KBox>, g, b, 0, s, __VA_ARGS__); break;          \
    case 1: hipLaunchKernelGGL(KFN<KHat>, g, b, 0, s, __VA_ARGS__); break;          \
    case 2: hipLaunchKernelGGL(KFN<KCatmullRom>, g, b, 0, s, __VA_ARGS__); break;   \
    case 3: hipLaunchKernelGGL(KFN<KMitchell>, g, b, 0, s, __VA_ARGS__); break;     \
    case 4: hipLaunchKernelGGL(KFN<KCardinalBSpline3>, g, b, 0, s, __VA_ARGS__); break; \
    case 5: hipLaunchKernelGGL(KFN<KCardinalOmoms3>, g, b, 0, s, __VA_ARGS__); break;   \
    default: return hipErrorInvalidValue;                                           \
  }

#define CVR_KERNEL_SWITCH_LDS(KFN, kernel, g, b, lds, s, ...)                          \
  switch (kernel) {                                                                  \
    case 0: hipLaunchKernelGGL(KFN<KBox>, g, b, lds, s, __VA_ARGS__); break;         \
    case 1: hipLaunchKernelGGL(KFN<KHat>, g, b, lds, s, __VA_ARGS__); break;         \
    case 2: hipLaunchKernelGGL(KFN<KCatmullRom>, g, b, lds, s, __VA_ARGS__); break;  \
    case 3: hipLaunchKernelGGL(KFN<KMitchell>, g, b, lds, s, __VA_ARGS__); break;    \
    case 4: hipLaunchKernelGGL(KFN<KCardinalBSpline3>, g, b, lds, s, __VA_ARGS__); break; \
    case 5: hipLaunchKernelGGL(KFN<KCardinalOmoms3>, g, b, lds, s, __VA_ARGS__); break;   \
    default: return hipErrorInvalidValue;                                            \
  }

// LDS bytes of digital_filter_seg_kernel for 2^shift lines of nn elements.
static size_t seg_lds_bytes(int shift, int nseg) {
  const size_t chains = (size_t)4 << shift;
  return chains * nseg * kSegPitch * 2 + (size_t)spare_slots((int)(chains * nseg)) * kSeg * 2 + chains * nseg * 12 + 8 +
         chains * ((nseg + 63) / 64) * 16;
}

hipError_t launch_digital(int kernel, uint2* img, int w, int h, hipStream_t s) {
  for (int dir = 0; dir < 2; dir++) {
    const int lines = dir == 0 ? h : w, nn = dir == 0 ? w : h;
    if (lines <= 0 || nn <= 0) continue;
    const int nseg = (nn + kSeg - 1) / kSeg;
    // lines per workgroup: enough workgroups for every CU (>= 256), at most 16 lines
    int shift = 0;
    while (shift < 4 && (lines >> (shift + 1)) >= 256) shift++;
    while (shift > 0 && seg_lds_bytes(shift, nseg) > kSegLdsMax) shift--;
    const size_t lds = seg_lds_bytes(shift, nseg);
    const int items = (4 << shift) * nseg;
    if (lds <= kSegLdsMax && items <= 8 * kSegMaxThreads) {
      // the dynamic-LDS limit is a per-device kernel attribute: set it once per
      // device (a bit per device id; two threads setting it together is harmless)
      static std::atomic<uint64_t> attr_devices{0};
      int dev = 0;
      if (hipGetDevice(&dev) != hipSuccess) dev = 0;
      const uint64_t bit = 1ull << (dev & 63);
      if (!(attr_devices.load(std::memory_order_acquire) & bit)) {
        hipError_t e = hipFuncSetAttribute(
            reinterpret_cast<const void*>(&digital_filter_seg_kernel<LCbs>),
            hipFuncAttributeMaxDynamicSharedMemorySize, (int)kSegLdsMax);
        if (e == hipSuccess)
          e = hipFuncSetAttribute(reinterpret_cast<const void*>(&digital_filter_seg_kernel<LOmoms>),
                                  hipFuncAttributeMaxDynamicSharedMemorySize, (int)kSegLdsMax);
        if (e != hipSuccess) return e;
        attr_devices.fetch_or(bit, std::memory_order_acq_rel);
      }
      const int thr = std::min(kSegMaxThreads, (items + 63) / 64 * 64);
      const dim3 g((lines + (1 << shift) - 1) >> shift), b(thr);
      uint16_t* p = (uint16_t*)img;
      if (kernel == 4)
        hipLaunchKernelGGL(digital_filter_seg_kernel<LCbs>, g, b, lds, s, p, w, h, dir, shift, nseg);
      else
        hipLaunchKernelGGL(digital_filter_seg_kernel<LOmoms>, g, b, lds, s, p, w, h, dir, shift, nseg);
      hipError_t e = hipGetLastError();
      if (e != hipSuccess) return e;
      continue;
    }
    // lines too long for LDS: one lane per chain in global memory
    const int lanes = 4 * lines;
    const dim3 g((lanes + 63) / 64), b(64);
    uint16_t* p = (uint16_t*)img;
    if (kernel == 4) hipLaunchKernelGGL(digital_filter_kernel<LCbs>, g, b, 0, s, p, w, h, dir);
    else hipLaunchKernelGGL(digital_filter_kernel<LOmoms>, g, b, 0, s, p, w, h, dir);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}

}  // namespace

hipError_t launch_multiscale(int mode, int kernel, void* frame, int fw, int fh, void* screen, int sw,
                             int sh, hipStream_t s) {
  const dim3 g((sw + 15) / 16, (sh + 15) / 16), b(256);
  uint2* src = (uint2*)frame;
  uint2* dst = (uint2*)screen;
  if (mode == 1) {
    hipLaunchKernelGGL(multisample_kernel, g, b, 0, s, src, fw, fh, dst, sw, sh);
    return hipGetLastError();
  }
  const bool cardinal = kernel == 4 || kernel == 5;
  if (mode == 2) {
    // taps per axis <= support * frame / screen + 2; the window of a 16x16 block
    // <= (16 + support) * frame / screen + 3 a side
    static const float support[6] = {1.0f, 2.0f, 4.0f, 4.0f, 4.0f, 4.0f};
    const float fr = std::max((float)fw / (float)sw, (float)fh / (float)sh);
    const float sup = support[kernel];
    const size_t side = (size_t)((16.0f + sup) * fr) + 4;
    const size_t lds = (side | 1) * side * sizeof(uint2);
    // the kernel's static weight tables (wcol, wrow) share the 64 KiB with the window
    constexpr size_t kDownStaticLds = sizeof(float) * 2 * 16 * kDownMaxTaps;
    if (sup * fr + 2.0f <= (float)kDownMaxTaps && lds + kDownStaticLds <= 64 * 1024) {
      CVR_KERNEL_SWITCH_LDS(downscale_lds_kernel, kernel, g, b, lds, s, src, fw, fh, dst, sw, sh);
    } else {
      CVR_KERNEL_SWITCH(downscale_kernel, kernel, g, b, s, src, fw, fh, dst, sw, sh);
    }
    hipError_t e = hipGetLastError();
    if (e != hipSuccess || !cardinal) return e;
    return launch_digital(kernel, dst, sw, sh, s);        // over the filtered screen
  }
  if (mode == 3) {
    if (cardinal) {
      hipError_t e = launch_digital(kernel, src, fw, fh, s);   // in place on the frame
      if (e != hipSuccess) return e;
    }
    CVR_KERNEL_SWITCH(upscale_kernel, kernel, g, b, s, src, fw, fh, dst, sw, sh);
    return hipGetLastError();
  }
  return hipErrorInvalidValue;
}

hipError_t launch_screenshot(const void* frame, int half, int w, int h, uint8_t* rgb,
                             hipStream_t s) {
  const size_t n = (size_t)w * h;
  if (n == 0) return hipSuccess;
  const dim3 g((unsigned)((n + 255) / 256)), b(256);
  if (half) hipLaunchKernelGGL(screenshot_kernel<true>, g, b, 0, s, frame, w, h, rgb);
  else hipLaunchKernelGGL(screenshot_kernel<false>, g, b, 0, s, frame, w, h, rgb);
  return hipGetLastError();
}

}  // namespace cvr
