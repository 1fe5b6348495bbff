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

// upscaling_filter.comp
template <class K>
__global__ void upscale_kernel(const uint2* __restrict__ src, int sw, int sh,
                               uint2* __restrict__ dst, int tw, int th) {
  const int jc = blockIdx.x * 16 + (threadIdx.x & 15), jr = blockIdx.y * 16 + (threadIdx.x >> 4);
  if (jc >= tw || jr >= th) return;
  const float kr = 0.5f * K::support;
  const float x_r = ((float)jr + 0.5f) / (float)th;
  const float xi_r = x_r * (float)sh - 0.5f;
  const int il_r = (int)ceilf(xi_r - kr), ir_r = (int)floorf(xi_r + kr);
  const float x_c = ((float)jc + 0.5f) / (float)tw;
  const float xi_c = x_c * (float)sw - 0.5f;
  const int il_c = (int)ceilf(xi_c - kr), ir_c = (int)floorf(xi_c + kr);
  float4 f = make_float4(0.f, 0.f, 0.f, 0.f);
  for (int ir = il_r; ir <= ir_r; ir++) {
    const float wr = K::w(xi_r - (float)ir);
    for (int ic = il_c; ic <= ir_c; ic++)
      f = madd(f, wr * K::w(xi_c - (float)ic), fetch_px(src, sw, sh, ic, ir));
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

// The same recursion with the lines staged in LDS.  One wave takes `lpw` lines
// (lpw * 4 chains, one lane per (line, channel)): the lines are read into LDS
// with coalesced 8-B pixel loads, de-interleaved into one plane of binary16 per
// chain (chain stride S halves: a multiple of 8, padded so that the 16 lanes of a
// ds_read_b128 group fall on distinct banks), both passes run on the planes 8
// elements per LDS access, and the lines are written back once.  Every step
// still rounds to binary16 and the next step reads the rounded value, as the
// global-memory kernel above and the reference's imageLoad/imageStore do.
template <int C> struct Head { static constexpr bool value = true; static constexpr int chunk = C; };
struct NoHead { static constexpr bool value = false; static constexpr int chunk = 0; };

// Staging: a workgroup of kDigitalThreads moves the lines in and out (memory-level
// parallelism for the one wave that then runs the sequential recursions).
constexpr int kDigitalThreads = 256;
constexpr int kDigitalUnroll = 8;

template <class LU>
__global__ void __launch_bounds__(kDigitalThreads)
digital_filter_lds_kernel(uint16_t* __restrict__ img, int w, int h, int dir, int lpw_shift, int S) {
  extern __shared__ uint4 lds_raw[];
  uint16_t* plane = reinterpret_cast<uint16_t*>(lds_raw);
  const int lpw = 1 << lpw_shift;
  const int lines = dir == 0 ? h : w, nn = dir == 0 ? w : h;
  const int l0 = blockIdx.x * lpw;
  const int nl = min(lpw, lines - l0);
  uint2* px = reinterpret_cast<uint2*>(img);
  auto put = [&](int l, int i, uint2 v) {
    uint16_t* q = plane + (size_t)(l * 4) * S + i;
    q[0] = (uint16_t)(v.x & 0xffffu);
    q[S] = (uint16_t)(v.x >> 16);
    q[2 * S] = (uint16_t)(v.y & 0xffffu);
    q[3 * S] = (uint16_t)(v.y >> 16);
  };
  auto get = [&](int l, int i) {
    const uint16_t* q = plane + (size_t)(l * 4) * S + i;
    return make_uint2((uint32_t)q[0] | ((uint32_t)q[S] << 16),
                      (uint32_t)q[2 * S] | ((uint32_t)q[3 * S] << 16));
  };
  // ---- stage in: all kDigitalThreads lanes, kDigitalUnroll loads in flight each ----
  // element e of the wave's nl lines: dir 0 -> (line e / nn, i = e % nn), rows are
  // contiguous in memory; dir 1 -> (line e % lpw, i = e >> lpw_shift), one image
  // row of lpw adjacent pixels per lpw elements
  const int tid = threadIdx.x;
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
  for (int e0 = 0; e0 < total; e0 += kDigitalThreads * kDigitalUnroll) {
    uint2 v[kDigitalUnroll];
#pragma unroll
    for (int u = 0; u < kDigitalUnroll; u++) {
      const int e = e0 + u * kDigitalThreads + tid;
      int l, i;
      const size_t a = src_of(e, l, i);
      if (e < total && l < nl) v[u] = px[a];
    }
#pragma unroll
    for (int u = 0; u < kDigitalUnroll; u++) {
      const int e = e0 + u * kDigitalThreads + tid;
      int l, i;
      src_of(e, l, i);
      if (e < total && l < nl) put(l, i, v[u]);
    }
  }
  __syncthreads();
  // ---- both passes on this lane's chain ----
  const int q = tid;   // the first wave runs the recursions (one lane per chain)
#ifdef CVR_DIGITAL_NO_COMPUTE   // cost probe only (tools/build_variant.sh): wrong images
  if (false) {
#else
  if (q < 64 && (q >> 2) < nl) {
#endif
    uint16_t* c = plane + (size_t)q * S;
    uint4* c4 = reinterpret_cast<uint4*>(c);
    const int m = LU::m;
    const float p_inv = 1.0f;
    const float L_inf = LU::L(m - 1), v_inv = L_inf / (1.f + L_inf);
    // forward pass: f[i] -= L * f[i-1], i = 1 .. nn-1; reverse pass: f[i] = L * (p_inv
    // * f[i] - f[i+1]), i = nn-2 .. 0.  8 elements per LDS access.  The first two
    // chunks (the steps whose coefficient comes from the table: i < m) are peeled
    // with compile-time coefficients, whole chunks run without bounds checks, and
    // the chunk holding element nn-1 checks bounds per element.
    // prev is kept as the stored binary16 bits: the next step reads it straight
    // from the half (v_fma_mix), one dependent conversion less per step
    uint32_t prev = 0u;
    const int nfull = nn >> 3;          // chunks entirely inside [0, nn)
    auto fwd = [&](uint4 v, int ch, auto head, bool check) {
      uint32_t wd[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
      for (int k = 0; k < 8; k++) {
        const int i = (ch << 3) + k;
        float l = L_inf;
        if (decltype(head)::value) {
          const int ic = (decltype(head)::chunk << 3) + k;   // == i at compile time
          if (ic == 0) { prev = wd[0] & 0xffffu; continue; }
          l = ic < m ? LU::L(ic - 1) : L_inf;
        }
        if (check && i >= nn) break;
        const uint32_t x = wd[k >> 1];
        const float p = mul_h16(l, prev);
        const uint32_t o = f2h((k & 1) ? half_minus<true>(x, p) : half_minus<false>(x, p));
        wd[k >> 1] = (k & 1) ? ((x & 0xffffu) | (o << 16)) : ((x & 0xffff0000u) | o);
        prev = o;
      }
      c4[ch] = make_uint4(wd[0], wd[1], wd[2], wd[3]);
    };
    auto rev = [&](uint4 v, int ch, auto head, bool check) {
      uint32_t wd[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
      for (int k = 7; k >= 0; k--) {
        const int i = (ch << 3) + k;
        float l = L_inf;
        if (decltype(head)::value) {
          const int ic = (decltype(head)::chunk << 3) + k;
          l = ic >= m - 1 ? L_inf : LU::L(ic);
        }
        if (check && i > nn - 2) continue;
        const uint32_t x = wd[k >> 1];
        // p_inv * f[i] = f[i] exactly (p_inv = 1)
        const uint32_t o = f2h(l * ((k & 1) ? half_minus_h16<true>(x, prev)
                                            : half_minus_h16<false>(x, prev)));
        wd[k >> 1] = (k & 1) ? ((x & 0xffffu) | (o << 16)) : ((x & 0xffff0000u) | o);
        prev = o;
      }
      c4[ch] = make_uint4(wd[0], wd[1], wd[2], wd[3]);
    };
    const int nch = (nn + 7) >> 3;
    uint4 nxt = c4[0];
    {
      const uint4 v = nxt;
      if (nch > 1) nxt = c4[1];
      fwd(v, 0, Head<0>{}, nfull < 1);
    }
    if (nch > 1) {
      const uint4 v = nxt;
      if (nch > 2) nxt = c4[2];
      fwd(v, 1, Head<1>{}, nfull < 2);
    }
    for (int ch = 2; ch < nfull; ch++) {   // the next chunk's read goes out first
      const uint4 v = nxt;
      if (ch + 1 < nch) nxt = c4[ch + 1];
      fwd(v, ch, NoHead{}, false);
    }
    if (nch > 2 && nfull < nch) fwd(nxt, nch - 1, NoHead{}, true);
    // f[nn-1] *= p_inv * v_inv  (prev holds the stored f[nn-1])
    {
      const uint32_t o = f2h(h2f((uint16_t)prev) * (p_inv * v_inv));
      c[nn - 1] = (uint16_t)o;
      prev = o;
    }
    if (nn >= 2) {
      const int top = (nn - 2) >> 3;            // chunk of element nn-2
      const bool top_partial = ((top << 3) + 7) > nn - 2;
      int ch = top;
      nxt = c4[ch];
      if (ch >= 2 && top_partial) {
        const uint4 v = nxt;
        nxt = c4[ch - 1];
        rev(v, ch, NoHead{}, true);
        ch--;
      }
      for (; ch >= 2; ch--) {
        const uint4 v = nxt;
        nxt = c4[ch - 1];
        rev(v, ch, NoHead{}, false);
      }
      if (ch == 1) {
        const uint4 v = nxt;
        nxt = c4[0];
        rev(v, 1, Head<1>{}, top == 1 && top_partial);
        ch--;
      }
      if (ch == 0) rev(nxt, 0, Head<0>{}, top == 0 && top_partial);
    }
  }
  __syncthreads();
  // ---- stage out ----
  for (int e0 = 0; e0 < total; e0 += kDigitalThreads * kDigitalUnroll) {
#pragma unroll
    for (int u = 0; u < kDigitalUnroll; u++) {
      const int e = e0 + u * kDigitalThreads + tid;
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

// LDS bytes of one wave of digital_filter_lds_kernel: lpw * 4 chains of S halves.
constexpr size_t kDigitalLdsMax = 160 * 1024;

hipError_t launch_digital(int kernel, uint2* img, int w, int h, hipStream_t s) {
  for (int dir = 0; dir < 2; dir++) {
    const int lines = dir == 0 ? h : w, nn = dir == 0 ? w : h;
    const int S = ((nn + 7) / 8) * 8 + 8;   // chain stride (halves): 16-B chunks + 4-bank pad
    int shift = 4;                          // 16 lines (64 chains) per wave, fewer for long lines
    while (shift > 0 && ((size_t)4 << shift) * S * 2 > kDigitalLdsMax) shift--;
    const size_t lds = ((size_t)4 << shift) * S * 2;
    if (lds <= kDigitalLdsMax && lines > 0 && nn > 0) {
      static bool attr = false;   // dynamic LDS beyond 64 KiB must be allowed per kernel
      if (!attr) {
        hipError_t e = hipFuncSetAttribute(
            reinterpret_cast<const void*>(&digital_filter_lds_kernel<LCbs>),
            hipFuncAttributeMaxDynamicSharedMemorySize, (int)kDigitalLdsMax);
        if (e == hipSuccess)
          e = hipFuncSetAttribute(reinterpret_cast<const void*>(&digital_filter_lds_kernel<LOmoms>),
                                  hipFuncAttributeMaxDynamicSharedMemorySize, (int)kDigitalLdsMax);
        if (e != hipSuccess) return e;
        attr = true;
      }
      const dim3 g((lines + (1 << shift) - 1) >> shift), b(kDigitalThreads);
      uint16_t* p = (uint16_t*)img;
      if (kernel == 4)
        hipLaunchKernelGGL(digital_filter_lds_kernel<LCbs>, g, b, lds, s, p, w, h, dir, shift, S);
      else
        hipLaunchKernelGGL(digital_filter_lds_kernel<LOmoms>, g, b, lds, s, p, w, h, dir, shift, S);
      hipError_t e = hipGetLastError();
      if (e != hipSuccess) return e;
      continue;
    }
    const int lanes = 4 * (dir == 0 ? h : w);
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
    CVR_KERNEL_SWITCH(downscale_kernel, kernel, g, b, s, src, fw, fh, dst, sw, sh);
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
