// raymarch.hip — gfx950 kernels of the structured single-pass ray-caster.
//
// Re-designs cppvolrend's ray_marching_1p.comp (rc1pass) for CDNA4:
//   * one wave64 = one 8x8 pixel tile (the reference's 8x8 local size,
//     rc1prenderer.cpp:77-86);
//   * no HIP texture objects on gfx950, so trilinear filtering is done in
//     software from a padded "cell8" layout: every sample is ONE 16-byte load of
//     the 8 fp16 corners GL_LINEAR + CLAMP_TO_EDGE would read from the R16F
//     volume (libs/volvis_utils/utils.cpp:20-56), bricked 4x4x4 for locality;
//   * the 1D transfer function (RGBA16F, GenerateTexture_1D_RGBt) lives in LDS;
//   * per-ray state in registers; K samples addressed and fetched per batch
//     (K x 16 B in flight per lane), classified, then composited in order with
//     the per-lane early ray termination (dst.a > 0.99);
//   * scheduling: one wave tile per workgroup; each XCD owns one horizontal
//     band of the screen (L2 locality) and receives its tiles longest-first
//     when the previous frame's per-tile costs are known (LPT), the longest
//     ones at raised wave priority.
//
// Arithmetic follows CVR-SPEC: explicit fmaf, IEEE div/sqrt, the
// polynomial cvr_expf / cvr_powf.  The file is compiled with -ffp-contract=off
// so results are bit-identical to oracle/cvr_oracle.cpp.
#include <hip/hip_runtime.h>
#include <cstdint>

#include "cvr_device.h"

namespace cvr {

constexpr int kMaxTfLds = 4096;

// ---------------------------------------------------------------------------
// Work decomposition
// ---------------------------------------------------------------------------

// Wave tile `t` (8x8 pixels) -> pixel of `lane` and its output index.
// Unpacked: tiles are row-major over the (W/8)x(H/8) grid.  Packed (screen
// split): tile t = k*(T/8)^2 + j is sub-tile j of this rank's k-th TxT tile.
__device__ __forceinline__ void tile_pixel(const Rc1passArgs& A, int t, int lane, int& px, int& py,
                                           long long& out_idx) {
  const int lx = lane & 7, ly = lane >> 3;
  if (!A.packed) {
    const int ntx8 = (A.W + 7) >> 3;
    const int ty = t / ntx8, tx = t - ty * ntx8;
    px = (tx << 3) | lx;
    py = (ty << 3) | ly;
    out_idx = (long long)py * A.W + px;
  } else {
    const int s = A.tile >> 3;               // 8x8 sub-tiles per tile row
    const int k = t / (s * s), j = t - k * s * s;
    const int g = A.rank + k * A.nranks;     // global tile index
    const int gy = g / A.ntx, gx = g - gy * A.ntx;
    const int ox = ((j % s) << 3) | lx, oy = ((j / s) << 3) | ly;
    px = gx * A.tile + ox;
    py = gy * A.tile + oy;
    out_idx = (long long)k * A.tile * A.tile + (long long)oy * A.tile + ox;
  }
}

// ---------------------------------------------------------------------------
// The ray
// ---------------------------------------------------------------------------

// One sample's cell address + weights (stage 1 of the batched march).
struct SamplePos { int idx; float ax, ay, az; int ix, iy, iz; };   // idx may be < 0 (linear: origin-relative)

template <int LAYOUT>
__device__ __forceinline__ SamplePos sample_pos(float x, float y, float z, const Rc1passArgs& A,
                                                uint32_t bxby) {
  // GL_LINEAR texel-centre convention.  Clamping to [-1, N-1] (one v_med3) is
  // value-neutral under CLAMP_TO_EDGE and keeps the padded cell index
  // floor(x)+1 inside [0, N].
  x = __builtin_amdgcn_fmed3f(x, -1.0f, A.nm1[0]);
  y = __builtin_amdgcn_fmed3f(y, -1.0f, A.nm1[1]);
  z = __builtin_amdgcn_fmed3f(z, -1.0f, A.nm1[2]);
  float fx = floorf(x), fy = floorf(y), fz = floorf(z);
  SamplePos p;
  p.ax = x - fx; p.ay = y - fy; p.az = z - fz;
  p.ix = (int)fx; p.iy = (int)fy; p.iz = (int)fz;
  if (LAYOUT == kLayoutLinear) {
    // cell (ix+1, iy+1, iz+1) of the (N+1)^3 grid; the +1 offsets live in the base pointer
    p.idx = __mul24(p.iz, A.cells.pitch_z) + __mul24(p.iy, A.cells.pitch_y) + p.ix;
  } else {
    uint32_t cx = (uint32_t)(p.ix + 1), cy = (uint32_t)(p.iy + 1), cz = (uint32_t)(p.iz + 1);
    uint32_t brick = __umul24(cz >> 2, bxby) + __umul24(cy >> 2, (uint32_t)A.cells.bx) + (cx >> 2);
    p.idx = (int)((brick << 6) | ((cz & 3u) << 4) | ((cy & 3u) << 2) | (cx & 3u));
  }
  return p;
}

// (float)hi - (float)lo of a packed fp16 pair, in ONE mixed-precision FMA
// (hi * 1.0 + (-lo), computed exactly then rounded once = the fp32 subtraction
// of the two exactly-converted halves).
__device__ __forceinline__ float pair_diff(uint32_t w) {
  float d;
  asm("v_fma_mix_f32 %0, %1, 1.0, -%1 op_sel:[1,0,0] op_sel_hi:[1,0,1]" : "=v"(d) : "v"(w));
  return d;
}

// lerp(lo, hi, t) of a packed fp16 pair = fmaf(t, hi - lo, lo): two v_fma_mix_f32.
__device__ __forceinline__ float pair_lerp(uint32_t w, float t) {
  half2_t p = __builtin_bit_cast(half2_t, w);
  return fmaf(t, pair_diff(w), (float)p.x);
}

__device__ __forceinline__ float trilerp_cell(uint4 raw, float ax, float ay, float az) {
  float c00 = pair_lerp(raw.x, ax);    // (v000, v100)
  float c10 = pair_lerp(raw.y, ax);    // (v010, v110)
  float c01 = pair_lerp(raw.z, ax);    // (v001, v101)
  float c11 = pair_lerp(raw.w, ax);    // (v011, v111)
  float c0 = lerpf(c00, c10, ay);
  float c1 = lerpf(c01, c11, ay);
  return lerpf(c0, c1, az);
}

// Blinn-Phong (ray_marching_1p.comp:48-81), CVR-SPEC arithmetic.
__device__ __forceinline__ void shade_phong(const Rc1passArgs& A, const uint2* __restrict__ grad,
                                            const SamplePos& sp, f3 dir, float t, f3 tpos, f3 hg,
                                            f3 eye, float4& src) {
  Texel tx;
  tx.ix = sp.ix; tx.iy = sp.iy; tx.iz = sp.iz;
  tx.ax = sp.ax; tx.ay = sp.ay; tx.az = sp.az;
  f3 g = sample_gradient(grad, A.N, tx);
  if (g.x != 0.0f || g.y != 0.0f || g.z != 0.0f) {
    f3 wp{fmaf(dir.x, t, tpos.x) - hg.x, fmaf(dir.y, t, tpos.y) - hg.y, fmaf(dir.z, t, tpos.z) - hg.z};
    f3 n = normalize3(g);
    f3 Ld = normalize3(f3{A.light[0] - wp.x, A.light[1] - wp.y, A.light[2] - wp.z});
    f3 Ve = normalize3(f3{eye.x - wp.x, eye.y - wp.y, eye.z - wp.z});
    f3 Hv = normalize3(f3{Ve.x + Ld.x, Ve.y + Ld.y, Ve.z + Ld.z});
    float dd = fmaxf(0.0f, dot3(n, Ld));
    float ds = fmaxf(0.0f, dot3(Hv, n));
    float pw = cvr_powf(ds, A.shininess);
    float f = fmaf(A.kd, dd, A.ka);
    src.x = fmaf(A.ispec[0] * A.ks, pw, src.x * f);
    src.y = fmaf(A.ispec[1] * A.ks, pw, src.y * f);
    src.z = fmaf(A.ispec[2] * A.ks, pw, src.z * f);
  }
}

// One ray of ray_marching_1p.comp:87-176.  The arithmetic per sample is
// exactly the reference's sequential loop (s accumulates h one step at a time);
// the batching only changes when the loads are issued.
template <int K, bool PHONG, int LAYOUT>
__device__ __forceinline__ void march_ray(const Rc1passArgs& A, const uint4* __restrict__ cells,
                                          const uint2* __restrict__ grad,
                                          const float4* __restrict__ tfp, int px, int py,
                                          float4& dst, uint32_t& cnt) {
  dst = make_float4(0.f, 0.f, 0.f, 0.f);
  cnt = 0;
  // ray generation, ray_marching_1p.comp:93-99
  float fx = (float)px + 0.5f, fy = (float)py + 0.5f;
  float vx = fmaf(fx / (float)A.W, 2.0f, -1.0f);
  float vy = fmaf(fy / (float)A.H, 2.0f, -1.0f);
  f3 c{(vx * A.tan_half_fovy) * A.aspect, vy * A.tan_half_fovy, -1.0f};
  f3 d{dot3(c, f3{A.col0[0], A.col0[1], A.col0[2]}), dot3(c, f3{A.col1[0], A.col1[1], A.col1[2]}),
       dot3(c, f3{A.col2[0], A.col2[1], A.col2[2]})};
  f3 dir = normalize3(normalize3(d));
  // slab test, ray_bbox_intersection.comp:18-30
  f3 inv{1.0f / dir.x, 1.0f / dir.y, 1.0f / dir.z};
  const f3 eye{A.eye[0], A.eye[1], A.eye[2]};
  const f3 hg{A.half_grid[0], A.half_grid[1], A.half_grid[2]};
  f3 ta{inv.x * (-hg.x - eye.x), inv.y * (-hg.y - eye.y), inv.z * (-hg.z - eye.z)};
  f3 tb{inv.x * (hg.x - eye.x), inv.y * (hg.y - eye.y), inv.z * (hg.z - eye.z)};
  float tnear = fmaxf(fmaxf(fminf(ta.x, tb.x), fminf(ta.y, tb.y)), fminf(ta.z, tb.z));
  float tfar = fminf(fminf(fmaxf(ta.x, tb.x), fmaxf(ta.y, tb.y)), fmaxf(ta.z, tb.z));
  bool hit = tfar > tnear;
  tnear = fmaxf(tnear, 0.0f);
  if (!hit) return;   // misses keep the cleared (0,0,0,0), renderoutputframe.cpp:187-190
  const float D = fabsf(tfar - tnear);
  const f3 tpos{fmaf(dir.x, tnear, eye.x) + hg.x, fmaf(dir.y, tnear, eye.y) + hg.y,
                fmaf(dir.z, tnear, eye.z) + hg.z};
  const f3 o{fmaf(tpos.x, A.n_over_g[0], -0.5f), fmaf(tpos.y, A.n_over_g[1], -0.5f),
             fmaf(tpos.z, A.n_over_g[2], -0.5f)};
  const f3 dt{dir.x * A.n_over_g[0], dir.y * A.n_over_g[1], dir.z * A.n_over_g[2]};
  const float step = A.step;
  const uint32_t bxby = (uint32_t)A.cells.bx * (uint32_t)A.cells.by;
  const int n = A.tf_n;
  const float fn = (float)n;
  float s = 0.0f;
  bool done = !(s < D);
  while (!done) {
    // stage 1: the next K sample positions (sequential s += h) and their loads
    float hj[K], tj[K];
    bool vj[K];
    SamplePos sp[K];
    uint4 raw[K];
    float ss = s;
#pragma unroll
    for (int j = 0; j < K; j++) {
      vj[j] = ss < D;
      hj[j] = fminf(step, D - ss);
      tj[j] = fmaf(hj[j], 0.5f, ss);
      ss = ss + hj[j];
      sp[j] = sample_pos<LAYOUT>(fmaf(dt.x, tj[j], o.x), fmaf(dt.y, tj[j], o.y),
                                 fmaf(dt.z, tj[j], o.z), A, bxby);
      raw[j] = cells[sp[j].idx];
    }
    // stage 2: density and transfer-function classification (padded LDS table:
    // x = d*n - 0.5 reads the adjacent entries tfp[floor(x)+1], tfp[floor(x)+2])
    float4 src[K];
#pragma unroll
    for (int j = 0; j < K; j++) {
      float dens = trilerp_cell(raw[j], sp[j].ax, sp[j].ay, sp[j].az);
      float x = fmaf(dens, fn, -0.5f);
      float fl = floorf(x);
      float a = x - fl;
      int i = (int)fl + 1;   // dens in [0,1] (a lerp of [0,1] values) -> i in [0, n]
      float4 t0 = tfp[i], t1 = tfp[i + 1];
      src[j] = make_float4(lerpf(t0.x, t1.x, a), lerpf(t0.y, t1.y, a), lerpf(t0.z, t1.z, a),
                           lerpf(t0.w, t1.w, a));
    }
    // stage 3: front-to-back composite + ERT, in sample order
#pragma unroll
    for (int j = 0; j < K; j++) {
      if (!done) {
        if (!vj[j]) {
          done = true;
        } else {
          cnt++;
          float4 sc = src[j];
          if (sc.w > 0.0f) {
            if (PHONG) shade_phong(A, grad, sp[j], dir, tj[j], tpos, hg, eye, sc);
            float a = 1.0f - cvr_expf_nb(-(sc.w * hj[j]));
            float om = 1.0f - dst.w;
            dst.x = fmaf(om, sc.x * a, dst.x);
            dst.y = fmaf(om, sc.y * a, dst.y);
            dst.z = fmaf(om, sc.z * a, dst.z);
            dst.w = fmaf(om, a, dst.w);
            if (dst.w > 0.99f) done = true;
          }
        }
      }
    }
    s = ss;
    if (!(s < D)) done = true;
  }
}

__device__ __forceinline__ void load_tf_lds(float4* tfp, const float4* __restrict__ tf_g, int n) {
  // Padded TF: tfp[k] = T[clamp(k-1, 0, n-1)], k in [0, n+1] (CLAMP_TO_EDGE folded in).
  for (int i = threadIdx.x; i < n + 2; i += blockDim.x) tfp[i] = tf_g[min(max(i - 1, 0), n - 1)];
  __syncthreads();
}

// Writes one wave tile's results; lanes outside the image store zeros only in
// the packed layout (edge-tile padding).
__device__ __forceinline__ void finish_tile(const Rc1passArgs& A, int t, int lane, bool inside,
                                            long long oidx, float4 dst, uint32_t cnt,
                                            float4* __restrict__ out, uint32_t* __restrict__ samples,
                                            unsigned long long* __restrict__ total,
                                            uint32_t* __restrict__ tile_cost) {
  if (inside || A.packed) {
    out[oidx] = dst;
    if (samples) samples[oidx] = cnt;
  }
  if (total) {
    unsigned long long v = cnt;
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
    if (lane == 0 && v) atomicAdd(total, v);
  }
  if (tile_cost) {   // the tile's critical path (its longest ray), for the next frame's order
    uint32_t m = cnt;
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) m = max(m, (uint32_t)__shfl_xor((int)m, off, 64));
    if (lane == 0) tile_cost[t] = m;
  }
}

// ---------------------------------------------------------------------------
// Kernels
// ---------------------------------------------------------------------------

// One workgroup = one wave = one 8x8 tile, so a long ray only ever holds its
// own wave slot.  Tile t comes from the LPT order when given (each XCD gets its
// screen band longest-first), else from the XCD-banded remap (blocks b and b+8
// share an XCD, so XCD b%8 gets one contiguous band of the screen).  The first
// `boost` tiles of every band (its longest, by the previous frame) raise their
// wave priority so their long dependency chains issue ahead of short tiles.
template <int K, bool PHONG, int LAYOUT>
__global__ void __launch_bounds__(64)
rc1pass_tile_kernel(Rc1passArgs A, const uint4* __restrict__ cells,
                    const uint2* __restrict__ grad, const float4* __restrict__ tf_g,
                    float4* __restrict__ out, uint32_t* __restrict__ samples,
                    unsigned long long* __restrict__ total, const int* __restrict__ order,
                    uint32_t* __restrict__ tile_cost, int boost) {
  extern __shared__ float4 tfp[];
  load_tf_lds(tfp, tf_g, A.tf_n);
  const int b = blockIdx.x, nt = A.ntiles;
  int t;
  if (order) {
    t = order[b];
    if (t < 0) return;   // padding slot of a shorter band
    if ((b >> 3) < boost) __builtin_amdgcn_s_setprio(2);
  } else if ((nt & 7) == 0) {
    t = (b & 7) * (nt >> 3) + (b >> 3);
  } else {
    t = b;
  }
  const int lane = threadIdx.x;
  unsigned long long t_start = 0;
  if (A.tile_stats) t_start = __builtin_amdgcn_s_memrealtime();
  int px, py;
  long long oidx;
  tile_pixel(A, t, lane, px, py, oidx);
  const bool inside = px < A.W && py < A.H;
  float4 dst = make_float4(0.f, 0.f, 0.f, 0.f);
  uint32_t cnt = 0;
  if (inside) march_ray<K, PHONG, LAYOUT>(A, cells, grad, tfp, px, py, dst, cnt);
  finish_tile(A, t, lane, inside, oidx, dst, cnt, out, samples, total, tile_cost);
  if (A.tile_stats) {   // diagnostics: 100 MHz start/end stamps, longest ray, placement
    uint32_t m = cnt;
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) m = max(m, (uint32_t)__shfl_xor((int)m, off, 64));
    unsigned long long t_end = __builtin_amdgcn_s_memrealtime();
    unsigned hw;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
    if (lane == 0) {
      A.tile_stats[t * 4 + 0] = t_start;
      A.tile_stats[t * 4 + 1] = t_end;
      A.tile_stats[t * 4 + 2] = m;
      A.tile_stats[t * 4 + 3] = ((unsigned long long)b << 32) | hw;
    }
  }
}

// LPT order from the previous frame's per-tile costs: workgroup `seg` sorts the
// tiles of XCD band seg (bitonic sort in LDS, descending cost, ties by index)
// and deals them to physical blocks seg, seg+8, seg+16, ... (the blocks XCD
// seg receives), so every XCD keeps its screen band and starts with its
// longest tiles.
__global__ void __launch_bounds__(1024)
tile_order_kernel(const uint32_t* __restrict__ tile_cost, int nunits, int* __restrict__ order) {
  extern __shared__ unsigned long long keys[];
  const int b0 = (blockIdx.x * nunits) >> 3, b1 = ((blockIdx.x + 1) * nunits) >> 3;
  const int seg = b1 - b0;
  int P = 1;
  while (P < seg) P <<= 1;
  for (int i = threadIdx.x; i < P; i += blockDim.x) {
    unsigned long long k = 0;
    if (i < seg) {
      uint32_t u = (uint32_t)(b0 + i);
      k = ((unsigned long long)tile_cost[u] << 32) | (0xffffffffu - u);
    }
    keys[i] = k;
  }
  __syncthreads();
  for (int size = 2; size <= P; size <<= 1) {
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      for (int i = threadIdx.x; i < P; i += blockDim.x) {
        int j = i ^ stride;
        if (j > i) {
          bool desc = (i & size) == 0;
          unsigned long long a = keys[i], b = keys[j];
          if ((a < b) == desc) { keys[i] = b; keys[j] = a; }
        }
      }
      __syncthreads();
    }
  }
  // band sizes differ by at most one: bands with the extra tile come last
  // ((b*n)>>3 rounding), so physical block seg + 8*i exists for every i < seg
  // as long as the grid is launched with 8*ceil(n/8) blocks, see launcher
  for (int i = threadIdx.x; i < seg; i += blockDim.x) {
    int u = (int)(0xffffffffu - (uint32_t)keys[i]);
    order[blockIdx.x + 8 * i] = u;
  }
}

// ---------------------------------------------------------------------------
// Launchers
// ---------------------------------------------------------------------------

template <int K, bool PHONG, int LAYOUT>
static hipError_t launch_kpl(const Ctx& c, const Rc1passArgs& a, float4* out, uint32_t* samples,
                             unsigned long long* total, const int* order, uint32_t* tile_cost,
                             const RenderPlan& plan, hipStream_t s) {
  size_t lds = (size_t)(a.tf_n + 2) * sizeof(float4);
  const uint4* cells = (const uint4*)c.d_cells;
  if (LAYOUT == kLayoutLinear) cells += c.cells.linear_origin;   // cell (1,1,1) <-> texel (0,0,0)
  // with an order the grid is 8*ceil(n/8) blocks; the padding blocks (unused
  // order slots) are marked -1 and exit at once
  int grid = order ? plan.order_slots : plan.ntiles;
  hipLaunchKernelGGL((rc1pass_tile_kernel<K, PHONG, LAYOUT>), dim3(grid), dim3(64), lds, s, a,
                     cells, (const uint2*)c.d_grad, (const float4*)c.d_tf, out, samples, total,
                     order, tile_cost, order ? plan.boost : 0);
  return hipGetLastError();
}

template <int K, bool PHONG>
static hipError_t launch_kp(const Ctx& c, const Rc1passArgs& a, float4* out, uint32_t* samples,
                            unsigned long long* total, const int* order, uint32_t* tile_cost,
                            const RenderPlan& plan, hipStream_t s) {
  return c.cells.layout == kLayoutLinear
             ? launch_kpl<K, PHONG, kLayoutLinear>(c, a, out, samples, total, order, tile_cost, plan, s)
             : launch_kpl<K, PHONG, kLayoutBrick>(c, a, out, samples, total, order, tile_cost, plan, s);
}

template <int K>
static hipError_t launch_k(const Ctx& c, const Rc1passArgs& a, bool phong, float4* out,
                           uint32_t* samples, unsigned long long* total, const int* order,
                           uint32_t* tile_cost, const RenderPlan& plan, hipStream_t s) {
  return phong ? launch_kp<K, true>(c, a, out, samples, total, order, tile_cost, plan, s)
               : launch_kp<K, false>(c, a, out, samples, total, order, tile_cost, plan, s);
}

hipError_t launch_rc1pass(const Ctx& c, const Rc1passArgs& a, bool phong, float4* out,
                          uint32_t* samples, unsigned long long* total, const int* order,
                          uint32_t* tile_cost, const RenderPlan& plan, hipStream_t s) {
  if (a.ntiles <= 0) return hipSuccess;
  if (a.tf_n > kMaxTfLds) return hipErrorInvalidValue;
  switch (c.batch) {
    case 2: return launch_k<2>(c, a, phong, out, samples, total, order, tile_cost, plan, s);
    case 8: return launch_k<8>(c, a, phong, out, samples, total, order, tile_cost, plan, s);
    default: return launch_k<4>(c, a, phong, out, samples, total, order, tile_cost, plan, s);
  }
}

__global__ void fill_int_kernel(int* p, int n, int v) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) p[i] = v;
}

hipError_t launch_tile_order(const uint32_t* tile_cost, const RenderPlan& plan, int* order,
                             hipStream_t s) {
  const int nunits = plan.ntiles;
  const int seg = (nunits + 7) >> 3;
  int P = 1;
  while (P < seg) P <<= 1;
  if (P > 16384) return hipErrorInvalidValue;
  if (plan.order_slots != nunits)   // padding slots of short bands
    hipLaunchKernelGGL(fill_int_kernel, dim3((plan.order_slots + 255) / 256), dim3(256), 0, s,
                       order, plan.order_slots, -1);
  hipLaunchKernelGGL(tile_order_kernel, dim3(8), dim3(1024), (size_t)P * 8, s, tile_cost, nunits,
                     order);
  return hipGetLastError();
}

}  // namespace cvr
