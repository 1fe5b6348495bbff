// march_common.h — device pieces shared by the ray-march kernels (rc1pass in
// raymarch.hip, directional occlusion in dos.hip): tile decomposition, the
// cell8 trilinear sample, TF classification, Blinn-Phong, ray setup, and the
// LDS TF staging / wave reductions.  CVR-SPEC arithmetic.
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>

#include "cvr_device.h"

namespace cvr {

// Pixel store: float4, or RGBA16F (round to nearest even, as imageStore into
// the reference's RGBA16F frame) packed in one uint2.
__device__ __forceinline__ void store_rgba(float4* out, long long i, float4 v, int half) {
  if (half) {
    const uint32_t x = f32_to_h16(v.x), y = f32_to_h16(v.y);
    const uint32_t z = f32_to_h16(v.z), w = f32_to_h16(v.w);
    reinterpret_cast<uint2*>(out)[i] = make_uint2(x | (y << 16), z | (w << 16));
  } else {
    out[i] = v;
  }
}

// ---------------------------------------------------------------------------
// Work decomposition
// ---------------------------------------------------------------------------

// Tile `t` (8x8 pixels), local pixel (lx, ly) -> pixel and output index.
// Unpacked: tiles are row-major over the (W/8)x(H/8) grid.  Packed (screen
// split): tile t = k*(T/8)^2 + j is sub-tile j of this rank's k-th TxT tile
// (split_tile, cvr_internal.h).
__device__ __forceinline__ void tile_pixel(const Rc1passArgs& A, int t, int lx, int ly, int& px,
                                           int& py, long long& out_idx) {
  if (!A.packed) {
    const int ntx8 = (A.W + 7) >> 3;
    const int ty = t / ntx8, tx = t - ty * ntx8;
    px = (tx << 3) | lx;
    py = (ty << 3) | ly;
    out_idx = (long long)py * A.W + px;
  } else {
    const int s = A.tile >> 3;               // 8x8 sub-tiles per tile row
    const int k = t / (s * s), j = t - k * s * s;
    int gx, gy;                              // this rank's k-th TxT tile
    split_tile(A.rank, A.nranks, k, A.ntx, gx, gy);
    const int ox = ((j % s) << 3) | lx, oy = ((j / s) << 3) | ly;
    px = gx * A.tile + ox;
    py = gy * A.tile + oy;
    out_idx = (long long)k * A.tile * A.tile + (long long)oy * A.tile + ox;
  }
}

// Workgroup b runs on XCD b % 8.  With t = b, tile column tx lands on XCD
// tx % 8 (every tile row has a multiple of 8 tiles at the bench sizes), so a
// tile's vertical neighbours share its XCD's L2 but its horizontal ones never
// do.  With column groups of G, columns [G c, G c + G)
// share an XCD instead, still dealt round-robin over the XCDs (balance), when
// the row has a multiple of 8 G tiles; otherwise t = b.  The shaded marches
// use G = 4 (CVR_SHADED_COLGROUP, tools/r02_s54.sh, frame ms, G = 1 -> 2 / 4 /
// 8): EBS 512^3 28.5 -> 27.2 / 27.0 / 30.0, DOS 15.56 -> 15.31 / 14.81 / 14.99.
template <int G>
__device__ __forceinline__ int screen_tile_of_block(const Rc1passArgs& A, int b, int nt) {
  if (G <= 1 || A.packed) return b;
  const int ntx8 = (A.W + 7) >> 3;
  if (ntx8 % (8 * G) != 0 || nt % ntx8 != 0) return b;
  const int per_row = ntx8 >> 3;               // tiles of one XCD in one row
  const int x = b & 7, j = b >> 3;
  const int ty = j / per_row, rem = j - ty * per_row;
  const int c = rem / G, r = rem - c * G;
  return ty * ntx8 + (c * 8 + x) * G + r;
}

// ---------------------------------------------------------------------------
// Sampling
// ---------------------------------------------------------------------------

// Buffer resource word 3 for gfx9-family raw buffers (32-bit data format, no
// swizzle); with num_records = 0xffffffff a 32-bit byte offset reaches 4 GiB.
constexpr int kBufferConfigDword = 0x00020000;

// 16-byte buffer load at a 32-bit byte offset from a scalar resource.
__device__ __forceinline__ uint4 buffer_load_u4(__amdgpu_buffer_rsrc_t r, uint32_t byte_off) {
  typedef unsigned int u4v __attribute__((ext_vector_type(4)));
  const u4v v = __builtin_amdgcn_raw_buffer_load_b128(r, (int)byte_off, 0, 0);
  return make_uint4(v.x, v.y, v.z, v.w);
}

// floor(x) as int in one instruction (x finite and in int range).
__device__ __forceinline__ int cvt_flr(float x) {
  int r;
  asm("v_cvt_flr_i32_f32 %0, %1" : "=v"(r) : "v"(x));
  return r;
}

// One sample's cell address + weights.  Along each axis the texel coordinate x
// lies in [-0.5, N-0.5] (a sample inside the box); cell floor(x)+1 of the
// (N+1)^3 cell grid holds texels (floor(x), floor(x)+1) clamped to the edge, so
// for x in [-1, 0) and [N-1, N) it holds one texel twice and any weight gives
// that texel exactly (fmaf(a, 0, v) = v for v >= 0) — the value GL's
// CLAMP_TO_EDGE and the oracle's clamped floor give.  Weight = v_fract(x).
struct SamplePos { uint32_t idx; float ax, ay, az; int ix, iy, iz; };

// a * b + c in one v_mad_i32_i24 (a, b signed 24-bit; the result mod 2^32)
__device__ __forceinline__ uint32_t mad_i24(int a, int b, uint32_t c) {
  uint32_t r;
  asm("v_mad_i32_i24 %0, %1, %2, %3" : "=v"(r) : "v"(a), "s"(b), "v"(c));
  return r;
}

__device__ __forceinline__ SamplePos sample_pos(float x, float y, float z, const Rc1passArgs& A) {
  SamplePos p;
  p.ax = __builtin_amdgcn_fractf(x); p.ay = __builtin_amdgcn_fractf(y); p.az = __builtin_amdgcn_fractf(z);
  p.ix = cvt_flr(x); p.iy = cvt_flr(y); p.iz = cvt_flr(z);
  // cell (ix+1, iy+1, iz+1), counted from the grid's first cell (ix, iy, iz >= -1)
  p.idx = (uint32_t)(__mul24(p.iz, A.cells.pitch_z) + __mul24(p.iy, A.cells.pitch_y) +
                     (p.ix + (int)A.cells.linear_origin));
  return p;
}

// The same for a position that may lie anywhere (not a live sample of a hit
// ray): clamped into the grid first, so the load stays in bounds.
__device__ __forceinline__ SamplePos sample_pos_clamped(float x, float y, float z,
                                                       const Rc1passArgs& A) {
  return sample_pos(__builtin_amdgcn_fmed3f(x, 0.0f, A.nm1[0]), __builtin_amdgcn_fmed3f(y, 0.0f, A.nm1[1]),
                    __builtin_amdgcn_fmed3f(z, 0.0f, A.nm1[2]), A);
}

// (float)hi - (float)lo of a packed fp16 pair, in ONE mixed-precision FMA
// (hi * 1.0 + (-lo), computed exactly then rounded once = the fp32 subtraction
// of the two exactly-converted halves).  ABS: |hi| - |lo| (the operand modifier
// is free): a density cell's sign bits carry the skip flags (cell_empty below).
template <bool ABS = false>
__device__ __forceinline__ float pair_diff(uint32_t w) {
  float d;
  if (ABS)
    asm("v_fma_mix_f32 %0, |%1|, 1.0, -|%1| op_sel:[1,0,0] op_sel_hi:[1,0,1]" : "=v"(d) : "v"(w));
  else
    asm("v_fma_mix_f32 %0, %1, 1.0, -%1 op_sel:[1,0,0] op_sel_hi:[1,0,1]" : "=v"(d) : "v"(w));
  return d;
}

// lerp(lo, hi, t) of a packed fp16 pair = fmaf(t, hi - lo, lo): two
// v_fma_mix_f32, the second taking lo straight from the low half.
template <bool ABS = false>
__device__ __forceinline__ float pair_lerp(uint32_t w, float t) {
  float r;
  if (ABS)
    asm("v_fma_mix_f32 %0, %1, %2, |%3| op_sel_hi:[0,0,1]" : "=v"(r) : "v"(t), "v"(pair_diff<true>(w)), "v"(w));
  else
    asm("v_fma_mix_f32 %0, %1, %2, %3 op_sel_hi:[0,0,1]" : "=v"(r) : "v"(t), "v"(pair_diff<false>(w)), "v"(w));
  return r;
}

typedef float f2v __attribute__((ext_vector_type(2)));

// cvr_expf_neg (cvr_device.h) of two arguments at once, bit for bit: every multiply
// and fma of the Cody-Waite reduction and the Horner polynomial is the same IEEE
// operation on each half (v_pk_mul_f32 / v_pk_fma_f32: two lanes' worth per issue
// slot on gfx950), only the rint, the conversion and the ldexp stay scalar.  For x
// in [-86, 0] (the host's exp_fast range); ~17 instructions for two samples instead
// of ~30.
__device__ __forceinline__ f2v cvr_expf_neg2(f2v x) {
  const f2v m = x * f2v{1.44269504088896341f, 1.44269504088896341f};
  const float n0 = rintf(m.x), n1 = rintf(m.y);
  const f2v n = {n0, n1};
  f2v r = __builtin_elementwise_fma(n, f2v{-0.693359375f, -0.693359375f}, x);
  r = __builtin_elementwise_fma(n, f2v{2.12194440e-4f, 2.12194440e-4f}, r);
  f2v p = {1.9875691500e-4f, 1.9875691500e-4f};
  p = __builtin_elementwise_fma(p, r, f2v{1.3981999507e-3f, 1.3981999507e-3f});
  p = __builtin_elementwise_fma(p, r, f2v{8.3334519073e-3f, 8.3334519073e-3f});
  p = __builtin_elementwise_fma(p, r, f2v{4.1665795894e-2f, 4.1665795894e-2f});
  p = __builtin_elementwise_fma(p, r, f2v{1.6666665459e-1f, 1.6666665459e-1f});
  p = __builtin_elementwise_fma(p, r, f2v{5.0000001201e-1f, 5.0000001201e-1f});
  const f2v r2 = r * r;
  const f2v v = __builtin_elementwise_fma(p, r2, r) + f2v{1.0f, 1.0f};
  return f2v{ldexpf(v.x, (int)n0), ldexpf(v.y, (int)n1)};
}

// Skip flags of the density cells (precompute.hip: build_cell_flags, rebuilt
// for every TF).  Densities are >= 0, so the 8 fp16 sign bits of a cell are
// free; every density read takes |corner| (ABS above, no extra instruction):
//  * bit 31 of .x: the cell is EMPTY — every density its corners can
//    interpolate to (a lerp stays within its end points) classifies to tau = 0,
//    so a sample there composites nothing (ray_marching_1p.comp:142);
//  * bits 31 of .y, .z, .w (an empty cell): q = min(d, 8) - 1, d = the
//    chessboard distance in cells to the nearest cell that is not empty, so
//    every cell within q of this one is empty too.
__device__ __forceinline__ bool cell_empty(uint4 r) { return (int)r.x < 0; }
__device__ __forceinline__ int cell_skip_q(uint4 r) {
  return (int)((r.y >> 31) | ((r.z >> 31) << 1) | ((r.w >> 31) << 2));
}
constexpr int kCellSkipCap = 8;            // distances stored up to 8 (q <= 7)
// The distance skip's margin in texels: absorbs the rounding of s and of the
// sample positions (raymarch.hip march_ray, shaded_march.h shaded_jobs_kernel).
constexpr float kSkipMarginTexels = 1.0f / 32.0f;

// PK: the two y lerps as one packed subtract and one packed fma, per lane the
// same two roundings as lerpf (the emission-absorption march: kernel -5 % with
// the buffer-offset and TF-weight changes of round 3; the Blinn-Phong march
// keeps the scalar form, where the register pairs cost it 10 %).  ABS (default):
// a density cell, whose sign bits are flags; the gradient cells are signed.
template <bool PK = false, bool ABS = true>
__device__ __forceinline__ float trilerp_cell(uint4 raw, float ax, float ay, float az) {
  float c00 = pair_lerp<ABS>(raw.x, ax);    // (v000, v100)
  float c10 = pair_lerp<ABS>(raw.y, ax);    // (v010, v110)
  float c01 = pair_lerp<ABS>(raw.z, ax);    // (v001, v101)
  float c11 = pair_lerp<ABS>(raw.w, ax);    // (v011, v111)
  if (PK) {
    const f2v lo = {c00, c01}, hi = {c10, c11};
    const f2v c = __builtin_elementwise_fma(f2v{ay, ay}, hi - lo, lo);
    return lerpf(c.x, c.y, az);
  }
  float c0 = lerpf(c00, c10, ay);
  float c1 = lerpf(c01, c11, ay);
  return lerpf(c0, c1, az);
}

// A GL_LINEAR weight at FB fraction bits (FB = 0: the exact float weight).
// rint(a * 2^FB) * 2^-FB: both scalings are exact, rint rounds half to even
// (the literal reading's nearbyint, oracle/glsl_literal.cpp weight()).
template <int FB>
__device__ __forceinline__ float filter_weight(float a) {
  if (FB == 0) return a;
  return __builtin_rintf(a * (float)(1 << FB)) * (1.0f / (float)(1 << FB));
}

template <int FB>
__device__ __forceinline__ void quantise_weights(SamplePos& p) {
  p.ax = filter_weight<FB>(p.ax);
  p.ay = filter_weight<FB>(p.ay);
  p.az = filter_weight<FB>(p.az);
}

// texture(TexTransferFunc, density) from the padded LDS table: x = d*n - 0.5
// reads the adjacent entries tfp[floor(x)+1], tfp[floor(x)+2]; d in [0,1]
// (a lerp of [0,1] values) keeps floor(x)+1 in [0, n].
template <int FB = 0>
__device__ __forceinline__ float4 classify(const float4* __restrict__ tfp, float fn, float dens) {
  float x = fmaf(dens, fn, -0.5f);
  // floor as int in one instruction and the weight as v_fract: equal to x -
  // floor(x) for x >= 0; for x in [-0.5, 0) both neighbours are T[0] (the
  // padded table), so the weight does not change the lerp
  float a = filter_weight<FB>(__builtin_amdgcn_fractf(x));
  int i = cvt_flr(x) + 1;
  float4 t0 = tfp[i], t1 = tfp[i + 1];
  return make_float4(lerpf(t0.x, t1.x, a), lerpf(t0.y, t1.y, a), lerpf(t0.z, t1.z, a),
                     lerpf(t0.w, t1.w, a));
}

// The gradient at a sample, from the gradient cell8 grid (precompute.hip:
// gradient_cells_kernel) at the volume cell's index: three 16-B loads, the same
// corners and lerp order as the per-voxel trilinear fetch.
__device__ __forceinline__ f3 sample_gradient_cell(const uint4* __restrict__ gcells,
                                                   const SamplePos& sp) {
  const uint4* g = gcells + 3 * (size_t)sp.idx;
  const uint4 gx = g[0], gy = g[1], gz = g[2];
  return f3{trilerp_cell<false, false>(gx, sp.ax, sp.ay, sp.az),
            trilerp_cell<false, false>(gy, sp.ax, sp.ay, sp.az),
            trilerp_cell<false, false>(gz, sp.ax, sp.ay, sp.az)};
}

// Blinn-Phong (ray_marching_1p.comp:48-81), CVR-SPEC arithmetic, for gradient g
// at world position wp (the sample's tex_pos minus half the grid).
__device__ __forceinline__ void phong_rgb(const Rc1passArgs& A, f3 g, f3 wp, f3 eye, float4& src) {
#ifdef CVR_PROBE_PHONG_NOMATH
  src.x *= g.x; src.y *= g.y; src.z *= g.z;
  return;
#endif
  if (g.x != 0.0f || g.y != 0.0f || g.z != 0.0f) {
    f3 n = normalize3(g);
    f3 Ld = normalize3(f3{A.light[0] - wp.x, A.light[1] - wp.y, A.light[2] - wp.z});
    f3 Ve = normalize3(f3{eye.x - wp.x, eye.y - wp.y, eye.z - wp.z});
    f3 Hv = normalize3(f3{Ve.x + Ld.x, Ve.y + Ld.y, Ve.z + Ld.z});
    float dd = fmaxf(0.0f, dot3(n, Ld));
    float ds = fmaxf(0.0f, dot3(Hv, n));
    float pw = cvr_powf_nb(ds, A.shininess);
    float f = fmaf(A.kd, dd, A.ka);
    src.x = fmaf(A.ispec[0] * A.ks, pw, src.x * f);
    src.y = fmaf(A.ispec[1] * A.ks, pw, src.y * f);
    src.z = fmaf(A.ispec[2] * A.ks, pw, src.z * f);
  }
}

__device__ __forceinline__ f3 phong_wpos(f3 dir, float t, f3 tpos, f3 hg) {
  return f3{fmaf(dir.x, t, tpos.x) - hg.x, fmaf(dir.y, t, tpos.y) - hg.y, fmaf(dir.z, t, tpos.z) - hg.z};
}

__device__ __forceinline__ f3 phong_gradient(const uint4* __restrict__ grad, const SamplePos& sp) {
#ifdef CVR_PROBE_PHONG_NOLOAD   // cost probes (tools/build_variant.sh), images wrong by design
  return f3{sp.ax, sp.ay, 1.0f};
#else
  return sample_gradient_cell(grad, sp);
#endif
}

// The sample's gradient fetch + Blinn-Phong, in the lane that marches it.
__device__ __forceinline__ void shade_phong(const Rc1passArgs& A, const uint4* __restrict__ grad,
                                            const SamplePos& sp, f3 dir, float t, f3 tpos, f3 hg,
                                            f3 eye, float4& src) {
  const f3 g = phong_gradient(grad, sp);
  phong_rgb(A, g, phong_wpos(dir, t, tpos, hg), eye, src);
}

// ---------------------------------------------------------------------------
// The ray
// ---------------------------------------------------------------------------

struct Ray {
  f3 cam;                // camera_dir: normalize(d * mat3(View)) (normalised once)
  f3 dir, tpos, o, dt;   // direction, entry point (texture space), texel-space origin/step
  f3 inv_dt;             // 1 / dt (macro-cell exits)
  float D;               // distance to evaluate, |tfar - tnear|
  float tnear, tfar;     // RayAABBIntersection's rtnear (clamped to >= 0) and rtfar
  bool outside;          // box behind the eye (tfar < 0): the march runs outside the grid
};

// Ray generation + slab test, ray_marching_1p.comp:93-121 and
// ray_bbox_intersection.comp:18-52.  Returns false for a miss.
__device__ __forceinline__ bool ray_setup(const Rc1passArgs& A, int px, int py, Ray& r) {
  float fx = (float)px + 0.5f, fy = (float)py + 0.5f;
  float vx = fmaf(fx / (float)A.W, 2.0f, -1.0f);
  float vy = fmaf(fy / (float)A.H, 2.0f, -1.0f);
  f3 c{(vx * A.tan_half_fovy) * A.aspect, vy * A.tan_half_fovy, -1.0f};
  f3 d{dot3(c, f3{A.col0[0], A.col0[1], A.col0[2]}), dot3(c, f3{A.col1[0], A.col1[1], A.col1[2]}),
       dot3(c, f3{A.col2[0], A.col2[1], A.col2[2]})};
  const f3 cam = normalize3(d);
  f3 dir = normalize3(cam);                // RayAABBIntersection normalises again (:219)
  r.cam = cam;
  f3 inv{1.0f / dir.x, 1.0f / dir.y, 1.0f / dir.z};
  const f3 eye{A.eye[0], A.eye[1], A.eye[2]};
  const f3 hg{A.half_grid[0], A.half_grid[1], A.half_grid[2]};
  f3 ta{inv.x * (-hg.x - eye.x), inv.y * (-hg.y - eye.y), inv.z * (-hg.z - eye.z)};
  f3 tb{inv.x * (hg.x - eye.x), inv.y * (hg.y - eye.y), inv.z * (hg.z - eye.z)};
  float tnear = fmaxf(fmaxf(fminf(ta.x, tb.x), fminf(ta.y, tb.y)), fminf(ta.z, tb.z));
  float tfar = fminf(fminf(fmaxf(ta.x, tb.x), fmaxf(ta.y, tb.y)), fmaxf(ta.z, tb.z));
  bool hit = tfar > tnear;
  // With tfar >= 0 the marched segment [max(tnear, 0), tfar] lies in the box;
  // a box behind the eye is still "hit" and marched from the eye outward
  // (the reference samples the clamped texture there), so those positions
  // must be clamped before addressing cells.
  r.outside = !(tfar >= 0.0f);
  tnear = fmaxf(tnear, 0.0f);
  r.tnear = tnear;
  r.tfar = tfar;
  r.dir = dir;
  r.D = fabsf(tfar - tnear);
  r.tpos = f3{fmaf(dir.x, tnear, eye.x) + hg.x, fmaf(dir.y, tnear, eye.y) + hg.y,
              fmaf(dir.z, tnear, eye.z) + hg.z};
  r.o = f3{fmaf(r.tpos.x, A.n_over_g[0], -0.5f), fmaf(r.tpos.y, A.n_over_g[1], -0.5f),
           fmaf(r.tpos.z, A.n_over_g[2], -0.5f)};
  r.dt = f3{dir.x * A.n_over_g[0], dir.y * A.n_over_g[1], dir.z * A.n_over_g[2]};
  if (A.occ) r.inv_dt = f3{1.0f / r.dt.x, 1.0f / r.dt.y, 1.0f / r.dt.z};
  return hit;
}

__device__ __forceinline__ void load_tf_lds(float4* tfp, const float4* __restrict__ tf_g, int n) {
  // Padded TF: tfp[k] = T[clamp(k-1, 0, n-1)], k in [0, n+1] (CLAMP_TO_EDGE folded in).
  for (int i = threadIdx.x; i < n + 2; i += blockDim.x) tfp[i] = tf_g[min(max(i - 1, 0), n - 1)];
  __syncthreads();
}

__device__ __forceinline__ uint32_t wave_max(uint32_t m) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) m = max(m, (uint32_t)__shfl_xor((int)m, off, 64));
  return m;
}

__device__ __forceinline__ unsigned long long wave_sum(unsigned long long v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
  return v;
}

}  // namespace cvr
