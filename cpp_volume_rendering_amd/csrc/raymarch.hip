// raymarch.hip — gfx950 kernels of the structured single-pass ray-caster.
//
// Re-designs cppvolrend's ray_marching_1p.comp (rc1pass) for CDNA4:
//   * one wave64 = one 8x8 pixel tile (the reference's 8x8 local size,
//     rc1prenderer.cpp:77-86), four waves per 256-thread block (16x16 px);
//   * no HIP texture objects on gfx950, so trilinear filtering is done in
//     software from a padded "cell8" layout: every sample is ONE 16-byte load of
//     the 8 fp16 corners GL_LINEAR + CLAMP_TO_EDGE would read from the R16F
//     volume (libs/volvis_utils/utils.cpp:20-56), bricked 4x4x4 for locality;
//   * the 1D transfer function (RGBA16F, GenerateTexture_1D_RGBt) lives in LDS;
//   * per-ray state in registers, per-lane early ray termination (dst.a > 0.99);
//   * blocks are remapped so that each XCD renders one contiguous band of the
//     screen (neighbouring rays share that XCD's L2).
//
// Arithmetic follows CVR-SPEC: explicit fmaf, IEEE div/sqrt, the
// polynomial cvr_expf / cvr_powf.  The file is compiled with -ffp-contract=off
// so results are bit-identical to oracle/cvr_oracle.cpp.
#include <hip/hip_runtime.h>
#include <cstdint>

#include "cvr_internal.h"

namespace cvr {

typedef _Float16 half2_t __attribute__((ext_vector_type(2)));

__device__ __forceinline__ float lerpf(float a, float b, float t) { return fmaf(t, b - a, a); }

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

// pow(x, y) for x >= 0, CVR-SPEC (identical to oracle cvr_powf)
__device__ __forceinline__ float cvr_powf(float x, float y) {
  if (x != x || y != y) return x + y;
  if (!(x > 0.0f) || x < 1.17549435e-38f) {
    if (y > 0.0f) return 0.0f;
    if (y == 0.0f) return 1.0f;
    return __builtin_inff();
  }
  if (x == __builtin_inff()) return y > 0.0f ? __builtin_inff() : (y == 0.0f ? 1.0f : 0.0f);
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
  lnx = fmaf(fe, 0.693359375f, lnx);
  return cvr_expf(y * lnx);
}

struct f3 { float x, y, z; };
__device__ __forceinline__ float dot3(f3 a, f3 b) { return fmaf(a.z, b.z, fmaf(a.y, b.y, a.x * b.x)); }
__device__ __forceinline__ f3 normalize3(f3 v) {
  float inv = 1.0f / sqrtf(dot3(v, v));
  return f3{v.x * inv, v.y * inv, v.z * inv};
}

__device__ __forceinline__ uint32_t brick_index(const CellGrid& g, int a, int b, int c) {
  uint32_t brick = ((uint32_t)(c >> 2) * (uint32_t)g.by + (uint32_t)(b >> 2)) * (uint32_t)g.bx + (uint32_t)(a >> 2);
  return (brick << 6) | ((uint32_t)(c & 3) << 4) | ((uint32_t)(b & 3) << 2) | (uint32_t)(a & 3);
}

// Texel-space coordinate -> cell index + fractional weights.  Clamping x to
// [-1, N-1] does not change the filtered value (CLAMP_TO_EDGE), it only keeps
// the cell index inside [0, N].
struct Texel { int ix, iy, iz; float ax, ay, az; };
__device__ __forceinline__ Texel texel(float x, float y, float z, const float nm1[3]) {
  x = fminf(fmaxf(x, -1.0f), nm1[0]);
  y = fminf(fmaxf(y, -1.0f), nm1[1]);
  z = fminf(fmaxf(z, -1.0f), nm1[2]);
  float fx = floorf(x), fy = floorf(y), fz = floorf(z);
  Texel t;
  t.ax = x - fx; t.ay = y - fy; t.az = z - fz;
  t.ix = (int)fx; t.iy = (int)fy; t.iz = (int)fz;
  return t;
}

__device__ __forceinline__ float sample_cells(const uint4* __restrict__ cells, const CellGrid& g,
                                              const Texel& t) {
  uint4 raw = cells[brick_index(g, t.ix + 1, t.iy + 1, t.iz + 1)];
  float v000, v100, v010, v110, v001, v101, v011, v111;
  h2f2(raw.x, v000, v100);
  h2f2(raw.y, v010, v110);
  h2f2(raw.z, v001, v101);
  h2f2(raw.w, v011, v111);
  float c00 = lerpf(v000, v100, t.ax);
  float c10 = lerpf(v010, v110, t.ax);
  float c01 = lerpf(v001, v101, t.ax);
  float c11 = lerpf(v011, v111, t.ax);
  float c0 = lerpf(c00, c10, t.ay);
  float c1 = lerpf(c01, c11, t.ay);
  return lerpf(c0, c1, t.az);
}

// Gradient: 4 x fp16 (x, y, z, 0) per voxel, x-fastest, trilinear per channel.
__device__ __forceinline__ f3 sample_gradient(const uint2* __restrict__ grad, const int N[3],
                                              const Texel& t) {
  int x0 = max(t.ix, 0), x1 = min(t.ix + 1, N[0] - 1);
  int y0 = max(t.iy, 0), y1 = min(t.iy + 1, N[1] - 1);
  int z0 = max(t.iz, 0), z1 = min(t.iz + 1, N[2] - 1);
  size_t sx = 1, sy = (size_t)N[0], sz = (size_t)N[0] * N[1];
  uint2 q[8];
  q[0] = grad[x0 * sx + y0 * sy + z0 * sz];
  q[1] = grad[x1 * sx + y0 * sy + z0 * sz];
  q[2] = grad[x0 * sx + y1 * sy + z0 * sz];
  q[3] = grad[x1 * sx + y1 * sy + z0 * sz];
  q[4] = grad[x0 * sx + y0 * sy + z1 * sz];
  q[5] = grad[x1 * sx + y0 * sy + z1 * sz];
  q[6] = grad[x0 * sx + y1 * sy + z1 * sz];
  q[7] = grad[x1 * sx + y1 * sy + z1 * sz];
  float vx[8], vy[8], vz[8];
#pragma unroll
  for (int i = 0; i < 8; i++) {
    float dummy;
    h2f2(q[i].x, vx[i], vy[i]);
    h2f2(q[i].y, vz[i], dummy);
  }
  f3 r;
  {
    float c00 = lerpf(vx[0], vx[1], t.ax), c10 = lerpf(vx[2], vx[3], t.ax);
    float c01 = lerpf(vx[4], vx[5], t.ax), c11 = lerpf(vx[6], vx[7], t.ax);
    r.x = lerpf(lerpf(c00, c10, t.ay), lerpf(c01, c11, t.ay), t.az);
  }
  {
    float c00 = lerpf(vy[0], vy[1], t.ax), c10 = lerpf(vy[2], vy[3], t.ax);
    float c01 = lerpf(vy[4], vy[5], t.ax), c11 = lerpf(vy[6], vy[7], t.ax);
    r.y = lerpf(lerpf(c00, c10, t.ay), lerpf(c01, c11, t.ay), t.az);
  }
  {
    float c00 = lerpf(vz[0], vz[1], t.ax), c10 = lerpf(vz[2], vz[3], t.ax);
    float c01 = lerpf(vz[4], vz[5], t.ax), c11 = lerpf(vz[6], vz[7], t.ax);
    r.z = lerpf(lerpf(c00, c10, t.ay), lerpf(c01, c11, t.ay), t.az);
  }
  return r;
}

// texture(TexTransferFunc, density): 1D linear, clamp-to-edge, from LDS.
__device__ __forceinline__ float4 tf_lookup(const float4* __restrict__ tf, int n, float density) {
  float x = fmaf(density, (float)n, -0.5f);
  x = fminf(fmaxf(x, -1.0f), (float)(n - 1));
  float fl = floorf(x);
  float a = x - fl;
  int i = (int)fl;
  float4 t0 = tf[max(i, 0)];
  float4 t1 = tf[min(i + 1, n - 1)];
  return make_float4(lerpf(t0.x, t1.x, a), lerpf(t0.y, t1.y, a), lerpf(t0.z, t1.z, a),
                     lerpf(t0.w, t1.w, a));
}

constexpr int kMaxTfLds = 4096;

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

// Pixel assignment of lane `lane` in wave `wave` of logical block `L`.
__device__ __forceinline__ void pixel_of(const Rc1passArgs& A, int L, int wave, int lane, int& px,
                                         int& py, long long& out_idx) {
  int lx = ((wave & 1) << 3) | (lane & 7);
  int ly = ((wave >> 1) << 3) | (lane >> 3);
  if (!A.packed) {
    int nbx = (A.W + 15) >> 4;
    px = (L % nbx) * 16 + lx;
    py = (L / nbx) * 16 + ly;
    out_idx = (long long)py * A.W + px;
  } else {
    int bpt_x = A.tile >> 4;               // 16x16 blocks per tile row
    int bpt = bpt_x * bpt_x;
    int k = L / bpt, j = L - k * bpt;
    int t = A.rank + k * A.nranks;
    int tx = t % A.ntx, ty = t / A.ntx;
    int ox = (j % bpt_x) * 16 + lx, oy = (j / bpt_x) * 16 + ly;
    px = tx * A.tile + ox;
    py = ty * A.tile + oy;
    out_idx = (long long)k * A.tile * A.tile + (long long)oy * A.tile + ox;
  }
}

// One sample's cell address + weights (stage 1 of the batched march).
struct SamplePos { uint32_t idx; float ax, ay, az; int ix, iy, iz; };

__device__ __forceinline__ SamplePos sample_pos(float x, float y, float z, const Rc1passArgs& A,
                                                uint32_t bxby) {
  // GL_LINEAR texel-centre convention; positions are inside [-0.5, N-0.5] for
  // every hit ray, so the CLAMP_TO_EDGE corner clamp is folded into the padded
  // cell grid (cell = floor(x)+1 in [0, N]; the integer clamp only guards memory).
  float fx = floorf(x), fy = floorf(y), fz = floorf(z);
  SamplePos p;
  p.ax = x - fx; p.ay = y - fy; p.az = z - fz;
  p.ix = (int)fx; p.iy = (int)fy; p.iz = (int)fz;
  uint32_t cx = (uint32_t)min(max(p.ix + 1, 0), A.N[0]);
  uint32_t cy = (uint32_t)min(max(p.iy + 1, 0), A.N[1]);
  uint32_t cz = (uint32_t)min(max(p.iz + 1, 0), A.N[2]);
  uint32_t brick = __umul24(cz >> 2, bxby) + __umul24(cy >> 2, (uint32_t)A.cells.bx) + (cx >> 2);
  p.idx = (brick << 6) | ((cz & 3u) << 4) | ((cy & 3u) << 2) | (cx & 3u);
  return p;
}

__device__ __forceinline__ float trilerp_cell(uint4 raw, float ax, float ay, float az) {
  float v000, v100, v010, v110, v001, v101, v011, v111;
  h2f2(raw.x, v000, v100);
  h2f2(raw.y, v010, v110);
  h2f2(raw.z, v001, v101);
  h2f2(raw.w, v011, v111);
  float c00 = lerpf(v000, v100, ax);
  float c10 = lerpf(v010, v110, ax);
  float c01 = lerpf(v001, v101, ax);
  float c11 = lerpf(v011, v111, ax);
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

// The ray-march.  K samples are addressed and fetched per batch (K 16-byte
// loads in flight per lane), then their densities are classified through the
// LDS transfer function, then composited front to back in order with the
// per-lane ERT exit.  The arithmetic per sample is exactly the sequential loop
// of ray_marching_1p.comp:124-172 (s accumulates h one step at a time).
template <int K, bool PHONG>
__global__ void __launch_bounds__(256)
rc1pass_kernel(Rc1passArgs A, const uint4* __restrict__ cells, const uint2* __restrict__ grad,
               const float4* __restrict__ tf_g, float4* __restrict__ out,
               uint32_t* __restrict__ samples, unsigned long long* __restrict__ total,
               const int* __restrict__ order, uint32_t* __restrict__ wave_cost, int nblocks) {
  // Padded TF: tfp[k] = T[clamp(k-1, 0, n-1)], k in [0, n+1]; a lookup at
  // x = d*n - 0.5 reads the two adjacent entries tfp[floor(x)+1], tfp[floor(x)+2].
  extern __shared__ float4 tfp[];
  const int n = A.tf_n;
  for (int i = threadIdx.x; i < n + 2; i += blockDim.x) tfp[i] = tf_g[min(max(i - 1, 0), n - 1)];
  __syncthreads();

  // Block -> screen tile: a cost-ordered permutation (longest tiles first) when
  // given, else an XCD-aware remap (blocks b and b+8 share an XCD; XCD b%8 gets
  // one contiguous band of logical blocks).
  const int b = blockIdx.x;
  int L;
  if (order) L = order[b];
  else if (A.xcd_remap && (nblocks & 7) == 0) L = (b & 7) * (nblocks >> 3) + (b >> 3);
  else L = b;

  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  int px, py;
  long long oidx;
  pixel_of(A, L, wave, lane, px, py, oidx);
  const bool inside = px < A.W && py < A.H;

  float4 dst = make_float4(0.f, 0.f, 0.f, 0.f);
  uint32_t cnt = 0;
  if (inside) {
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
    if (hit) {
      const float D = fabsf(tfar - tnear);
      const f3 tpos{fmaf(dir.x, tnear, eye.x) + hg.x, fmaf(dir.y, tnear, eye.y) + hg.y,
                    fmaf(dir.z, tnear, eye.z) + hg.z};
      const f3 o{fmaf(tpos.x, A.n_over_g[0], -0.5f), fmaf(tpos.y, A.n_over_g[1], -0.5f),
                 fmaf(tpos.z, A.n_over_g[2], -0.5f)};
      const f3 dt{dir.x * A.n_over_g[0], dir.y * A.n_over_g[1], dir.z * A.n_over_g[2]};
      const float step = A.step;
      const uint32_t bxby = (uint32_t)A.cells.bx * (uint32_t)A.cells.by;
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
          sp[j] = sample_pos(fmaf(dt.x, tj[j], o.x), fmaf(dt.y, tj[j], o.y), fmaf(dt.z, tj[j], o.z),
                             A, bxby);
          raw[j] = cells[sp[j].idx];
        }
        // stage 2: density and transfer-function classification
        float4 src[K];
#pragma unroll
        for (int j = 0; j < K; j++) {
          float dens = trilerp_cell(raw[j], sp[j].ax, sp[j].ay, sp[j].az);
          float x = fmaf(dens, fn, -0.5f);
          float fl = floorf(x);
          float a = x - fl;
          int i = min(max((int)fl + 1, 0), n);
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
    out[oidx] = dst;   // misses store the cleared (0,0,0,0), renderoutputframe.cpp:187-190
    if (samples) samples[oidx] = cnt;
  } else if (A.packed) {
    out[oidx] = dst;   // padding pixels of edge tiles
    if (samples) samples[oidx] = 0;
  }
  if (total) {
    unsigned long long v = cnt;
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
    if (lane == 0 && v) atomicAdd(total, v);
  }
  if (wave_cost) {   // the wave's critical path (its longest ray) for the next frame's order
    uint32_t m = cnt;
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) m = max(m, (uint32_t)__shfl_xor((int)m, off, 64));
    if (lane == 0) wave_cost[L * 4 + wave] = m;
  }
}

// Longest-processing-time-first block order from the previous frame's wave
// costs: segment s (one workgroup) sorts logical blocks [s*seg, (s+1)*seg) by
// descending cost (bitonic sort in LDS) and assigns them to physical blocks
// s, s+nseg, s+2*nseg, ... (nseg = 8: one XCD band per segment; nseg = 1: global).
__global__ void __launch_bounds__(1024)
tile_order_kernel(const uint32_t* __restrict__ wave_cost, int nblocks, int nseg,
                  int* __restrict__ order) {
  extern __shared__ unsigned long long keys[];
  const int seg = nblocks / nseg;
  const int base = blockIdx.x * seg;
  int P = 1;
  while (P < seg) P <<= 1;
  for (int i = threadIdx.x; i < P; i += blockDim.x) {
    unsigned long long k = 0;
    if (i < seg) {
      uint32_t L = (uint32_t)(base + i);
      uint32_t c = wave_cost[L * 4] + wave_cost[L * 4 + 1] + wave_cost[L * 4 + 2] + wave_cost[L * 4 + 3];
      k = ((unsigned long long)c << 32) | (0xffffffffu - L);
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
  for (int i = threadIdx.x; i < seg; i += blockDim.x) {
    int L = (int)(0xffffffffu - (uint32_t)keys[i]);
    order[nseg == 1 ? i : (blockIdx.x + nseg * i)] = L;
  }
}

hipError_t launch_tile_order(const uint32_t* wave_cost, int nblocks, int nseg, int* order,
                             hipStream_t s) {
  if (nblocks % nseg) return hipErrorInvalidValue;
  int seg = nblocks / nseg, P = 1;
  while (P < seg) P <<= 1;
  if (P > 16384) return hipErrorInvalidValue;
  hipLaunchKernelGGL(tile_order_kernel, dim3(nseg), dim3(1024), (size_t)P * 8, s, wave_cost,
                     nblocks, nseg, order);
  return hipGetLastError();
}

template <int K>
static hipError_t launch_k(const Ctx& c, const Rc1passArgs& a, bool phong, float4* out,
                           uint32_t* samples, unsigned long long* total, const int* order,
                           uint32_t* wave_cost, int nblocks, hipStream_t s) {
  dim3 grid(nblocks), block(256);
  size_t lds = (size_t)(a.tf_n + 2) * sizeof(float4);
  if (phong)
    hipLaunchKernelGGL((rc1pass_kernel<K, true>), grid, block, lds, s, a, (const uint4*)c.d_cells,
                       (const uint2*)c.d_grad, (const float4*)c.d_tf, out, samples, total, order,
                       wave_cost, nblocks);
  else
    hipLaunchKernelGGL((rc1pass_kernel<K, false>), grid, block, lds, s, a, (const uint4*)c.d_cells,
                       (const uint2*)c.d_grad, (const float4*)c.d_tf, out, samples, total, order,
                       wave_cost, nblocks);
  return hipGetLastError();
}

hipError_t launch_rc1pass(const Ctx& c, const Rc1passArgs& a, bool phong, float4* out,
                          uint32_t* samples, unsigned long long* total, const int* order,
                          uint32_t* wave_cost, int nblocks, hipStream_t s) {
  if (nblocks <= 0) return hipSuccess;
  if (a.tf_n > kMaxTfLds) return hipErrorInvalidValue;
  switch (c.batch) {
    case 1: return launch_k<1>(c, a, phong, out, samples, total, order, wave_cost, nblocks, s);
    case 2: return launch_k<2>(c, a, phong, out, samples, total, order, wave_cost, nblocks, s);
    case 8: return launch_k<8>(c, a, phong, out, samples, total, order, wave_cost, nblocks, s);
    default: return launch_k<4>(c, a, phong, out, samples, total, order, wave_cost, nblocks, s);
  }
}

// ---------------------------------------------------------------------------
// Precompute kernels
// ---------------------------------------------------------------------------

// Build the padded, bricked cell8 layout from raw voxels using the host-made
// value table lut[v] = half(float(v / 255.0)) (GL_R16F upload of
// GetNormalizedSample, utils.cpp:20-56).
template <typename VT>
__global__ void build_cells_kernel(const VT* __restrict__ vox, const uint16_t* __restrict__ lut,
                                   int nx, int ny, int nz, CellGrid g, uint4* __restrict__ cells,
                                   size_t ncells) {
  size_t idx = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= ncells) return;
  uint32_t i = (uint32_t)idx;
  uint32_t inner = i & 63u, brick = i >> 6;
  int a = (int)(inner & 3u), b = (int)((inner >> 2) & 3u), c = (int)(inner >> 4);
  int bxi = (int)(brick % (uint32_t)g.bx);
  uint32_t rest = brick / (uint32_t)g.bx;
  int byi = (int)(rest % (uint32_t)g.by), bzi = (int)(rest / (uint32_t)g.by);
  a += bxi * 4; b += byi * 4; c += bzi * 4;
  uint4 r = make_uint4(0, 0, 0, 0);
  if (a < g.cx && b < g.cy && c < g.cz) {
    int x0 = max(a - 1, 0), x1 = min(a, nx - 1);
    int y0 = max(b - 1, 0), y1 = min(b, ny - 1);
    int z0 = max(c - 1, 0), z1 = min(c, nz - 1);
    auto q = [&](int x, int y, int z) -> uint32_t {
      return lut[vox[(size_t)x + (size_t)y * nx + (size_t)z * nx * ny]];
    };
    r.x = q(x0, y0, z0) | (q(x1, y0, z0) << 16);
    r.y = q(x0, y1, z0) | (q(x1, y1, z0) << 16);
    r.z = q(x0, y0, z1) | (q(x1, y0, z1) << 16);
    r.w = q(x0, y1, z1) | (q(x1, y1, z1) << 16);
  }
  cells[idx] = r;
}

hipError_t launch_build_cells_impl(const void* vox, int bpv, const uint16_t* lut, const int N[3],
                                   const CellGrid& g, void* cells, hipStream_t s) {
  size_t n = cell_count(g);
  int bs = 256;
  size_t nb = (n + bs - 1) / bs;
  if (bpv == 1)
    hipLaunchKernelGGL(build_cells_kernel<uint8_t>, dim3((unsigned)nb), dim3(bs), 0, s,
                       (const uint8_t*)vox, lut, N[0], N[1], N[2], g, (uint4*)cells, n);
  else
    hipLaunchKernelGGL(build_cells_kernel<uint16_t>, dim3((unsigned)nb), dim3(bs), 0, s,
                       (const uint16_t*)vox, lut, N[0], N[1], N[2], g, (uint4*)cells, n);
  return hipGetLastError();
}

// GetNormalizedSample in double (structuredgridvolume.cpp:121-151), 0 outside.
template <typename VT>
__device__ __forceinline__ double norm_sample(const VT* vox, int nx, int ny, int nz, int x, int y,
                                              int z, double inv_max) {
  if (x < 0 || y < 0 || z < 0 || x >= nx || y >= ny || z >= nz) return 0.0;
  return (double)vox[(size_t)x + (size_t)y * nx + (size_t)z * nx * ny] / inv_max;
}

__device__ __forceinline__ uint32_t f2h_bits(float f) {
  _Float16 h = (_Float16)f;
  return (uint32_t)__builtin_bit_cast(uint16_t, h);
}

// GenerateGradientTexture (utils.cpp:146-190) with its defaults, and
// GenerateSobelFeldmanGradientTexture (utils.cpp:287-333); stored RGB16F.
template <typename VT>
__global__ void gradient_kernel(const VT* __restrict__ vox, int nx, int ny, int nz, int mode,
                                double maxv, uint2* __restrict__ grad) {
  size_t idx = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  size_t n = (size_t)nx * ny * nz;
  if (idx >= n) return;
  int x = (int)(idx % (size_t)nx);
  size_t r = idx / (size_t)nx;
  int y = (int)(r % (size_t)ny), z = (int)(r / (size_t)ny);
  double gx = 0, gy = 0, gz = 0;
  if (mode == CVR_GRADIENT_FINITE_DIFFERENCES) {
    gx = norm_sample(vox, nx, ny, nz, x + 1, y, z, maxv) - norm_sample(vox, nx, ny, nz, x - 1, y, z, maxv);
    gy = norm_sample(vox, nx, ny, nz, x, y + 1, z, maxv) - norm_sample(vox, nx, ny, nz, x, y - 1, z, maxv);
    gz = norm_sample(vox, nx, ny, nz, x, y, z + 1, maxv) - norm_sample(vox, nx, ny, nz, x, y, z - 1, maxv);
    double sqr = gx * gx + gy * gy + gz * gz;
    double inv = 1.0 / sqrt(sqr);
    gx *= inv; gy *= inv; gz *= inv;
    if (gx != gx) { gx = 0.0; gy = 0.0; gz = 0.0; }
  } else {
    for (int v1 = -1; v1 <= 1; v1++)
      for (int v2 = -1; v2 <= 1; v2++) {
        int m = abs(v1) + abs(v2);
        double wgt = m == 0 ? 1.0 : (m == 1 ? 2.0 : 4.0);   // pow(2, |v1|+|v2|)
        gz += norm_sample(vox, nx, ny, nz, x + v1, y + v2, z - 1, maxv) * (4.0 / wgt)
            + norm_sample(vox, nx, ny, nz, x + v1, y + v2, z + 1, maxv) * (-4.0 / wgt);
        gy += norm_sample(vox, nx, ny, nz, x + v1, y - 1, z + v2, maxv) * (4.0 / wgt)
            + norm_sample(vox, nx, ny, nz, x + v1, y + 1, z + v2, maxv) * (-4.0 / wgt);
        gx += norm_sample(vox, nx, ny, nz, x - 1, y + v2, z + v1, maxv) * (4.0 / wgt)
            + norm_sample(vox, nx, ny, nz, x + 1, y + v2, z + v1, maxv) * (-4.0 / wgt);
      }
  }
  uint2 o;
  o.x = f2h_bits((float)gx) | (f2h_bits((float)gy) << 16);
  o.y = f2h_bits((float)gz);
  grad[idx] = o;
}

hipError_t launch_gradient(const Ctx& c, int mode, hipStream_t s) {
  size_t n = (size_t)c.N[0] * c.N[1] * c.N[2];
  int bs = 256;
  size_t nb = (n + bs - 1) / bs;
  if (c.bpv == 1)
    hipLaunchKernelGGL(gradient_kernel<uint8_t>, dim3((unsigned)nb), dim3(bs), 0, s,
                       (const uint8_t*)c.d_vox, c.N[0], c.N[1], c.N[2], mode, 255.0,
                       (uint2*)c.d_grad);
  else
    hipLaunchKernelGGL(gradient_kernel<uint16_t>, dim3((unsigned)nb), dim3(bs), 0, s,
                       (const uint16_t*)c.d_vox, c.N[0], c.N[1], c.N[2], mode, 65535.0,
                       (uint2*)c.d_grad);
  return hipGetLastError();
}

// Scatter packed per-rank tiles (screen-tile split) into the W x H image.
__global__ void unpack_tiles_kernel(const float4* __restrict__ packed, float4* __restrict__ out,
                                    int W, int H, int tile, int nranks, int tpr_max, int ntx,
                                    size_t n) {
  size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  size_t tt = (size_t)tile * tile;
  size_t slot = i / tt;                     // rank * tpr_max + k
  int inner = (int)(i - slot * tt);
  int r = (int)(slot / (size_t)tpr_max), k = (int)(slot % (size_t)tpr_max);
  int t = r + k * nranks;
  int tx = t % ntx, ty = t / ntx;
  int px = tx * tile + inner % tile, py = ty * tile + inner / tile;
  if (px < W && py < H && ty * tile < H) out[(size_t)py * W + px] = packed[i];
}

hipError_t launch_unpack_tiles(const float4* packed, float4* out, int W, int H, int tile,
                               int nranks, int tpr_max, hipStream_t s) {
  int ntx = (W + tile - 1) / tile;
  size_t n = (size_t)nranks * tpr_max * tile * tile;
  int bs = 256;
  size_t nb = (n + bs - 1) / bs;
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(unpack_tiles_kernel, dim3((unsigned)nb), dim3(bs), 0, s, packed, out, W, H,
                     tile, nranks, tpr_max, ntx, n);
  return hipGetLastError();
}

}  // namespace cvr
