// dos.hip — directional-occlusion shading (cppvolrend rc1pdosct) on gfx950.
//
//  * the extinction-coefficient mip volume (ExtinctionCoefficientVolume, custom
//    resolution path: extcoefvolumegenerator.cpp:230-408 and glslextgen/*.comp):
//    level 0 = 7^3-tap Gaussian of the TF opacity over the volume, level L = the
//    same Gaussian (sigma 2^L) over level L-1, then tau = -log(1 - opacity);
//    every level stored as fp16 (GL_R16F), x-fastest, levels concatenated;
//  * the ray-march of ray_bbox_marching.comp:658-734 with ShadeSample (:607-656):
//    for every sample with alpha > 0, a cone-traced ambient occlusion toward the
//    eye (Cone1/3/7RayOcclusion, :116-333) and a cone-traced shadow toward the
//    light (Cone1/3/7RayShadow, :337-562), each a trapezoid accumulation of
//    Gaussian-filtered extinctions along 1 -> 3 -> 7 rays.
//
// Arithmetic follows CVR-SPEC exactly as oracle/cvr_oracle.cpp (oracle_ext_volume,
// oracle_render_dos) so results are bit-identical.  Compiled -ffp-contract=off.
#include <hip/hip_runtime.h>
#include <cstdint>

#include "cvr_device.h"
#include "march_common.h"
#include "shaded_march.h"

namespace cvr {

// ---------------------------------------------------------------------------
// fp16 level sampling (trilinear, clamp-to-edge, texel-centre convention)
// ---------------------------------------------------------------------------

__device__ __forceinline__ float h2f(uint16_t h) { return (float)__builtin_bit_cast(_Float16, h); }

// float -> binary16, round to nearest even (v_cvt_f16_f32)
__device__ __forceinline__ uint16_t f2h_rne(float f) { return (uint16_t)f32_to_h16(f); }

// x, y, z in texel space of a d[0] x d[1] x d[2] level.  Clamping to [0, d-1]
// gives the same values as GL's CLAMP_TO_EDGE on [-1, d-1] (see sample_pos).
__device__ __forceinline__ float sample_level(const uint16_t* __restrict__ lv, const int d[3],
                                              float x, float y, float z) {
  x = __builtin_amdgcn_fmed3f(x, 0.0f, (float)(d[0] - 1));
  y = __builtin_amdgcn_fmed3f(y, 0.0f, (float)(d[1] - 1));
  z = __builtin_amdgcn_fmed3f(z, 0.0f, (float)(d[2] - 1));
  const int ix = (int)x, iy = (int)y, iz = (int)z;
  const float ax = __builtin_amdgcn_fractf(x), ay = __builtin_amdgcn_fractf(y),
              az = __builtin_amdgcn_fractf(z);
  const int x1 = min(ix + 1, d[0] - 1), y1 = min(iy + 1, d[1] - 1), z1 = min(iz + 1, d[2] - 1);
  const long long sy = d[0], sz = (long long)d[0] * d[1];
  const long long r00 = iz * sz + iy * sy, r10 = iz * sz + y1 * sy;
  const long long r01 = z1 * sz + iy * sy, r11 = z1 * sz + y1 * sy;
  const float c00 = lerpf(h2f(lv[r00 + ix]), h2f(lv[r00 + x1]), ax);
  const float c10 = lerpf(h2f(lv[r10 + ix]), h2f(lv[r10 + x1]), ax);
  const float c01 = lerpf(h2f(lv[r01 + ix]), h2f(lv[r01 + x1]), ax);
  const float c11 = lerpf(h2f(lv[r11 + ix]), h2f(lv[r11 + x1]), ax);
  return lerpf(lerpf(c00, c10, ay), lerpf(c01, c11, ay), az);
}

// ---------------------------------------------------------------------------
// Extinction-coefficient volume
// ---------------------------------------------------------------------------

struct ExtBuildArgs {
  // the volume (cell8 layout, see sample_pos) and the opacity TF
  CellGrid cells;
  float nm1[3];
  int N[3];
  float G[3];                 // VolumeGridSize
  int tf_n;
  // this level
  int L;
  int d[3], pd[3];            // this level's and the previous level's dimensions
  float S;                    // sigma0 * 2^L
  float vs[3];                // G / d (voxel size)
};

// One thread per voxel of level L (gen_extcoefvol_anysize.comp:36-76 for L = 0,
// gen_extcoefvol_anysize_mmlevel.comp:35-78 for L >= 1).  The 343 tap weights are
// shared by the block (LDS).  L = 0 samples the volume cells and the opacity TF
// (padded alpha table in LDS); L >= 1 samples level L-1 (`prev`).
__global__ void __launch_bounds__(256)
ext_level_kernel(ExtBuildArgs E, const uint4* __restrict__ cells, const float4* __restrict__ tf,
                 const uint16_t* __restrict__ prev, uint16_t* __restrict__ out) {
  __shared__ float w_lds[343];
  __shared__ float a_lds[kMaxTfLds + 2];
  const float S = E.S, S3 = (S * S) * S, den = (2.0f * S) * S;
  for (int t = threadIdx.x; t < 343; t += blockDim.x) {
    const int tx = t / 49 - 3, ty = (t / 7) % 7 - 3, tz = t % 7 - 3;
    const float fx = (float)tx * S, fy = (float)ty * S, fz = (float)tz * S;
    w_lds[t] = S3 * cvr_expf(-((fx * fx + fy * fy) + fz * fz) / den);
  }
  if (E.L == 0)
    for (int i = threadIdx.x; i < E.tf_n + 2; i += blockDim.x)
      a_lds[i] = tf[min(max(i - 1, 0), E.tf_n - 1)].w;
  __syncthreads();
  const long long nv = (long long)E.d[0] * E.d[1] * E.d[2];
  const long long v = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (v >= nv) return;
  const int i = (int)(v % E.d[0]), j = (int)((v / E.d[0]) % E.d[1]),
            k = (int)(v / ((long long)E.d[0] * E.d[1]));
  const float gx = ((float)i + 0.5f) * E.vs[0], gy = ((float)j + 0.5f) * E.vs[1],
              gz = ((float)k + 0.5f) * E.vs[2];
  const float fn = (float)E.tf_n;
  float swc = 0.0f, sw = 0.0f;
  int t = 0;
  for (int tx = -3; tx <= 3; tx++)
    for (int ty = -3; ty <= 3; ty++)
      for (int tz = -3; tz <= 3; tz++, t++) {
        const float w = w_lds[t];
        const float px = gx + (float)tx * S, py = gy + (float)ty * S, pz = gz + (float)tz * S;
        const float ux = px / E.G[0], uy = py / E.G[1], uz = pz / E.G[2];
        float c = 0.0f;
        if (!(ux < 0.0f || uy < 0.0f || uz < 0.0f || ux > 1.0f || uy > 1.0f || uz > 1.0f)) {
          if (E.L == 0) {
            Rc1passArgs A;   // sample_pos reads only nm1 and the cell pitches
            A.nm1[0] = E.nm1[0]; A.nm1[1] = E.nm1[1]; A.nm1[2] = E.nm1[2];
            A.cells = E.cells;
            const SamplePos sp = sample_pos(fmaf(ux, (float)E.N[0], -0.5f),
                                            fmaf(uy, (float)E.N[1], -0.5f),
                                            fmaf(uz, (float)E.N[2], -0.5f), A);
            const float dens = trilerp_cell(cells[sp.idx], sp.ax, sp.ay, sp.az);
            // texture(TF, d).a: padded table, x = d*n - 0.5
            const float xt = fmaf(dens, fn, -0.5f);
            const float fl = floorf(xt);
            const int ti = (int)fl + 1;
            c = lerpf(a_lds[ti], a_lds[ti + 1], xt - fl);
          } else {
            c = sample_level(prev, E.pd, fmaf(ux, (float)E.pd[0], -0.5f),
                             fmaf(uy, (float)E.pd[1], -0.5f), fmaf(uz, (float)E.pd[2], -0.5f));
          }
        }
        swc = swc + w * c;
        sw = sw + w;
      }
  out[v] = f2h_rne(swc / sw);
}

// backtotau.comp:11-34: tau = -1 * log(1 - opacity), in place over all levels.
__global__ void ext_to_tau_kernel(uint16_t* __restrict__ lv, long long n) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) lv[i] = f2h_rne(-1.0f * cvr_logf(1.0f - h2f(lv[i])));
}

// The cone fetches read cell8 texels: texel (i, j, k) of a level holds its 8
// trilinear corners (i|i+1, j|j+1, k|k+1, the +1 clamped to the edge) as fp16,
// so one dwordx4 load feeds one fetch (the volume's own layout, see sample_pos).
__global__ void ext_cells_kernel(const uint16_t* __restrict__ lv, uint4* __restrict__ cells, int dx,
                                 int dy, int dz) {
  const long long n = (long long)dx * dy * dz;
  const long long v = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (v >= n) return;
  const int i = (int)(v % dx), j = (int)((v / dx) % dy), k = (int)(v / ((long long)dx * dy));
  const int i1 = min(i + 1, dx - 1), j1 = min(j + 1, dy - 1), k1 = min(k + 1, dz - 1);
  const long long sy = dx, sz = (long long)dx * dy;
  auto at = [&](int x, int y, int z) -> uint32_t { return lv[z * sz + y * sy + x]; };
  uint4 c;
  c.x = at(i, j, k) | (at(i1, j, k) << 16);
  c.y = at(i, j1, k) | (at(i1, j1, k) << 16);
  c.z = at(i, j, k1) | (at(i1, j, k1) << 16);
  c.w = at(i, j1, k1) | (at(i1, j1, k1) << 16);
  cells[v] = c;
}

hipError_t launch_ext_volume(const Ctx& c, const float4* d_tf_rgba, int tf_n, const int res[3],
                             float sigma0, int nlevels, const long long* off, uint16_t* d_ext,
                             uint4* d_ext_cells, hipStream_t s) {
  if (tf_n > kMaxTfLds) return hipErrorInvalidValue;
  ExtBuildArgs E{};
  E.cells = c.cells;
  for (int i = 0; i < 3; i++) {
    E.N[i] = c.N[i];
    E.nm1[i] = (float)(c.N[i] - 1);
    E.G[i] = (float)c.N[i] * c.scale[i];
  }
  E.tf_n = tf_n;
  const uint4* cells = (const uint4*)c.d_cells;   // sample_pos indexes from the first cell
  for (int L = 0; L < nlevels; L++) {
    E.L = L;
    for (int i = 0; i < 3; i++) {
      E.d[i] = res[i] >> L > 1 ? res[i] >> L : 1;
      E.pd[i] = L == 0 ? 1 : (res[i] >> (L - 1) > 1 ? res[i] >> (L - 1) : 1);
      E.vs[i] = E.G[i] / (float)E.d[i];
    }
    E.S = L == 0 ? sigma0 : sigma0 * (float)(1 << L);
    const long long nv = (long long)E.d[0] * E.d[1] * E.d[2];
    hipLaunchKernelGGL(ext_level_kernel, dim3((unsigned)((nv + 255) / 256)), dim3(256), 0, s, E,
                       cells, d_tf_rgba, L == 0 ? nullptr : d_ext + off[L - 1], d_ext + off[L]);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
  }
  const long long n = off[nlevels];
  hipLaunchKernelGGL(ext_to_tau_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, d_ext, n);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  for (int L = 0; L < nlevels; L++) {
    int d[3];
    for (int i = 0; i < 3; i++) d[i] = res[i] >> L > 1 ? res[i] >> L : 1;
    const long long nv = off[L + 1] - off[L];
    hipLaunchKernelGGL(ext_cells_kernel, dim3((unsigned)((nv + 255) / 256)), dim3(256), 0, s,
                       d_ext + off[L], d_ext_cells + off[L], d[0], d[1], d[2]);
    e = hipGetLastError();
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}

// ---------------------------------------------------------------------------
// Cone tracing
// ---------------------------------------------------------------------------

// GetGaussianExtinction (:92-112): textureLod at an integer level (clamped to the
// pyramid; the level is wave-uniform, a section-table entry), plus the
// CONSIDER_BORDERS attenuation outside the volume box.  Split in two so that a
// batch of fetches issues all its loads before any of them is consumed.
struct ExtTap {
  uint32_t off;       // byte offset of the cell8 texel
  float ax, ay, az;
};

// A level's addressing, by scalar loads (the index is wave-uniform).
__device__ __forceinline__ ExtLevel load_level(const ExtLevel* lv, int L) {
#if __HIP_DEVICE_COMPILE__
  return ((const __attribute__((address_space(4))) ExtLevel*)lv)[L];
#else
  return lv[L];
#endif
}

// The cone code's template int M: bits 0-7 the GL_LINEAR weights' fraction bits
// (filter_bits; 0 = exact), bit 8 (kDosNativeExp) the border attenuation's exp as
// v_exp_f32 (option native_exp: tolerance mode, not CVR-SPEC).
constexpr int kDosNativeExp = 0x100;

template <int FB>   // FB: GL_LINEAR weights at FB fraction bits (filter_bits; 0 = exact)
__device__ __forceinline__ ExtTap ext_tap(const ExtLevel& l, f3 p) {
  const float x = __builtin_amdgcn_fmed3f(fmaf(p.x, l.sx, -0.5f), 0.0f, l.mx);
  const float y = __builtin_amdgcn_fmed3f(fmaf(p.y, l.sy, -0.5f), 0.0f, l.my);
  const float z = __builtin_amdgcn_fmed3f(fmaf(p.z, l.sz, -0.5f), 0.0f, l.mz);
  ExtTap t;
  // dims <= 2^12 and < 2^28 cells in all (checked on the host): 24-bit multiplies
  const uint32_t row = __umul24((uint32_t)z, (uint32_t)l.dy) + (uint32_t)y;
  t.off = (__umul24(row, (uint32_t)l.dx) + (uint32_t)x + (uint32_t)l.off) << 4;
  t.ax = filter_weight<(FB & 0xff)>(__builtin_amdgcn_fractf(x));
  t.ay = filter_weight<(FB & 0xff)>(__builtin_amdgcn_fractf(y));
  t.az = filter_weight<(FB & 0xff)>(__builtin_amdgcn_fractf(z));
  return t;
}

// The CONSIDER_BORDERS exponent of a tap outside the box: -(dist) / ((2 sg) sg)
// with sg = pow(2, mip); the divisor is 2^(2 mip + 1), so the quotient is exactly
// the product with 2^-(2 mip + 1).  dist = |clamp(p, 0, G) - p|^2.
__device__ __forceinline__ float border_exponent(const DosArgs& Q, f3 p, float mip) {
  const float inv = ldexpf(1.0f, -(2 * (int)mip + 1));
  // clamp(p, 0, G) - p (positions are finite: med3 == min(max()))
  const float cx = __builtin_amdgcn_fmed3f(p.x, 0.0f, Q.G[0]) - p.x;
  const float cy = __builtin_amdgcn_fmed3f(p.y, 0.0f, Q.G[1]) - p.y;
  const float cz = __builtin_amdgcn_fmed3f(p.z, 0.0f, Q.G[2]) - p.z;
  const float dist = (cx * cx + cy * cy) + cz * cz;
  return -(dist) * inv;
}

__device__ __forceinline__ bool outside_box(const DosArgs& Q, f3 p) {
  return (p.x < 0.0f) | (p.x > Q.G[0]) | (p.y < 0.0f) | (p.y > Q.G[1]) | (p.z < 0.0f) |
         (p.z > Q.G[2]);
}

template <int M>
__device__ __forceinline__ float ext_value(const DosArgs& Q, uint4 raw, const ExtTap& t,
                                           bool outside, float xb) {
  float rg = trilerp_cell<false, false>(raw, t.ax, t.ay, t.az);   // extinction cells: no flags
#ifdef CVR_DOS_EXPERIMENT_NO_BORDER   // cost probes only (tools/build_variant.sh): wrong images
  return rg;
#endif
  // tolerance mode (native_exp): v_exp_f32 of the border exponent (~6 % of the C4
  // frame); the CVR-SPEC exp otherwise
  if (outside) rg = rg * ((M & kDosNativeExp) ? cvr_expf_native(xb) : cvr_expf_nonpos(xb));
  return rg;
}

__device__ __forceinline__ f3 cone_axis(const float* a, f3 k, f3 u, f3 v) {
  return f3{fmaf(v.x, a[0], fmaf(u.x, a[1], k.x * a[2])), fmaf(v.y, a[0], fmaf(u.y, a[1], k.y * a[2])),
            fmaf(v.z, a[0], fmaf(u.z, a[1], k.z * a[2]))};
}

// The level of a section (uniform: every lane walks the same table entry).
__device__ __forceinline__ int level_of(const DosArgs& Q, float mip) {
  return __builtin_amdgcn_readfirstlane(min(max((int)mip, 0), Q.ext_levels - 1));
}

// Sections of a J-ray stage, U at a time: the positions of U consecutive
// sections depend only on the (uniform) table, so their U*J loads are issued
// together, and the trapezoid sums then run in section order (the same
// arithmetic as one section at a time).
// The section table is read-only for the kernel's lifetime: read it through the
// constant address space so that its (uniform) entries come in by scalar loads.
__device__ __forceinline__ float4 load_section(const float4* sec, int i) {
#if __HIP_DEVICE_COMPILE__
  return ((const __attribute__((address_space(4))) float4*)sec)[i];
#else
  return sec[i];
#endif
}
typedef const float4* ConstSections;

// Sections per batch of the 1-ray and 3-ray stages (loads in flight per lane:
// U and 3U; the 7-ray stage issues 4 + 3)
#ifndef CVR_DOS_U1
#define CVR_DOS_U1 4
#endif
#ifndef CVR_DOS_SPLIT7
#define CVR_DOS_SPLIT7 4   // the 7-ray stage's fetches in groups of 4 + 3 rays (3: 3+2+2, 2: 2+2+2+1)
#endif
#ifndef CVR_DOS_U3
#define CVR_DOS_U3 2
#endif
template <int J, int U, int J0, int JN, int FB>
__device__ __forceinline__ void cone_sections(const DosArgs& Q, const DosCone& C,
                                              const uint4* __restrict__ ext, const float4 (&e)[U],
                                              const float (&tr)[U], const f3 (&vk)[J], f3 pos,
                                              float (&rays)[7], float (&last)[7], uint32_t& nf) {
  ExtTap tap[U][JN];
  uint4 raw[U][JN];
  float xb[U][JN];
  bool out[U][JN], zero[U][JN];
#pragma unroll
  for (int q = 0; q < U; q++) {
    const ExtLevel l = load_level(Q.levels, level_of(Q, e[q].y));
#pragma unroll
    for (int j = 0; j < JN; j++) {
      const f3 p = vmad(vk[J0 + j], tr[q], pos);
      tap[q][j] = ext_tap<FB>(l, p);
      // The border exponent is -0 inside the box, so "outside" is xb < 0: a tap
      // outside whose exponent is still -0 (a distance that underflows) gets the
      // factor exp(-0) = 1 exactly, the inside value (no 6-compare box test)
      xb[q][j] = border_exponent(Q, p, e[q].y);
      out[q][j] = xb[q][j] < 0.0f;
      // Far outside the box the border factor is exactly 0 (exp below -86), and
      // so is the tap (a finite extinction times 0): no fetch, no filter
      zero[q][j] = Q.zero_skip && xb[q][j] < -86.0f;
#ifdef CVR_DOS_EXPERIMENT_NO_FETCH    // cost probes only: wrong images
      raw[q][j] = make_uint4(tap[q][j].off, tap[q][j].off, tap[q][j].off, tap[q][j].off);
#else
      if (!zero[q][j]) raw[q][j] = *(const uint4*)((const char*)ext + tap[q][j].off);
#endif
    }
  }
  if (Q.count_taps) {   // measurement only: the taps actually fetched (uniform branch)
#pragma unroll
    for (int q = 0; q < U; q++)
#pragma unroll
      for (int j = 0; j < JN; j++) nf += zero[q][j] ? 0u : 1u;
  }
#pragma unroll
  for (int q = 0; q < U; q++)
#pragma unroll
    for (int j = 0; j < JN; j++) {
      const float v =
          zero[q][j] ? 0.0f : ext_value<FB>(Q, raw[q][j], tap[q][j], out[q][j], xb[q][j]) * e[q].w;
      rays[J0 + j] += ((last[J0 + j] + v) * e[q].z) * C.ui_weight;
      last[J0 + j] = v;
    }
}

// U sections of a J-ray stage starting at table entry s (uniform).  The 7-ray
// stage is split 4 + 3 rays to bound the fetches (registers) in flight.
template <int J, int U, int FB>
__device__ __forceinline__ void cone_step(const DosArgs& Q, const DosCone& C,
                                          const uint4* __restrict__ ext, ConstSections sec, int s,
                                          float& track, const f3 (&vk)[J], f3 pos,
                                          float (&rays)[7], float (&last)[7], uint32_t& nf) {
  float4 e[U];
  float tr[U];
#pragma unroll
  for (int q = 0; q < U; q++) {
    e[q] = load_section(sec, s + q);
    tr[q] = track;
    track += e[q].x;
  }
  if (J == 7 && CVR_DOS_SPLIT7 == 2) {
    cone_sections<J, U, 0, 2, FB>(Q, C, ext, e, tr, vk, pos, rays, last, nf);
    cone_sections<J, U, 2, 2, FB>(Q, C, ext, e, tr, vk, pos, rays, last, nf);
    cone_sections<J, U, 4, 2, FB>(Q, C, ext, e, tr, vk, pos, rays, last, nf);
    cone_sections<J, U, 6, 1, FB>(Q, C, ext, e, tr, vk, pos, rays, last, nf);
  } else if (J == 7 && CVR_DOS_SPLIT7 == 3) {
    cone_sections<J, U, 0, 3, FB>(Q, C, ext, e, tr, vk, pos, rays, last, nf);
    cone_sections<J, U, 3, 2, FB>(Q, C, ext, e, tr, vk, pos, rays, last, nf);
    cone_sections<J, U, 5, 2, FB>(Q, C, ext, e, tr, vk, pos, rays, last, nf);
  } else if (J == 7) {
    cone_sections<J, U, 0, 4, FB>(Q, C, ext, e, tr, vk, pos, rays, last, nf);
    cone_sections<J, U, 4, 3, FB>(Q, C, ext, e, tr, vk, pos, rays, last, nf);
  } else {
    cone_sections<J, U, 0, J, FB>(Q, C, ext, e, tr, vk, pos, rays, last, nf);
  }
}

// Early exit, exact: once a ray has left the box and its last tap was 0, every
// later tap of the stage is 0 too when the border exponent provably stays below
// -86.  The box is convex and axis-aligned: on an axis where the ray is outside
// and moving outward, the excess e grows linearly, e(t') = e + |k_a| (t' - t),
// and the distance to the box is at least e(t').  The border scale
// 2^-(2 floor(mip) + 1) is constant over each run of sections (ConeStageExit), so
// the smallest exponent magnitude of a run is at its first section.  The test
// keeps a margin (1e-2 in distance, 0.1 % in slope, 1 % in the exponent) far
// beyond the float error of the kernel's own positions and distances.  Such taps
// add exactly 0 to the ray's sum (last == 0, v == 0), so the stage ends at once:
// s and track jump to its end, rays/last are final.
__device__ __forceinline__ bool ray_gone(const DosArgs& Q, const ConeStageExit& X, f3 k, f3 pos,
                                         float track, int s_next, float inv_next) {
  const f3 p = vmad(k, track, pos);
  float e = -1.0f, slope = 0.0f;
  auto axis = [&](float pa, float ka, float Ga) {
    const float ea = ka > 0.0f ? pa - Ga : (ka < 0.0f ? -pa : -1.0f);
    if (ea > e) { e = ea; slope = fabsf(ka); }
  };
  axis(p.x, k.x, Q.G[0]);
  axis(p.y, k.y, Q.G[1]);
  axis(p.z, k.z, Q.G[2]);
  e -= 1e-2f;
  slope *= 0.999f;
  if (!(e > 0.0f)) return false;
  constexpr float kLimit = 86.0f * 1.01f;
  if (!(e * e * inv_next > kLimit)) return false;   // the run holding section s_next
  for (int r = 0; r < X.nruns; r++) {
    if (X.run_first[r] <= s_next) continue;
    const float d = fmaf(slope, X.run_t[r] - track, e);
    if (!(d * d * X.run_inv[r] > kLimit)) return false;
  }
  return true;
}

template <int J, int U, int FB>
__device__ __forceinline__ void cone_stage(const DosArgs& Q, const DosCone& C,
                                           const uint4* __restrict__ ext, ConstSections sec, int& s,
                                           int n, float& track, const f3 (&vk)[J], f3 pos,
                                           float (&rays)[7], float (&last)[7], uint32_t& nf,
                                           const ConeStageExit& X) {
  int i = 0;
  for (; i + U <= n; i += U, s += U) {
    cone_step<J, U, FB>(Q, C, ext, sec, __builtin_amdgcn_readfirstlane(s), track, vk, pos, rays, last,
                    nf);
    if (X.nruns > 0 && i + U < n) {
      bool zero = true;
#pragma unroll
      for (int j = 0; j < J; j++) zero = zero && last[j] == 0.0f;
      if (__all(zero)) {   // every lane's rays just took a 0 tap: worth the full test
        const int sn = __builtin_amdgcn_readfirstlane(s + U);
        const float mip = load_section(sec, sn).y;
        const float inv = ldexpf(1.0f, -(2 * (int)mip + 1));
        bool gone = true;
#pragma unroll
        for (int j = 0; j < J; j++) gone = gone && ray_gone(Q, X, vk[j], pos, track, sn, inv);
        if (__all(gone)) {
          s = X.end_s;
          track = X.end_track;
          return;
        }
      }
    }
  }
  for (; i < n; i++, s++)
    cone_step<J, 1, FB>(Q, C, ext, sec, __builtin_amdgcn_readfirstlane(s), track, vk, pos, rays, last,
                    nf);
}

// Cone1/3/7 RayOcclusion and Cone1/3/7 RayShadow (the same accumulation): the
// visibility exp(-sum) of a cone from `pos` along k, split 1 -> 3 -> 7 rays.
// Every lane walks the same section table (wave-uniform loads and levels).
template <int FB>
__device__ __forceinline__ float cone_trace(const DosArgs& Q, const DosCone& C, const uint4* __restrict__ ext,
                            f3 pos, f3 k, f3 u, f3 v, uint32_t& nf) {
  float rays[7], last[7];
  float track = C.initial_step;
  rays[0] = 0.0f;
  last[0] = 0.0f;
  const ConstSections sec = C.sections;
  int s = 0;
  {
    const f3 vk[1] = {k};
    cone_stage<1, CVR_DOS_U1, FB>(Q, C, ext, sec, s, C.counts[0], track, vk, pos, rays, last, nf, C.exit[0]);
  }
  if (C.counts[1] + C.counts[2] == 0) return cvr_expf(-rays[0]);
  rays[2] = rays[0]; rays[1] = rays[0];
  last[2] = last[0]; last[1] = last[0];
  {
    f3 vk[3];
#pragma unroll
    for (int j = 0; j < 3; j++) vk[j] = cone_axis(C.axes + 3 * j, k, u, v);
    cone_stage<3, CVR_DOS_U3, FB>(Q, C, ext, sec, s, C.counts[1], track, vk, pos, rays, last, nf, C.exit[1]);
  }
  if (C.counts[2] == 0)
    return ((cvr_expf(-rays[0]) + cvr_expf(-rays[1])) + cvr_expf(-rays[2])) / 3.0f;
  // transform 3 to 7 (:127-139)
  rays[6] = rays[5] = rays[2];
  rays[4] = rays[3] = rays[1];
  const float avg = ((rays[2] + rays[1]) + rays[0]) / 3.0f;
  rays[2] = rays[1] = rays[0];
  rays[0] = avg;
  last[6] = last[5] = last[2];
  last[4] = last[3] = last[1];
  const float avgt = ((last[2] + last[1]) + last[0]) / 3.0f;
  last[2] = last[1] = last[0];
  last[0] = avgt;
  {
    f3 vk[7];
#pragma unroll
    for (int j = 0; j < 7; j++) vk[j] = cone_axis(C.axes + 3 * (3 + j), k, u, v);
    cone_stage<7, 1, FB>(Q, C, ext, sec, s, C.counts[2], track, vk, pos, rays, last, nf, C.exit[2]);
  }
  float side = cvr_expf(-rays[1]);
#pragma unroll
  for (int j = 2; j < 7; j++) side = side + cvr_expf(-rays[j]);
  return (cvr_expf(-rays[0]) + side * C.ray7w) / (1.0f + C.ray7w * 6.0f);
}

// ---------------------------------------------------------------------------
// ShadeSample (ray_bbox_marching.comp:607-656) for the deferred march
// ---------------------------------------------------------------------------

#ifndef CVR_DOS_FLAT_WAVES
#define CVR_DOS_FLAT_WAVES 5   // flat shading: 96 VGPRs, 5 waves/SIMD (19 spilled): 11.2 -> 11.0 ms per frame; 4 / 6 waves: 11.2 / 12.6 ms
#endif
#ifndef CVR_DOS_WAVES
#define CVR_DOS_WAVES 3
#endif
template <int FB>
struct DosShaderT {
  using Args = DosArgs;
  static constexpr int kFB = FB & 0xff;   // GL_LINEAR weights of every fetch (filter_bits)
  // register budget: 3 waves/SIMD (168 VGPRs; the compiler alone takes 172 -> 2 waves):
  // kernel 21.1 -> 18.0 ms, 4 waves 18.8 ms (spills)
  static constexpr int kMinWavesPerEU = CVR_DOS_WAVES;
  static constexpr int kFlatWavesPerEU = CVR_DOS_FLAT_WAVES;   // flat_shade_kernel
  using Data = const uint4*;   // the cell8 extinction pyramid

  // The two halves of ShadeSample (:607-656), so that flat shading keeps only the
  // job's position live across the cone traces (its colour, opacity and gradient
  // are read back from the job list afterwards, shaded_march.h flat_shade_kernel):
  //   visibility: the occlusion and shadow cones' transmittances (iocc, isdw);
  //     `lit` counts the shadow cones traced, `fetches` the extinction taps
  //     actually fetched (Q.count_taps; taps whose border factor is exactly 0
  //     are skipped and not counted);
  //   combine: the shaded colour from them.
  // shade = combine(visibility), the per-wave kernel's single call.
  static constexpr bool kSplit = true;
  struct Vis {
    float iocc, isdw;
  };
  // wp = tx - half_grid, recomputed from an opaque copy of tx where needed so that
  // the compiler does not keep it live across a cone trace (96-VGPR budget)
  __device__ static __forceinline__ f3 world_pos(const DosArgs& Q, f3 tx) {
    asm volatile("" : "+v"(tx.x), "+v"(tx.y), "+v"(tx.z));
    const Rc1passArgs& A = Q.a;
    return f3{tx.x - A.half_grid[0], tx.y - A.half_grid[1], tx.z - A.half_grid[2]};
  }
  __device__ static __forceinline__ Vis visibility(const DosArgs& Q, const uint4* __restrict__ ext, f3 tx,
                                                   f3 wp, f3 cam, uint32_t& lit, uint32_t& fetches) {
    const Rc1passArgs& A = Q.a;
    Vis r{0.0f, 0.0f};
    if (Q.apply_occlusion) {
      const f3 eye{A.eye[0], A.eye[1], A.eye[2]};
      // eye-space frame of the occlusion cones (:681-684)
      const f3 v_right = normalize3(cross3(cam, f3{0.0f, 1.0f, 0.0f}));
      const f3 v_up = normalize3(cross3(f3{-cam.x, -cam.y, -cam.z}, v_right));
      const f3 k = normalize3(f3{eye.x - wp.x, eye.y - wp.y, eye.z - wp.z});
      r.iocc = cone_trace<FB>(Q, Q.occ, ext, tx, k, v_up, v_right, fetches);
      wp = world_pos(Q, tx);
    }
    if (Q.apply_shadow) {
      const f3 light{A.light[0], A.light[1], A.light[2]};
      f3 k, u, v;
      bool on = true;
      const f3 lf{Q.lfwd[0], Q.lfwd[1], Q.lfwd[2]};
      if (Q.shadow_type == 2) {
        k = lf;
        v = f3{Q.lup[0], Q.lup[1], Q.lup[2]};
        u = f3{Q.lright[0], Q.lright[1], Q.lright[2]};
      } else {
        k = normalize3(f3{light.x - wp.x, light.y - wp.y, light.z - wp.z});
        u = normalize3(cross3(k, f3{Q.lright[0], Q.lright[1], Q.lright[2]}));
        v = normalize3(cross3(k, u));
        if (Q.shadow_type == 1 && dot3(k, lf) < Q.spot_cos) on = false;
      }
      // Cone1RayShadow(pos, k, v, u) is called as (pos, k, u, v): swapped (:559-561)
      if (on) {
        r.isdw = cone_trace<FB>(Q, Q.sdw, ext, tx, k, v, u, fetches);
        lit++;
      }
    }
    return r;
  }
  __device__ static __forceinline__ f3 combine(const DosArgs& Q, Vis r, f3 wp, f3 rgb, const f3* g) {
    const Rc1passArgs& A = Q.a;
    const float inv_k = 1.0f / (Q.ka + Q.kd);
    if (g) {   // ApplyPhongShading
      if (g->x != 0.0f || g->y != 0.0f || g->z != 0.0f) {
        const f3 eye{A.eye[0], A.eye[1], A.eye[2]};
        const f3 light{A.light[0], A.light[1], A.light[2]};
        const f3 nrm = normalize3(*g);
        const f3 L = normalize3(f3{light.x - wp.x, light.y - wp.y, light.z - wp.z});
        const f3 Ve = normalize3(f3{eye.x - wp.x, eye.y - wp.y, eye.z - wp.z});
        const f3 Hv = normalize3(f3{Ve.x + L.x, Ve.y + L.y, Ve.z + L.z});
        const float dd = fmaxf(0.0f, dot3(nrm, L));
        const float ds = fmaxf(0.0f, dot3(Hv, nrm));
        const float diff = inv_k * (r.iocc * Q.ka + (r.isdw * Q.kd) * dd);
        const float spec = (r.isdw * Q.ks) * cvr_powf_nb(ds, A.shininess);
        return f3{fmaf(A.ispec[0], spec, rgb.x * diff), fmaf(A.ispec[1], spec, rgb.y * diff),
                  fmaf(A.ispec[2], spec, rgb.z * diff)};
      }
      return rgb;
    }
    return f3{inv_k * ((rgb.x * r.iocc) * Q.ka + (rgb.x * r.isdw) * Q.kd),
              inv_k * ((rgb.y * r.iocc) * Q.ka + (rgb.y * r.isdw) * Q.kd),
              inv_k * ((rgb.z * r.iocc) * Q.ka + (rgb.z * r.isdw) * Q.kd)};
  }
  // Forced inline: as a call (the inliner's choice for filter_bits 8, or after small
  // changes to the taps) the kernel-argument block Q is copied to scratch, ~1.9 KB
  // per lane, and the frame runs ~7x slower (72 -> 11 ms)
  __device__ static __forceinline__ f3 shade(const DosArgs& Q, const uint4* __restrict__ ext, f3 tx, f3 wp,
                                             f3 cam, f3 rgb, const f3* g, uint32_t& lit, uint32_t& fetches) {
    const Vis r = visibility(Q, ext, tx, wp, cam, lit, fetches);
    return combine(Q, r, wp, rgb, g);
  }
};

template <class SH>
static hipError_t launch_dos_fb(const Ctx& c, const DosArgs& q, float4* out, uint32_t* samples,
                                unsigned long long* shade, unsigned long long* tile_samples, hipStream_t s) {
  if (c.shade_flat)
    return launch_shaded_flat<SH>(c, q, q.phong != 0, c.d_ext_cells, out, samples, shade, tile_samples, s);
  return launch_shaded_march<SH>(c, q, q.phong != 0, c.d_ext_cells, out, samples, shade, tile_samples, s);
}

hipError_t launch_dos(const Ctx& c, const DosArgs& q, float4* out, uint32_t* samples,
                      unsigned long long* shade, unsigned long long* tile_samples, hipStream_t s) {
  if (q.a.filter_bits == 8)   // GL texture-unit weights (CVR-SPEC-8)
    return launch_dos_fb<DosShaderT<8>>(c, q, out, samples, shade, tile_samples, s);
  if (q.a.exp_native)         // tolerance mode: the border attenuation's exp in hardware
    return launch_dos_fb<DosShaderT<kDosNativeExp>>(c, q, out, samples, shade, tile_samples, s);
  return launch_dos_fb<DosShaderT<0>>(c, q, out, samples, shade, tile_samples, s);
}

}  // namespace cvr
