// ebs.hip — extinction-based shading (cppvolrend rc1pextbsd) on gfx950.
//
// The march of shaded_march.h with ShadeSample of ebs_ray_bbox_marching.comp
// (:498-550): an ambient occlusion from 15 concentric SAT boxes around the
// sample (ExtinctionAmbientOcclusion :109-146, 120 SAT fetches) and a shadow
// from a chain of SAT boxes along the dominant axis of the light direction,
// widened by the cone angle (ExtinctionDirectionalShadows / ConeX|Y|ZAxis
// :187-481; up to ~N/2 boxes of 8 fetches).  A SAT fetch is the GL_LINEAR
// texture(TexVolumeSAT3D, p / (G + 2 s)) of the float SAT (sat.hip).
// Arithmetic follows CVR-SPEC as oracle/cvr_oracle.cpp (oracle_render_ebs_rows)
// does, op for op, so the images are bit-identical.  Compiled -ffp-contract=off.
#include <hip/hip_runtime.h>
#include <cstdint>

#include "cvr_device.h"
#include "march_common.h"
#include "shaded_march.h"

namespace cvr {

namespace {

// The two device layouts of the float SAT (option "sat_layout"; addressing:
// sat_texel_index, cvr_internal.h).  corners(idx) gives a texel's 8 GL_LINEAR
// corners as lo = (x, x+1 of row y; x, x+1 of row y+1) of plane z and hi, the
// same of plane z + 1.
//  * SatCell4: the cell4 copy (a float4 of a plane's 4 corners per texel, plus
//    one repeated top plane; sat.hip sat_cells_kernel): two dwordx4 loads;
//  * SatPlain: the plain x-fastest float SAT (4x smaller), four float pairs.  A
//    clamped texel's +1 neighbours (weight exactly 0) are the next row / plane's
//    first element or the zero planes past the SAT (kSatPlainPadPlanes), all
//    finite, so each lerp returns its first operand as the cell4 copy's
//    repeated corner does: the same bits.
struct SatCell4 {
  using Ptr = const float4*;
  static constexpr int kFB = 0;   // GL_LINEAR weights at kFB fraction bits (filter_bits; 0 = exact)
  __device__ static __forceinline__ void corners(Ptr sat, uint32_t idx, uint32_t w, uint32_t pz,
                                                 float4& lo, float4& hi) {
    lo = sat[idx];
    hi = sat[idx + pz];
  }
};
struct SatPlain {
  using Ptr = const float*;
  static constexpr int kFB = 0;
  typedef float f2a __attribute__((ext_vector_type(2), aligned(4)));   // dwordx2 at 4-byte alignment
  __device__ static __forceinline__ void corners(Ptr sat, uint32_t idx, uint32_t w, uint32_t pz,
                                                 float4& lo, float4& hi) {
    const f2a a = *reinterpret_cast<const f2a*>(sat + idx);
    const f2a b = *reinterpret_cast<const f2a*>(sat + (idx + w));
    const f2a c = *reinterpret_cast<const f2a*>(sat + (idx + pz));
    const f2a d = *reinterpret_cast<const f2a*>(sat + (idx + pz + w));
    lo = make_float4(a.x, a.y, b.x, b.y);
    hi = make_float4(c.x, c.y, d.x, d.y);
  }
};

// A layout whose fetches round their GL_LINEAR weights to FB fraction bits
// (option filter_bits, CVR-SPEC-8: as a GPU texture unit filters texture()).
template <class Base, int FB>
struct SatFB : Base {
  static constexpr int kFB = FB;
};

// GetSummed3Density (:77-83): trilinear of the float SAT at u = p * inv_vol_scaled.
template <class L>
__device__ __forceinline__ float sat_fetch(const EbsArgs& Q, typename L::Ptr __restrict__ sat, float x,
                                           float y, float z) {
  const float tx = __builtin_amdgcn_fmed3f(fmaf(x * Q.inv_vs[0], Q.nsat[0], -0.5f), 0.0f, Q.nsat_m1[0]);
  const float ty = __builtin_amdgcn_fmed3f(fmaf(y * Q.inv_vs[1], Q.nsat[1], -0.5f), 0.0f, Q.nsat_m1[1]);
  const float tz = __builtin_amdgcn_fmed3f(fmaf(z * Q.inv_vs[2], Q.nsat[2], -0.5f), 0.0f, Q.nsat_m1[2]);
  // < 2^31 texels (checked on the host): 32-bit index, 24-bit row products
  const uint32_t idx = sat_texel_index((uint32_t)tx, (uint32_t)ty, (uint32_t)tz, (uint32_t)Q.sat_dims[0],
                                       (uint32_t)Q.sat_dims[1]);
  float4 lo, hi;
  L::corners(sat, idx, (uint32_t)Q.sat_dims[0], Q.sat_pz, lo, hi);
  const float ax = filter_weight<L::kFB>(__builtin_amdgcn_fractf(tx)),
              ay = filter_weight<L::kFB>(__builtin_amdgcn_fractf(ty)),
              az = filter_weight<L::kFB>(__builtin_amdgcn_fractf(tz));
  const float c00 = lerpf(lo.x, lo.y, ax), c10 = lerpf(lo.z, lo.w, ax);
  const float c01 = lerpf(hi.x, hi.y, ax), c11 = lerpf(hi.z, hi.w, ax);
  return lerpf(lerpf(c00, c10, ay), lerpf(c01, c11, ay), az);
}

// EvaluateSAT3D (:85-99)
template <class L>
__device__ __forceinline__ float sat_box(const EbsArgs& Q, typename L::Ptr __restrict__ sat, f3 p1, f3 p2) {
  const float V1 = sat_fetch<L>(Q, sat, p2.x, p2.y, p2.z), V2 = sat_fetch<L>(Q, sat, p1.x, p2.y, p2.z);
  const float V3 = sat_fetch<L>(Q, sat, p2.x, p2.y, p1.z), V4 = sat_fetch<L>(Q, sat, p1.x, p2.y, p1.z);
  const float V5 = sat_fetch<L>(Q, sat, p2.x, p1.y, p2.z), V6 = sat_fetch<L>(Q, sat, p1.x, p1.y, p2.z);
  const float V7 = sat_fetch<L>(Q, sat, p2.x, p1.y, p1.z), V8 = sat_fetch<L>(Q, sat, p1.x, p1.y, p1.z);
  return (V1 - V2 - V3 + V4 - V5 + V6 + V7 - V8);
}

// clamp(p + VolumeScales, MinSATPosition, MaxSATPosition)
__device__ __forceinline__ f3 sat_offset(const EbsArgs& Q, f3 p) {
  return f3{fminf(fmaxf(p.x + Q.S[0], Q.min_sat[0]), Q.max_sat[0]),
            fminf(fmaxf(p.y + Q.S[1], Q.min_sat[1]), Q.max_sat[1]),
            fminf(fmaxf(p.z + Q.S[2], Q.min_sat[2]), Q.max_sat[2])};
}

// z_mean / d of a cone edge: by the reciprocal (div_by_recip, exact for a normal
// d and 1/d) when the host has proven d >= cos(89 deg) for every sample (cone
// angle <= 44 deg: the dominant-axis projection is within 45 deg of its axis and
// the cone turns it by at most the cone angle), else the IEEE division (d -> 0
// as the cone angle nears 90 deg: z_mean / 0 = inf, where the reciprocal path
// would give NaN).
template <bool R>
__device__ __forceinline__ float cone_div(float a, float d, float rd) {
  return R ? div_by_recip(a, d, rd) : a / d;
}

// EvaluateShadowSAT3D (:148-185, the texture path)
template <class L>
__device__ __forceinline__ float shadow_box(const EbsArgs& Q, typename L::Ptr __restrict__ sat, f3 p1, f3 p2,
                                           f3 rS) {
  const float volquery = (div_by_recip(fabsf(p1.x - p2.x), Q.S[0], rS.x)) *
                         (div_by_recip(fabsf(p1.y - p2.y), Q.S[1], rS.y)) *
                         (div_by_recip(fabsf(p1.z - p2.z), Q.S[2], rS.z));
  return ((sat_box<L>(Q, sat, sat_offset(Q, p1), sat_offset(Q, p2)) / volquery)) * Q.ui_weight;
}

// The same shadow box as a software pipeline, half a box deep.  A box's eight
// SAT fetches fall in two halves, V1..V4 (at p2.y) and V5..V8 (at p1.y).  The
// chain issues the second half of box i, finishes the first half, issues the
// first half of box i+1 and finishes the second half of box i, so eight cell
// loads are always in flight behind the lerps while only two half-boxes (64
// VGPRs, as many as one whole box) are held.  The operations and their order
// are shadow_box's, so the bits are too.  The loads of a box past the end of a
// chain are in bounds (its coordinates are clamped as for any box) and unused.
// (A generic NP-part version, 2 / 4 / 8 parts with NP-1 in flight and the next
// box's coordinates computed at the top, measured slower at every depth: EBS
// 512^3 kernel 37.6 ms at 4 parts, 36.0 at 2, 36.3 at 8, vs 36.1 unpipelined and
// 32.9 for this one; profiles/r02_ebs_pipe_ab.txt.)
struct SatBoxCoord {
  float tx[2], ty[2], tz[2];         // texel coordinates of p1 / p2 (after sat_offset)
  float vq;                          // volquery
};

__device__ __forceinline__ float sat_texel(float x, float inv_vs, float n, float n_m1) {
  return __builtin_amdgcn_fmed3f(fmaf(x * inv_vs, n, -0.5f), 0.0f, n_m1);
}

__device__ __forceinline__ SatBoxCoord shadow_box_coord(const EbsArgs& Q, f3 p1, f3 p2, f3 rS) {
  SatBoxCoord C;
  C.vq = (div_by_recip(fabsf(p1.x - p2.x), Q.S[0], rS.x)) *
         (div_by_recip(fabsf(p1.y - p2.y), Q.S[1], rS.y)) *
         (div_by_recip(fabsf(p1.z - p2.z), Q.S[2], rS.z));
  const f3 q1 = sat_offset(Q, p1), q2 = sat_offset(Q, p2);
  C.tx[0] = sat_texel(q1.x, Q.inv_vs[0], Q.nsat[0], Q.nsat_m1[0]);
  C.tx[1] = sat_texel(q2.x, Q.inv_vs[0], Q.nsat[0], Q.nsat_m1[0]);
  C.ty[0] = sat_texel(q1.y, Q.inv_vs[1], Q.nsat[1], Q.nsat_m1[1]);
  C.ty[1] = sat_texel(q2.y, Q.inv_vs[1], Q.nsat[1], Q.nsat_m1[1]);
  C.tz[0] = sat_texel(q1.z, Q.inv_vs[2], Q.nsat[2], Q.nsat_m1[2]);
  C.tz[1] = sat_texel(q2.z, Q.inv_vs[2], Q.nsat[2], Q.nsat_m1[2]);
  return C;
}

// V_k (k = 0..7 for V1..V8) is the fetch at p1.x if k & 1, p1.z if k & 2,
// p1.y if k & 4 (else p2): half H holds k = 4H .. 4H+3.
template <int H, class L>
__device__ __forceinline__ void shadow_half_issue(const EbsArgs& Q, typename L::Ptr __restrict__ sat,
                                                  const SatBoxCoord& C, float4 (&c)[8]) {
  const uint32_t ty = (uint32_t)C.ty[H ? 0 : 1];
#pragma unroll
  for (int j = 0; j < 4; j++) {
    const int k = 4 * H + j;
    const int xi = (k & 1) ? 0 : 1, zi = (k & 2) ? 0 : 1;
    const uint32_t idx = sat_texel_index((uint32_t)C.tx[xi], ty, (uint32_t)C.tz[zi],
                                         (uint32_t)Q.sat_dims[0], (uint32_t)Q.sat_dims[1]);
    L::corners(sat, idx, (uint32_t)Q.sat_dims[0], Q.sat_pz, c[2 * j], c[2 * j + 1]);
  }
}

template <int H, int FB>
__device__ __forceinline__ void shadow_half_finish(const SatBoxCoord& C, const float4 (&c)[8], float (&V)[4]) {
  const float ay = filter_weight<FB>(__builtin_amdgcn_fractf(C.ty[H ? 0 : 1]));
#pragma unroll
  for (int j = 0; j < 4; j++) {
    const int k = 4 * H + j;
    const int xi = (k & 1) ? 0 : 1, zi = (k & 2) ? 0 : 1;
    const float ax = filter_weight<FB>(__builtin_amdgcn_fractf(C.tx[xi])),
                az = filter_weight<FB>(__builtin_amdgcn_fractf(C.tz[zi]));
    const float4 lo = c[2 * j], hi = c[2 * j + 1];
    const float c00 = lerpf(lo.x, lo.y, ax), c10 = lerpf(lo.z, lo.w, ax);
    const float c01 = lerpf(hi.x, hi.y, ax), c11 = lerpf(hi.z, hi.w, ax);
    V[j] = lerpf(lerpf(c00, c10, ay), lerpf(c01, c11, ay), az);
  }
}

#ifndef CVR_EBS_PIPE
#define CVR_EBS_PIPE 1
#endif

// The box chain of a cone: while cond(w) { Stau += box(w); w += si }, with
// box_at(w, p1, p2) giving the box corners at axis position w (ConeZAxis
// :240-272 and its Y / X twins).  Pipelined half a box deep (CVR_EBS_PIPE).
template <class L, class Cond, class BoxAt>
__device__ __forceinline__ float shadow_chain(const EbsArgs& Q, typename L::Ptr __restrict__ sat, f3 rS,
                                              float w, float si, Cond cond, BoxAt box_at,
                                              uint32_t& boxes) {
  float Stau = 0.0f;
  f3 p1, p2;
  if (!CVR_EBS_PIPE) {
    while (cond(w)) {
      box_at(w, p1, p2);
      Stau += shadow_box<L>(Q, sat, p1, p2, rS);
      boxes++;
      w = w + si;
    }
    return Stau;
  }
  if (!cond(w)) return Stau;
  box_at(w, p1, p2);
  SatBoxCoord C = shadow_box_coord(Q, p1, p2, rS);
  float4 F[8], S[8];
  float V[4];
  shadow_half_issue<0, L>(Q, sat, C, F);
  for (;;) {
    shadow_half_issue<1, L>(Q, sat, C, S);
    __builtin_amdgcn_sched_barrier(0);   // keep the loads ahead of the lerps
    shadow_half_finish<0, L::kFB>(C, F, V);
    float sum = V[0] - V[1] - V[2] + V[3];
    const float wn = w + si;
    const bool more = cond(wn);
    box_at(wn, p1, p2);
    const SatBoxCoord Cn = shadow_box_coord(Q, p1, p2, rS);
    shadow_half_issue<0, L>(Q, sat, Cn, F);
    __builtin_amdgcn_sched_barrier(0);
    shadow_half_finish<1, L::kFB>(C, S, V);
    sum = sum - V[0] + V[1] + V[2] - V[3];
    Stau += (sum / C.vq) * Q.ui_weight;
    boxes++;
    if (!more) break;
    w = wn;
    C = Cn;
  }
  return Stau;
}

// ExtinctionAmbientOcclusion (:109-146)
template <class L>
__device__ float ebs_occlusion(const EbsArgs& Q, typename L::Ptr __restrict__ sat, f3 tx) {
  const float R = Q.occ_radius;
  const f3 r0{R * Q.S[0], R * Q.S[1], R * Q.S[2]};
  const float SAT_Sh0 = sat_box<L>(Q, sat, sat_offset(Q, f3{tx.x - r0.x, tx.y - r0.y, tx.z - r0.z}),
                                sat_offset(Q, f3{tx.x + r0.x, tx.y + r0.y, tx.z + r0.z}));
  // the weights 1 / r^2 and W_A are the same for every sample: Q.ao_w / Q.ao_wa,
  // computed on the host by the same float expressions
  const bool tab = Q.occ_shells <= EbsArgs::kMaxAoShells;
  const float tSh0 = SAT_Sh0 * (tab ? Q.ao_w[0] : 1.0f / (R * R));
  float SAT_Shi = SAT_Sh0, tshi = tSh0;
  for (int i = 1; i < Q.occ_shells; i++) {
    const float r1 = R * (float)(i + 1);
    const f3 ri{r1 * Q.S[0], r1 * Q.S[1], r1 * Q.S[2]};
    const float SAT_Shi_1 = sat_box<L>(Q, sat, sat_offset(Q, f3{tx.x - ri.x, tx.y - ri.y, tx.z - ri.z}),
                                    sat_offset(Q, f3{tx.x + ri.x, tx.y + ri.y, tx.z + ri.z}));
    const float tshi_1 = tshi + (SAT_Shi_1 - SAT_Shi) * (tab ? Q.ao_w[i] : 1.0f / (r1 * r1));
    SAT_Shi = SAT_Shi_1;
    tshi = tshi_1;
  }
  const float rshi = R * (float)Q.occ_shells;
  const float W_A = tab ? Q.ao_wa : 1.0f / (rshi * rshi);
  const float Stau = W_A * tshi;
  return cvr_expf(-(Stau));
}

// ConeZAxis (:187-275)
template <class L, bool R>
__device__ float cone_z(const EbsArgs& Q, typename L::Ptr __restrict__ sat, f3 pos, f3 cv,
                        uint32_t& boxes) {
  float signal = 1.0f;
  if (cv.z < 0) signal = -1.0f;
  const float p_cs = Q.p_cs, p_sn = Q.p_sn, n_cs = Q.n_cs, n_sn = Q.n_sn;
  const f3 rS{1.0f / Q.S[0], 1.0f / Q.S[1], 1.0f / Q.S[2]};   // loop-invariant divisors
  const f3 proj_y = normalize3(f3{0.0f, cv.y, cv.z});
  const f3 proj_x = normalize3(f3{cv.x, 0.0f, cv.z});
  const f3 pj_x1 = normalize3(f3{proj_x.x * n_cs - proj_x.z * n_sn, 0.0f, proj_x.x * n_sn + proj_x.z * n_cs});
  const f3 pj_x2 = normalize3(f3{proj_x.x * p_cs - proj_x.z * p_sn, 0.0f, proj_x.x * p_sn + proj_x.z * p_cs});
  const f3 pj_y1 = normalize3(f3{0.0f, proj_y.y * n_cs - proj_y.z * n_sn, proj_y.y * n_sn + proj_y.z * n_cs});
  const f3 pj_y2 = normalize3(f3{0.0f, proj_y.y * p_cs - proj_y.z * p_sn, proj_y.y * p_sn + proj_y.z * p_cs});
  const float si = Q.interval * signal * Q.S[2];
  float z_pos = Q.initial_step * signal * Q.S[2];
  const float vmin = Q.S[2] * 0.5f, vmax = Q.G[2] - Q.S[2] * 0.5f;
  const float d_x1 = fabsf(pj_x1.z), d_x2 = fabsf(pj_x2.z), d_y1 = fabsf(pj_y1.z), d_y2 = fabsf(pj_y2.z);
  const float r_x1 = 1.0f / d_x1, r_x2 = 1.0f / d_x2, r_y1 = 1.0f / d_y1, r_y2 = 1.0f / d_y2;
  const float rc = 1.0f / cv.z;
  auto cond = [&](float z_pos) {
    return div_by_recip(z_pos, cv.z, rc) < Q.max_distance &&
           (pos.z + (z_pos + si) > vmin && pos.z + (z_pos + si) < vmax);
  };
  auto box_at = [&](float z_pos, f3& p1, f3& p2) {
    const float z_mean = fabsf(z_pos + si * 0.5f);
    const float p_x1 = pj_x1.x * cone_div<R>(z_mean, d_x1, r_x1);
    const float p_x2 = pj_x2.x * cone_div<R>(z_mean, d_x2, r_x2);
    const float p_y1 = pj_y1.y * cone_div<R>(z_mean, d_y1, r_y1);
    const float p_y2 = pj_y2.y * cone_div<R>(z_mean, d_y2, r_y2);
    float x1 = fminf(p_x1, p_x2), x2 = fmaxf(p_x1, p_x2);
    float y1 = fminf(p_y1, p_y2), y2 = fmaxf(p_y1, p_y2);
    const float xdiff = fabsf(x2 - x1), ydiff = fabsf(y2 - y1);
    const float xq = div_by_recip(xdiff, Q.S[0], rS.x), yq = div_by_recip(ydiff, Q.S[1], rS.y);
    const float xs = (ceilf(xq) - xq) * 0.5f;
    const float ys = (ceilf(yq) - yq) * 0.5f;
    x1 = x1 - xs * Q.S[0]; x2 = x2 + xs * Q.S[0];
    y1 = y1 - ys * Q.S[1]; y2 = y2 + ys * Q.S[1];
    const float z1 = fminf(z_pos, z_pos + si), z2 = fmaxf(z_pos, z_pos + si);
    p1 = f3{pos.x + x1, pos.y + y1, pos.z + z1};
    p2 = f3{pos.x + x2, pos.y + y2, pos.z + z2};
  };
  return shadow_chain<L>(Q, sat, rS, z_pos, si, cond, box_at, boxes);
}

// ConeYAxis (:277-364)
template <class L, bool R>
__device__ float cone_y(const EbsArgs& Q, typename L::Ptr __restrict__ sat, f3 pos, f3 cv,
                        uint32_t& boxes) {
  float signal = 1.0f;
  if (cv.y < 0) signal = -1.0f;
  const float p_cs = Q.p_cs, p_sn = Q.p_sn, n_cs = Q.n_cs, n_sn = Q.n_sn;
  const f3 rS{1.0f / Q.S[0], 1.0f / Q.S[1], 1.0f / Q.S[2]};   // loop-invariant divisors
  const f3 proj_x = normalize3(f3{cv.x, cv.y, 0.0f});
  const f3 proj_z = normalize3(f3{0.0f, cv.y, cv.z});
  const f3 pj_x1 = normalize3(f3{proj_x.x * n_cs - proj_x.y * n_sn, proj_x.x * n_sn + proj_x.y * n_cs, 0.0f});
  const f3 pj_x2 = normalize3(f3{proj_x.x * p_cs - proj_x.y * p_sn, proj_x.x * p_sn + proj_x.y * p_cs, 0.0f});
  const f3 pj_z1 = normalize3(f3{0.0f, proj_z.z * n_sn + proj_z.y * n_cs, proj_z.z * n_cs - proj_z.y * n_sn});
  const f3 pj_z2 = normalize3(f3{0.0f, proj_z.z * p_sn + proj_z.y * p_cs, proj_z.z * p_cs - proj_z.y * p_sn});
  const float si = Q.interval * signal * Q.S[1];
  float y_pos = Q.initial_step * signal * Q.S[1];
  const float vmin = Q.S[1] * 0.5f, vmax = Q.G[1] - Q.S[1] * 0.5f;
  const float d_x1 = fabsf(pj_x1.y), d_x2 = fabsf(pj_x2.y), d_z1 = fabsf(pj_z1.y), d_z2 = fabsf(pj_z2.y);
  const float r_x1 = 1.0f / d_x1, r_x2 = 1.0f / d_x2, r_z1 = 1.0f / d_z1, r_z2 = 1.0f / d_z2;
  const float rc = 1.0f / cv.y;
  auto cond = [&](float y_pos) {
    return div_by_recip(y_pos, cv.y, rc) < Q.max_distance &&
           (pos.y + (y_pos + si) > vmin && pos.y + (y_pos + si) < vmax);
  };
  auto box_at = [&](float y_pos, f3& p1, f3& p2) {
    const float y_mean = fabsf(y_pos + si * 0.5f);
    const float p_x1 = pj_x1.x * cone_div<R>(y_mean, d_x1, r_x1);
    const float p_x2 = pj_x2.x * cone_div<R>(y_mean, d_x2, r_x2);
    const float p_z1 = pj_z1.z * cone_div<R>(y_mean, d_z1, r_z1);
    const float p_z2 = pj_z2.z * cone_div<R>(y_mean, d_z2, r_z2);
    float x1 = fminf(p_x1, p_x2), x2 = fmaxf(p_x1, p_x2);
    float z1 = fminf(p_z1, p_z2), z2 = fmaxf(p_z1, p_z2);
    const float xdiff = fabsf(x2 - x1), zdiff = fabsf(z2 - z1);
    const float xq = div_by_recip(xdiff, Q.S[0], rS.x), zq = div_by_recip(zdiff, Q.S[2], rS.z);
    const float xs = (ceilf(xq) - xq) * 0.5f;
    const float zs = (ceilf(zq) - zq) * 0.5f;
    x1 = x1 - xs * Q.S[0]; x2 = x2 + xs * Q.S[0];
    z1 = z1 - zs * Q.S[2]; z2 = z2 + zs * Q.S[2];
    const float y1 = fminf(y_pos, y_pos + si), y2 = fmaxf(y_pos, y_pos + si);
    p1 = f3{pos.x + x1, pos.y + y1, pos.z + z1};
    p2 = f3{pos.x + x2, pos.y + y2, pos.z + z2};
  };
  return shadow_chain<L>(Q, sat, rS, y_pos, si, cond, box_at, boxes);
}

// ConeXAxis (:366-453)
template <class L, bool R>
__device__ float cone_x(const EbsArgs& Q, typename L::Ptr __restrict__ sat, f3 pos, f3 cv,
                        uint32_t& boxes) {
  float signal = 1.0f;
  if (cv.x < 0) signal = -1.0f;
  const float p_cs = Q.p_cs, p_sn = Q.p_sn, n_cs = Q.n_cs, n_sn = Q.n_sn;
  const f3 rS{1.0f / Q.S[0], 1.0f / Q.S[1], 1.0f / Q.S[2]};   // loop-invariant divisors
  const f3 proj_y = normalize3(f3{cv.x, cv.y, 0.0f});
  const f3 proj_z = normalize3(f3{cv.x, 0.0f, cv.z});
  const f3 pj_y1 = normalize3(f3{proj_y.y * n_sn + proj_y.x * n_cs, proj_y.y * n_cs - proj_y.x * n_sn, 0.0f});
  const f3 pj_y2 = normalize3(f3{proj_y.y * p_sn + proj_y.x * p_cs, proj_y.y * p_cs - proj_y.x * p_sn, 0.0f});
  const f3 pj_z1 = normalize3(f3{proj_z.z * n_sn + proj_z.x * n_cs, 0.0f, proj_z.z * n_cs - proj_z.x * n_sn});
  const f3 pj_z2 = normalize3(f3{proj_z.z * p_sn + proj_z.x * p_cs, 0.0f, proj_z.z * p_cs - proj_z.x * p_sn});
  const float si = Q.interval * signal * Q.S[0];
  float x_pos = Q.initial_step * signal * Q.S[0];
  const float vmin = Q.S[0] * 0.5f, vmax = Q.G[0] - Q.S[0] * 0.5f;
  const float d_y1 = fabsf(pj_y1.x), d_y2 = fabsf(pj_y2.x), d_z1 = fabsf(pj_z1.x), d_z2 = fabsf(pj_z2.x);
  const float r_y1 = 1.0f / d_y1, r_y2 = 1.0f / d_y2, r_z1 = 1.0f / d_z1, r_z2 = 1.0f / d_z2;
  const float rc = 1.0f / cv.x;
  auto cond = [&](float x_pos) {
    return div_by_recip(x_pos, cv.x, rc) < Q.max_distance &&
           (pos.x + (x_pos + si) > vmin && pos.x + (x_pos + si) < vmax);
  };
  auto box_at = [&](float x_pos, f3& p1, f3& p2) {
    const float x_mean = fabsf(x_pos + si * 0.5f);
    const float p_y1 = pj_y1.y * cone_div<R>(x_mean, d_y1, r_y1);
    const float p_y2 = pj_y2.y * cone_div<R>(x_mean, d_y2, r_y2);
    const float p_z1 = pj_z1.z * cone_div<R>(x_mean, d_z1, r_z1);
    const float p_z2 = pj_z2.z * cone_div<R>(x_mean, d_z2, r_z2);
    float y1 = fminf(p_y1, p_y2), y2 = fmaxf(p_y1, p_y2);
    float z1 = fminf(p_z1, p_z2), z2 = fmaxf(p_z1, p_z2);
    const float ydiff = fabsf(y2 - y1), zdiff = fabsf(z2 - z1);
    const float yq = div_by_recip(ydiff, Q.S[1], rS.y), zq = div_by_recip(zdiff, Q.S[2], rS.z);
    const float ys = (ceilf(yq) - yq) * 0.5f;
    const float zs = (ceilf(zq) - zq) * 0.5f;
    y1 = y1 - ys * Q.S[1]; y2 = y2 + ys * Q.S[1];
    z1 = z1 - zs * Q.S[2]; z2 = z2 + zs * Q.S[2];
    const float x1 = fminf(x_pos, x_pos + si), x2 = fmaxf(x_pos, x_pos + si);
    p1 = f3{pos.x + x1, pos.y + y1, pos.z + z1};
    p2 = f3{pos.x + x2, pos.y + y2, pos.z + z2};
  };
  return shadow_chain<L>(Q, sat, rS, x_pos, si, cond, box_at, boxes);
}

}  // namespace

#ifndef CVR_EBS_FLAT_WAVES
#define CVR_EBS_FLAT_WAVES 1   // flat shading: the compiler's 128 VGPRs, 4 waves/SIMD
#endif
#ifndef CVR_EBS_WAVES
#define CVR_EBS_WAVES 1
#endif
template <bool RECIP_CONE, class LY>
struct EbsShaderT {
  using Args = EbsArgs;
  static constexpr int kMinWavesPerEU = CVR_EBS_WAVES;   // register budget (1: compiler's choice)
  static constexpr int kFlatWavesPerEU = CVR_EBS_FLAT_WAVES;   // flat_shade_kernel
  static constexpr bool kSplit = false;   // flat_shade_kernel calls shade() whole
  using Data = typename LY::Ptr;   // the float SAT, cell4 or plain
  static constexpr int kFB = LY::kFB;   // GL_LINEAR weights of every fetch (filter_bits)

  // ShadeSample (:498-550); `lit` counts the shadow box chains traced.
  __device__ static f3 shade(const EbsArgs& Q, typename LY::Ptr __restrict__ sat, f3 tx, f3 wp, f3,
                             f3 rgb, const f3* g, uint32_t& lit, uint32_t& fetches) {
    const Rc1passArgs& A = Q.a;
    const f3 eye{A.eye[0], A.eye[1], A.eye[2]};
    const f3 light{A.light[0], A.light[1], A.light[2]};
    float iocc = 0.0f, isdw = 0.0f;
    if (Q.apply_occlusion) {
      iocc = ebs_occlusion<LY>(Q, sat, tx);
      fetches += 8 * Q.occ_shells;
    }
    if (Q.apply_shadow) {
      // ExtinctionDirectionalShadows (:455-481)
      const f3 cv = Q.shadow_type == 0 ? normalize3(f3{light.x - wp.x, light.y - wp.y, light.z - wp.z})
                                       : normalize3(f3{Q.lfwd[0], Q.lfwd[1], Q.lfwd[2]});
      const f3 ac{fabsf(cv.x), fabsf(cv.y), fabsf(cv.z)};
      float Stau;
      uint32_t boxes = 0;
      if (ac.z > ac.x && ac.z > ac.y) Stau = cone_z<LY, RECIP_CONE>(Q, sat, tx, cv, boxes);
      else if (ac.y > ac.x) Stau = cone_y<LY, RECIP_CONE>(Q, sat, tx, cv, boxes);
      else Stau = cone_x<LY, RECIP_CONE>(Q, sat, tx, cv, boxes);
      fetches += 8 * boxes;
      isdw = cvr_expf(-Stau);
      lit++;
    }
    const float inv_k = 1.0f / (Q.ka + Q.kd);
    if (g) {   // ApplyPhongShading
      if (g->x != 0.0f || g->y != 0.0f || g->z != 0.0f) {
        const f3 nrm = normalize3(*g);
        const f3 L = normalize3(f3{light.x - wp.x, light.y - wp.y, light.z - wp.z});
        const f3 Ve = normalize3(f3{eye.x - wp.x, eye.y - wp.y, eye.z - wp.z});
        const f3 Hv = normalize3(f3{Ve.x + L.x, Ve.y + L.y, Ve.z + L.z});
        const float dd = fmaxf(0.0f, dot3(nrm, L));
        const float ds = fmaxf(0.0f, dot3(Hv, nrm));
        const float pw = cvr_powf_nb(ds, A.shininess);
        // (1/(ka+kd)) * (L*IOcc*ka + IShadow*(L*kd*dot_diff)) + IShadow*(ks*Ispecular*pow) (:528-530)
        return f3{inv_k * ((rgb.x * iocc) * Q.ka + isdw * ((rgb.x * Q.kd) * dd)) + isdw * ((Q.ks * A.ispec[0]) * pw),
                  inv_k * ((rgb.y * iocc) * Q.ka + isdw * ((rgb.y * Q.kd) * dd)) + isdw * ((Q.ks * A.ispec[1]) * pw),
                  inv_k * ((rgb.z * iocc) * Q.ka + isdw * ((rgb.z * Q.kd) * dd)) + isdw * ((Q.ks * A.ispec[2]) * pw)};
      }
      return rgb;
    }
    return f3{inv_k * ((rgb.x * iocc) * Q.ka + (rgb.x * isdw) * Q.kd),
              inv_k * ((rgb.y * iocc) * Q.ka + (rgb.y * isdw) * Q.kd),
              inv_k * ((rgb.z * iocc) * Q.ka + (rgb.z * isdw) * Q.kd)};
  }
};

template <class L>
static hipError_t launch_ebs_layout(const Ctx& c, const EbsArgs& q, typename L::Ptr sat, float4* out,
                                    uint32_t* samples, unsigned long long* shade,
                                    unsigned long long* tile_samples, hipStream_t s) {
  const bool ph = q.phong != 0;
  if (c.shade_flat)
    return q.recip_cone
               ? launch_shaded_flat<EbsShaderT<true, L>>(c, q, ph, sat, out, samples, shade, tile_samples, s)
               : launch_shaded_flat<EbsShaderT<false, L>>(c, q, ph, sat, out, samples, shade, tile_samples, s);
  if (q.recip_cone)
    return launch_shaded_march<EbsShaderT<true, L>>(c, q, ph, sat, out, samples, shade, tile_samples, s);
  return launch_shaded_march<EbsShaderT<false, L>>(c, q, ph, sat, out, samples, shade, tile_samples, s);
}

hipError_t launch_ebs(const Ctx& c, const EbsArgs& q, float4* out, uint32_t* samples,
                      unsigned long long* shade, unsigned long long* tile_samples, hipStream_t s) {
  if (q.a.filter_bits == 8)   // GL texture-unit weights (CVR-SPEC-8): the cell4 copy only
    return c.sat_layout == 1 ? hipErrorInvalidValue
                             : launch_ebs_layout<SatFB<SatCell4, 8>>(c, q, c.d_sat_cells, out, samples,
                                                                     shade, tile_samples, s);
  if (c.sat_layout == 1)
    return launch_ebs_layout<SatPlain>(c, q, c.d_sat, out, samples, shade, tile_samples, s);
  return launch_ebs_layout<SatCell4>(c, q, c.d_sat_cells, out, samples, shade, tile_samples, s);
}

}  // namespace cvr
