// raymarch.hip — gfx950 kernels of the structured single-pass ray-caster.
//
// Re-designs cppvolrend's ray_marching_1p.comp (rc1pass) for CDNA4:
//   * no HIP texture objects on gfx950, so trilinear filtering is done in
//     software from a padded "cell8" layout: every sample is ONE 16-byte load of
//     the 8 fp16 corners GL_LINEAR + CLAMP_TO_EDGE would read from the R16F
//     volume (libs/volvis_utils/utils.cpp:20-56); the x-lerps run as
//     mixed-precision FMAs straight on the packed halves;
//   * the 1D transfer function (RGBA16F, GenerateTexture_1D_RGBt) lives in LDS;
//   * two ways to march a ray, chosen per 8x8 screen tile:
//       - ray-parallel: one lane per ray, K samples addressed and fetched per
//         batch (K x 16 B in flight per lane), composited in order;
//       - sample-parallel ("quad"): four lanes per ray, each fetching and
//         classifying one of the next four samples, then an in-order composite
//         over the quad with DPP broadcasts.  Optional (option "quad", off by
//         default: measured slower than ray-parallel even for the longest
//         tiles) and compiled into a separate kernel;
//   * scheduling: one wave per workgroup; each XCD owns one horizontal band of
//     the screen (L2 locality) and, from the previous frame's per-tile critical
//     paths, receives its band longest-first (LPT).
//
// Arithmetic follows CVR-SPEC: explicit fmaf, IEEE div/sqrt, the
// polynomial cvr_expf.  Compiled with -ffp-contract=off; both march variants
// produce bit-identical results, equal to oracle/cvr_oracle.cpp.
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdint>

#include "cvr_device.h"
#include "march_common.h"

namespace cvr {

constexpr int kQuadFlag = 1 << 28;   // order entry = tile | (quarter + 1) << 28 for quad tiles
#ifdef CVR_PHONG_CLASSIFY_FULL
constexpr bool kPhongClassifyFull = true;
#else
constexpr bool kPhongClassifyFull = false;
#endif


// Macro-cell skip.  The macro cell m (2^mshift texels a side) of a sample is
// taken from its clamped texel coordinate exactly as sample_pos computes it; its
// occupancy byte says whether any trilinear density over texels
// [m*2^s, (m+1)*2^s] can have alpha > 0.  Samples are stepped over while their
// centre t stays below the ray's exit from the macro box shrunk by
// kMacroMargin texels (which absorbs the rounding of t_exit and of the sample
// positions, ~1e-4 texels), so every skipped sample lies in the cell.
// Returns true if at least one sample was skipped.
constexpr float kMacroMargin = 1.0f / 64.0f;

__device__ __forceinline__ bool skip_empty(const Rc1passArgs& A, const Ray& r, float step, float D,
                                           float& s, uint32_t& cnt) {
  const float h0 = fminf(step, D - s);
  const float t0 = fmaf(h0, 0.5f, s);
  const float x = __builtin_amdgcn_fmed3f(fmaf(r.dt.x, t0, r.o.x), 0.0f, A.nm1[0]);
  const float y = __builtin_amdgcn_fmed3f(fmaf(r.dt.y, t0, r.o.y), 0.0f, A.nm1[1]);
  const float z = __builtin_amdgcn_fmed3f(fmaf(r.dt.z, t0, r.o.z), 0.0f, A.nm1[2]);
  const int sh = A.mshift;
  const int mx = (int)x >> sh, my = (int)y >> sh, mz = (int)z >> sh;
  if (A.occ[(mz * A.mdim[1] + my) * A.mdim[0] + mx]) return false;
  const float w = (float)(1 << sh);
  // exit parameter of the shrunk box on each axis (1/dt = +-inf on a parallel
  // axis gives +-inf or NaN, both ignored by fminf against the other axes)
  const float bx = r.dt.x > 0.0f ? (float)(mx + 1) * w - kMacroMargin : (float)mx * w + kMacroMargin;
  const float by = r.dt.y > 0.0f ? (float)(my + 1) * w - kMacroMargin : (float)my * w + kMacroMargin;
  const float bz = r.dt.z > 0.0f ? (float)(mz + 1) * w - kMacroMargin : (float)mz * w + kMacroMargin;
  const float t_exit = fminf(fminf((bx - r.o.x) * r.inv_dt.x, (by - r.o.y) * r.inv_dt.y),
                             (bz - r.o.z) * r.inv_dt.z);
  const float s_in = s;
  while (s < D) {
    const float h = fminf(step, D - s);
    if (!(fmaf(h, 0.5f, s) < t_exit)) break;
    s = s + h;
    cnt++;
  }
  return s != s_in;
}

// Ray-parallel march (one lane per ray) of ray_marching_1p.comp:124-172.  The
// arithmetic per sample is exactly the reference's sequential loop (s
// accumulates h one step at a time); batching only changes when loads issue.
// Per-cell skip (CS, option "cell_skip", march_common.h cell_empty):
//  * CS >= 1: when sample j of every marching lane lies in an EMPTY cell (a
//    wave-uniform ballot of one sign bit per load), its trilinear density, TF
//    lookup and composite test are skipped: its tau is exactly 0, so the
//    reference composites nothing (:142) and only counts it;
//  * CS == 2: after a batch whose last sample lies in an empty cell at chessboard
//    distance d >= 2 from any non-empty cell, the next m samples are counted and
//    stepped over with the same s += h recurrence, without loads: m full steps
//    move the position by at most m * step * max|dt| <= d - 1 - kSkipMarginTexels
//    texels on every axis, so each of those samples lies in a cell within d - 1
//    of the last one (all empty), and m stays 2 steps short of the ray's end, so
//    every skipped h is the full step.
// Both leave the image and the sample count bit for bit as the plain march.

// The composite's exp two samples per packed instruction (-DCVR_PAIR_EXP; DESIGN
// §5‴): bit-exact and 45.7 -> 38.7 VALU per sample on the headline, but 4.7 %
// slower (0.0731 -> 0.0765 ms per frame, A/B in one session, profiles/r06/s12-s13):
// the march waits on dependencies, not on VALU issue.  Off by default.
#ifdef CVR_PAIR_EXP
constexpr bool kNoPairExp = false;
#else
constexpr bool kNoPairExp = true;
#endif
#ifndef CVR_PAIR_FROM
#define CVR_PAIR_FROM 2
#endif
#ifndef CVR_RECOMPUTE_TF
#define CVR_RECOMPUTE_TF 1
#endif
constexpr bool kRecomputeTf = CVR_RECOMPUTE_TF != 0;

template <int K, bool PHONG, bool SKIP, int XF, int BUF, int FB, int CS>
__device__ __forceinline__ void march_ray(const Rc1passArgs& A, const uint4* __restrict__ cells,
                                          const uint4* __restrict__ grad,
                                          const float4* __restrict__ tfp, int px, int py,
                                          float4& dst, uint32_t& cnt, uint32_t& nshade,
                                          uint32_t& nbatch, uint32_t& nskip, uint32_t& npm,
                                          uint32_t& npc) {
  dst = make_float4(0.f, 0.f, 0.f, 0.f);
  cnt = 0;
  Ray r;
  if (!ray_setup(A, px, py, r)) return;   // misses keep (0,0,0,0), renderoutputframe.cpp:187-190
  const f3 eye{A.eye[0], A.eye[1], A.eye[2]};
  const f3 hg{A.half_grid[0], A.half_grid[1], A.half_grid[2]};
  const float step = A.step, D = r.D, fn = (float)A.tf_n;
  float s = 0.0f;
  bool done = !(s < D);
  bool probe = true;
  const bool wave_in_box = __ballot(r.outside) == 0;   // the usual case: no clamps
  // BUF (cell grid < 4 GiB): buffer loads with a 32-bit byte offset from one
  // scalar resource instead of 64-bit per-lane addresses (two fewer VALU
  // instructions and VGPRs per load; -3 % on the headline frame)
  const __amdgpu_buffer_rsrc_t crs =
      __builtin_amdgcn_make_buffer_rsrc((void*)cells, 0, -1, kBufferConfigDword);
  // BUF 2 (16 * pitch_z fits a signed 24-bit operand): the byte offset in three
  // instructions, two v_mad_i32_i24 whose sums wrap mod 2^32 to the exact
  // offset (< 4 GiB); BUF 1: the cell index times 16
  auto load_cell = [&](const SamplePos& p) -> uint4 {
    if (BUF == 2)
      return buffer_load_u4(crs, mad_i24(p.iz, A.cells.bpitch_z,
                                         mad_i24(p.iy, A.cells.bpitch_y, ((uint32_t)p.ix << 4) + A.cells.borigin)));
    if (BUF == 1) return buffer_load_u4(crs, p.idx << 4);
    return cells[p.idx];
  };
  while (!done) {
    if (CS > 0) nbatch++;   // the LPT cost with skipping: loop rounds, not samples
    // Empty-space skipping (bit-exact): if the macro cell holding the next
    // sample is transparent for the current TF (every density its texels can
    // interpolate to classifies to alpha <= 0), the samples whose positions stay
    // inside it are counted and stepped over with the same s += h recurrence,
    // without loads: the reference composites nothing for them (:142).
    // Probed only after a batch that composited nothing: inside visible
    // material the lookup would add a dependent memory round trip per batch.
    if (SKIP && probe) {
      probe = false;
      if (skip_empty(A, r, step, D, s, cnt)) {
        probe = true;
        if (!(s < D)) done = true;
        continue;
      }
    }
    // stage 1: the next K sample positions (sequential s += h) and their loads.
    // Away from the ray's end every h is the full step: when D - s_(K-1) >=
    // step for every active lane (s_j = s + step + ... + step, the same adds),
    // the min / compare of each step are skipped (wave-uniform branch).
    float hj[K], tj[K];
    bool vj[K];
    SamplePos sp[K];
    uint4 raw[K];
    float ss;
    {
      float c[K + 1];
      c[0] = s;
#pragma unroll
      for (int j = 0; j < K; j++) c[j + 1] = c[j] + step;
      if (__ballot(!(D - c[K - 1] >= step)) == 0) {
#pragma unroll
        for (int j = 0; j < K; j++) {
          vj[j] = true;
          hj[j] = step;
          tj[j] = fmaf(step, 0.5f, c[j]);
        }
        ss = c[K];
      } else {
        ss = s;
#pragma unroll
        for (int j = 0; j < K; j++) {
          vj[j] = ss < D;
          hj[j] = fminf(step, D - ss);
          // a sample past the ray's end is not composited; its (discarded) load
          // goes to the entry point so that it stays inside the grid
          tj[j] = vj[j] ? fmaf(hj[j], 0.5f, ss) : 0.0f;
          ss = ss + hj[j];
        }
      }
    }
    if (wave_in_box) {
#pragma unroll
      for (int j = 0; j < K; j++) {
        sp[j] = sample_pos(fmaf(r.dt.x, tj[j], r.o.x), fmaf(r.dt.y, tj[j], r.o.y),
                           fmaf(r.dt.z, tj[j], r.o.z), A);
#ifdef CVR_PROBE_LDS_CELLS   // cost probe only: every sample from a 4 KiB LDS table (wrong images)
        {
          const uint4 v = reinterpret_cast<const uint4*>(tfp)[(sp[j].idx * 7u) & 255u];
          raw[j] = make_uint4((v.x & 0x01ff01ffu) | 0x00000000u, (v.y & 0x01ff01ffu) | 0x00000000u,
                              (v.z & 0x01ff01ffu) | 0x00000000u, (v.w & 0x01ff01ffu) | 0x00000000u);
        }
#else
        raw[j] = load_cell(sp[j]);
#endif
      }
    } else {
#pragma unroll
      for (int j = 0; j < K; j++) {
        sp[j] = sample_pos_clamped(fmaf(r.dt.x, tj[j], r.o.x), fmaf(r.dt.y, tj[j], r.o.y),
                                   fmaf(r.dt.z, tj[j], r.o.z), A);
        raw[j] = load_cell(sp[j]);
      }
    }
    if (FB) {   // GL texture-unit weights (filter_bits): volume and gradient fetches
#pragma unroll
      for (int j = 0; j < K; j++) quantise_weights<FB>(sp[j]);
    }
    // stage 2: density and transfer-function classification
    float4 src[K];
    // Emission-absorption: alpha first (two 4-B LDS reads); the rgb lerps (two
    // 16-B reads) only for visible samples, ~1 in 5 on the headline frame
    int tfi[K];
    float tfa[K];
    float txd[K];   // kPairExp: the TF coordinate, its index and weight recomputed at the rgb lerps
    // we[j], wave-uniform: sample j of every marching lane lies in an empty cell.
    // Each is tested right before its sample's math, so the loads of the later
    // samples stay in flight behind it (testing all four first waited for all).
    bool we[K];
    int qlast = 0;   // the last sample's skip distance (0: no skip), read before raw[] dies
    // Blinn-Phong too (CVR_PHONG_CLASSIFY_FULL: the round-3 full classify of every
    // sample): its shading needs the rgb only for the visible samples as well
    constexpr bool kAlphaFirst = !PHONG || !kPhongClassifyFull;
    if (kAlphaFirst) {
#pragma unroll
      for (int j = 0; j < K; j++) {
        we[j] = CS > 0 && __ballot(!cell_empty(raw[j])) == 0;
        if (CS >= 2 && j == K - 1) qlast = cell_empty(raw[j]) ? cell_skip_q(raw[j]) : 0;
        if (CS > 0 && we[j]) {
          tfa[j] = 0.0f; tfi[j] = 0; txd[j] = 0.0f; src[j].w = 0.0f;
        } else {
          const float xd = fmaf(trilerp_cell<!PHONG>(raw[j], sp[j].ax, sp[j].ay, sp[j].az), fn, -0.5f);
          tfa[j] = filter_weight<FB>(__builtin_amdgcn_fractf(xd));   // see classify
          tfi[j] = cvt_flr(xd) + 1;
          txd[j] = xd;
          src[j].w = lerpf(tfp[tfi[j]].w, tfp[tfi[j] + 1].w, tfa[j]);
        }
      }
    } else {
#pragma unroll
      for (int j = 0; j < K; j++) {
        we[j] = CS > 0 && __ballot(!cell_empty(raw[j])) == 0;
        if (CS >= 2 && j == K - 1) qlast = cell_empty(raw[j]) ? cell_skip_q(raw[j]) : 0;
        if (CS > 0 && we[j]) src[j] = make_float4(0.f, 0.f, 0.f, 0.f);
        else src[j] = classify<FB>(tfp, fn, trilerp_cell(raw[j], sp[j].ax, sp[j].ay, sp[j].az));
      }
    }
    bool visible = false;
    // Alphas two samples per packed exp (cvr_expf_neg2, the same bits as the scalar
    // cvr_expf_neg): a_j depends on sample j's extinction only, not on the
    // composite before it, so at each even j the pair (j, j+1) is computed when some
    // lane of the wave may composite either of them (empty space skips it, as the
    // composite's branches do).  Computed at the pair rather than for the whole
    // batch up front, which held four more registers across the composite and
    // spilled (13 VGPRs, 0.073 -> 0.080 ms per frame).
    constexpr bool kPairExp = XF == 1 && kAlphaFirst && (K % 2 == 0) && !kNoPairExp;
    float a_odd = 0.0f;   // the pair's second alpha, used by the next sample
    // the samples from kPairFrom on go in pairs (the first ones keep the scalar exp:
    // at j = 0 the batch's registers peak)
    constexpr int kPairFrom = CVR_PAIR_FROM;
#ifdef CVR_PROBE_SHADE_PASSES   // cost probe (tools/phong_pass_probe.py): shading passes per batch
    bool shj[K];
    if (PHONG) {
      int nv = 0;
#pragma unroll
      for (int j = 0; j < K; j++) {
        shj[j] = false;
        nv += (!done && vj[j] && !(CS > 0 && we[j]) && src[j].w > 0.0f) ? 1 : 0;
      }
      // one pass per sample the busiest lane must shade (ballots: active lanes only)
#pragma unroll
      for (int q = 1; q <= K; q++) npm += __ballot(nv >= q) != 0 ? 1u : 0u;
    }
#endif
    // stage 3: front-to-back composite + ERT, in sample order.  The branches
    // matter: a wave whose samples are all transparent (empty space) skips
    // the exp and the composite together (a branch-free select form measured
    // 1.4x slower on the headline frame).
#pragma unroll
    for (int j = 0; j < K; j++) {
      float a_even = 0.0f;
      if (kPairExp && j >= kPairFrom && ((j - kPairFrom) & 1) == 0) {
        const bool may = !done && ((vj[j] && !(CS > 0 && we[j]) && src[j].w > 0.0f) ||
                                   (vj[j + 1] && !(CS > 0 && we[j + 1]) && src[j + 1].w > 0.0f));
        if (__ballot(may) != 0) {
          const f2v e = cvr_expf_neg2(f2v{-(src[j].w * hj[j]), -(src[j + 1].w * hj[j + 1])});
          a_even = 1.0f - e.x;
          a_odd = 1.0f - e.y;
        }
      }
      if (!done) {
        if (!vj[j]) {
          done = true;
        } else {
          cnt++;
          float4 sc = src[j];
          if (!(CS > 0 && we[j]) && sc.w > 0.0f) {
            visible = true;
            if (kAlphaFirst) {   // classify's rgb, same lerps
              // (kPairExp: index and weight again from the coordinate -- two VALU per
              // visible sample for two registers fewer per batch sample across the composite)
              const int ti = kPairExp && kRecomputeTf ? cvt_flr(txd[j]) + 1 : tfi[j];
              const float ta = kPairExp && kRecomputeTf ? filter_weight<FB>(__builtin_amdgcn_fractf(txd[j])) : tfa[j];
              const float4 t0 = tfp[ti], t1 = tfp[ti + 1];
              sc.x = lerpf(t0.x, t1.x, ta);
              sc.y = lerpf(t0.y, t1.y, ta);
              sc.z = lerpf(t0.z, t1.z, ta);
            }
            if (PHONG) {
              shade_phong(A, grad, sp[j], r.dir, tj[j], r.tpos, hg, eye, sc);
              nshade++;
#ifdef CVR_PROBE_SHADE_PASSES
              shj[j] = true;
#endif
            }
            const float x = -(sc.w * hj[j]);
            const float a = (kPairExp && j >= kPairFrom) ? (((j - kPairFrom) & 1) ? a_odd : a_even)
                                     : 1.0f - (XF == 2 ? cvr_expf_native(x) : XF ? cvr_expf_neg(x) : cvr_expf_nb(x));
            const float om = 1.0f - dst.w;
            dst.x = fmaf(om, sc.x * a, dst.x);
            dst.y = fmaf(om, sc.y * a, dst.y);
            dst.z = fmaf(om, sc.z * a, dst.z);
            dst.w = fmaf(om, a, dst.w);
            if (dst.w > 0.99f) done = true;
          }
        }
      }
    }
#ifdef CVR_PROBE_SHADE_PASSES
    if (PHONG) {
#pragma unroll
      for (int j = 0; j < K; j++) npc += __ballot(shj[j]) != 0 ? 1u : 0u;   // passes run today
    }
#endif
    s = ss;
    if (!(s < D)) done = true;
    probe = !visible;
    if (CS >= 2 && wave_in_box) {
      const bool ok = !done && qlast > 0 && vj[K - 1];
      // CS 3: only when every marching lane can skip (one ballot, so a wave with
      // any lane in occupied space pays nothing more)
      if ((CS != 3 || __ballot(!ok) == 0) && ok) {
        // samples per texel of the largest per-axis move: 1 / (step * max|dt|),
        // recomputed here (the opaque copies keep the compiler from hoisting it
        // out of the loop, where it took a register and spilled)
        float dx = r.dt.x, dy = r.dt.y, dz = r.dt.z;
        asm volatile("" : "+v"(dx), "+v"(dy), "+v"(dz));
        const float kinv = __builtin_amdgcn_rcpf(step * fmaxf(fmaxf(fabsf(dx), fabsf(dy)), fabsf(dz)));
        int m = min(cvt_flr(((float)qlast - kSkipMarginTexels) * kinv), cvt_flr((D - s) * A.inv_step) - 2);
        if (CS == 2) {   // each lane its own m
          if (m > 0) {
            cnt += (uint32_t)m;
            nskip += (uint32_t)m;
            for (; m >= 4; m -= 4) {
              s = s + step;
              s = s + step;
              s = s + step;
              s = s + step;
            }
            for (; m > 0; m--) s = s + step;
          }
        } else {
          // 3 (every marching lane) / 4 (the lanes that can): they skip the same
          // number of samples, the fewest any of them may, so they stay at one
          // sample index and a wave load keeps touching neighbouring cells
          int i = 0;
          for (; __all(i < m); i++) s = s + step;
          cnt += (uint32_t)i;
          nskip += (uint32_t)i;
        }
      }
    }
  }
}

// Value of `v` in lane L of this lane's quad (DPP quad_perm broadcast).
template <int L>
__device__ __forceinline__ float quad_bcast(float v) {
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), L | (L << 2) | (L << 4) | (L << 6),
                                                 0xf, 0xf, false));
}

// One premultiplied sample of the quad march: (alpha, r*alpha, g*alpha, b*alpha).
struct QSample { float a, r, g, b; };

// Composite sample k (owned by quad lane L) into dst, in sample order.
template <int L>
__device__ __forceinline__ void quad_composite(const QSample& q, bool valid, bool& done,
                                               float4& dst, uint32_t& cnt) {
  const float ak = quad_bcast<L>(q.a), rk = quad_bcast<L>(q.r);
  const float gk = quad_bcast<L>(q.g), bk = quad_bcast<L>(q.b);
  if (!done) {
    if (valid) {
      cnt++;
      const float om = 1.0f - dst.w;
      dst.x = fmaf(om, rk, dst.x);
      dst.y = fmaf(om, gk, dst.y);
      dst.z = fmaf(om, bk, dst.z);
      dst.w = fmaf(om, ak, dst.w);
      if (dst.w > 0.99f) done = true;
    } else {
      done = true;
    }
  }
}

// Sample-parallel march: the 4 lanes of a quad share one ray.  Each iteration
// covers the ray's next 4K samples (positions from the same sequential s += h
// recurrence); sample 4k+j belongs to quad lane j, which fetches and classifies
// its K samples with all K loads in flight.  Every lane then composites the 4K
// samples in order (DPP quad broadcasts) and applies the ERT exit, so all four
// hold the ray's identical state.  A transparent sample enters the composite as
// exact zeros, which leaves dst bit-unchanged — the same result as the
// reference skipping it (:142).  One memory round trip advances a ray 4K
// samples instead of K: the longest tiles' critical path shrinks ~4x.
// Must be called by all 64 lanes (DPP reads neighbours); `active` = lane's ray is live.
template <int K, bool PHONG, int XF>
__device__ __forceinline__ void march_ray_quad(const Rc1passArgs& A,
                                               const uint4* __restrict__ cells,
                                               const uint4* __restrict__ grad,
                                               const float4* __restrict__ tfp, int px, int py,
                                               bool active, float4& dst, uint32_t& cnt) {
  const int j = threadIdx.x & 3;
  dst = make_float4(0.f, 0.f, 0.f, 0.f);
  cnt = 0;
  Ray r;
  bool hit = ray_setup(A, px, py, r);
  const float D = (active && hit) ? r.D : 0.0f;
  const f3 eye{A.eye[0], A.eye[1], A.eye[2]};
  const f3 hg{A.half_grid[0], A.half_grid[1], A.half_grid[2]};
  const float step = A.step, fn = (float)A.tf_n;
  const unsigned qshift = threadIdx.x & ~3u;
  float s = 0.0f;
  bool done = !(s < D);
  while (!__all(done)) {
    // this lane's samples: steps 4k+j of the sequential recurrence from s
    float sj[K], hj[K];
    float ss = s;
#pragma unroll
    for (int k = 0; k < K; k++) {
#pragma unroll
      for (int l = 0; l < 4; l++) {
        const float h = fminf(step, D - ss);
        if (l == j) { sj[k] = ss; hj[k] = h; }
        ss = ss + h;
      }
    }
    SamplePos sp[K];
    uint4 raw[K];
    float tj[K];
#pragma unroll
    for (int k = 0; k < K; k++) {
      tj[k] = fmaf(hj[k], 0.5f, sj[k]);
      // quad lanes of dead rays or past a ray's end load too (results dropped)
      sp[k] = sample_pos_clamped(fmaf(r.dt.x, tj[k], r.o.x), fmaf(r.dt.y, tj[k], r.o.y),
                                 fmaf(r.dt.z, tj[k], r.o.z), A);
      raw[k] = cells[sp[k].idx];
    }
    QSample q[K];
    unsigned qv[K];
#pragma unroll
    for (int k = 0; k < K; k++) {
      float4 sc = classify(tfp, fn, trilerp_cell(raw[k], sp[k].ax, sp[k].ay, sp[k].az));
      const bool vj = !done && sj[k] < D;
      q[k] = QSample{0.0f, 0.0f, 0.0f, 0.0f};
      if (vj && sc.w > 0.0f) {
        if (PHONG) shade_phong(A, grad, sp[k], r.dir, tj[k], r.tpos, hg, eye, sc);
        const float x = -(sc.w * hj[k]);
        const float a = 1.0f - (XF == 2 ? cvr_expf_native(x) : XF ? cvr_expf_neg(x) : cvr_expf_nb(x));
        q[k] = QSample{a, sc.x * a, sc.y * a, sc.z * a};
      }
      qv[k] = (unsigned)(__ballot(vj) >> qshift) & 0xfu;
    }
    // in-order composite of the 4K samples (every lane of the quad)
#pragma unroll
    for (int k = 0; k < K; k++) {
      quad_composite<0>(q[k], qv[k] & 1u, done, dst, cnt);
      quad_composite<1>(q[k], qv[k] & 2u, done, dst, cnt);
      quad_composite<2>(q[k], qv[k] & 4u, done, dst, cnt);
      quad_composite<3>(q[k], qv[k] & 8u, done, dst, cnt);
    }
    s = ss;
  }
}

// ---------------------------------------------------------------------------
// Kernel
// ---------------------------------------------------------------------------

// One workgroup = one wave.  Entry e of the launch order is a whole 8x8 tile
// (one lane per ray) or, for the longest tiles, one 4x4 quarter of a tile
// (four lanes per ray).  Without an order, block b -> tile in XCD bands
// (blocks b and b+8 share an XCD, so XCD b%8 gets one contiguous band).
// Waves of the `boost` longest tiles of each band raise their priority.
// Register budget: the plain emission-absorption march at K = 4 (the headline
// kernel, 69 VGPRs by itself -> 7 waves/SIMD) is held to 64 VGPRs for 8
// waves/SIMD (2 spilled): one kernel takes the same time (0.1207 vs 0.1217 ms)
// but frames in flight overlap better, 0.1070 -> 0.1018 ms per frame on the
// driver's command.  Blinn-Phong at K = 2 is held to 80 VGPRs, 6 waves/SIMD (the
// compiler's 93 give 5): kernel 0.3094 -> 0.3148 ms, frame 0.2723 -> 0.2608 ms.
// Every other variant is left to the compiler (Phong K = 4 at 4 waves: neutral).
// (CVR_RC1_WAVES_PER_EU: residency experiments, tools/build_variant.sh)
template <int K, bool PHONG, bool SKIP, bool QUAD>
constexpr int rc1_waves_per_eu() {
#ifdef CVR_RC1_WAVES_PER_EU
  return CVR_RC1_WAVES_PER_EU;
#else
#ifndef CVR_RC1_PHONG_WAVES2
#define CVR_RC1_PHONG_WAVES2 6
#endif
#ifndef CVR_RC1_PHONG_WAVES4
#define CVR_RC1_PHONG_WAVES4 1
#endif
  if (PHONG && !SKIP && !QUAD) return K == 2 ? CVR_RC1_PHONG_WAVES2 : CVR_RC1_PHONG_WAVES4;
  return (K == 4 && !PHONG && !SKIP && !QUAD) ? 8 : 1;
#endif
}
// Waves (8x8 tiles) per workgroup: they share one TF copy in LDS and one
// dispatch.  Slot b of the launch (launch order, bands, frames: as with one wave
// per workgroup) is wave w of workgroup B = 8 q + x with b = 8 (W q + w) + x, so
// it still runs on XCD b % 8.  (The quad march keeps one wave per workgroup.)
#ifndef CVR_RC1_WPG
#define CVR_RC1_WPG 1
#endif
template <bool QUAD>
constexpr int rc1_waves_per_group() { return QUAD ? 1 : CVR_RC1_WPG; }

template <int K, bool PHONG, bool SKIP, bool QUAD, int XF, int BUF, int FB, int CS>
__global__ void __launch_bounds__(64 * rc1_waves_per_group<QUAD>())
__attribute__((amdgpu_waves_per_eu(rc1_waves_per_eu<K, PHONG, SKIP, QUAD>())))
rc1pass_tile_kernel(Rc1passArgs A0, const uint4* __restrict__ cells,
                    const uint4* __restrict__ grad, const float4* __restrict__ tf_g,
                    float4* __restrict__ out0, uint32_t* __restrict__ samples0,
                    unsigned long long* __restrict__ tile_samples, const int* __restrict__ order,
                    uint32_t* __restrict__ tile_cost, int boost, LaunchFrames LF) {
  extern __shared__ float4 tfp[];
  // Several frames per launch (LF.n > 1, cvr_render_rc1pass_frames): workgroup
  // blockIdx.x marches block b of frame f with that frame's view and outputs.
  // Only frame 0 records the tile costs of the next launch order; the per-tile
  // sample counts of all frames add up (the launch's total).
  Rc1passArgs A = A0;
  float4* __restrict__ out = out0;
  uint32_t* __restrict__ samples = samples0;
  constexpr int WG = rc1_waves_per_group<QUAD>();
  int b = WG > 1 ? (((WG * ((int)blockIdx.x >> 3) + (int)(threadIdx.x >> 6)) << 3) | ((int)blockIdx.x & 7))
                 : (int)blockIdx.x;
  int f = 0;
  const int nt = A.ntiles;
  if (LF.n > 1) {
    if (LF.interleave) {          // b = 8 (n e + f) + x -> frame f, block 8 e + x
      const int x = b & 7, q = b >> 3;
      const int e = q / LF.n;
      f = q - e * LF.n;
      b = (e << 3) | x;
    } else {
      f = b / LF.grid;
      b -= f * LF.grid;
    }
    const FrameView& v = LF.view[f];
#pragma unroll
    for (int i = 0; i < 3; i++) {
      A.eye[i] = v.eye[i];
      A.col0[i] = v.col0[i];
      A.col1[i] = v.col1[i];
      A.col2[i] = v.col2[i];
    }
    A.tan_half_fovy = v.tan_half_fovy;
    A.aspect = v.aspect;
    out = LF.out[f];
    samples = LF.samples[f];
    if (f != 0) tile_cost = nullptr;
  }
  int t = 0, quarter = -1;
  bool pad = false;   // a slot past a band's entries (or past the tiles): the wave exits
  if (order) {
    const int e = order[b];
    pad = e < 0;
    t = e & (kQuadFlag - 1);
    if (QUAD) quarter = (e >> 28) - 1;
    if (!pad && (b >> 3) < boost) __builtin_amdgcn_s_setprio(2);
  } else if (b >= nt) {
    pad = true;
  } else if ((nt & 7) == 0 && !A.interleave) {
    t = (b & 7) * (nt >> 3) + (b >> 3);
  } else {
    t = b;
  }
  if (WG == 1 && pad) return;               // (whole workgroup)
  load_tf_lds(tfp, tf_g, A.tf_n);           // every wave of the workgroup takes part (barrier)
  if (pad) return;
  const int lane = (int)(threadIdx.x & 63);
  unsigned long long t_start = 0;
  if (A.tile_stats || A.cost_time) t_start = __builtin_amdgcn_s_memrealtime();
  int px, py;
  long long oidx;
  float4 dst;
  // nskip: samples stepped over without a load (measurement); the EA march has
  // no shaded-sample count, so it shares that register
  uint32_t cnt, nshade = 0, nbatch = 0, nskip_own = 0, npm = 0, npc = 0;
  uint32_t& nskip = PHONG ? nskip_own : nshade;
  bool writer;
  if (!QUAD || quarter < 0) {   // whole tile, one lane per ray
    tile_pixel(A, t, lane & 7, lane >> 3, px, py, oidx);
    const bool inside = px < A.W && py < A.H;
    dst = make_float4(0.f, 0.f, 0.f, 0.f);
    cnt = 0;
    if (inside) march_ray<K, PHONG, SKIP, XF, BUF, FB, CS>(A, cells, grad, tfp, px, py, dst, cnt, nshade,
                                                          nbatch, nskip, npm, npc);
    writer = inside || A.packed;
    if (CS > 0) {
      // the output index again, from the lane id (v_mbcnt) and the wave's tile
      // (scalar) rather than held across the march, where it spilled (16 B per
      // lane of scratch traffic)
      const int ln = (int)__lane_id();
      int px2, py2;
      tile_pixel(A, t, ln & 7, ln >> 3, px2, py2, oidx);
    }
  } else {                    // quarter of a tile, four lanes per ray
    const int ray = lane >> 2;
    tile_pixel(A, t, ((quarter & 1) << 2) | (ray & 3), ((quarter >> 1) << 2) | (ray >> 2), px, py,
               oidx);
    const bool inside = px < A.W && py < A.H;
    march_ray_quad<K, PHONG, XF>(A, cells, grad, tfp, px, py, inside, dst, cnt);
    writer = (lane & 3) == 0 && (inside || A.packed);
    if ((lane & 3) != 0) cnt = 0;           // one count per ray
  }
  if (writer) {
    store_rgba(out, oidx, dst, A.out_half);
    if (samples) samples[oidx] = cnt;
  }
  if (A.shade_ctr) {   // measurement only: shaded samples (the gradient's bytes), skipped samples
    if (PHONG) {
      const unsigned long long v = wave_sum(nshade);
      if (lane == 0 && v) atomicAdd(&A.shade_ctr[0], v);
    }
#ifdef CVR_PROBE_SHADE_PASSES
    if (PHONG) {   // [1] passes if each lane shaded its visible samples in turn, [2] passes today
      // every active lane adds each batch's wave-wide count: the longest-lived lane has it all
      const uint32_t pm = wave_max(npm), pc = wave_max(npc);
      if (lane == 0) {
        atomicAdd(&A.shade_ctr[1], (unsigned long long)pm);
        atomicAdd(&A.shade_ctr[2], (unsigned long long)pc);
      }
    }
#else
    if (CS >= 2) {
      const unsigned long long v = wave_sum(nskip);
      if (lane == 0 && v) atomicAdd(&A.shade_ctr[1], v);
    }
    if (CS > 0 && !PHONG) {   // the wave's march rounds (K cell loads each): bench.py's vmem roofline
      const uint32_t r = wave_max(nbatch);
      if (lane == 0 && r) atomicAdd(&A.shade_ctr[2], (unsigned long long)r);
    }
#endif
  }
  if (tile_samples) {   // per-tile sample count; summed by tile_order_kernel (no hot atomic)
    unsigned long long v = wave_sum(cnt);
    if (lane == 0) {
      if ((QUAD && quarter >= 0) || LF.n > 1) {
        if (v) atomicAdd(&tile_samples[t], v);
      } else {
        tile_samples[t] = v;
      }
    }
  }
  uint32_t m = 0;
  if (tile_cost || A.tile_stats) m = wave_max(cnt);
  // with the per-cell skip the samples no longer measure a tile's time (a skipped
  // sample costs one add): its march rounds do (x 4, the scale of the samples)
  uint32_t mb = 0;
  if (CS > 0 && tile_cost) mb = 4u * wave_max(nbatch);
  if (tile_cost && lane == 0) {   // next frame's order: the tile's measured time or its longest ray
    uint32_t c = CS > 0 ? mb : m;
    if (A.cost_time) {
      const unsigned long long d = __builtin_amdgcn_s_memrealtime() - t_start;   // 100 MHz ticks
      c = d > 0xffffffffull ? 0xffffffffu : (uint32_t)d;
    }
    if (quarter < 0) tile_cost[t] = c;
    else atomicMax(&tile_cost[t], c);
  }
  if (A.tile_stats) {   // diagnostics: 100 MHz start/end stamps, longest ray, placement
    unsigned long long t_end = __builtin_amdgcn_s_memrealtime();
    unsigned hw;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
    if (lane == 0 && quarter <= 0 && f == 0) {
      A.tile_stats[t * 4 + 0] = t_start;
      A.tile_stats[t * 4 + 1] = t_end;
      A.tile_stats[t * 4 + 2] = m;
      A.tile_stats[t * 4 + 3] = ((unsigned long long)b << 32) | hw;
    }
  }
}

// ---------------------------------------------------------------------------
// Launch order (LPT) from the previous frame
// ---------------------------------------------------------------------------

// Per-frame epilogue, one workgroup per XCD band:
//  * `tile_samples` (optional): sums the band's per-tile sample counts into
//    *total (one atomic per band instead of one per wave on a single word) and
//    resets them;
//  * `tile_cost` (optional): builds the next frame's launch order.  The screen
//    (row-major wave tiles) is cut into 8 contiguous bands of equal predicted
//    work — weight = the tile's critical path + kTileWeightBias, prefix-summed
//    over the whole frame — so every XCD finishes together while keeping a
//    compact screen region (L2 locality).  A band that would exceed `max_seg`
//    tiles (option band_cap) has its boundaries moved the least that fits.  Each band is ordered by
//    descending critical path (bucketed into 256 cost levels: O(n), ties in any
//    order — the order never changes a pixel), its longest `nquad` tiles are
//    expanded into four quad quarters, and the entries are dealt to physical
//    blocks band, band+8, ... (the blocks XCD `band` receives); slots past the
//    band's entries are -1.  Resets tile_cost for the next frame's atomicMax.
constexpr int kOrderThreads = 1024;
constexpr unsigned kTileWeightBias = 8;
constexpr int kGroupChunk = 256;    // 64-tile groups scanned per pass of the boundary search

__global__ void __launch_bounds__(kOrderThreads)
tile_epilogue_kernel(uint32_t* __restrict__ tile_cost, unsigned long long* __restrict__ tile_samples,
                     unsigned long long* __restrict__ total, int ntiles, int quad_pct,
                     int slots_per_band, int max_seg, int keep, int stop_after,
                     int* __restrict__ order) {
  __shared__ unsigned hist[256];
  __shared__ unsigned start[256];
  __shared__ unsigned maxc;
  __shared__ unsigned long long wsum[kOrderThreads / 64];
  __shared__ int bounds[9];
  __shared__ unsigned long long gsum[kGroupChunk];
  __shared__ unsigned long long gcarry;
  extern __shared__ int dyn_lds[];   // gpref[ngroups] (u64), then sorted[max_seg]
  unsigned long long* gpref = reinterpret_cast<unsigned long long*>(dyn_lds);
  int* sorted = dyn_lds + 2 * ((ntiles + 63) >> 6);
  const int band = blockIdx.x, tid = threadIdx.x;
  if (tile_samples) {
    const int s0 = (band * ntiles) >> 3, s1 = ((band + 1) * ntiles) >> 3;
    unsigned long long acc = 0;
    for (int i = s0 + tid; i < s1; i += kOrderThreads) {
      acc += tile_samples[i];
      tile_samples[i] = 0ull;
    }
    acc = wave_sum(acc);
    if ((tid & 63) == 0) wsum[tid >> 6] = acc;
    __syncthreads();
    if (tid == 0) {
      unsigned long long t = 0;
      for (int w = 0; w < kOrderThreads / 64; w++) t += wsum[w];
      if (total && t) atomicAdd(total, t);
    }
  }
  if (!tile_cost || stop_after == 9) return;

  // 1) work-balanced band boundaries (every block computes all 8, identically),
  //    at the granularity of 64-tile groups: a wave reads a group with one
  //    coalesced load and reduces it; one wave scans the group sums; band k
  //    starts after the group whose prefix reaches k/8 of the total weight.
  //    (Per-thread contiguous chunks made every load instruction touch 64
  //    cache lines: ~20 us for this phase alone.)
  const int ngroups = (ntiles + 63) >> 6;
  const int lane = tid & 63, wid = tid >> 6;
  __syncthreads();   // gsum aliases wsum's neighbours in LDS below
  constexpr int kGroupsPerWave = kGroupChunk / (kOrderThreads / 64);
  for (int g0 = 0; g0 < ngroups; g0 += kGroupChunk) {
    const int gend = min(g0 + kGroupChunk, ngroups);
    uint32_t w[kGroupsPerWave];   // all loads in flight before any reduction
#pragma unroll
    for (int j = 0; j < kGroupsPerWave; j++) {
      const int g = g0 + wid + j * (kOrderThreads / 64), i = (g << 6) + lane;
      w[j] = (g < gend && i < ntiles) ? tile_cost[i] + kTileWeightBias : 0u;
    }
#pragma unroll
    for (int j = 0; j < kGroupsPerWave; j++) {
      const int g = g0 + wid + j * (kOrderThreads / 64);
      const unsigned long long v = wave_sum((unsigned long long)w[j]);
      if (lane == 0 && g < gend) gsum[g - g0] = v;
    }
    __syncthreads();
    if (wid == 0) {   // inclusive scan of this chunk of group sums, carried across chunks
      const int n = min(kGroupChunk, ngroups - g0);
      unsigned long long carry = g0 == 0 ? 0ull : gcarry;
      for (int base = 0; base < n; base += 64) {
        unsigned long long v = base + lane < n ? gsum[base + lane] : 0ull;
#pragma unroll
        for (int off = 1; off < 64; off <<= 1) {
          const unsigned long long o = __shfl_up(v, off, 64);
          if (lane >= off) v += o;
        }
        v += carry;
        if (base + lane < n) gsum[base + lane] = v;
        carry = __shfl(v, 63, 64);
      }
      if (lane == 0) gcarry = carry;
    }
    __syncthreads();
    // record the chunk's inclusive prefixes for the boundary search
    for (int g = g0 + tid; g < min(g0 + kGroupChunk, ngroups); g += kOrderThreads)
      gpref[g] = gsum[g - g0];
    __syncthreads();
  }
  if (tid < 9) bounds[tid] = tid == 8 ? ntiles : (tid == 0 ? 0 : -1);
  if (tid == 0) maxc = 0;
  if (tid < 256) hist[tid] = 0;
  __syncthreads();
  const unsigned long long wtot = gpref[ngroups - 1];
  for (int g = tid; g < ngroups; g += kOrderThreads) {
    const unsigned long long end = gpref[g], beg = g == 0 ? 0ull : gpref[g - 1];
    for (int k = 1; k < 8; k++) {
      const unsigned long long target = (wtot * (unsigned long long)k) >> 3;
      if (beg < target && target <= end) bounds[k] = min((g + 1) << 6, ntiles);
    }
  }
  __syncthreads();
  bool balanced = true;
  for (int k = 1; k < 8; k++) {
    if (bounds[k] < 0) balanced = false;
  }
  if (balanced) {
    // Held to the cap (max_seg >= ceil(ntiles / 8), so this is always feasible):
    // each boundary moves the least that leaves its band <= max_seg tiles and
    // the bands after it room for the rest.
    if (tid == 0) {
      for (int k = 1; k < 8; k++) {
        const int lo = max(bounds[k - 1], ntiles - (8 - k) * max_seg);
        bounds[k] = min(max(bounds[k], lo), bounds[k - 1] + max_seg);
      }
    }
    __syncthreads();
    for (int k = 0; k < 8; k++)
      if (bounds[k + 1] < bounds[k] || bounds[k + 1] - bounds[k] > max_seg) balanced = false;
  }
  const int b0 = balanced ? bounds[band] : (band * ntiles) >> 3;
  const int b1 = balanced ? bounds[band + 1] : ((band + 1) * ntiles) >> 3;
  const int seg = b1 - b0;
  if (stop_after == 1) return;

  // 2) LPT order of the band: bucket sort by critical path.  The band's costs
  //    are read once into registers (kBandRegs per thread; longer bands loop).
  constexpr int kBandRegs = 4;
  uint32_t cst[kBandRegs];
#pragma unroll
  for (int k = 0; k < kBandRegs; k++) {
    const int i = tid + k * kOrderThreads;
    cst[k] = i < seg ? tile_cost[b0 + i] : 0u;
  }
  unsigned lmax = 0;
#pragma unroll
  for (int k = 0; k < kBandRegs; k++) lmax = max(lmax, cst[k]);
  for (int i = tid + kBandRegs * kOrderThreads; i < seg; i += kOrderThreads)
    lmax = max(lmax, tile_cost[b0 + i]);
  lmax = wave_max(lmax);
  if ((tid & 63) == 0) atomicMax(&maxc, lmax);
  __syncthreads();
  if (stop_after == 2) return;
  const unsigned long long mc = (unsigned long long)maxc + 1;
  auto bucket_of = [mc](uint32_t c) { return 255u - (unsigned)(((unsigned long long)c * 256u) / mc); };
#pragma unroll
  for (int k = 0; k < kBandRegs; k++)
    if (tid + k * kOrderThreads < seg) atomicAdd(&hist[bucket_of(cst[k])], 1u);
  for (int i = tid + kBandRegs * kOrderThreads; i < seg; i += kOrderThreads)
    atomicAdd(&hist[bucket_of(tile_cost[b0 + i])], 1u);
  __syncthreads();
  if (stop_after == 3) return;
  if (tid < 64) {   // exclusive scan of the 256 counts by one wave (4 per lane)
    const unsigned h0 = hist[4 * tid], h1 = hist[4 * tid + 1], h2 = hist[4 * tid + 2],
                   h3 = hist[4 * tid + 3];
    const unsigned part = h0 + h1 + h2 + h3;
    unsigned inc = part;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
      const unsigned o = (unsigned)__shfl_up((int)inc, off, 64);
      if (tid >= off) inc += o;
    }
    unsigned ex = inc - part;
    start[4 * tid] = ex; ex += h0;
    start[4 * tid + 1] = ex; ex += h1;
    start[4 * tid + 2] = ex; ex += h2;
    start[4 * tid + 3] = ex;
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < kBandRegs; k++) {
    const int i = tid + k * kOrderThreads;
    if (i < seg) sorted[atomicAdd(&start[bucket_of(cst[k])], 1u)] = b0 + i;
  }
  for (int i = tid + kBandRegs * kOrderThreads; i < seg; i += kOrderThreads)
    sorted[atomicAdd(&start[bucket_of(tile_cost[b0 + i])], 1u)] = b0 + i;
  __syncthreads();
  if (stop_after == 4) return;
  const int nquad = (int)(((long long)seg * quad_pct) / 100);
  const int nent = keep > 0 ? min(seg + 3 * nquad, keep) : seg + 3 * nquad;
  for (int e = tid; e < slots_per_band; e += kOrderThreads) {
    int v = -1;
    if (e < 4 * nquad) v = sorted[e >> 2] | (((e & 3) + 1) << 28);
    else if (e < nent) v = sorted[e - 3 * nquad];
    order[band + 8 * e] = v;
  }
  // tile_cost is not cleared here: every block reads all of it for the
  // boundaries (see launch_tile_epilogue)
}

// Clears tile_cost for the next frame's atomicMax (after every band has read it).
__global__ void clear_u32_kernel(uint32_t* __restrict__ p, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) p[i] = 0u;
}

// ---------------------------------------------------------------------------
// Launchers
// ---------------------------------------------------------------------------

// Kernel variant: K (batch), PHONG, SKIP (empty-space skipping compiled in),
// QUAD (quad path compiled in), XF (exp: 0 CVR-SPEC, 1 CVR-SPEC without range
// selects, 2 the native v_exp_f32 -- tolerance mode, option native_exp).  Paths a frame does not
// use are compiled out: they would cost the hot loop registers (occupancy).
template <int K, bool PHONG, bool SKIP, bool QUAD, int XF, int BUF, int FB = 0, int CS = 0>
static hipError_t launch_variant(const Ctx& c, const Rc1passArgs& a, float4* out, uint32_t* samples,
                                 unsigned long long* tile_samples, const int* order,
                                 uint32_t* tile_cost, const RenderPlan& plan, hipStream_t s) {
  size_t lds = (size_t)(a.tf_n + 2) * sizeof(float4);
  if (c.max_waves_cu > 0) lds = std::max(lds, (size_t)(160 * 1024 / c.max_waves_cu) & ~(size_t)255);
  // cell (1,1,1) <-> texel (0,0,0)
  const uint4* cells = (const uint4*)c.d_cells;   // sample_pos indexes from the first cell
  constexpr int WG = rc1_waves_per_group<QUAD>();
  // slots: a multiple of 8 x WG (the order's bands hold a multiple of 4 slots,
  // cvr_api.cpp; the slots past the tiles exit at once)
  int grid = order ? plan.order_slots : plan.ntiles;
  grid = (grid + 8 * WG - 1) / (8 * WG) * (8 * WG);
  if (order && grid != plan.order_slots) return hipErrorInvalidValue;
  LaunchFrames lf;
  lf.n = 1;
  lf.interleave = 0;
  if (plan.frames && plan.frames->n > 1) {
    lf = *plan.frames;
    lf.grid = grid;
    lf.interleave = (order && (grid & 7) == 0 && c.launch_interleave) ? 1 : 0;
    grid *= lf.n;
  }
  hipLaunchKernelGGL((rc1pass_tile_kernel<K, PHONG, SKIP, QUAD, XF, BUF, FB, CS>), dim3(grid / WG), dim3(64 * WG), lds, s,
                     a, cells, (const uint4*)c.d_grad, (const float4*)c.d_tf, out, samples,
                     tile_samples, order, tile_cost, order ? plan.boost : 0, lf);
  return hipGetLastError();
}

template <int K, bool PHONG, bool SKIP>
static hipError_t launch_kps(const Ctx& c, const Rc1passArgs& a, float4* out, uint32_t* samples,
                             unsigned long long* ts, const int* order, uint32_t* tile_cost,
                             const RenderPlan& plan, hipStream_t s) {
  // buffer loads address the cell grid with 32-bit byte offsets (BUF 2: the
  // 24-bit multiply-add form, while 16 * pitch_z < 2^23, i.e. up to 723^3)
  const int buf = c.cells_bytes >= (size_t(1) << 32) ? 0
                  : (c.cells.bpitch_z > 0 && c.cells.bpitch_z < (1 << 23)) ? 2 : 1;
  if (a.filter_bits == 8) {   // GL texture-unit weights: the ray-parallel march only
    if (buf == 2)
      return a.exp_fast ? launch_variant<K, PHONG, SKIP, false, true, 2, 8>(c, a, out, samples, ts, order, tile_cost, plan, s)
                        : launch_variant<K, PHONG, SKIP, false, false, 2, 8>(c, a, out, samples, ts, order, tile_cost, plan, s);
    if (buf == 1)
      return a.exp_fast ? launch_variant<K, PHONG, SKIP, false, true, 1, 8>(c, a, out, samples, ts, order, tile_cost, plan, s)
                        : launch_variant<K, PHONG, SKIP, false, false, 1, 8>(c, a, out, samples, ts, order, tile_cost, plan, s);
    return a.exp_fast ? launch_variant<K, PHONG, SKIP, false, true, 0, 8>(c, a, out, samples, ts, order, tile_cost, plan, s)
                      : launch_variant<K, PHONG, SKIP, false, false, 0, 8>(c, a, out, samples, ts, order, tile_cost, plan, s);
  }
  const bool quad = order && plan.quad_pct > 0;
  if (!SKIP && !quad && a.cell_skip > 0) {   // per-cell skip flags (a.occ is null then)
#define CVR_CS_LAUNCH(CSV)                                                                                 \
    if (buf == 2)                                                                                          \
      return a.exp_fast ? launch_variant<K, PHONG, false, false, true, 2, 0, CSV>(c, a, out, samples, ts, order, tile_cost, plan, s) \
                        : launch_variant<K, PHONG, false, false, false, 2, 0, CSV>(c, a, out, samples, ts, order, tile_cost, plan, s); \
    if (buf == 1)                                                                                          \
      return a.exp_fast ? launch_variant<K, PHONG, false, false, true, 1, 0, CSV>(c, a, out, samples, ts, order, tile_cost, plan, s) \
                        : launch_variant<K, PHONG, false, false, false, 1, 0, CSV>(c, a, out, samples, ts, order, tile_cost, plan, s); \
    return a.exp_fast ? launch_variant<K, PHONG, false, false, true, 0, 0, CSV>(c, a, out, samples, ts, order, tile_cost, plan, s) \
                      : launch_variant<K, PHONG, false, false, false, 0, 0, CSV>(c, a, out, samples, ts, order, tile_cost, plan, s);
    // tolerance mode (option native_exp): the headline's variants only (buffer
    // addressing, exact weights, cell skip 3, either shading) -- DESIGN §5‴
    if (a.exp_native && buf == 2 && a.cell_skip == 3)
      return launch_variant<K, PHONG, false, false, 2, 2, 0, 3>(c, a, out, samples, ts, order, tile_cost, plan, s);
    if (a.cell_skip == 1) { CVR_CS_LAUNCH(1) }
    if (a.cell_skip == 3) { CVR_CS_LAUNCH(3) }
    if (a.cell_skip == 4) { CVR_CS_LAUNCH(4) }
    CVR_CS_LAUNCH(2)
#undef CVR_CS_LAUNCH
  }
  if (quad)
    return a.exp_fast ? launch_variant<K, PHONG, SKIP, true, true, 0>(c, a, out, samples, ts, order, tile_cost, plan, s)
                      : launch_variant<K, PHONG, SKIP, true, false, 0>(c, a, out, samples, ts, order, tile_cost, plan, s);
  if (buf == 2)
    return a.exp_fast ? launch_variant<K, PHONG, SKIP, false, true, 2>(c, a, out, samples, ts, order, tile_cost, plan, s)
                      : launch_variant<K, PHONG, SKIP, false, false, 2>(c, a, out, samples, ts, order, tile_cost, plan, s);
  if (buf == 1)
    return a.exp_fast ? launch_variant<K, PHONG, SKIP, false, true, 1>(c, a, out, samples, ts, order, tile_cost, plan, s)
                      : launch_variant<K, PHONG, SKIP, false, false, 1>(c, a, out, samples, ts, order, tile_cost, plan, s);
  return a.exp_fast ? launch_variant<K, PHONG, SKIP, false, true, 0>(c, a, out, samples, ts, order, tile_cost, plan, s)
                    : launch_variant<K, PHONG, SKIP, false, false, 0>(c, a, out, samples, ts, order, tile_cost, plan, s);
}

template <int K, bool PHONG>
static hipError_t launch_kp(const Ctx& c, const Rc1passArgs& a, float4* out, uint32_t* samples,
                            unsigned long long* ts, const int* order, uint32_t* tile_cost,
                            const RenderPlan& plan, hipStream_t s) {
  return a.occ ? launch_kps<K, PHONG, true>(c, a, out, samples, ts, order, tile_cost, plan, s)
               : launch_kps<K, PHONG, false>(c, a, out, samples, ts, order, tile_cost, plan, s);
}

template <int K>
static hipError_t launch_k(const Ctx& c, const Rc1passArgs& a, bool phong, float4* out,
                           uint32_t* samples, unsigned long long* ts, const int* order,
                           uint32_t* tile_cost, const RenderPlan& plan, hipStream_t s) {
  return phong ? launch_kp<K, true>(c, a, out, samples, ts, order, tile_cost, plan, s)
               : launch_kp<K, false>(c, a, out, samples, ts, order, tile_cost, plan, s);
}

hipError_t launch_rc1pass(const Ctx& c, const Rc1passArgs& a, bool phong, float4* out,
                          uint32_t* samples, unsigned long long* tile_samples, const int* order,
                          uint32_t* tile_cost, const RenderPlan& plan, hipStream_t s) {
  if (a.ntiles <= 0) return hipSuccess;
  if (a.tf_n > kMaxTfLds) return hipErrorInvalidValue;
  if (c.batch == 2 || (c.batch == 0 && phong)) return launch_k<2>(c, a, phong, out, samples, tile_samples, order, tile_cost, plan, s);
  return launch_k<4>(c, a, phong, out, samples, tile_samples, order, tile_cost, plan, s);
}

hipError_t launch_tile_epilogue(uint32_t* tile_cost, unsigned long long* tile_samples,
                                unsigned long long* total, const RenderPlan& plan, int* order,
                                hipStream_t s) {
  const int max_seg = plan.max_seg;
  if (tile_cost && (max_seg > kMaxBandTiles || max_seg < (plan.ntiles + 7) / 8))
    return hipErrorInvalidValue;
  const size_t lds = tile_cost ? (size_t)((plan.ntiles + 63) >> 6) * 8 + (size_t)max_seg * sizeof(int)
                              : 0;
  hipLaunchKernelGGL(tile_epilogue_kernel, dim3(8), dim3(kOrderThreads), lds, s, tile_cost, tile_samples,
                     total, plan.ntiles, plan.quad_pct, plan.order_slots / 8, max_seg, plan.keep,
                     plan.epi_stop, order);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess || !tile_cost) return e;
  // quad quarters atomicMax into tile_cost: it must start the next frame at zero
  if (plan.quad_pct > 0) {
    hipLaunchKernelGGL(clear_u32_kernel, dim3((plan.ntiles + 255) / 256), dim3(256), 0, s,
                       tile_cost, plan.ntiles);
    e = hipGetLastError();
  }
  return e;
}

}  // namespace cvr
