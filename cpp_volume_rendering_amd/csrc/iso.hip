// iso.hip — the sibling isosurface ray-casters of cppvolrend
// on gfx950, both first-hit isosurface marches with block-based empty-space
// skipping over a min/max block grid and adaptive steps:
//
//   variant 0  "1-Pass - Custom Isosurface Raycaster Adaptive"
//              (cppvolrend/structured/rc1pisocustom: custom_ray_marching_1p_iso_adapt.comp
//              :98-129, 133-290; 4^3 blocks, rc1custompisoadaptrenderer.cpp:173)
//   variant 2  "1-Pass - Isosurface Raycaster Adaptive" (cppvolrend/structured/
//              rc1pisoadapt: ray_marching_1p_iso_adapt.comp:113-172), no blocks
//   variant 1  "Empty Space Skipping V2"
//              (cppvolrend/structured/rc1pisodfscustom: the same file :100-141, 144-227;
//              32^3 blocks, rc1custompisoadaptdfsrenderer.cpp:190)
//
// One lane per ray (8x8 tile per wave, the rc1pass tiling), the loop of the
// shader per lane.  Volume samples are the R16F trilinear texture() fetches of
// the rc1pass march (one 16-B cell8 load each); the block min/max tables
// (GL_R32F, GL_NEAREST, default GL_REPEAT wrap: an out-of-range block index
// wraps modulo the block count) are read through the cache.  Every GLSL float
// expression is evaluated in the shader's order without contraction
// (-ffp-contract=off), as oracle/cvr_oracle.cpp (oracle_render_iso) does.
// Deviation: a lane stops after kIsoMaxIter iterations (the reference can
// loop without end when Color.a is 0; the default colour's alpha is 1).
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdint>

#include "cvr_device.h"
#include "march_common.h"

namespace cvr {

namespace {

constexpr uint32_t kIsoMaxIter = 1u << 22;
#ifndef CVR_ISO_SPEC
#define CVR_ISO_SPEC 4
#endif
constexpr int kIsoSpec = CVR_ISO_SPEC;   // speculative steps per round trip (variant 2)

// texture(TexVolume, tex / VolumeGridSize).r: the rc1pass trilinear fetch at the
// texel coordinate fma(tex, N/G, -0.5), clamped to the grid (CLAMP_TO_EDGE).
__device__ __forceinline__ float iso_density(const Rc1passArgs& A, const uint4* __restrict__ cells,
                                             f3 tex, SamplePos& sp) {
  sp = sample_pos_clamped(fmaf(tex.x, A.n_over_g[0], -0.5f), fmaf(tex.y, A.n_over_g[1], -0.5f),
                          fmaf(tex.z, A.n_over_g[2], -0.5f), A);
  return trilerp_cell(cells[sp.idx], sp.ax, sp.ay, sp.az);
}

// r.Origin + r.Dir * t + VolumeGridSize * 0.5
__device__ __forceinline__ f3 iso_tex(f3 eye, f3 dir, float t, f3 hg) {
  return f3{fmaf(dir.x, t, eye.x) + hg.x, fmaf(dir.y, t, eye.y) + hg.y, fmaf(dir.z, t, eye.z) + hg.z};
}

// getBlockIndex (:86-89): floor((pos + G/2) / G * numBlocks), pos = r.Origin + t * r.Dir
// Fast path: x * (1/G) * nb is within ~2e-5 of the exact value for the block
// counts used (<= 1024 blocks), so away from an integer its floor is the
// exact one; near an integer the correctly rounded division decides.
__device__ __forceinline__ void iso_block(const IsoArgs& Q, f3 eye, f3 dir, float t, int b[3]) {
  const float p[3] = {fmaf(dir.x, t, eye.x), fmaf(dir.y, t, eye.y), fmaf(dir.z, t, eye.z)};
#pragma unroll
  for (int i = 0; i < 3; i++) {
    const float x = p[i] + Q.a.half_grid[i];
    const float ya = (x * Q.inv_g[i]) * Q.nb[i];
    const float fa = floorf(ya);
    const float margin = fmaxf(1e-3f, fabsf(ya) * 1e-5f);
    const bool sure = (ya - fa) > margin && (fa + 1.0f - ya) > margin;
    b[i] = (int)(sure ? fa : floorf((x / Q.G[i]) * Q.nb[i]));
  }
}

// texture(TexBlockMin/Max, (idx + 0.5) / numBlocks), NEAREST + REPEAT
__device__ __forceinline__ float2 iso_block_range(const IsoArgs& Q, const float2* __restrict__ mm,
                                                  const int b[3]) {
  int w[3];
#pragma unroll
  for (int i = 0; i < 3; i++) {
    const int n = Q.nbi[i];
    const int v = b[i];
    w[i] = (v >= 0 && v < n) ? v : (v < 0 && v >= -n ? v + n : (v >= n && v < 2 * n ? v - n : ((v % n) + n) % n));
  }
  return mm[((size_t)w[2] * Q.nbi[1] + w[1]) * Q.nbi[0] + w[0]];
}

// Blinn-Phong of the iso shaders (ShadeBlinnPhong :50-84): the gradient texture at
// the hit, light / eye / halfway vectors from the world position.
__device__ __forceinline__ f3 iso_phong(const Rc1passArgs& A, const uint4* __restrict__ grad,
                                        const SamplePos& sp, f3 tex, f3 hg, f3 eye, f3 clr) {
  const f3 g = sample_gradient_cell(grad, sp);
  if (g.x != 0.0f || g.y != 0.0f || g.z != 0.0f) {
    const f3 wp{tex.x - hg.x, tex.y - hg.y, tex.z - hg.z};
    const f3 L = normalize3(f3{A.light[0] - wp.x, A.light[1] - wp.y, A.light[2] - wp.z});
    const f3 E = normalize3(f3{eye.x - wp.x, eye.y - wp.y, eye.z - wp.z});
    const f3 H = normalize3(f3{E.x + L.x, E.y + L.y, E.z + L.z});
    const f3 n = normalize3(g);
    const float dd = fmaxf(0.0f, dot3(n, L));
    const float ds = fmaxf(0.0f, dot3(H, n));
    const float pw = cvr_powf_nb(ds, A.shininess);
    const float f = fmaf(A.kd, dd, A.ka);        // the rc1pass Blinn-Phong (CVR-SPEC)
    clr = f3{fmaf(A.ispec[0] * A.ks, pw, clr.x * f), fmaf(A.ispec[1] * A.ks, pw, clr.y * f),
             fmaf(A.ispec[2] * A.ks, pw, clr.z * f)};
  }
  return clr;
}

// Front-to-back composition of the hit colour: src.rgb *= src.a; dst += (1 - dst.a) * src
__device__ __forceinline__ void iso_composite(const IsoArgs& Q, f3 c, float4& dst) {
  const float a = Q.color[3];
  const float om = 1.0f - dst.w;
  dst.x = fmaf(om, c.x * a, dst.x);
  dst.y = fmaf(om, c.y * a, dst.y);
  dst.z = fmaf(om, c.z * a, dst.z);
  dst.w = fmaf(om, a, dst.w);
}

// The hit colour (Color, optionally Blinn-Phong shaded at the refined position).
template <bool PHONG>
__device__ __forceinline__ f3 iso_hit_colour(const IsoArgs& Q, const uint4* __restrict__ grad,
                                             f3 st, f3 hg, f3 eye) {
  f3 c{Q.color[0], Q.color[1], Q.color[2]};
  if (PHONG) {
    const Rc1passArgs& A = Q.a;
    const SamplePos gp = sample_pos_clamped(fmaf(st.x, A.n_over_g[0], -0.5f),
                                            fmaf(st.y, A.n_over_g[1], -0.5f),
                                            fmaf(st.z, A.n_over_g[2], -0.5f), A);
    c = iso_phong(A, grad, gp, st, hg, eye, c);
  }
  return c;
}

// One ray of the shader's main loop.  `pd` is the shader's prevDensity variable
// and `dc` the density fetched at the current t when `have` says so: a fetch at
// an unchanged t returns the same value, so it is reused (but counted, as the
// shader fetches it).
template <int VARIANT, bool PHONG>
__device__ void iso_march(const IsoArgs& Q, const uint4* __restrict__ cells,
                          const uint4* __restrict__ grad, const float2* __restrict__ mm, int px,
                          int py, float4& dst, uint32_t& fetches, uint32_t& iters) {
  const Rc1passArgs& A = Q.a;
  dst = make_float4(0.f, 0.f, 0.f, 0.f);
  fetches = iters = 0;
  Ray r;
  if (!ray_setup(A, px, py, r)) return;
  const f3 eye{A.eye[0], A.eye[1], A.eye[2]};
  const f3 hg{A.half_grid[0], A.half_grid[1], A.half_grid[2]};
  const f3 dir = r.dir;
  const float tfar = r.tfar;
  const float iso = Q.iso;
  SamplePos sp;
  if (VARIANT == 2) {
    // RayCasting1PassIsoAdapt (rc1pisoadapt/ray_marching_1p_iso_adapt.comp:113-172):
    // adaptive steps over s in [0, D) from the entry point, no blocks.  Each step
    // size depends on the density just fetched, so one lane would have one load
    // in flight.  Instead kIsoSpec steps are issued at once, all of the size the
    // current decision gives (s += min(step, D - s) evaluated as the shader
    // does); they are consumed in order while each new density keeps that
    // decision, and the rest are dropped.  Results and counts are the shader's.
    const f3 tp = r.tpos;
    const float D = r.D;
    float prev = iso_density(A, cells, tp, sp);
    fetches++;
    float s = 0.0f;
    while (s < D && iters < kIsoMaxIter) {
      const bool near = fabsf(prev - iso) < Q.step_range;
      const float step = near ? Q.step_small : Q.step_large;
      uint4 c[kIsoSpec];
      SamplePos ps[kIsoSpec];
      float hk[kIsoSpec];
      bool ok[kIsoSpec];
      float ss = s;
#pragma unroll
      for (int k = 0; k < kIsoSpec; k++) {
        ok[k] = ss < D;
        const float h = fminf(step, D - ss);
        const float sh = ss + h;
        ps[k] = sample_pos_clamped(fmaf(fmaf(dir.x, sh, tp.x), A.n_over_g[0], -0.5f),
                                   fmaf(fmaf(dir.y, sh, tp.y), A.n_over_g[1], -0.5f),
                                   fmaf(fmaf(dir.z, sh, tp.z), A.n_over_g[2], -0.5f), A);
        c[k] = cells[ps[k].idx];
        hk[k] = h;
        ss = sh;
      }
      bool done = false;
#pragma unroll
      for (int k = 0; k < kIsoSpec; k++) {
        if (k > 0 && (!ok[k] || iters >= kIsoMaxIter || (fabsf(prev - iso) < Q.step_range) != near))
          break;
        iters++;
        const float h = hk[k];
        const float dens = trilerp_cell(c[k], ps[k].ax, ps[k].ay, ps[k].az);
        fetches++;
        if ((prev <= iso && iso < dens) || (prev >= iso && iso > dens)) {
          const float tt = (iso - prev) / (dens - prev);
          const float st = fmaf(tt, h, s);
          const f3 hp{fmaf(dir.x, st, tp.x), fmaf(dir.y, st, tp.y), fmaf(dir.z, st, tp.z)};
          iso_composite(Q, iso_hit_colour<PHONG>(Q, grad, hp, hg, eye), dst);
          if (dst.w > 0.99f) { done = true; break; }
        }
        prev = dens;
        s = s + h;
      }
      if (done) break;
    }
    return;
  }
  // rayDirRecip of the V2 file (:107-110), per ray
  float rdir[3];
  {
    const float dd[3] = {dir.x, dir.y, dir.z};
#pragma unroll
    for (int i = 0; i < 3; i++)
      rdir[i] = fabsf(dd[i]) > 1e-6f ? 1.0f / dd[i]
                                     : (dd[i] > 0.0f ? 1e6f : (dd[i] < 0.0f ? -1e6f : 0.0f));
  }
  float t = r.tnear;
  float pd = iso_density(A, cells, iso_tex(eye, dir, t, hg), sp);   // prevDensity at tnear
  fetches++;
  float dc = pd;
  bool have = true;
  while (t < tfar && iters < kIsoMaxIter) {
    if (have) {
      // Speculative run of the in-block path: kIsoSpec steps of the size the
      // density at t gives, their block lookups and volume fetches issued
      // together, consumed in order while the block is not skippable, the step
      // decision holds and no surface is hit; anything else falls back to the
      // one-step path below at the same t.
      // (variant 0 sizes the step from the old prevDensity, variant 1 from the
      // density at t)
      const bool near0 = fabsf((VARIANT == 0 ? pd : dc) - iso) < Q.step_range;
      const float sstep = near0 ? Q.step_small
                                : (VARIANT == 0 ? Q.step_large : fminf(Q.step_large, Q.half_block_len));
      float tk[kIsoSpec + 1], hk[kIsoSpec];
      uint4 ck[kIsoSpec];
      SamplePos pk[kIsoSpec];
      float2 mk[kIsoSpec];
      tk[0] = t;
#pragma unroll
      for (int k = 0; k < kIsoSpec; k++) {
        hk[k] = fminf(sstep, tfar - tk[k]);
        tk[k + 1] = tk[k] + hk[k];
        const f3 q = iso_tex(eye, dir, tk[k + 1], hg);
        pk[k] = sample_pos_clamped(fmaf(q.x, A.n_over_g[0], -0.5f), fmaf(q.y, A.n_over_g[1], -0.5f),
                                   fmaf(q.z, A.n_over_g[2], -0.5f), A);
        ck[k] = cells[pk[k].idx];
      }
      // Block of each step start.  The index floor((fma(d, t, e) + G/2) / G * nb)
      // is a composition of correctly rounded monotone operations, so it is
      // monotone in t: equal at the first and last start (the starts not
      // decreasing) means equal at every start in between.
      {
        int b0[3], bl[3];
        iso_block(Q, eye, dir, tk[0], b0);
        iso_block(Q, eye, dir, tk[kIsoSpec - 1], bl);
        bool mono = true;                  // every h >= 0: the starts do not decrease
#pragma unroll
        for (int k = 0; k + 1 < kIsoSpec; k++) mono = mono && hk[k] >= 0.0f;
        const bool same = mono && b0[0] == bl[0] && b0[1] == bl[1] && b0[2] == bl[2];
        mk[0] = iso_block_range(Q, mm, b0);
        if (same) {
#pragma unroll
          for (int k = 1; k < kIsoSpec; k++) mk[k] = mk[0];
        } else {
#pragma unroll
          for (int k = 1; k < kIsoSpec; k++) {
            int bk[3];
            iso_block(Q, eye, dir, tk[k], bk);
            mk[k] = iso_block_range(Q, mm, bk);
          }
        }
      }
      int used = 0;
      bool done = false;
#pragma unroll
      for (int k = 0; k < kIsoSpec; k++) {
        if (!(t < tfar) || iters >= kIsoMaxIter) break;
        if (VARIANT == 0 ? (iso < mk[k].x || iso > mk[k].y)
                         : (iso < mk[k].x - 0.001f || iso > mk[k].y + 0.001f))
          break;
        if (k > 0 && (fabsf((VARIANT == 0 ? pd : dc) - iso) < Q.step_range) != near0) break;
        iters++;
        used++;
        fetches++;                       // prevDensity / currentDensity at t (= dc)
        pd = dc;
        const float h = hk[k];
        t = tk[k + 1];                   // t += h
        const float dens = trilerp_cell(ck[k], pk[k].ax, pk[k].ay, pk[k].az);
        fetches++;
        dc = dens;
        if ((pd <= iso && iso < dens) || (pd >= iso && iso > dens)) {
          if (VARIANT == 0) {
            t -= (dens - iso) / (dens - pd);
          } else {
            const float tt = (iso - pd) / (dens - pd);
            t = t - h * (1.0f - tt);
          }
          have = false;
          iso_composite(Q, iso_hit_colour<PHONG>(Q, grad, iso_tex(eye, dir, t, hg), hg, eye), dst);
          if (dst.w > 0.99f) done = true;
          break;
        }
      }
      if (done) break;
      if (used > 0) continue;
    }
    iters++;
    // The in-block path's next fetch depends on t and a density already known
    // (variant 0: the old prevDensity; variant 1: the density at t when `have`),
    // not on the block table: issue it before the table lookup so both loads are
    // in flight together.  It is used only when that path runs at this t.
    const float known = VARIANT == 0 ? pd : dc;
    const float sstep = fabsf(known - iso) < Q.step_range
                            ? Q.step_small
                            : (VARIANT == 0 ? Q.step_large : fminf(Q.step_large, Q.half_block_len));
    const float sh = fminf(sstep, tfar - t);
    // (variant 1 without the density at t: the hoisted fetch is that density,
    // currentDensity, instead)
    const float st2 = (VARIANT == 1 && !have) ? t : t + sh;
    const SamplePos sp2 = sample_pos_clamped(fmaf(iso_tex(eye, dir, st2, hg).x, A.n_over_g[0], -0.5f),
                                             fmaf(iso_tex(eye, dir, st2, hg).y, A.n_over_g[1], -0.5f),
                                             fmaf(iso_tex(eye, dir, st2, hg).z, A.n_over_g[2], -0.5f), A);
    const uint4 c2 = cells[sp2.idx];
    int b[3];
    iso_block(Q, eye, dir, t, b);
    const float2 m = iso_block_range(Q, mm, b);
    // block bounds in world space (getBlockBounds), from the unwrapped index
    float bmin[3], bmax[3];
#pragma unroll
    for (int i = 0; i < 3; i++) {
      bmin[i] = Q.nhg[i] + Q.bs[i] * (float)b[i];
      bmax[i] = bmin[i] + Q.bs[i];
    }
    const float d[3] = {dir.x, dir.y, dir.z};
    const float op[3] = {fmaf(dir.x, t, eye.x), fmaf(dir.y, t, eye.y), fmaf(dir.z, t, eye.z)};
    if (VARIANT == 0) {
      bool tilted = false;
      if (iso < m.x || iso > m.y) {
        float dt;
        // calculateNextBlockIntersection (:97-129): the ray's chord through the block
        if (fabsf(d[0]) < 0.01f || fabsf(d[1]) < 0.01f || fabsf(d[2]) < 0.01f) {
          dt = -1.0f;
        } else {
          float tmin[3], tmax[3];
#pragma unroll
          for (int i = 0; i < 3; i++) {
            const float t1 = (bmin[i] - op[i]) / d[i], t2 = (bmax[i] - op[i]) / d[i];
            tmin[i] = fminf(t1, t2);
            tmax[i] = fmaxf(t1, t2);
          }
          dt = fminf(fminf(tmax[0], tmax[1]), tmax[2]) - fmaxf(fmaxf(tmin[0], tmin[1]), tmin[2]);
        }
        if (dt == -1.0f) tilted = true;
        if (dt <= Q.step_small) dt = Q.step_small;
        t += dt;
        have = false;
        if (!tilted) continue;
      }
      // adaptive step: the size from the OLD prevDensity, then prevDensity at t
      const float step = fabsf(pd - iso) < Q.step_range ? Q.step_small : Q.step_large;
      const bool fresh = !tilted;   // t and the old prevDensity as at the hoisted fetch
      pd = have ? dc : iso_density(A, cells, iso_tex(eye, dir, t, hg), sp);
      fetches++;
      const float h = fminf(step, tfar - t);
      t += h;
      const float dens = fresh ? trilerp_cell(c2, sp2.ax, sp2.ay, sp2.az)
                               : iso_density(A, cells, iso_tex(eye, dir, t, hg), sp);
      fetches++;
      dc = dens;
      have = true;
      if ((pd <= iso && iso < dens) || (pd >= iso && iso > dens)) {
        const float tt = (dens - iso) / (dens - pd);
        t -= tt;
        have = false;
        iso_composite(Q, iso_hit_colour<PHONG>(Q, grad, iso_tex(eye, dir, t, hg), hg, eye), dst);
        if (dst.w > 0.99f) break;
      }
    } else {
      // isBlockSkippable (:137-141)
      if (iso < m.x - 0.001f || iso > m.y + 0.001f) {
        // calculateNextBlockIntersection of the V2 file (:105-135): exit distance + offsets
        float tmax[3];
#pragma unroll
        for (int i = 0; i < 3; i++) tmax[i] = fmaxf((bmin[i] - op[i]) * rdir[i], (bmax[i] - op[i]) * rdir[i]);
        float exitT = fminf(fminf(tmax[0], tmax[1]), tmax[2]);
        if (fabsf(exitT - tmax[0]) < 1e-5f) exitT += 1e-4f;
        if (fabsf(exitT - tmax[1]) < 1e-5f) exitT += 1e-4f;
        if (fabsf(exitT - tmax[2]) < 1e-5f) exitT += 1e-4f;
        t += fmaxf(Q.step_small, exitT);
        // prevDensity = texture(newPos): fetched by the shader, overwritten before use
        fetches++;
        have = false;
        continue;
      }
      const bool fresh = have;              // the hoisted fetch used dc = density at t
      const float cur = have ? dc : trilerp_cell(c2, sp2.ax, sp2.ay, sp2.az);
      fetches++;
      const float step = fabsf(cur - iso) < Q.step_range ? Q.step_small
                                                          : fminf(Q.step_large, Q.half_block_len);
      const float h = fminf(step, tfar - t);
      pd = cur;
      t += h;
      const float dens = fresh ? trilerp_cell(c2, sp2.ax, sp2.ay, sp2.az)
                               : iso_density(A, cells, iso_tex(eye, dir, t, hg), sp);
      fetches++;
      dc = dens;
      have = true;
      if ((pd <= iso && iso < dens) || (pd >= iso && iso > dens)) {
        const float tt = (iso - pd) / (dens - pd);
        t = t - h * (1.0f - tt);
        have = false;
        iso_composite(Q, iso_hit_colour<PHONG>(Q, grad, iso_tex(eye, dir, t, hg), hg, eye), dst);
        if (dst.w > 0.99f) break;
      }
    }
  }
}

// Register budget per variant (waves/SIMD; 1 = the compiler's choice): 6 / 6 / 8
// (80 / 80 / 63 VGPRs; the compiler alone: 84 / 88 / 67 -> 5 / 5 / 7 waves).  One
// kernel takes the same time, frames in flight overlap better: frame 2.20 ->
// 2.11, 1.59 -> 1.53, 1.54 -> 1.50 ms.
#ifndef CVR_ISO_WAVES0
#define CVR_ISO_WAVES0 6
#endif
#ifndef CVR_ISO_WAVES1
#define CVR_ISO_WAVES1 6
#endif
#ifndef CVR_ISO_WAVES2
#define CVR_ISO_WAVES2 8
#endif
#ifndef CVR_ISO_COLGROUP
#define CVR_ISO_COLGROUP 4   // iso 2.11 -> 2.09 ms, isoadapt 1.494 -> 1.483, isodfs neutral (tools/r02_s56.sh)
#endif
template <int VARIANT, bool PHONG>
constexpr int iso_waves_per_eu() {
  return PHONG ? 1 : (VARIANT == 0 ? CVR_ISO_WAVES0 : (VARIANT == 1 ? CVR_ISO_WAVES1 : CVR_ISO_WAVES2));
}
template <int VARIANT, bool PHONG>
__global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(iso_waves_per_eu<VARIANT, PHONG>())))
iso_tile_kernel(IsoArgs Q, const uint4* __restrict__ cells, const uint4* __restrict__ grad,
                const float2* __restrict__ mm, float4* __restrict__ out,
                uint32_t* __restrict__ samples, unsigned long long* __restrict__ tile_samples) {
  const Rc1passArgs& A = Q.a;
  const int b = blockIdx.x, nt = A.ntiles;
  // groups of 4 tile columns dealt round-robin over the XCDs: every XCD gets a
  // share of every screen region, so the long iso rays spread evenly (contiguous
  // XCD bands measured 4-8 % slower), and neighbouring tiles share an L2
  const int t = screen_tile_of_block<CVR_ISO_COLGROUP>(A, b, nt);
  const int lane = threadIdx.x;
  int px, py;
  long long oidx;
  tile_pixel(A, t, lane & 7, lane >> 3, px, py, oidx);
  const bool inside = px < A.W && py < A.H;
  float4 dst = make_float4(0.f, 0.f, 0.f, 0.f);
  uint32_t fetches = 0, iters = 0;
  if (inside) iso_march<VARIANT, PHONG>(Q, cells, grad, mm, px, py, dst, fetches, iters);
  if (inside || A.packed) {
    store_rgba(out, oidx, dst, A.out_half);
    if (samples) samples[oidx] = fetches;
  }
  if (tile_samples) {
    const unsigned long long v = wave_sum(fetches);
    if (lane == 0) tile_samples[t] = v;
  }
}

// Block min / max of the normalised voxel values (ComputeBlocksFromVolume,
// rc1custompisoadaptrenderer.cpp:20-117): blocks of ceil(N / nb) voxels per
// axis, [start, min(start + size, N)); raw integer extremes here, normalised by
// the host (v / 255 or v / 65535 in double, then float, the R32F texture).
// Workgroup (block, slab): `zc` planes of one block, folded in by atomics, so a
// 4^3 table still spreads over the whole chip.
__global__ void block_minmax_init(uint2* __restrict__ out, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) out[i] = make_uint2(0xffffffffu, 0u);
}

template <typename VT>
__global__ void __launch_bounds__(256)
block_minmax_kernel(const VT* __restrict__ vox, int nx, int ny, int nz, int nbx, int nby, int bsx,
                    int bsy, int bsz, int zc, int nslab, uint2* __restrict__ out) {
  const int blk = blockIdx.x / nslab, slab = blockIdx.x % nslab;
  const int bx = blk % nbx, by = (blk / nbx) % nby, bz = blk / (nbx * nby);
  const int x0 = bx * bsx, y0 = by * bsy, zb = bz * bsz;
  const int x1 = min(x0 + bsx, nx), y1 = min(y0 + bsy, ny), zb1 = min(zb + bsz, nz);
  const int z0 = zb + slab * zc, z1 = min(z0 + zc, zb1);
  uint32_t lo = 0xffffffffu, hi = 0;
  const int w = x1 - x0, h = y1 - y0, dpt = z1 - z0;
  const long long n = (w > 0 && h > 0 && dpt > 0) ? (long long)w * h * dpt : 0;
  for (long long i = threadIdx.x; i < n; i += blockDim.x) {
    const int x = x0 + (int)(i % w), y = y0 + (int)((i / w) % h), z = z0 + (int)(i / ((long long)w * h));
    const uint32_t v = vox[((size_t)z * ny + y) * nx + x];
    lo = min(lo, v);
    hi = max(hi, v);
  }
  __shared__ uint32_t slo[256], shi[256];
  slo[threadIdx.x] = lo;
  shi[threadIdx.x] = hi;
  __syncthreads();
  for (int s = blockDim.x / 2; s > 0; s >>= 1) {
    if ((int)threadIdx.x < s) {
      slo[threadIdx.x] = min(slo[threadIdx.x], slo[threadIdx.x + s]);
      shi[threadIdx.x] = max(shi[threadIdx.x], shi[threadIdx.x + s]);
    }
    __syncthreads();
  }
  if (threadIdx.x == 0 && n > 0) {
    atomicMin(&out[blk].x, slo[0]);
    atomicMax(&out[blk].y, shi[0]);
  }
}

}  // namespace

hipError_t launch_block_minmax(const void* vox, int bpv, const int N[3], const int nb[3], uint2* out,
                               hipStream_t s) {
  const int bs[3] = {(N[0] + nb[0] - 1) / nb[0], (N[1] + nb[1] - 1) / nb[1],
                     (N[2] + nb[2] - 1) / nb[2]};
  const int nblk = nb[0] * nb[1] * nb[2];
  // slabs of >= 4 planes until the grid has ~4096 workgroups
  const int want = std::max(1, std::min((4096 + nblk - 1) / nblk, (bs[2] + 3) / 4));
  const int zc = (bs[2] + want - 1) / want;
  const int nslab = (bs[2] + zc - 1) / zc;
  hipLaunchKernelGGL(block_minmax_init, dim3((unsigned)((nblk + 255) / 256)), dim3(256), 0, s, out,
                     nblk);
  const dim3 g((unsigned)((long long)nblk * nslab)), b(256);
  if (bpv == 1)
    hipLaunchKernelGGL(block_minmax_kernel<uint8_t>, g, b, 0, s, (const uint8_t*)vox, N[0], N[1],
                       N[2], nb[0], nb[1], bs[0], bs[1], bs[2], zc, nslab, out);
  else
    hipLaunchKernelGGL(block_minmax_kernel<uint16_t>, g, b, 0, s, (const uint16_t*)vox, N[0], N[1],
                       N[2], nb[0], nb[1], bs[0], bs[1], bs[2], zc, nslab, out);
  return hipGetLastError();
}

hipError_t launch_iso(const Ctx& c, const IsoArgs& q, int variant, bool phong, const float2* mm,
                      float4* out, uint32_t* samples, unsigned long long* tile_samples,
                      hipStream_t s) {
  if (q.a.ntiles <= 0) return hipSuccess;
  const uint4* cells = (const uint4*)c.d_cells;
  const uint4* grad = (const uint4*)c.d_grad;
  const dim3 g((unsigned)q.a.ntiles), b(64);
#define CVR_ISO_LAUNCH(V, P)                                                                   \
  hipLaunchKernelGGL((iso_tile_kernel<V, P>), g, b, 0, s, q, cells, grad, mm, out, samples,   \
                     tile_samples)
  if (variant == 0) {
    if (phong) CVR_ISO_LAUNCH(0, true); else CVR_ISO_LAUNCH(0, false);
  } else if (variant == 2) {
    if (phong) CVR_ISO_LAUNCH(2, true); else CVR_ISO_LAUNCH(2, false);
  } else {
    if (phong) CVR_ISO_LAUNCH(1, true); else CVR_ISO_LAUNCH(1, false);
  }
#undef CVR_ISO_LAUNCH
  return hipGetLastError();
}

}  // namespace cvr
