// shaded_march.h — the single-pass march of the shaded renderers (rc1pdosct,
// rc1pextbsd) with their per-sample shading deferred into full-wave batches.
//
// ray_bbox_marching.comp:658-734 and ebs_ray_bbox_marching.comp:552-625 march
// exactly as rc1pass does and, for every sample with alpha > 0, call an
// expensive ShadeSample (cone tracing / SAT boxes: 10^2..10^3 fetches).  The
// opacity of a sample, and with it the ERT break and the sample count, does not
// depend on its shading (ShadeSample changes rgb only).  So each lane marches
// its ray and, for every such sample, appends a shading job (position, TF
// colour, alpha, 1 - dst.a before it) to its queue in LDS, advancing dst.a at
// once.  When the wave holds >= 64 jobs (or no lane can march further) the jobs
// are compacted and shaded 64 at a time, one per lane, so the shading runs at
// full wave occupancy whatever the rays' divergence.  Each lane then folds its
// own results into dst.rgb in sample order with the same fma as the sequential
// loop: the image is bit-identical to it.
//
// A shader is a struct with
//   using Args = ...;   // holds `Rc1passArgs a` (ray, volume, TF, tiles)
//   using Data = ...;   // its device tables (passed by value)
//   static f3 shade(const Args&, Data, f3 tx, f3 wp, f3 cam, f3 rgb, const f3* g, uint32_t& lit,
//                   uint32_t& fetches);
// (tx: position in the [0, G] box, wp: world position, cam: the ray's camera
// direction, g: the gradient sample when Phong shading is on, else null; lit
// and fetches count the shadow traces and the secondary texture fetches, for the
// roofline).
#pragma once

#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdint>

#include "cvr_device.h"
#include "cvr_internal.h"
#include "march_common.h"

namespace cvr {

constexpr int kJobsPerLane = 4;
constexpr int kJobSlots = 64 * kJobsPerLane;

__device__ __forceinline__ f3 vmad(f3 d, float t, f3 p) {
  return f3{fmaf(d.x, t, p.x), fmaf(d.y, t, p.y), fmaf(d.z, t, p.z)};
}
__device__ __forceinline__ f3 cross3(f3 x, f3 y) {   // glm / GLSL cross, no fma
  return f3{x.y * y.z - y.y * x.z, x.z * y.x - y.z * x.x, x.x * y.y - y.x * x.y};
}

#ifndef CVR_SHADED_COLGROUP
#define CVR_SHADED_COLGROUP 4
#endif

// One wave = one 8x8 tile.
template <class SH, bool PHONG>
__global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(SH::kMinWavesPerEU)))
shaded_march_kernel(typename SH::Args Q, const uint4* __restrict__ cells,
                    const uint4* __restrict__ grad, const float4* __restrict__ tf_g,
                    typename SH::Data data, float4* __restrict__ out,
                    uint32_t* __restrict__ samples, unsigned long long* __restrict__ shade_ctr,
                    unsigned long long* __restrict__ tile_samples,
                    const unsigned long long* __restrict__ run_if) {
  // run_if: the flat pipeline's totals; this kernel is its fallback and renders
  // only a frame whose job list did not fit (run_if[2] set by flat_scan_kernel)
  if (run_if && !run_if[2]) return;
  extern __shared__ float4 tfp[];
  __shared__ float jpx[kJobSlots], jpy[kJobSlots], jpz[kJobSlots];   // tx_pos
  __shared__ float jr[kJobSlots], jg[kJobSlots], jb[kJobSlots];      // TF rgb -> shaded rgb * a
  __shared__ float ja[kJobSlots], jom[kJobSlots];                    // alpha, 1 - dst.a
  __shared__ float jnx[PHONG ? kJobSlots : 1], jny[PHONG ? kJobSlots : 1],
      jnz[PHONG ? kJobSlots : 1];                                     // gradient (Phong)
  __shared__ uint16_t jlist[kJobSlots];
  __shared__ float lane_cam[3][64];
  load_tf_lds(tfp, tf_g, Q.a.tf_n);
  const Rc1passArgs& A = Q.a;
  const int b = blockIdx.x, nt = A.ntiles;
  // column groups dealt round-robin over the XCDs: each XCD gets a share of
  // every screen region, so the costly shading regions spread over all XCDs
  // (contiguous XCD bands: DOS kernel 23.5 vs 21.1 ms, EBS 512^3 42.0 vs 35.1 ms)
  const int t = screen_tile_of_block<CVR_SHADED_COLGROUP>(A, b, nt);
  const int lane = threadIdx.x;
  int px, py;
  long long oidx;
  tile_pixel(A, t, lane & 7, lane >> 3, px, py, oidx);
  const bool inside = px < A.W && py < A.H;
  float4 dst = make_float4(0.f, 0.f, 0.f, 0.f);
  uint32_t cnt = 0, nshade = 0, nlit = 0, nfetch = 0;
  Ray r;
  bool active = inside && ray_setup(A, px, py, r);
  if (active) {
    lane_cam[0][lane] = r.cam.x;
    lane_cam[1][lane] = r.cam.y;
    lane_cam[2][lane] = r.cam.z;
    active = 0.0f < r.D;
  }
  const f3 hg{A.half_grid[0], A.half_grid[1], A.half_grid[2]};
  const float step = A.step, fn = (float)A.tf_n;
  float s = 0.0f;
  const bool wave_in_box = __ballot(active && r.outside) == 0;   // else clamp positions

  for (;;) {
    // ---- march until the wave holds a full batch of jobs --------------------
    int n = 0;            // this lane's queued jobs
    int queued = 0;       // the wave's (uniform)
    for (;;) {
      const bool can = active && n < kJobsPerLane;
      if (__ballot(can) == 0) break;
      bool pushed = false;
      if (can) {
        const float h = fminf(step, r.D - s);
        const float tt = fmaf(h, 0.5f, s);
        const float x = fmaf(r.dt.x, tt, r.o.x), y = fmaf(r.dt.y, tt, r.o.y),
                    z = fmaf(r.dt.z, tt, r.o.z);
        SamplePos sp = wave_in_box ? sample_pos(x, y, z, A) : sample_pos_clamped(x, y, z, A);
        if (SH::kFB) quantise_weights<SH::kFB>(sp);   // filter_bits: volume and gradient weights
        const float4 sc = classify<SH::kFB>(tfp, fn, trilerp_cell(cells[sp.idx], sp.ax, sp.ay, sp.az));
        cnt++;
        if (sc.w > 0.0f) {
          const int slot = lane * kJobsPerLane + n;
          const f3 tx = vmad(r.dir, tt, r.tpos);        // tx_pos, box at [0, G]
          jpx[slot] = tx.x; jpy[slot] = tx.y; jpz[slot] = tx.z;
          jr[slot] = sc.x; jg[slot] = sc.y; jb[slot] = sc.z;
          const float a = 1.0f - cvr_expf(-(sc.w * h));
          const float om = 1.0f - dst.w;
          ja[slot] = a;
          jom[slot] = om;
          if (PHONG) {
            const f3 g = sample_gradient_cell(grad, sp);
            jnx[slot] = g.x; jny[slot] = g.y; jnz[slot] = g.z;
          }
          dst.w = fmaf(om, a, dst.w);
          n++;
          pushed = true;
          if (dst.w > 0.99f) active = false;
        }
        if (active) {
          s = s + h;
          active = s < r.D;
        }
      }
      queued += __popcll(__ballot(pushed));
      if (queued >= 64) break;
    }
    if (queued == 0) break;   // nobody could march: every ray is done

    // ---- compact the queues: exclusive prefix of n from its bit planes -----
    const unsigned long long lt = (1ull << lane) - 1ull;
    const unsigned long long b0 = __ballot(n & 1), b1 = __ballot(n & 2), b2 = __ballot(n & 4);
    const int first = __popcll(b0 & lt) + 2 * __popcll(b1 & lt) + 4 * __popcll(b2 & lt);
    for (int j = 0; j < kJobsPerLane; j++)
      if (j < n) jlist[first + j] = (uint16_t)(lane * kJobsPerLane + j);
    __syncthreads();

    // ---- shade 64 jobs at a time -------------------------------------------
    for (int base = 0; base < queued; base += 64) {
      const int f = base + lane;
      if (f < queued) {
        const int slot = jlist[f];
        const int owner = slot / kJobsPerLane;
        const f3 tx{jpx[slot], jpy[slot], jpz[slot]};
        const f3 wp{tx.x - hg.x, tx.y - hg.y, tx.z - hg.z};
        const f3 cam{lane_cam[0][owner], lane_cam[1][owner], lane_cam[2][owner]};
        const f3 rgb{jr[slot], jg[slot], jb[slot]};
        f3 g;
        if (PHONG) g = f3{jnx[slot], jny[slot], jnz[slot]};
        const f3 c = SH::shade(Q, data, tx, wp, cam, rgb, PHONG ? &g : nullptr, nlit, nfetch);
        const float a = ja[slot];
        jr[slot] = c.x * a;
        jg[slot] = c.y * a;
        jb[slot] = c.z * a;
      }
    }
    __syncthreads();

    // ---- fold the results in sample order (front-to-back) -------------------
    for (int j = 0; j < kJobsPerLane; j++)
      if (j < n) {
        const int slot = lane * kJobsPerLane + j;
        const float om = jom[slot];
        dst.x = fmaf(om, jr[slot], dst.x);
        dst.y = fmaf(om, jg[slot], dst.y);
        dst.z = fmaf(om, jb[slot], dst.z);
      }
    nshade += n;
    __syncthreads();
  }

  if (inside || A.packed) {
    store_rgba(out, oidx, dst, A.out_half);
    if (samples) samples[oidx] = cnt;
  }
  if (tile_samples) {
    const unsigned long long v = wave_sum(cnt);
    if (lane == 0) tile_samples[t] = v;
  }
  if (shade_ctr) {   // measurement only (secondary-fetch count of the roofline)
    const unsigned long long sa = wave_sum(nshade), sl = wave_sum(nlit), sf = wave_sum(nfetch);
    if (lane == 0) {
      atomicAdd(&shade_ctr[0], sa);
      atomicAdd(&shade_ctr[1], sl);
      atomicAdd(&shade_ctr[2], sf);
    }
  }
}

// ---------------------------------------------------------------------------
// Flat shading (option "shade_flat", the default).  The per-wave batches above
// tie a tile's shading to its wave, so a frame lasts as long as its longest
// tile: with fewer tiles per GPU (the screen split) the longest waves set the
// frame time (one 1024^3 EBS wave runs for ~45 ms; 8 ranks: 2.1x, not 8x).
// Flat shading cuts the frame at the job instead:
//   1. shaded_jobs_kernel<count>: the march, counting per tile the jobs
//      (samples with alpha > 0 before the ERT break; opacity does not depend on
//      shading, so the march is exact without it) and the march rounds in which
//      at least one lane made a job;
//   2. flat_scan_kernel: both counts to exclusive offsets and frame totals,
//      and whether they fit the stream's buffer set (sized from earlier
//      frames' totals, read back without blocking; a frame that does not fit
//      is rendered by the per-wave kernel, launched behind the fold with the
//      flag as its condition, so the host never waits on a frame);
//   3. shaded_jobs_kernel<emit>: the same march; each round's jobs are written
//      contiguously (lane order, so the stores coalesce: position, alpha, TF
//      rgb, pixel slot; + gradient with Phong) and the round's ballot mask kept;
//   4. flat_shade_kernel: one job per lane over the whole list, 64-job chunks
//      dealt to the XCDs in groups of flat_group consecutive chunks (one XCD's
//      L2 sees neighbouring rays' neighbouring samples);
//   5. flat_fold_kernel: the tile's rounds replayed from their masks, each
//      lane folding its results front to back with the sequential loop's fma
//      order (dst.a from the alphas), so the image is bit-identical to the
//      per-wave kernel and to the oracle.
// ---------------------------------------------------------------------------

template <class SH, bool PHONG, bool EMIT>
__global__ void __launch_bounds__(64)
shaded_jobs_kernel(typename SH::Args Q, const uint4* __restrict__ cells,
                   const uint4* __restrict__ grad, const float4* __restrict__ tf_g, FlatJobs J,
                   uint32_t* __restrict__ samples, unsigned long long* __restrict__ shade_ctr,
                   unsigned long long* __restrict__ tile_samples) {
  if (EMIT && J.total[2]) return;   // the list does not fit: the per-wave fallback renders
  extern __shared__ float4 tfp[];
  load_tf_lds(tfp, tf_g, Q.a.tf_n);
  const Rc1passArgs& A = Q.a;
  const int t = screen_tile_of_block<CVR_SHADED_COLGROUP>(A, blockIdx.x, A.ntiles);
  const int lane = threadIdx.x;
  const int slot = t * 64 + lane;
  const unsigned long long lt = (1ull << lane) - 1ull;
  int px, py;
  long long oidx;
  tile_pixel(A, t, lane & 7, lane >> 3, px, py, oidx);
  const bool inside = px < A.W && py < A.H;
  Ray r;
  bool active = inside && ray_setup(A, px, py, r);
  active = active && 0.0f < r.D;
  const bool wave_in_box = __ballot(active && r.outside) == 0;   // else clamp positions
  size_t jbase = 0, rbase = 0;                                    // EMIT: the tile's next job / round
  if (EMIT) {
    jbase = J.tile_off[t];
    rbase = J.tile_roff[t];
  }
  const float step = A.step, fn = (float)A.tf_n;
  float s = 0.0f, dst_a = 0.0f;
  uint32_t cnt = 0, rounds = 0, tjobs = 0;   // rounds, tjobs: wave-uniform
  bool any_job = false;
  const bool skip = A.cell_skip > 0;   // per-cell skip flags (march_common.h cell_empty)
  for (;;) {   // one sample per live lane per round (wave-uniform loop)
    if (__ballot(active) == 0) break;
    bool pushed = false;
    float4 q0, q1, q2;
    float h = 0.0f, tt = 0.0f;
    SamplePos sp;
    uint4 raw;
    bool empty = true;
    if (active) {
      h = fminf(step, r.D - s);
      tt = fmaf(h, 0.5f, s);
      const float x = fmaf(r.dt.x, tt, r.o.x), y = fmaf(r.dt.y, tt, r.o.y), z = fmaf(r.dt.z, tt, r.o.z);
      sp = wave_in_box ? sample_pos(x, y, z, A) : sample_pos_clamped(x, y, z, A);
      raw = cells[sp.idx];
      empty = cell_empty(raw);
    }
    // every marching lane's sample in an empty cell: tau is exactly 0 for all of
    // them (no job, no alpha), so the round only counts and steps (bit-exact)
    const bool wave_empty = skip && __ballot(!empty) == 0;
    if (active) {
      float4 sc = make_float4(0.f, 0.f, 0.f, 0.f);
      if (!wave_empty) {
        if (SH::kFB) quantise_weights<SH::kFB>(sp);   // filter_bits: volume and gradient weights
        sc = classify<SH::kFB>(tfp, fn, trilerp_cell(raw, sp.ax, sp.ay, sp.az));
      }
      cnt++;
      if (sc.w > 0.0f) {
        const float a = 1.0f - cvr_expf(-(sc.w * h));
        if (EMIT) {
          const f3 tx = vmad(r.dir, tt, r.tpos);        // tx_pos, box at [0, G]
          q0 = make_float4(tx.x, tx.y, tx.z, a);
          q1 = make_float4(sc.x, sc.y, sc.z, __int_as_float(slot));
          if (PHONG) {
            const f3 g = sample_gradient_cell(grad, sp);
            q2 = make_float4(g.x, g.y, g.z, 0.0f);
          }
        }
        dst_a = fmaf(1.0f - dst_a, a, dst_a);
        pushed = true;
        any_job = true;
        if (dst_a > 0.99f) active = false;
      }
      if (active) {
        s = s + h;
        active = s < r.D;
      }
    }
    // the distance skip of an all-empty round (raymarch.hip march_ray, CS 3): when
    // every lane still marching sits in an empty cell at distance >= 2 from any
    // occupied one, all of them step over the same number of samples without
    // loads (the fewest any may: lanes stay at one sample index).  Skipped samples
    // make no job and no round, so the job list and its masks are unchanged.
    if (wave_empty && wave_in_box) {
      const int q = active ? cell_skip_q(raw) : 0;
      if (__ballot(active && q == 0) == 0 && __ballot(active) != 0 && active) {
        float dx = r.dt.x, dy = r.dt.y, dz = r.dt.z;
        asm volatile("" : "+v"(dx), "+v"(dy), "+v"(dz));
        const float kinv = __builtin_amdgcn_rcpf(step * fmaxf(fmaxf(fabsf(dx), fabsf(dy)), fabsf(dz)));
        const int msk = min(cvt_flr(((float)q - kSkipMarginTexels) * kinv),
                            cvt_flr((r.D - s) * A.inv_step) - 2);
        int i = 0;
        for (; __all(i < msk); i++) s = s + step;
        cnt += (uint32_t)i;
      }
    }
    const unsigned long long m = __ballot(pushed);
    if (m) {
      if (EMIT) {
        if (pushed) {
          float4* jp = J.jobs + (jbase + __popcll(m & lt)) * (PHONG ? 3 : 2);
          jp[0] = q0;
          jp[1] = q1;
          if (PHONG) jp[2] = q2;
        }
        if (lane == 0) J.masks[rbase + rounds] = m;
        jbase += __popcll(m);
      }
      tjobs += __popcll(m);
      rounds++;
    }
  }
  if (EMIT) return;
  J.cam[slot] = any_job ? make_float4(r.cam.x, r.cam.y, r.cam.z, 0.0f) : make_float4(0.f, 0.f, 0.f, 0.f);
  if (lane == 0) {
    J.tile_off[t] = tjobs;
    J.tile_roff[t] = rounds;
  }
  if ((inside || A.packed) && samples) samples[oidx] = cnt;
  if (tile_samples) {
    const unsigned long long v = wave_sum(cnt);
    if (lane == 0) tile_samples[t] = v;
  }
  if (shade_ctr && lane == 0) atomicAdd(&shade_ctr[0], (unsigned long long)tjobs);
}

template <class SH, bool PHONG>
__global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(SH::kFlatWavesPerEU)))
flat_shade_kernel(typename SH::Args Q, typename SH::Data data, FlatJobs J, int nchunks, int group,
                  unsigned long long* __restrict__ shade_ctr) {
  // the grid covers the set's capacity; this frame's total is on the device
  const unsigned long long total = J.total[0];
  if (J.total[2]) return;   // did not fit: the per-wave fallback renders the frame
  // block b runs on XCD b % 8; XCD x takes chunk groups x, x + 8, ... in order
  const int b = blockIdx.x, x = b & 7, k = b >> 3;
  const int chunk = ((k / group) * 8 + x) * group + (k % group);
  if (chunk >= nchunks || (unsigned long long)chunk * 64 >= total) return;
  const int lane = threadIdx.x;
  const unsigned long long i = (unsigned long long)chunk * 64 + lane;
  uint32_t nlit = 0, nfetch = 0;
  if constexpr (SH::kSplit) {
    if (i < total) {
      // Only the position (and the pixel slot, for the camera ray) is live across
      // the cone traces; opacity, colour and gradient are read after them, and the
      // job index is rebuilt from the block (the shader's visibility / combine
      // halves: 32 B of spills per lane at the 96-VGPR budget instead of 72)
      const float* jf = (const float*)(J.jobs + i * (PHONG ? 3 : 2));
      const f3 tx{jf[0], jf[1], jf[2]};
      const float4 cm = J.cam[__float_as_int(jf[7])];
      const typename SH::Vis vis =
          SH::visibility(Q, data, tx, SH::world_pos(Q, tx), f3{cm.x, cm.y, cm.z}, nlit, nfetch);
      // (the lane from mbcnt, which the compiler does not equate with the thread
      // index: the first index and address are not kept live or spilled)
      const unsigned long long i2 =
          (unsigned long long)chunk * 64 + __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u));
      const float* jf2 = (const float*)(J.jobs + i2 * (PHONG ? 3 : 2));
      f3 g;
      if (PHONG) g = f3{jf2[8], jf2[9], jf2[10]};
      const f3 tx2{jf2[0], jf2[1], jf2[2]};
      const f3 c = SH::combine(Q, vis, SH::world_pos(Q, tx2), f3{jf2[4], jf2[5], jf2[6]},
                               PHONG ? &g : nullptr);
      const float a = jf2[3];
      J.res[i2] = make_float4(c.x * a, c.y * a, c.z * a, a);
    }
  } else if (i < total) {
    const float4* jp = J.jobs + i * (PHONG ? 3 : 2);
    const float4 q0 = jp[0], q1 = jp[1];
    const f3 tx{q0.x, q0.y, q0.z};
    const f3 hg{Q.a.half_grid[0], Q.a.half_grid[1], Q.a.half_grid[2]};
    const f3 wp{tx.x - hg.x, tx.y - hg.y, tx.z - hg.z};
    const float4 cm = J.cam[__float_as_int(q1.w)];
    const f3 cam{cm.x, cm.y, cm.z};
    const f3 rgb{q1.x, q1.y, q1.z};
    f3 g;
    if (PHONG) {
      const float4 q2 = jp[2];
      g = f3{q2.x, q2.y, q2.z};
    }
    const f3 c = SH::shade(Q, data, tx, wp, cam, rgb, PHONG ? &g : nullptr, nlit, nfetch);
    const float a = q0.w;
    J.res[i] = make_float4(c.x * a, c.y * a, c.z * a, a);
  }
  if (shade_ctr) {   // measurement only (secondary-fetch count of the roofline)
    const unsigned long long sl = wave_sum(nlit), sf = wave_sum(nfetch);
    if (lane == 0) {
      atomicAdd(&shade_ctr[1], sl);
      atomicAdd(&shade_ctr[2], sf);
    }
  }
}

template <class SH>
hipError_t launch_shaded_march(const Ctx& c, const typename SH::Args& q, bool phong,
                               typename SH::Data data, float4* out, uint32_t* samples,
                               unsigned long long* shade_ctr, unsigned long long* tile_samples,
                               hipStream_t s, const unsigned long long* run_if = nullptr);
hipError_t launch_flat_scan(FlatJobs& J, int ntiles, unsigned long long cap, unsigned long long rcap,
                            unsigned long long* shade_ctr, hipStream_t s);
hipError_t launch_flat_fold(const Rc1passArgs& a, FlatJobs& J, float4* out, hipStream_t s);
hipError_t flat_reserve(FlatJobs& J, int ntiles, size_t jobs, size_t rounds, hipStream_t s);
FlatJobs& flat_set(const Ctx& c, hipStream_t s);

template <class SH>
hipError_t launch_shaded_flat(const Ctx& c, const typename SH::Args& q, bool phong,
                              typename SH::Data data, float4* out, uint32_t* samples,
                              unsigned long long* shade_ctr, unsigned long long* tile_samples,
                              hipStream_t s) {
  const int nt = q.a.ntiles;
  if (nt <= 0) return hipSuccess;
  if (q.a.tf_n > kMaxTfLds) return hipErrorInvalidValue;
  FlatJobs& J = flat_set(c, s);
  hipError_t e = flat_reserve(J, nt, 0, 0, s);
  if (e != hipSuccess) return e;
  const size_t lds = (size_t)(q.a.tf_n + 2) * sizeof(float4);
  const uint4* cells = (const uint4*)c.d_cells;
  const uint4* grad = (const uint4*)c.d_grad;
  const float4* tf = (const float4*)c.d_tf;
  // The set's capacity from the totals of its earlier frames, read back without
  // blocking: the copy of a frame's totals lands in pinned memory behind it
  // (ev_read), and is read by a later call once it has.
  if (J.pending_read && hipEventQuery(J.ev_read) == hipSuccess) {
    J.want_jobs = std::max(J.want_jobs, (size_t)J.h_total[0]);
    J.want_rounds = std::max(J.want_rounds, (size_t)J.h_total[1]);
    J.pending_read = false;
  }
  const bool first = J.cap == 0;   // no estimate yet: this frame reads its totals synchronously
  if (!first && (J.want_jobs > J.cap || J.want_rounds > J.rcap)) {
    if (flat_reserve(J, nt, J.want_jobs, J.want_rounds, s) != hipSuccess) {
      (void)hipGetLastError();   // too large to hold: keep the old size (frames fall back)
      J.want_jobs = std::min(J.want_jobs, J.cap);
      J.want_rounds = std::min(J.want_rounds, J.rcap);
    }
  }
  if (phong)
    hipLaunchKernelGGL((shaded_jobs_kernel<SH, true, false>), dim3(nt), dim3(64), lds, s, q, cells,
                       grad, tf, J, samples, shade_ctr, tile_samples);
  else
    hipLaunchKernelGGL((shaded_jobs_kernel<SH, false, false>), dim3(nt), dim3(64), lds, s, q, cells,
                       grad, tf, J, samples, shade_ctr, tile_samples);
  if ((e = hipGetLastError()) != hipSuccess) return e;
  const unsigned long long kNoLimit = ~0ull;
  // (debug_flat_limit: a smaller capacity, to exercise the device-side fallback)
  const unsigned long long lim = c.debug_flat_limit > 0 ? (unsigned long long)c.debug_flat_limit : kNoLimit;
  if ((e = launch_flat_scan(J, nt, first ? kNoLimit : std::min<unsigned long long>(J.cap, lim),
                            first ? kNoLimit : J.rcap, shade_ctr, s)) != hipSuccess)
    return e;
  if (first) {
    if ((e = hipMemcpyAsync(J.h_total, J.total, 3 * sizeof(unsigned long long), hipMemcpyDeviceToHost,
                            s)) != hipSuccess)
      return e;
    if ((e = hipStreamSynchronize(s)) != hipSuccess) return e;
    const unsigned long long total = J.h_total[0], rounds = J.h_total[1];
    J.want_jobs = (size_t)total;
    J.want_rounds = (size_t)rounds;
    if (flat_reserve(J, nt, std::max<size_t>((size_t)total, 1), std::max<size_t>((size_t)rounds, 1), s) !=
        hipSuccess) {
      // more jobs than 32-bit offsets or the free memory hold: the per-wave kernel
      // renders the same frame, bit for bit, without a job list
      (void)hipGetLastError();
      if (shade_ctr && (e = hipMemsetAsync(shade_ctr, 0, 3 * sizeof(unsigned long long), s)) != hipSuccess)
        return e;
      return launch_shaded_march<SH>(c, q, phong, data, out, samples, shade_ctr, tile_samples, s);
    }
  }
  if (phong)
    hipLaunchKernelGGL((shaded_jobs_kernel<SH, true, true>), dim3(nt), dim3(64), lds, s, q, cells,
                       grad, tf, J, nullptr, nullptr, nullptr);
  else
    hipLaunchKernelGGL((shaded_jobs_kernel<SH, false, true>), dim3(nt), dim3(64), lds, s, q, cells,
                       grad, tf, J, nullptr, nullptr, nullptr);
  if ((e = hipGetLastError()) != hipSuccess) return e;
  // the shade grid covers the set's capacity; blocks past the frame's total exit
  const unsigned long long nch = ((unsigned long long)J.cap + 63) / 64;
  if (nch > (1ull << 30)) return hipErrorInvalidValue;
  const int nchunks = (int)nch, group = c.flat_group;
  const long long span = 8LL * group;                           // chunks per round of the XCDs
  const long long nb = (nchunks + span - 1) / span * span;      // every XCD gets whole groups
  if (phong)
    hipLaunchKernelGGL((flat_shade_kernel<SH, true>), dim3((unsigned)nb), dim3(64), 0, s, q, data, J,
                       nchunks, group, shade_ctr);
  else
    hipLaunchKernelGGL((flat_shade_kernel<SH, false>), dim3((unsigned)nb), dim3(64), 0, s, q, data, J,
                       nchunks, group, shade_ctr);
  if ((e = hipGetLastError()) != hipSuccess) return e;
  if ((e = launch_flat_fold(q.a, J, out, s)) != hipSuccess) return e;
  // the device-side fallback: renders the frame only if its list did not fit
  if ((e = launch_shaded_march<SH>(c, q, phong, data, out, samples, shade_ctr, tile_samples, s,
                                   J.total)) != hipSuccess)
    return e;
  if (!first) {
    if ((e = hipMemcpyAsync(J.h_total, J.total, 3 * sizeof(unsigned long long), hipMemcpyDeviceToHost,
                            s)) != hipSuccess)
      return e;
    if ((e = hipEventRecord(J.ev_read, s)) != hipSuccess) return e;
    J.pending_read = true;
  }
  return hipEventRecord(J.ev_done, s);
}

template <class SH>
hipError_t launch_shaded_march(const Ctx& c, const typename SH::Args& q, bool phong,
                               typename SH::Data data, float4* out, uint32_t* samples,
                               unsigned long long* shade_ctr, unsigned long long* tile_samples,
                               hipStream_t s, const unsigned long long* run_if) {
  if (q.a.ntiles <= 0) return hipSuccess;
  if (q.a.tf_n > kMaxTfLds) return hipErrorInvalidValue;
  const size_t lds = (size_t)(q.a.tf_n + 2) * sizeof(float4);
  const uint4* cells = (const uint4*)c.d_cells;   // sample_pos indexes from the first cell
  if (phong)
    hipLaunchKernelGGL((shaded_march_kernel<SH, true>), dim3(q.a.ntiles), dim3(64), lds, s, q,
                       cells, (const uint4*)c.d_grad, (const float4*)c.d_tf, data, out, samples,
                       shade_ctr, tile_samples, run_if);
  else
    hipLaunchKernelGGL((shaded_march_kernel<SH, false>), dim3(q.a.ntiles), dim3(64), lds, s, q,
                       cells, (const uint4*)c.d_grad, (const float4*)c.d_tf, data, out, samples,
                       shade_ctr, tile_samples, run_if);
  return hipGetLastError();
}

}  // namespace cvr
