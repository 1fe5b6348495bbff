// flat.hip — the non-template parts of flat shading (shaded_march.h): the tile
// scan, the front-to-back fold and the job buffers.
#include <hip/hip_runtime.h>
#include <cstdint>

#include "cvr_device.h"
#include "cvr_internal.h"
#include "march_common.h"
#include "shaded_march.h"

namespace cvr {

// Exclusive scans (in place) of the per-tile job and round counts, each with
// its total at index n and in total[0] / total[1].  One workgroup walks the
// array in coalesced blocks of 4096 counts (a uint4 per thread), scanning each
// block through LDS and carrying its sum into the next.
__device__ void flat_scan_one(uint32_t* __restrict__ a, int n, unsigned long long* __restrict__ total,
                              unsigned long long* part) {
  const int t = threadIdx.x;
  unsigned long long carry = 0;
  for (int base = 0; base < n; base += 4096) {
    const int i0 = base + 4 * t;
    uint32_t v[4];
#pragma unroll
    for (int k = 0; k < 4; k++) v[k] = i0 + k < n ? a[i0 + k] : 0u;
    const unsigned long long sum = (unsigned long long)v[0] + v[1] + v[2] + v[3];
    part[t] = sum;
    __syncthreads();
    for (int d = 1; d < 1024; d <<= 1) {          // Hillis-Steele inclusive scan
      const unsigned long long x = t >= d ? part[t - d] : 0ull;
      __syncthreads();
      part[t] += x;
      __syncthreads();
    }
    unsigned long long run = carry + part[t] - sum;
#pragma unroll
    for (int k = 0; k < 4; k++) {
      if (i0 + k < n) a[i0 + k] = (uint32_t)run;
      run += v[k];
    }
    carry += part[1023];
    __syncthreads();
  }
  if (t == 0) {
    *total = carry;
    a[n] = (uint32_t)carry;
  }
  __syncthreads();
}

// After the scans: total[2] = 1 when the frame's jobs or rounds exceed the
// set's capacity.  The emit, shade and fold kernels then do nothing and the
// per-wave kernel renders the frame (the same bits); the count kernel's shade
// counters (measurement) are cleared for it.
__global__ void __launch_bounds__(1024) flat_scan_kernel(uint32_t* __restrict__ tile_off,
                                                         uint32_t* __restrict__ tile_roff, int n,
                                                         unsigned long long* __restrict__ total,
                                                         unsigned long long cap,
                                                         unsigned long long rcap,
                                                         unsigned long long* __restrict__ shade_ctr) {
  __shared__ unsigned long long part[1024];
  flat_scan_one(tile_off, n, total + 0, part);
  flat_scan_one(tile_roff, n, total + 1, part);
  if (threadIdx.x == 0) {
    const bool over = total[0] > cap || total[1] > rcap;
    total[2] = over ? 1ull : 0ull;
    if (over && shade_ctr) shade_ctr[0] = shade_ctr[1] = shade_ctr[2] = 0ull;
  }
}

// Per pixel: its jobs' results folded in sample order, dst.a replayed from the
// alphas (the sequential loop: om = 1 - dst.a; dst.a = fma(om, a, dst.a);
// dst.rgb = fma(om, rgb * a, dst.rgb)).  The tile's march rounds are replayed
// from their ballot masks: round r's results sit contiguously in lane order.
__global__ void __launch_bounds__(64) flat_fold_kernel(Rc1passArgs A, FlatJobs J,
                                                       float4* __restrict__ out) {
  if (J.total[2]) return;   // the list did not fit: the per-wave kernel writes the frame
  const int t = blockIdx.x, lane = threadIdx.x;
  const unsigned long long lt = (1ull << lane) - 1ull;
  int px, py;
  long long oidx;
  tile_pixel(A, t, lane & 7, lane >> 3, px, py, oidx);
  size_t j = J.tile_off[t];
  const uint32_t r0 = J.tile_roff[t], r1 = J.tile_roff[t + 1];
  float4 dst = make_float4(0.f, 0.f, 0.f, 0.f);
  for (uint32_t r = r0; r < r1; r++) {
    const unsigned long long m = J.masks[r];
    if ((m >> lane) & 1ull) {
      const float4 v = J.res[j + __popcll(m & lt)];
      const float om = 1.0f - dst.w;
      dst.w = fmaf(om, v.w, dst.w);
      dst.x = fmaf(om, v.x, dst.x);
      dst.y = fmaf(om, v.y, dst.y);
      dst.z = fmaf(om, v.z, dst.z);
    }
    j += __popcll(m);
  }
  if ((px < A.W && py < A.H) || A.packed) store_rgba(out, oidx, dst, A.out_half);
}

hipError_t launch_flat_scan(FlatJobs& J, int ntiles, unsigned long long cap, unsigned long long rcap,
                            unsigned long long* shade_ctr, hipStream_t s) {
  hipLaunchKernelGGL(flat_scan_kernel, dim3(1), dim3(1024), 0, s, J.tile_off, J.tile_roff, ntiles,
                     J.total, cap, rcap, shade_ctr);
  return hipGetLastError();
}

hipError_t launch_flat_fold(const Rc1passArgs& a, FlatJobs& J, float4* out, hipStream_t s) {
  if (a.ntiles <= 0) return hipSuccess;
  hipLaunchKernelGGL(flat_fold_kernel, dim3(a.ntiles), dim3(64), 0, s, a, J, out);
  return hipGetLastError();
}

static void free_ptr(void*& p) {
  if (p) (void)hipFree(p);
  p = nullptr;
}

// Buffers for `ntiles` 8x8 tiles, `jobs` jobs and `rounds` round masks (0: the
// per-tile part only), for frames on stream s.  Grows, never shrinks; the job list and the masks get
// 1/4 headroom so a slowly moving camera does not re-allocate every frame.
// Blocks the calling thread only when it allocates.
hipError_t flat_reserve(FlatJobs& J, int ntiles, size_t jobs, size_t rounds, hipStream_t s) {
  hipError_t e = hipSuccess;
  // growing frees buffers the set's last frame may still read: wait for that
  // frame only (its own event), not for the device
  if ((J.tiles < ntiles && J.tiles > 0) || (jobs > J.cap && J.cap > 0) || (rounds > J.rcap && J.rcap > 0))
    if (J.ev_done && (e = hipEventSynchronize(J.ev_done)) != hipSuccess) return e;
  if (!J.ev_done && (e = hipEventCreateWithFlags(&J.ev_done, hipEventDisableTiming)) != hipSuccess) return e;
  if (!J.ev_read && (e = hipEventCreateWithFlags(&J.ev_read, hipEventDisableTiming)) != hipSuccess) return e;
  if (J.tiles < ntiles) {
    void* p = J.tile_off; free_ptr(p); J.tile_off = nullptr;
    p = J.tile_roff; free_ptr(p); J.tile_roff = nullptr;
    p = J.cam; free_ptr(p); J.cam = nullptr;
    J.tiles = 0;
    const size_t slots = (size_t)ntiles * 64;
    if ((e = hipMalloc((void**)&J.tile_off, ((size_t)ntiles + 1) * sizeof(uint32_t))) != hipSuccess) return e;
    if ((e = hipMalloc((void**)&J.tile_roff, ((size_t)ntiles + 1) * sizeof(uint32_t))) != hipSuccess) return e;
    if ((e = hipMalloc((void**)&J.cam, slots * sizeof(float4))) != hipSuccess) return e;
    J.tiles = ntiles;
  }
  if (!J.total) {
    if ((e = hipMalloc((void**)&J.total, 3 * sizeof(unsigned long long))) != hipSuccess) return e;
    // on the render stream, ordered before the set's first count/scan: a plain
    // hipMemset runs on the null stream, which the caller's non-blocking render
    // streams do not wait for -- it could land after the first frame's scan and
    // zero its totals (round 4: a DOS frame on a fresh stream came out empty)
    if ((e = hipMemsetAsync(J.total, 0, 3 * sizeof(unsigned long long), s)) != hipSuccess) return e;
  }
  if (!J.h_total && (e = hipHostMalloc((void**)&J.h_total, 3 * sizeof(unsigned long long))) != hipSuccess)
    return e;
  if (jobs >= (1ull << 32) || rounds >= (1ull << 32)) return hipErrorInvalidValue;   // 32-bit offsets
  if (jobs > J.cap) {
    void* p = J.jobs; free_ptr(p); J.jobs = nullptr;
    p = J.res; free_ptr(p); J.res = nullptr;
    J.cap = 0;
    const size_t cap = jobs + jobs / 4 + 1024;
    if ((e = hipMalloc((void**)&J.jobs, cap * 3 * sizeof(float4))) != hipSuccess) return e;
    if ((e = hipMalloc((void**)&J.res, cap * sizeof(float4))) != hipSuccess) return e;
    J.cap = cap;
  }
  if (rounds > J.rcap) {
    void* p = J.masks; free_ptr(p); J.masks = nullptr;
    J.rcap = 0;
    const size_t cap = rounds + rounds / 4 + 1024;
    if ((e = hipMalloc((void**)&J.masks, cap * sizeof(unsigned long long))) != hipSuccess) return e;
    J.rcap = cap;
  }
  return hipSuccess;
}

// The buffer set of render stream s: the one it used before, else the least
// recently used set (a set taken over from another stream first waits, on the
// device, for that stream's last frame with it).
FlatJobs& flat_set(const Ctx& c, hipStream_t s) {
  FlatJobs* best = nullptr;
  for (auto& J : c.flat)
    if (J.owned && J.stream == s) best = &J;
  if (!best) {
    for (auto& J : c.flat)
      if (!best || J.last_use < best->last_use) best = &J;
    if (best->owned && best->ev_done) (void)hipStreamWaitEvent(s, best->ev_done, 0);
    best->owned = true;
    best->stream = s;
  }
  best->last_use = ++c.flat_clock;
  return *best;
}

void flat_release(FlatJobs& J) {
  if (J.ev_done) (void)hipEventSynchronize(J.ev_done);
  if (J.ev_done) (void)hipEventDestroy(J.ev_done);
  if (J.ev_read) (void)hipEventDestroy(J.ev_read);
  void* p = J.tile_off; free_ptr(p);
  p = J.tile_roff; free_ptr(p);
  p = J.masks; free_ptr(p);
  p = J.cam; free_ptr(p);
  p = J.total; free_ptr(p);
  p = J.jobs; free_ptr(p);
  p = J.res; free_ptr(p);
  if (J.h_total) (void)hipHostFree(J.h_total);
  J = FlatJobs();
}

}  // namespace cvr
