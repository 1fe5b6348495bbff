// flat.hip — the non-template parts of flat shading (shaded_march.h): the tile
// scan, the front-to-back fold and the job buffers.
#include <hip/hip_runtime.h>
#include <cstdint>

#include "cvr_device.h"
#include "cvr_internal.h"
#include "march_common.h"
#include "shaded_march.h"

namespace cvr {

// Exclusive scan of the per-tile job counts (in place) and the frame total.
// One workgroup: a contiguous run of tiles per thread, then a scan of the runs.
__global__ void __launch_bounds__(1024) flat_scan_kernel(uint32_t* __restrict__ tile_off, int n,
                                                         unsigned long long* __restrict__ total) {
  __shared__ unsigned long long part[1024];
  const int t = threadIdx.x;
  const int per = (n + 1023) / 1024;
  const int lo = min(n, t * per), hi = min(n, lo + per);
  unsigned long long sum = 0;
  for (int i = lo; i < hi; i++) sum += tile_off[i];
  part[t] = sum;
  __syncthreads();
  for (int d = 1; d < 1024; d <<= 1) {          // Hillis-Steele inclusive scan of the runs
    const unsigned long long v = t >= d ? part[t - d] : 0ull;
    __syncthreads();
    part[t] += v;
    __syncthreads();
  }
  unsigned long long run = part[t] - sum;       // exclusive start of this thread's run
  for (int i = lo; i < hi; i++) {
    const uint32_t v = tile_off[i];
    tile_off[i] = (uint32_t)run;
    run += v;
  }
  if (t == 1023) *total = part[1023];
}

// Per pixel: its jobs' results folded in sample order, dst.a replayed from the
// alphas (the sequential loop: om = 1 - dst.a; dst.a = fma(om, a, dst.a);
// dst.rgb = fma(om, rgb * a, dst.rgb)).
__global__ void __launch_bounds__(64) flat_fold_kernel(Rc1passArgs A, FlatJobs J,
                                                       float4* __restrict__ out) {
  const int t = blockIdx.x, lane = threadIdx.x, slot = t * 64 + lane;
  int px, py;
  long long oidx;
  tile_pixel(A, t, lane & 7, lane >> 3, px, py, oidx);
  const uint32_t n = J.lane_jobs[slot];
  size_t i = (size_t)J.tile_off[t] + wave_excl_scan(n, lane);
  float4 dst = make_float4(0.f, 0.f, 0.f, 0.f);
  for (uint32_t j = 0; j < n; j++, i++) {
    const float4 r = J.res[i];
    const float om = 1.0f - dst.w;
    dst.w = fmaf(om, r.w, dst.w);
    dst.x = fmaf(om, r.x, dst.x);
    dst.y = fmaf(om, r.y, dst.y);
    dst.z = fmaf(om, r.z, dst.z);
  }
  if ((px < A.W && py < A.H) || A.packed) store_rgba(out, oidx, dst, A.out_half);
}

hipError_t launch_flat_scan(FlatJobs& J, int ntiles, hipStream_t s) {
  hipLaunchKernelGGL(flat_scan_kernel, dim3(1), dim3(1024), 0, s, J.tile_off, ntiles, J.total);
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

// Buffers for `ntiles` 8x8 tiles and `jobs` jobs (0: the per-pixel part only).
// Grows, never shrinks; the job list gets 1/4 headroom so a slowly moving camera
// does not re-allocate every frame.  Blocks the calling thread only when it allocates.
hipError_t flat_reserve(FlatJobs& J, int ntiles, size_t jobs, int /*phong*/) {
  hipError_t e = hipSuccess;
  if (J.tiles < ntiles) {
    void* p = J.lane_jobs; free_ptr(p); J.lane_jobs = nullptr;
    p = J.tile_off; free_ptr(p); J.tile_off = nullptr;
    p = J.cam; free_ptr(p); J.cam = nullptr;
    J.tiles = 0;
    const size_t slots = (size_t)ntiles * 64;
    if ((e = hipMalloc((void**)&J.lane_jobs, slots * sizeof(uint32_t))) != hipSuccess) return e;
    if ((e = hipMalloc((void**)&J.tile_off, ((size_t)ntiles + 1) * sizeof(uint32_t))) != hipSuccess) return e;
    if ((e = hipMalloc((void**)&J.cam, slots * sizeof(float4))) != hipSuccess) return e;
    J.tiles = ntiles;
  }
  if (!J.total && (e = hipMalloc((void**)&J.total, sizeof(unsigned long long))) != hipSuccess) return e;
  if (!J.h_total && (e = hipHostMalloc((void**)&J.h_total, sizeof(unsigned long long))) != hipSuccess)
    return e;
  if (jobs >= (1ull << 32)) return hipErrorInvalidValue;   // 32-bit tile offsets
  if (jobs > J.cap) {
    void* p = J.jobs; free_ptr(p); J.jobs = nullptr;
    p = J.res; free_ptr(p); J.res = nullptr;
    J.cap = 0;
    const size_t cap = jobs + jobs / 4 + 1024;
    if ((e = hipMalloc((void**)&J.jobs, cap * 3 * sizeof(float4))) != hipSuccess) return e;
    if ((e = hipMalloc((void**)&J.res, cap * sizeof(float4))) != hipSuccess) return e;
    J.cap = cap;
  }
  return hipSuccess;
}

void flat_release(FlatJobs& J) {
  void* p = J.lane_jobs; free_ptr(p);
  p = J.tile_off; free_ptr(p);
  p = J.cam; free_ptr(p);
  p = J.total; free_ptr(p);
  p = J.jobs; free_ptr(p);
  p = J.res; free_ptr(p);
  if (J.h_total) (void)hipHostFree(J.h_total);
  J = FlatJobs();
}

}  // namespace cvr
