// wg_probe.hip — the cost of a workgroup's life around the rc1pass march, on
// gfx950: how long G workgroups of one wave take when each does only the parts of
// rc1pass_tile_kernel that do not depend on the ray's length.  Not product code: it
// measures the per-tile fixed cost behind DESIGN §5′ ("the per-frame fixed cost").
//
// Stages (cumulative, template mask):
//   0      empty kernel (dispatch only)
//   STORE  one 8-B RGBA16F store per lane (the frame write)
//   ORDER  the tile index from a launch-order table (a dependent scalar load)
//   TF     the transfer function, 258 float4 from global into dynamic LDS + barrier
//   SETUP  ray set-up arithmetic of the march (~90 VALU: 2 exact normalisations,
//          3 reciprocals, the slab test)
//   ARGS   a 1-KiB by-value argument block (the size of Rc1passArgs + LaunchFrames),
//          a few fields read
// WPB = waves per workgroup (one 8x8 tile per wave; one TF fill per workgroup).
//
//   hipcc --offload-arch=gfx950 -O3 -o tools/wg_probe tools/wg_probe.hip
//   ./tools/wg_probe          (one JSON line per case)
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>
#include <algorithm>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { \
  fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); return 1; } } while (0)

enum { STORE = 1, ORDER = 2, TF = 4, SETUP = 8, ARGS = 16 };

struct BigArgs { float v[256]; };

__device__ __forceinline__ float nrm_inv(float x, float y, float z) {
  const float d = fmaf(z, z, fmaf(y, y, x * x));
  const float s = __builtin_amdgcn_sqrtf(d);
  const float sm = __uint_as_float(__float_as_uint(s) - 1u), sp = __uint_as_float(__float_as_uint(s) + 1u);
  const float rm = fmaf(-sm, s, d), rp = fmaf(-sp, s, d);
  float r = rm <= 0.0f ? sm : s;
  r = rp > 0.0f ? sp : r;
  const float y0 = __builtin_amdgcn_rcpf(r);
  return fmaf(fmaf(-r, y0, 1.0f), y0, y0);
}

template <int M, int WPB>
__global__ void __launch_bounds__(64 * WPB) wg_kernel(BigArgs A, const float4* __restrict__ tf, int tf_n,
                                                      const int* __restrict__ order, int W,
                                                      uint2* __restrict__ out) {
  extern __shared__ float4 tfp[];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  int t = blockIdx.x * WPB + wave;
  if (M & ORDER) t = order[t];
  float acc = 0.0f;
  if (M & TF) {
    for (int i = threadIdx.x; i < tf_n + 2; i += blockDim.x) tfp[i] = tf[min(max(i - 1, 0), tf_n - 1)];
    __syncthreads();
    acc += tfp[(lane * 3) & 255].w;
  }
  const int tpr = W >> 3;
  const int px = (t % tpr) * 8 + (lane & 7), py = (t / tpr) * 8 + (lane >> 3);
  if (M & SETUP) {
    const float a0 = (M & ARGS) ? A.v[3] : 0.7f, a1 = (M & ARGS) ? A.v[17] : 0.3f;
    const float a2 = (M & ARGS) ? A.v[101] : 0.2f, a3 = (M & ARGS) ? A.v[250] : 0.9f;
    const float vx = fmaf(((float)px + 0.5f) / (float)W, 2.0f, -1.0f);
    const float vy = fmaf(((float)py + 0.5f) / (float)W, 2.0f, -1.0f);
    float cx = vx * a0, cy = vy * a1, cz = -1.0f;
    float dx = fmaf(cz, a2, fmaf(cy, a1, cx * a0)), dy = fmaf(cz, a0, fmaf(cy, a3, cx * a2));
    float dz = fmaf(cz, a3, fmaf(cy, a2, cx * a1));
    float k = nrm_inv(dx, dy, dz);
    dx *= k; dy *= k; dz *= k;
    k = nrm_inv(dx, dy, dz);
    dx *= k; dy *= k; dz *= k;
    const float ix = 1.0f / dx, iy = 1.0f / dy, iz = 1.0f / dz;
    const float tax = ix * (-256.f - a0), tbx = ix * (256.f - a0);
    const float tay = iy * (-256.f - a1), tby = iy * (256.f - a1);
    const float taz = iz * (-256.f - a2), tbz = iz * (256.f - a2);
    const float tn = fmaxf(fmaxf(fminf(tax, tbx), fminf(tay, tby)), fminf(taz, tbz));
    const float tf2 = fminf(fminf(fmaxf(tax, tbx), fmaxf(tay, tby)), fmaxf(taz, tbz));
    acc += (tf2 > tn) ? tf2 - tn : 0.0f;
  } else if (M & ARGS) {
    acc += A.v[3] + A.v[250];
  }
  if (M & STORE) {
    typedef _Float16 h2 __attribute__((ext_vector_type(2)));
    const h2 rg = {(_Float16)acc, (_Float16)(float)px}, ba = {(_Float16)(float)py, (_Float16)1.0f};
    out[(size_t)py * W + px] = make_uint2(__builtin_bit_cast(uint32_t, rg), __builtin_bit_cast(uint32_t, ba));
  }
}

template <int M, int WPB>
static int run(const char* name, int W, const float4* tf, const int* order, uint2* out, hipStream_t s) {
  const int tiles = (W / 8) * (W / 8);
  const int grid = tiles / WPB;
  const size_t lds = (M & TF) ? 258 * sizeof(float4) : 0;
  BigArgs A;
  for (int i = 0; i < 256; i++) A.v[i] = 0.25f + 0.001f * i;
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int i = 0; i < 50; i++)
    hipLaunchKernelGGL((wg_kernel<M, WPB>), dim3(grid), dim3(64 * WPB), lds, s, A, tf, 256, order, W, out);
  std::vector<float> ms;
  for (int r = 0; r < 30; r++) {
    CK(hipEventRecord(e0, s));
    hipLaunchKernelGGL((wg_kernel<M, WPB>), dim3(grid), dim3(64 * WPB), lds, s, A, tf, 256, order, W, out);
    CK(hipEventRecord(e1, s));
    CK(hipEventSynchronize(e1));
    float x;
    CK(hipEventElapsedTime(&x, e0, e1));
    ms.push_back(x);
  }
  // 30 launches back to back: the rate when launches queue (no event gaps)
  CK(hipEventRecord(e0, s));
  for (int r = 0; r < 30; r++)
    hipLaunchKernelGGL((wg_kernel<M, WPB>), dim3(grid), dim3(64 * WPB), lds, s, A, tf, 256, order, W, out);
  CK(hipEventRecord(e1, s));
  CK(hipEventSynchronize(e1));
  float bb;
  CK(hipEventElapsedTime(&bb, e0, e1));
  std::sort(ms.begin(), ms.end());
  printf("{\"case\": \"%s\", \"W\": %d, \"tiles\": %d, \"waves_per_wg\": %d, \"lone_ms_median\": %.5f, "
         "\"back_to_back_ms\": %.5f, \"ns_per_tile_b2b\": %.4f}\n",
         name, W, tiles, WPB, ms[ms.size() / 2], bb / 30, bb / 30 * 1e6 / tiles);
  CK(hipEventDestroy(e0));
  CK(hipEventDestroy(e1));
  return 0;
}

int main() {
  const int Wmax = 2048;
  const int tiles_max = (Wmax / 8) * (Wmax / 8);
  float4* tf;
  int* order;
  uint2* out;
  CK(hipMalloc(&tf, 256 * sizeof(float4)));
  CK(hipMemset(tf, 0, 256 * sizeof(float4)));
  CK(hipMalloc(&order, tiles_max * sizeof(int)));
  CK(hipMalloc(&out, (size_t)Wmax * Wmax * sizeof(uint2)));
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  for (int W : {1024, 2048}) {
    const int tiles = (W / 8) * (W / 8);
    std::vector<int> h(tiles);
    for (int i = 0; i < tiles; i++) h[i] = (int)(((long long)i * 7919) % tiles);   // a permutation
    CK(hipMemcpy(order, h.data(), tiles * sizeof(int), hipMemcpyHostToDevice));
    if (run<0, 1>("empty", W, tf, order, out, s)) return 1;
    if (run<ARGS, 1>("args", W, tf, order, out, s)) return 1;
    if (run<STORE, 1>("store", W, tf, order, out, s)) return 1;
    if (run<STORE | ORDER, 1>("store+order", W, tf, order, out, s)) return 1;
    if (run<STORE | ORDER | TF, 1>("store+order+tf", W, tf, order, out, s)) return 1;
    if (run<STORE | ORDER | TF | SETUP, 1>("store+order+tf+setup", W, tf, order, out, s)) return 1;
    if (run<STORE | ORDER | TF | SETUP | ARGS, 1>("all", W, tf, order, out, s)) return 1;
    if (run<STORE | ORDER | SETUP | ARGS, 1>("all-but-tf", W, tf, order, out, s)) return 1;
    if (run<STORE | ORDER | TF | SETUP | ARGS, 2>("all", W, tf, order, out, s)) return 1;
    if (run<STORE | ORDER | TF | SETUP | ARGS, 4>("all", W, tf, order, out, s)) return 1;
  }
  CK(hipDeviceSynchronize());
  return 0;
}
