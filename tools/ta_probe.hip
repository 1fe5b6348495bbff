// ta_probe.hip — cost of one 16-B-per-lane wave-load (buffer_load_dwordx4) on
// gfx950 as a function of how its 64 addresses fall into 128-B lines, and of
// where the lines are served from.  Not product code: it sets the cost model
// behind the rc1pass cell layout ("what a wave-load costs").
//
// Every wave issues R rounds of U = 8 independent loads with almost no VALU, so
// the vector-memory pipe is the only busy unit.  Within one load, lane i reads
// (patterns; line = 128 B, slot = 16 B):
//   rr L   : line i % L, slot (i / L) % 8        (consecutive lanes, different lines)
//   blk L  : line i * L / 64, slot i % 8         (consecutive lanes share lines)
//   cells F: cell i * F / 64 of F distinct cells laid out 4 to a line (64 B used
//            per line; neighbouring lanes share a cell, as neighbouring rays do)
// Regimes (where the lines come from):
//   l1  : the same 64 KiB every round (L1/L2 resident)
//   l2  : each wave walks its own window of a 2 MiB table (L2 resident, L1 misses)
//   hbm : each wave walks its own window of a 2 GiB table (every line new)
// Output: one JSON line per (regime, pattern): ns per wave-load per CU and the
// cycles at 2.4 GHz.
//
//   hipcc --offload-arch=gfx950 -O3 -o tools/ta_probe tools/ta_probe.hip
//   ./tools/ta_probe [regime]
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstring>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { \
  fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); return 1; } } while (0)

constexpr int kU = 8;        // loads in flight per wave

__global__ void __launch_bounds__(256) probe(const uint4* __restrict__ tab, uint32_t tab_bytes,
                                             const uint32_t* __restrict__ offs, int rounds,
                                             uint32_t adv, uint32_t wave_stride, uint32_t mask,
                                             uint32_t* __restrict__ sink) {
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void*)tab, 0, (int)tab_bytes, 0x00020000);
  const int lane = threadIdx.x & 63;
  const uint32_t wave = blockIdx.x * 4 + (threadIdx.x >> 6);
  uint32_t off[kU];
#pragma unroll
  for (int u = 0; u < kU; u++) off[u] = offs[u * 64 + lane];
  uint32_t base = wave * wave_stride;
  uint32_t acc = 0;
  for (int r = 0; r < rounds; r++) {
    typedef unsigned int u4v __attribute__((ext_vector_type(4)));
    u4v v[kU];
#pragma unroll
    for (int u = 0; u < kU; u++) v[u] = __builtin_amdgcn_raw_buffer_load_b128(rs, (int)((base + off[u]) & mask), 0, 0);
#pragma unroll
    for (int u = 0; u < kU; u++) acc ^= v[u].x ^ v[u].w;
    base += adv;
  }
  if (acc == 0x12345678u) sink[blockIdx.x & 1023] = acc;
}

int main(int argc, char** argv) {
  hipDeviceProp_t prop;
  CK(hipGetDeviceProperties(&prop, 0));
  const int cus = prop.multiProcessorCount;
  const char* only = argc > 1 ? argv[1] : nullptr;
  const size_t big = size_t(2) << 30;
  uint4* tab; uint32_t* offs; uint32_t* sink;
  CK(hipMalloc(&tab, big));
  CK(hipMemset(tab, 1, big));
  CK(hipMalloc(&offs, kU * 64 * 4));
  CK(hipMalloc(&sink, 4096));
  const int waves_per_cu = 16, blocks = cus * waves_per_cu / 4;
  const int nwaves = blocks * 4;
  struct Pat { const char* name; int L; int kind; };
  std::vector<Pat> pats;
  for (int L : {1, 4, 8, 16, 32, 64}) pats.push_back({"rr", L, 0});
  for (int L : {1, 2, 4, 8, 16, 32, 64}) pats.push_back({"blk", L, 1});
  for (int F : {8, 16, 24, 32, 48, 64}) pats.push_back({"cells", F, 2});
  struct Reg { const char* name; uint32_t tab; uint32_t adv; uint32_t wstride; int rounds; };
  // l1: 8 loads x 8 KiB slices of one 64 KiB table, every round the same lines
  // l2: 2 MiB table, each wave starts at its own 8 KiB-aligned spot and advances 64 KiB a round
  // hbm: 2 GiB table, each wave its own 8 MiB window, advancing 64 KiB a round
  const Reg regs[] = {{"l1", 64u << 10, 0u, 0u, 4096},
                      {"l2", 2u << 20, 64u << 10, 8u << 10, 2048},
                      {"hbm", 0x80000000u, 64u << 10, 0u, 64}};
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  for (const Reg& g : regs) {
    if (only && strcmp(only, g.name)) continue;
    const uint32_t wstride = g.wstride ? g.wstride : (uint32_t)(big / nwaves) & ~0xffffu;
    for (const Pat& p : pats) {
      std::vector<uint32_t> h(kU * 64);
      for (int u = 0; u < kU; u++) {
        const uint32_t base = (uint32_t)u * 8192u;   // each load its own 8 KiB slice
        for (int i = 0; i < 64; i++) {
          uint32_t line = 0, slot = 0;
          if (p.kind == 0) { line = i % p.L; slot = (i / p.L) % 8; }
          else if (p.kind == 1) { line = i * p.L / 64; slot = i % 8; }
          else { const int c = i * p.L / 64; line = c / 4; slot = c % 4; }
          h[u * 64 + i] = base + line * 128u + slot * 16u;
        }
      }
      CK(hipMemcpy(offs, h.data(), h.size() * 4, hipMemcpyHostToDevice));
      const uint32_t mask = g.tab - 1;
      float ms = 0;
      for (int rep = 0; rep < 3; rep++) {   // the first two warm the clocks
        CK(hipEventRecord(e0));
        hipLaunchKernelGGL(probe, dim3(blocks), dim3(256), 0, 0, tab, g.tab, offs, g.rounds, g.adv,
                           wstride, mask, sink);
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        CK(hipEventElapsedTime(&ms, e0, e1));
      }
      const double wave_loads_per_cu = (double)waves_per_cu * g.rounds * kU;
      const double ns = ms * 1e6 / wave_loads_per_cu;
      const double bytes = (double)nwaves * g.rounds * kU * 1024.0;
      printf("{\"regime\": \"%s\", \"pattern\": \"%s\", \"param\": %d, \"ms\": %.4f, "
             "\"ns_per_wave_load_per_cu\": %.4f, \"cycles_at_2.4GHz\": %.2f, \"lane_TB_s\": %.2f}\n",
             g.name, p.name, p.L, ms, ns, ns * 2.4, bytes / (ms * 1e-3) / 1e12);
      fflush(stdout);
    }
  }
  return 0;
}
