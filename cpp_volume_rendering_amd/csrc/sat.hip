// sat.hip — the extinction summed-area table of the EBS renderer on gfx950.
//
// RC1PExtinctionBasedShading::GenerateExtinctionSAT3DTex (ebsrenderer.cpp:
// 624-716) fills a (W+2)(H+2)(D+2) grid, zero on its border, with the voxel
// extinctions and runs SummedAreaTable3D<double>::BuildSAT (summedareatable.h:
// 218-278) serially on the CPU.  Its interior step
//     S(x,y,z) = V + S(x-1,y-1,z-1) + S(x,y,z-1) + S(x,y-1,z) + S(x-1,y,z)
//                  - S(x-1,y-1,z) - S(x,y-1,z-1) - S(x-1,y,z-1)
// (double, left to right) depends only on the seven lower neighbours, and the
// lower planes x=0 / y=0 / z=0 are all zero.  Any order that evaluates a cell
// after those seven reproduces every double bit for bit, so:
//   * the (x, y) plane is cut into 8x8 column tiles, one wave each; tiles on one
//     anti-diagonal tx + ty = k are independent (one launch per k);
//   * inside a tile, lane (lx, ly) owns a column and visits z at time
//     t = z - 1 + lx + ly (a skewed pipeline): its left / upper / diagonal
//     neighbours reached the same z one or two steps earlier, so their values
//     come by cross-lane shuffles of a 3-deep history, no barrier per step;
//   * the tile's left face, upper face and corner column (finished by earlier
//     launches) and its voxel extinctions are staged in LDS 64 steps at a time.
// Only the tile's last row / column is kept in double (what later tiles read);
// every cell is stored as float, the texture the shader samples (GL_R32F).
#include <hip/hip_runtime.h>
#include <cstdint>

#include "cvr_internal.h"

namespace cvr {

namespace {

constexpr int kSatCh = 64;                    // steps per staging chunk
constexpr int kSatSkew = 14;                  // max lx + ly
constexpr int kSatBnd = kSatCh + kSatSkew + 1;  // boundary window (z and z - 1)
constexpr int kSatVal = kSatCh + kSatSkew;    // voxel window

struct SatArgs {
  int W, H, D;          // volume
  int w, h, d;          // SAT grid (W+2, H+2, D+2)
  int TY, k;            // tile rows; this launch's anti-diagonal
  int bpv;
  const void* vox;
  const float* lut;     // extinction per voxel value
  double* sd;           // double values of the tiles' last row / column
  float* sf;            // the float SAT
};

template <int BPV>
__global__ void __launch_bounds__(64) sat_tile_kernel(SatArgs P) {
  __shared__ double bnd[17][kSatBnd];   // left face (8), upper face (8), corner
  __shared__ float val[kSatVal][64];    // V(x, y, z) of the tile's columns
  const int lane = threadIdx.x, lx = lane & 7, ly = lane >> 3;
  const int tx = max(0, P.k - (P.TY - 1)) + (int)blockIdx.x, ty = P.k - tx;
  const int x0 = 1 + 8 * tx, y0 = 1 + 8 * ty;
  const int x = x0 + lx, y = y0 + ly;
  const bool in_xy = x <= P.w - 1 && y <= P.h - 1;
  const long long sy = P.w, sz = (long long)P.w * P.h;
  const int nsteps = P.d + kSatSkew - 1;   // lane with skew 14 reaches z = d - 1
  const bool keep = (lx == 7 || ly == 7);  // read back by the next tiles
  double h0 = 0.0, h1 = 0.0, h2 = 0.0;     // own column at z-1, z-2, z-3
  for (int t0 = 0; t0 < nsteps; t0 += kSatCh) {
    __syncthreads();
    // boundary columns, z in [t0 - 14, t0 + 64]
    for (int i = lane; i < 17 * kSatBnd; i += 64) {
      const int col = i / kSatBnd, zi = i - col * kSatBnd, z = t0 - kSatSkew + zi;
      const int cx = col < 8 ? x0 - 1 : (col < 16 ? x0 + col - 8 : x0 - 1);
      const int cy = col < 8 ? y0 + col : y0 - 1;
      double v = 0.0;
      if (z >= 1 && z <= P.d - 1 && cx >= 1 && cy >= 1 && cx <= P.w - 1 && cy <= P.h - 1)
        v = P.sd[cx + cy * sy + z * sz];
      bnd[col][zi] = v;
    }
    // voxel extinctions of the tile's columns, z in [t0 - 13, t0 + 64]
    for (int zi = 0; zi < kSatVal; zi++) {
      const int z = t0 - (kSatSkew - 1) + zi;
      float v = 0.0f;
      if (in_xy && z >= 1 && z <= P.D && x <= P.W && y <= P.H) {
        const long long i = (long long)(x - 1) + (long long)(y - 1) * P.W +
                            (long long)(z - 1) * P.W * P.H;
        const uint32_t q = BPV == 1 ? ((const uint8_t*)P.vox)[i] : ((const uint16_t*)P.vox)[i];
        v = P.lut[q];
      }
      val[zi][lane] = v;
    }
    __syncthreads();
    const int tend = min(t0 + kSatCh, nsteps);
    for (int t = t0; t < tend; t++) {
      const int z = 1 + t - (lx + ly);
      double L0 = __shfl(h0, lane - 1, 64), L1 = __shfl(h1, lane - 1, 64);
      double T0 = __shfl(h0, lane - 8, 64), T1 = __shfl(h1, lane - 8, 64);
      double D1 = __shfl(h1, lane - 9, 64), D2 = __shfl(h2, lane - 9, 64);
      double nh = 0.0;
      if (in_xy && z >= 1 && z <= P.d - 1) {
        const int zb = z - (t0 - kSatSkew);
        if (lx == 0) { L0 = bnd[ly][zb]; L1 = bnd[ly][zb - 1]; }
        if (ly == 0) { T0 = bnd[8 + lx][zb]; T1 = bnd[8 + lx][zb - 1]; }
        if (lx == 0 && ly == 0) { D1 = bnd[16][zb]; D2 = bnd[16][zb - 1]; }
        else if (lx == 0) { D1 = bnd[ly - 1][zb]; D2 = bnd[ly - 1][zb - 1]; }
        else if (ly == 0) { D1 = bnd[8 + lx - 1][zb]; D2 = bnd[8 + lx - 1][zb - 1]; }
        const double v = (double)val[z - (t0 - (kSatSkew - 1))][lane];
        const double s = v + D2 + h0 + T0 + L0 - D1 - T1 - L1;
        const long long o = x + y * sy + z * sz;
        P.sf[o] = (float)s;
        if (keep) P.sd[o] = s;
        nh = s;
      }
      h2 = h1;
      h1 = h0;
      h0 = nh;
    }
  }
}

// The shader's fetch layout: texel (i, j, k) holds its 8 trilinear corners
// (i|i+1, j|j+1, k|k+1, the +1 clamped to the edge) as two float4, so one
// GL_LINEAR fetch of the SAT is two dwordx4 loads from one 32-byte run.
__global__ void sat_cells_kernel(const float* __restrict__ sf, float4* __restrict__ cells, int w,
                                 int h, int d) {
  const long long n = (long long)w * h * d;
  const long long v = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (v >= n) return;
  const int i = (int)(v % w), j = (int)((v / w) % h), k = (int)(v / ((long long)w * h));
  const int i1 = min(i + 1, w - 1), j1 = min(j + 1, h - 1), k1 = min(k + 1, d - 1);
  const long long sy = w, sz = (long long)w * h;
  auto at = [&](int x, int y, int z) { return sf[z * sz + y * sy + x]; };
  cells[2 * v] = make_float4(at(i, j, k), at(i1, j, k), at(i, j1, k), at(i1, j1, k));
  cells[2 * v + 1] = make_float4(at(i, j, k1), at(i1, j, k1), at(i, j1, k1), at(i1, j1, k1));
}

}  // namespace

hipError_t launch_sat_cells(const Ctx& c, const float* d_sf, float4* d_cells, hipStream_t s) {
  const int w = c.N[0] + 2, h = c.N[1] + 2, d = c.N[2] + 2;
  const long long n = (long long)w * h * d;
  hipLaunchKernelGGL(sat_cells_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, d_sf,
                     d_cells, w, h, d);
  return hipGetLastError();
}

hipError_t launch_sat_build(const Ctx& c, const float* d_lut, double* d_sd, float* d_sf,
                            hipStream_t s) {
  SatArgs P{};
  P.W = c.N[0]; P.H = c.N[1]; P.D = c.N[2];
  P.w = P.W + 2; P.h = P.H + 2; P.d = P.D + 2;
  P.bpv = c.bpv;
  P.vox = c.d_vox;
  P.lut = d_lut;
  P.sd = d_sd;
  P.sf = d_sf;
  const int TX = (P.w - 1 + 7) / 8;   // columns x in [1, w-1] (the far border plane included)
  const int TY = (P.h - 1 + 7) / 8;
  P.TY = TY;
  hipError_t e = hipMemsetAsync(d_sf, 0, (size_t)P.w * P.h * P.d * sizeof(float), s);
  if (e != hipSuccess) return e;
  for (int k = 0; k <= TX + TY - 2; k++) {
    P.k = k;
    const int lo = k - (TY - 1) > 0 ? k - (TY - 1) : 0;
    const int hi = k < TX - 1 ? k : TX - 1;
    const int n = hi - lo + 1;
    if (n <= 0) continue;
    if (c.bpv == 1)
      hipLaunchKernelGGL(sat_tile_kernel<1>, dim3(n), dim3(64), 0, s, P);
    else
      hipLaunchKernelGGL(sat_tile_kernel<2>, dim3(n), dim3(64), 0, s, P);
    e = hipGetLastError();
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}

}  // namespace cvr
