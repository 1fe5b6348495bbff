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
//   * the z axis is cut into chunks; work item (tile, chunk) depends only on
//     the left / upper / diagonal tiles' same chunk and on its own previous
//     chunk, so items with tx + ty + chunk = k are independent: one launch per k
//     (critical path ~ (tiles along x + along y + chunks) x chunk length instead
//     of tiles x depth);
//   * inside an item, lane (lx, ly) owns a column and visits z at time
//     t = z - z0 + lx + ly (a skewed pipeline): its left / upper / diagonal
//     neighbours reached the same z one or two steps earlier, so their values
//     come by cross-lane shuffles of a 3-deep history, no barrier per step;
//   * the tile's left face, upper face and corner column (finished by earlier
//     launches), its own column below the chunk, and its voxel extinctions are
//     staged in LDS / registers when the item starts.
// Double values are kept for what later items read (the tiles' last row /
// column, the chunks' last two planes); every cell is stored as float, the
// texture the shader samples (GL_R32F).
#include <hip/hip_runtime.h>
#include <cstdint>

#include "cvr_internal.h"

namespace cvr {

namespace {

constexpr int kSatChMax = 64;                 // largest z chunk
constexpr int kSatSkew = 14;                  // max lx + ly

struct SatArgs {
  int W, H, D;          // volume
  int w, h, d;          // SAT grid (W+2, H+2, D+2)
  int TX, TY, NC, C;    // tiles along x / y, z chunks of C planes
  int k;                // this launch's anti-diagonal tx + ty + chunk
  int bpv;
  const void* vox;
  const float* lut;     // extinction per voxel value
  double* sd;           // double values read back by later items
  float* sf;            // the float SAT
};

template <int BPV>
__global__ void __launch_bounds__(64) sat_tile_kernel(SatArgs P) {
  __shared__ double bnd[17][kSatChMax + 1];   // left face (8), upper face (8), corner; z0-1 .. z1
  __shared__ float val[kSatChMax][64];        // V(x, y, z) of the tile's columns, z0 .. z1
  const int tx = (int)blockIdx.x % P.TX, cz = (int)blockIdx.x / P.TX;
  const int ty = P.k - tx - cz;
  if (ty < 0 || ty >= P.TY) return;           // not on this anti-diagonal (whole wave)
  const int lane = threadIdx.x, lx = lane & 7, ly = lane >> 3;
  const int x0 = 1 + 8 * tx, y0 = 1 + 8 * ty;
  const int x = x0 + lx, y = y0 + ly;
  const int z0 = 1 + cz * P.C, z1 = min(z0 + P.C - 1, P.d - 1);
  const int nz = z1 - z0 + 1;
  const bool in_xy = x <= P.w - 1 && y <= P.h - 1;
  const long long sy = P.w, sz = (long long)P.w * P.h;
  // the own column below the chunk (z0 - 1, z0 - 2): the history's start
  double h0 = 0.0, h1 = 0.0, h2 = 0.0;
  if (in_xy) {
    if (z0 - 1 >= 1) h0 = P.sd[x + y * sy + (z0 - 1) * sz];
    if (z0 - 2 >= 1) h1 = P.sd[x + y * sy + (z0 - 2) * sz];
  }
  // boundary columns, z in [z0 - 1, z1]
  for (int i = lane; i < 17 * (nz + 1); i += 64) {
    const int col = i / (nz + 1), zi = i - col * (nz + 1), z = z0 - 1 + zi;
    const int cx = col < 8 ? x0 - 1 : (col < 16 ? x0 + col - 8 : x0 - 1);
    const int cy = col < 8 ? y0 + col : y0 - 1;
    double v = 0.0;
    if (z >= 1 && cx >= 1 && cy >= 1 && cx <= P.w - 1 && cy <= P.h - 1)
      v = P.sd[cx + cy * sy + z * sz];
    bnd[col][zi] = v;
  }
  // voxel extinctions of the tile's columns, z in [z0, z1]
  for (int zi = 0; zi < nz; zi++) {
    const int z = z0 + zi;
    float v = 0.0f;
    if (in_xy && z <= P.D && x <= P.W && y <= P.H) {
      const long long i = (long long)(x - 1) + (long long)(y - 1) * P.W +
                          (long long)(z - 1) * P.W * P.H;
      const uint32_t q = BPV == 1 ? ((const uint8_t*)P.vox)[i] : ((const uint16_t*)P.vox)[i];
      v = P.lut[q];
    }
    val[zi][lane] = v;
  }
  __syncthreads();
  const bool keep_col = (lx == 7 || ly == 7);   // read by the next tiles (all z)
  const int nsteps = nz + kSatSkew;
  for (int t = 0; t < nsteps; t++) {
    const int z = z0 + t - (lx + ly);
    double L0 = __shfl(h0, lane - 1, 64), L1 = __shfl(h1, lane - 1, 64);
    double T0 = __shfl(h0, lane - 8, 64), T1 = __shfl(h1, lane - 8, 64);
    double D1 = __shfl(h1, lane - 9, 64), D2 = __shfl(h2, lane - 9, 64);
    double nh;
    if (in_xy && z >= z0 && z <= z1) {
      const int zb = z - (z0 - 1);
      if (lx == 0) { L0 = bnd[ly][zb]; L1 = bnd[ly][zb - 1]; }
      if (ly == 0) { T0 = bnd[8 + lx][zb]; T1 = bnd[8 + lx][zb - 1]; }
      if (lx == 0 && ly == 0) { D1 = bnd[16][zb]; D2 = bnd[16][zb - 1]; }
      else if (lx == 0) { D1 = bnd[ly - 1][zb]; D2 = bnd[ly - 1][zb - 1]; }
      else if (ly == 0) { D1 = bnd[8 + lx - 1][zb]; D2 = bnd[8 + lx - 1][zb - 1]; }
      const double v = (double)val[z - z0][lane];
      const double s = v + D2 + h0 + T0 + L0 - D1 - T1 - L1;
      const long long o = x + y * sy + z * sz;
      P.sf[o] = (float)s;
      if (keep_col || z >= z1 - 1) P.sd[o] = s;
      nh = s;
    } else {
      // before its first z the lane's history is the column below the chunk
      // (already in h0, h1); after its last z nothing reads it
      nh = z < z0 ? h0 : 0.0;
    }
    if (z >= z0 || !in_xy) {
      h2 = h1;
      h1 = h0;
      h0 = nh;
    }
  }
}

// The shader's fetch layout ("cell4"): texel (i, j, k) holds the 4 corners of
// its plane (i|i+1, j|j+1, the +1 clamped to the edge) as one float4, and one
// extra plane k = d repeats plane d - 1 (the clamped k + 1).  A GL_LINEAR fetch
// of the SAT is then two dwordx4 loads, texel (i, j, k) and the texel one plane
// above.  The earlier cell8 form (all 8 corners per texel, one 32-B run) made
// the same two loads at twice the footprint: cell4 halves the L2 working set of
// the shadow chains, 80.5 -> 73.5 ms per 1024^3 frame and 42.5 -> 36.5 ms per
// SAT build (profiles/r03_s29_*).
__global__ void sat_cells_kernel(const float* __restrict__ sf, float4* __restrict__ cells, int w,
                                 int h, int d) {
  const long long n = (long long)w * h * (d + 1);
  const long long v = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (v >= n) return;
  const int i = (int)(v % w), j = (int)((v / w) % h), k = min((int)(v / ((long long)w * h)), d - 1);
  const int i1 = min(i + 1, w - 1), j1 = min(j + 1, h - 1);
  const long long sy = w, sz = (long long)w * h;
  auto at = [&](int x, int y, int z) { return sf[z * sz + y * sy + x]; };
  cells[v] = make_float4(at(i, j, k), at(i1, j, k), at(i, j1, k), at(i1, j1, k));
}

}  // namespace

size_t sat_cells_float4s(int w, int h, int d) { return (size_t)w * h * (d + 1); }

hipError_t launch_sat_cells(const Ctx& c, const float* d_sf, float4* d_cells, hipStream_t s) {
  const int w = c.N[0] + 2, h = c.N[1] + 2, d = c.N[2] + 2;
  const long long n = (long long)w * h * (d + 1);
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
  P.TX = (P.w - 1 + 7) / 8;   // columns x in [1, w-1] (the far border plane included)
  P.TY = (P.h - 1 + 7) / 8;
  P.C = c.sat_chunk > 0 && c.sat_chunk <= kSatChMax ? c.sat_chunk : 32;
  P.NC = (P.d - 1 + P.C - 1) / P.C;   // planes z in [1, d-1]
  hipError_t e = hipMemsetAsync(d_sf, 0, (size_t)P.w * P.h * P.d * sizeof(float), s);
  if (e != hipSuccess) return e;
  const unsigned grid = (unsigned)(P.TX * P.NC);
  for (int k = 0; k <= P.TX + P.TY + P.NC - 3; k++) {
    P.k = k;
    if (c.bpv == 1)
      hipLaunchKernelGGL(sat_tile_kernel<1>, dim3(grid), dim3(64), 0, s, P);
    else
      hipLaunchKernelGGL(sat_tile_kernel<2>, dim3(grid), dim3(64), 0, s, P);
    e = hipGetLastError();
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}

}  // namespace cvr
