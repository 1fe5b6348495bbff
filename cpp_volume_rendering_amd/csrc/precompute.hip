// precompute.hip — one-time device precompute of the ray-caster's inputs:
// the padded cell8 volume layout (GL_R16F semantics), the gradient
// volume (finite differences / Sobel-Feldman, RGB16F), and the rank-0 tile
// unpack of the screen-tile split.
#include <hip/hip_runtime.h>
#include <hip/hip_fp16.h>
#include <cstdint>
#include <utility>

#include "cvr_device.h"
#include "cvr_internal.h"
#include "march_common.h"

namespace cvr {

// Build the padded cell8 layout (x-fastest (N+1)^3 cells) from raw voxels using the host-made
// value table lut[v] = half(float(v / 255.0)) (GL_R16F upload of
// GetNormalizedSample, utils.cpp:20-56).
template <typename VT>
__global__ void build_cells_kernel(const VT* __restrict__ vox, const uint16_t* __restrict__ lut,
                                   int nx, int ny, int nz, CellGrid g, uint4* __restrict__ cells,
                                   size_t ncells) {
  size_t idx = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= ncells) return;
  uint32_t i = (uint32_t)idx;
  const int a = (int)(i % (uint32_t)g.cx);
  const uint32_t rest = i / (uint32_t)g.cx;
  const int b = (int)(rest % (uint32_t)g.cy);
  const int c = (int)(rest / (uint32_t)g.cy);
  uint4 r = make_uint4(0, 0, 0, 0);
  if (a < g.cx && b < g.cy && c < g.cz) {
    int x0 = max(a - 1, 0), x1 = min(a, nx - 1);
    int y0 = max(b - 1, 0), y1 = min(b, ny - 1);
    int z0 = max(c - 1, 0), z1 = min(c, nz - 1);
    auto q = [&](int x, int y, int z) -> uint32_t {
      return lut[vox[(size_t)x + (size_t)y * nx + (size_t)z * nx * ny]];
    };
    r.x = q(x0, y0, z0) | (q(x1, y0, z0) << 16);
    r.y = q(x0, y1, z0) | (q(x1, y1, z0) << 16);
    r.z = q(x0, y0, z1) | (q(x1, y0, z1) << 16);
    r.w = q(x0, y1, z1) | (q(x1, y1, z1) << 16);
  }
  cells[idx] = r;
}

hipError_t launch_build_cells_impl(const void* vox, int bpv, const uint16_t* lut, const int N[3],
                                   const CellGrid& g, void* cells, hipStream_t s) {
  size_t n = cell_count(g);
  int bs = 256;
  size_t nb = (n + bs - 1) / bs;
  if (bpv == 1)
    hipLaunchKernelGGL(build_cells_kernel<uint8_t>, dim3((unsigned)nb), dim3(bs), 0, s,
                       (const uint8_t*)vox, lut, N[0], N[1], N[2], g, (uint4*)cells, n);
  else
    hipLaunchKernelGGL(build_cells_kernel<uint16_t>, dim3((unsigned)nb), dim3(bs), 0, s,
                       (const uint16_t*)vox, lut, N[0], N[1], N[2], g, (uint4*)cells, n);
  return hipGetLastError();
}

// GetNormalizedSample in double (structuredgridvolume.cpp:121-151), 0 outside.
template <typename VT>
__device__ __forceinline__ double norm_sample(const VT* vox, int nx, int ny, int nz, int x, int y,
                                              int z, double inv_max) {
  if (x < 0 || y < 0 || z < 0 || x >= nx || y >= ny || z >= nz) return 0.0;
  return (double)vox[(size_t)x + (size_t)y * nx + (size_t)z * nx * ny] / inv_max;
}

__device__ __forceinline__ uint32_t f2h_bits(float f) { return f32_to_h16(f); }

// GenerateGradientTexture (utils.cpp:146-190) with its defaults, and
// GenerateSobelFeldmanGradientTexture (utils.cpp:287-333); stored RGB16F.
template <typename VT>
__global__ void gradient_kernel(const VT* __restrict__ vox, int nx, int ny, int nz, int mode,
                                double maxv, uint2* __restrict__ grad) {
  size_t idx = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  size_t n = (size_t)nx * ny * nz;
  if (idx >= n) return;
  int x = (int)(idx % (size_t)nx);
  size_t r = idx / (size_t)nx;
  int y = (int)(r % (size_t)ny), z = (int)(r / (size_t)ny);
  double gx = 0, gy = 0, gz = 0;
  if (mode == CVR_GRADIENT_FINITE_DIFFERENCES) {
    gx = norm_sample(vox, nx, ny, nz, x + 1, y, z, maxv) - norm_sample(vox, nx, ny, nz, x - 1, y, z, maxv);
    gy = norm_sample(vox, nx, ny, nz, x, y + 1, z, maxv) - norm_sample(vox, nx, ny, nz, x, y - 1, z, maxv);
    gz = norm_sample(vox, nx, ny, nz, x, y, z + 1, maxv) - norm_sample(vox, nx, ny, nz, x, y, z - 1, maxv);
    double sqr = gx * gx + gy * gy + gz * gz;
    double inv = 1.0 / sqrt(sqr);
    gx *= inv; gy *= inv; gz *= inv;
    if (gx != gx) { gx = 0.0; gy = 0.0; gz = 0.0; }
  } else {
    for (int v1 = -1; v1 <= 1; v1++)
      for (int v2 = -1; v2 <= 1; v2++) {
        int m = abs(v1) + abs(v2);
        double wgt = m == 0 ? 1.0 : (m == 1 ? 2.0 : 4.0);   // pow(2, |v1|+|v2|)
        gz += norm_sample(vox, nx, ny, nz, x + v1, y + v2, z - 1, maxv) * (4.0 / wgt)
            + norm_sample(vox, nx, ny, nz, x + v1, y + v2, z + 1, maxv) * (-4.0 / wgt);
        gy += norm_sample(vox, nx, ny, nz, x + v1, y - 1, z + v2, maxv) * (4.0 / wgt)
            + norm_sample(vox, nx, ny, nz, x + v1, y + 1, z + v2, maxv) * (-4.0 / wgt);
        gx += norm_sample(vox, nx, ny, nz, x - 1, y + v2, z + v1, maxv) * (4.0 / wgt)
            + norm_sample(vox, nx, ny, nz, x + 1, y + v2, z + v1, maxv) * (-4.0 / wgt);
      }
  }
  uint2 o;
  o.x = f2h_bits((float)gx) | (f2h_bits((float)gy) << 16);
  o.y = f2h_bits((float)gz);
  grad[idx] = o;
}

// The gradient in the volume's cell8 grid: cell i holds, per component, the 8
// corners the trilinear fetch of cell i reads (same convention as
// build_cells_kernel), as three uint4 of packed fp16 pairs (x, y, z).  One
// shaded sample reads 48 contiguous bytes at the volume cell's index.
__global__ void gradient_cells_kernel(const uint2* __restrict__ grad, int nx, int ny, int nz,
                                      CellGrid g, uint4* __restrict__ gcells, size_t ncells) {
  size_t idx = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= ncells) return;
  uint32_t i = (uint32_t)idx;
  const int a = (int)(i % (uint32_t)g.cx);
  const uint32_t rest = i / (uint32_t)g.cx;
  const int b = (int)(rest % (uint32_t)g.cy);
  const int c = (int)(rest / (uint32_t)g.cy);
  const int x0 = max(a - 1, 0), x1 = min(a, nx - 1);
  const int y0 = max(b - 1, 0), y1 = min(b, ny - 1);
  const int z0 = max(c - 1, 0), z1 = min(c, nz - 1);
  auto q = [&](int x, int y, int z) { return grad[(size_t)x + (size_t)y * nx + (size_t)z * nx * ny]; };
  const uint2 g000 = q(x0, y0, z0), g100 = q(x1, y0, z0), g010 = q(x0, y1, z0), g110 = q(x1, y1, z0);
  const uint2 g001 = q(x0, y0, z1), g101 = q(x1, y0, z1), g011 = q(x0, y1, z1), g111 = q(x1, y1, z1);
  auto lo = [](uint32_t w) { return w & 0xffffu; };
  auto hi = [](uint32_t w) { return w >> 16; };
  // component x: low half of .x; y: high half of .x; z: low half of .y
  gcells[3 * idx + 0] = make_uint4(lo(g000.x) | (lo(g100.x) << 16), lo(g010.x) | (lo(g110.x) << 16),
                                   lo(g001.x) | (lo(g101.x) << 16), lo(g011.x) | (lo(g111.x) << 16));
  gcells[3 * idx + 1] = make_uint4(hi(g000.x) | (hi(g100.x) << 16), hi(g010.x) | (hi(g110.x) << 16),
                                   hi(g001.x) | (hi(g101.x) << 16), hi(g011.x) | (hi(g111.x) << 16));
  gcells[3 * idx + 2] = make_uint4(lo(g000.y) | (lo(g100.y) << 16), lo(g010.y) | (lo(g110.y) << 16),
                                   lo(g001.y) | (lo(g101.y) << 16), lo(g011.y) | (lo(g111.y) << 16));
}

// Per-voxel gradient (RGB16F + pad) into `tmp`, then its cell8 form into c.d_grad.
hipError_t launch_gradient(const Ctx& c, int mode, uint2* tmp, hipStream_t s) {
  size_t n = (size_t)c.N[0] * c.N[1] * c.N[2];
  int bs = 256;
  size_t nb = (n + bs - 1) / bs;
  if (c.bpv == 1)
    hipLaunchKernelGGL(gradient_kernel<uint8_t>, dim3((unsigned)nb), dim3(bs), 0, s,
                       (const uint8_t*)c.d_vox, c.N[0], c.N[1], c.N[2], mode, 255.0, tmp);
  else
    hipLaunchKernelGGL(gradient_kernel<uint16_t>, dim3((unsigned)nb), dim3(bs), 0, s,
                       (const uint16_t*)c.d_vox, c.N[0], c.N[1], c.N[2], mode, 65535.0, tmp);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  const size_t nc = cell_count(c.cells);
  hipLaunchKernelGGL(gradient_cells_kernel, dim3((unsigned)((nc + 255) / 256)), dim3(256), 0, s, tmp,
                     c.N[0], c.N[1], c.N[2], c.cells, (uint4*)c.d_grad, nc);
  return hipGetLastError();
}

// Scatter packed per-rank tiles (screen-tile split) into the W x H image.
// PX = float4 (RGBA32F) or uint2 (RGBA16F): pixels are moved, not converted.
// Rank r's k-th tile sits at tile slot r * rank_stride + k of `packed` (rank_stride
// = tpr_max for one frame per exchange; nframes * tpr_max when several frames
// travel together and `packed` points at frame j's first slot).
// One workgroup per tile slot: the slot's rank, index and screen position are
// worked out once (wave-uniform 32-bit math; round 3 did it per pixel with 64-bit
// divisions, ~10 us per 1024^2 frame), then 256 lanes copy the tile's pixels,
// coalesced on both sides (a 16-pixel row is 128 B of RGBA16F).
template <typename PX>
__global__ void __launch_bounds__(256)
unpack_tiles_kernel(const PX* __restrict__ packed, PX* __restrict__ out, int W, int H, int tile,
                    int nranks, int tpr_max, size_t rank_stride, int ntx) {
  const int slot = blockIdx.x;                       // rank * tpr_max + k
  const int r = slot / tpr_max, k = slot - r * tpr_max;
  int tx, ty;
  split_tile(r, nranks, k, ntx, tx, ty);
  if (ty * tile >= H) return;                        // a padding slot past the rank's tiles
  const PX* __restrict__ src = packed + ((size_t)r * rank_stride + k) * ((size_t)tile * tile);
  const int x0 = tx * tile, y0 = ty * tile;
  if (tile == 16 && sizeof(PX) == 8 && (W & 1) == 0) {
    // RGBA16F: 16 B (two pixels) per lane, 128 lanes per tile (a 16-pixel row = 8 lanes)
    const int t = threadIdx.x;
    if (t >= 128) return;
    const int px = x0 + ((t & 7) << 1), py = y0 + (t >> 3);
    if (py < H) {
      const uint4 v = reinterpret_cast<const uint4*>(src)[t];
      if (px + 1 < W)
        *reinterpret_cast<uint4*>(out + (size_t)py * W + px) = v;
      else if (px < W)
        *reinterpret_cast<uint2*>(out + (size_t)py * W + px) = make_uint2(v.x, v.y);
    }
    return;
  }
  if (tile == 16) {
    const int inner = threadIdx.x, px = x0 + (inner & 15), py = y0 + (inner >> 4);
    if (px < W && py < H) out[(size_t)py * W + px] = src[inner];
    return;
  }
  for (int inner = threadIdx.x; inner < tile * tile; inner += blockDim.x) {
    const int px = x0 + inner % tile, py = y0 + inner / tile;
    if (px < W && py < H) out[(size_t)py * W + px] = src[inner];
  }
}

// per-pixel sample counts (uint32) of packed tiles, for the single-process group
hipError_t launch_unpack_tiles_u32(const uint32_t* packed, uint32_t* out, int W, int H, int tile,
                                   int nranks, int tpr_max, hipStream_t s, size_t rank_stride) {
  const int ntx = (W + tile - 1) / tile;
  const long long nslots = (long long)nranks * tpr_max;
  if (nslots == 0) return hipSuccess;
  if (nslots > 0x7fffffffLL) return hipErrorInvalidValue;
  if (rank_stride == 0) rank_stride = (size_t)tpr_max;
  hipLaunchKernelGGL(unpack_tiles_kernel<uint32_t>, dim3((unsigned)nslots), dim3(256), 0, s, packed, out, W,
                     H, tile, nranks, tpr_max, rank_stride, ntx);
  return hipGetLastError();
}

hipError_t launch_unpack_tiles(const void* packed, void* out, int half, int W, int H, int tile,
                               int nranks, int tpr_max, hipStream_t s, size_t rank_stride) {
  int ntx = (W + tile - 1) / tile;
  const long long nslots = (long long)nranks * tpr_max;
  if (nslots == 0) return hipSuccess;
  if (nslots > 0x7fffffffLL) return hipErrorInvalidValue;
  if (rank_stride == 0) rank_stride = (size_t)tpr_max;
  if (half)
    hipLaunchKernelGGL(unpack_tiles_kernel<uint2>, dim3((unsigned)nslots), dim3(256), 0, s,
                       (const uint2*)packed, (uint2*)out, W, H, tile, nranks, tpr_max, rank_stride,
                       ntx);
  else
    hipLaunchKernelGGL(unpack_tiles_kernel<float4>, dim3((unsigned)nslots), dim3(256), 0, s,
                       (const float4*)packed, (float4*)out, W, H, tile, nranks, tpr_max,
                       rank_stride, ntx);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------
// Empty-space skipping: macro-cell value ranges and TF occupancy
// ---------------------------------------------------------------------------

// Raw-value range (max << 16 | min) of texels [m*w, m*w + w] (clamped) on every
// axis: the texels a trilinear sample whose floor lies in macro cell m reads.
template <typename VT>
__global__ void macro_minmax_kernel(const VT* __restrict__ vox, int nx, int ny, int nz, int shift,
                                    int mx, int my, int mz, uint32_t* __restrict__ out) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= mx * my * mz) return;
  const int cx = i % mx, cy = (i / mx) % my, cz = i / (mx * my);
  const int w = 1 << shift;
  const int x0 = cx * w, x1 = min(x0 + w, nx - 1);
  const int y0 = cy * w, y1 = min(y0 + w, ny - 1);
  const int z0 = cz * w, z1 = min(z0 + w, nz - 1);
  uint32_t lo = 0xffffu, hi = 0u;
  for (int z = z0; z <= z1; z++)
    for (int y = y0; y <= y1; y++) {
      const VT* row = vox + ((size_t)z * ny + y) * nx;
      for (int x = x0; x <= x1; x++) {
        const uint32_t v = row[x];
        lo = min(lo, v);
        hi = max(hi, v);
      }
    }
  out[i] = (hi << 16) | lo;
}

hipError_t launch_macro_minmax(const Ctx& c, int shift, const int mdim[3], uint32_t* out,
                               hipStream_t s) {
  const int n = mdim[0] * mdim[1] * mdim[2];
  const int bs = 128;
  if (c.bpv == 1)
    hipLaunchKernelGGL(macro_minmax_kernel<uint8_t>, dim3((n + bs - 1) / bs), dim3(bs), 0, s,
                       (const uint8_t*)c.d_vox, c.N[0], c.N[1], c.N[2], shift, mdim[0], mdim[1],
                       mdim[2], out);
  else
    hipLaunchKernelGGL(macro_minmax_kernel<uint16_t>, dim3((n + bs - 1) / bs), dim3(bs), 0, s,
                       (const uint16_t*)c.d_vox, c.N[0], c.N[1], c.N[2], shift, mdim[0], mdim[1],
                       mdim[2], out);
  return hipGetLastError();
}

// Occupancy byte of a macro cell for the current TF.  A density d reads the
// padded TF entries k = floor(fmaf(d, n, -0.5)) + 1 and k + 1 (classify in
// raymarch.hip); the alpha there is a lerp of those two, so it is <= 0 when
// both are.  The densities of the cell lie in [lut[min], lut[max]] (widened by
// 2^-10 against the rounding of the trilinear lerps); the cell is empty when
// no padded entry in the range has alpha > 0 (`prefix` counts them).
__global__ void occupancy_kernel(const uint32_t* __restrict__ minmax, int n_macro,
                                 const uint16_t* __restrict__ lut, const int* __restrict__ prefix,
                                 int tf_n, uint8_t* __restrict__ occ,
                                 unsigned int* __restrict__ n_empty) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n_macro) return;
  const uint32_t mm = minmax[i];
  const float lo = __half2float(__ushort_as_half(lut[mm & 0xffffu])) - 1.0f / 1024.0f;
  const float hi = __half2float(__ushort_as_half(lut[mm >> 16])) + 1.0f / 1024.0f;
  const float fn = (float)tf_n;
  int kl = (int)floorf(fmaf(lo, fn, -0.5f)) + 1;
  int kh = (int)floorf(fmaf(hi, fn, -0.5f)) + 2;
  kl = max(kl, 0);
  kh = min(kh, tf_n + 1);
  const bool o = kl <= kh && prefix[kh + 1] - prefix[kl] > 0;
  occ[i] = o ? 1 : 0;
  const unsigned long long e = __ballot(!o);   // one atomic per wave
  if ((threadIdx.x & 63) == 0 && e) atomicAdd(n_empty, (unsigned)__popcll(e));
}

hipError_t launch_occupancy(const uint32_t* minmax, int n_macro, const uint16_t* lut,
                            const int* prefix, int tf_n, uint8_t* occ, unsigned int* n_empty,
                            hipStream_t s) {
  const int bs = 256;
  hipLaunchKernelGGL(occupancy_kernel, dim3((n_macro + bs - 1) / bs), dim3(bs), 0, s, minmax,
                     n_macro, lut, prefix, tf_n, occ, n_empty);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------
// Skip flags of the density cells (march_common.h: cell_empty, cell_skip_q),
// rebuilt whenever the volume or the TF changes.
// ---------------------------------------------------------------------------

// Pass 0: is the cell EMPTY?  Its densities lie in [min, max] of its 8 corners
// (every lerp fmaf(t, b - a, a) with t in [0, 1] stays between a and b), and the
// TF entries a density reads grow with it (as occupancy_kernel; the range is
// widened by 2^-10, which also covers 8-bit filter weights).  Non-negative fp16
// bit patterns order like their values, so min/max run on the integer halves.
// Writes 0 (not empty) or kCellSkipCap (empty) per cell.
__global__ void cell_empty_kernel(const uint4* __restrict__ cells, size_t n,
                                  const int* __restrict__ prefix, int tf_n, uint8_t* __restrict__ d0) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint4 r = cells[i];
  const uint32_t w[4] = {r.x & 0x7fff7fffu, r.y & 0x7fff7fffu, r.z & 0x7fff7fffu, r.w & 0x7fff7fffu};
  uint32_t lo = 0xffffu, hi = 0u;
#pragma unroll
  for (int k = 0; k < 4; k++) {
    lo = min(lo, min(w[k] & 0xffffu, w[k] >> 16));
    hi = max(hi, max(w[k] & 0xffffu, w[k] >> 16));
  }
  float flo, fhi, dummy;
  h2f2(lo, flo, dummy);
  h2f2(hi, fhi, dummy);
  const float fn = (float)tf_n;
  int kl = (int)floorf(fmaf(flo - 1.0f / 1024.0f, fn, -0.5f)) + 1;
  int kh = (int)floorf(fmaf(fhi + 1.0f / 1024.0f, fn, -0.5f)) + 2;
  kl = max(kl, 0);
  kh = min(kh, tf_n + 1);
  const bool occupied = kl <= kh && prefix[kh + 1] - prefix[kl] > 0;
  d0[i] = occupied ? 0 : (uint8_t)kCellSkipCap;
}

// One axis of the chessboard distance transform, capped at kCellSkipCap:
// out(p) = min over |k| < cap (p + k e inside the grid) of max(|k|, in(p + k e)).
// Applied along x to the 0 / cap map of pass 0, then y, then z, it gives
// min over non-empty q of max(|dx|, |dy|, |dz|) (max distributes over min).
// Cells outside the grid count as empty: no sample position leaves the grid.
__global__ void cell_dist_axis_kernel(const uint8_t* __restrict__ in, uint8_t* __restrict__ out,
                                      size_t n, int cx, int cy, int cz, int axis) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint32_t a = (uint32_t)(i % (uint32_t)cx);
  const uint32_t rest = (uint32_t)(i / (uint32_t)cx);
  const uint32_t b = rest % (uint32_t)cy, c = rest / (uint32_t)cy;
  const int pos = axis == 0 ? (int)a : axis == 1 ? (int)b : (int)c;
  const int dim = axis == 0 ? cx : axis == 1 ? cy : cz;
  const long long stride = axis == 0 ? 1 : axis == 1 ? (long long)cx : (long long)cx * cy;
  int d = in[i];
  for (int k = 1; k < kCellSkipCap && k < d; k++) {
    if (pos - k >= 0) d = min(d, max(k, (int)in[(long long)i - k * stride]));
    if (pos + k < dim) d = min(d, max(k, (int)in[(long long)i + k * stride]));
  }
  out[i] = (uint8_t)d;
}

// Final pass: the distance into the cells' sign bits (flag + 3-bit q).
__global__ void cell_flags_write_kernel(uint4* __restrict__ cells, const uint8_t* __restrict__ dist,
                                        size_t n) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int d = dist[i];
  const uint32_t e = d >= 1 ? 1u : 0u;
  const uint32_t q = d >= 1 ? (uint32_t)(min(d, kCellSkipCap) - 1) : 0u;
  uint4 r = cells[i];
  r.x = (r.x & 0x7fff7fffu) | (e << 31);
  r.y = (r.y & 0x7fff7fffu) | ((q & 1u) << 31);
  r.z = (r.z & 0x7fff7fffu) | (((q >> 1) & 1u) << 31);
  r.w = (r.w & 0x7fff7fffu) | (((q >> 2) & 1u) << 31);
  cells[i] = r;
}

__global__ void fill_u8_kernel(uint8_t* __restrict__ p, size_t n, uint8_t v) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) p[i] = v;
}

// clear = true: strip every flag (the cells hold plain |densities| again)
hipError_t launch_cell_flags(const Ctx& c, bool clear, uint8_t* t0, uint8_t* t1, hipStream_t s) {
  const size_t n = cell_count(c.cells);
  const int bs = 256;
  const dim3 grid((unsigned)((n + bs - 1) / bs));
  uint4* cells = (uint4*)c.d_cells;
  if (clear) {
    hipLaunchKernelGGL(fill_u8_kernel, grid, dim3(bs), 0, s, t0, n, (uint8_t)0);
  } else {
    hipLaunchKernelGGL(cell_empty_kernel, grid, dim3(bs), 0, s, (const uint4*)cells, n,
                       c.d_tf_prefix, c.tf_n, t0);
    for (int axis = 0; axis < 3; axis++) {
      hipLaunchKernelGGL(cell_dist_axis_kernel, grid, dim3(bs), 0, s, (const uint8_t*)t0, t1, n,
                         c.cells.cx, c.cells.cy, c.cells.cz, axis);
      std::swap(t0, t1);
    }
  }
  hipLaunchKernelGGL(cell_flags_write_kernel, grid, dim3(bs), 0, s, cells, (const uint8_t*)t0, n);
  return hipGetLastError();
}

}  // namespace cvr
