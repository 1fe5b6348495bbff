// Lossless per-tile code of RGBA16F screen tiles: the bytes of the
// multi-GPU exchange.  At every world size the frame is bound by rank 0's xGMI
// inbound, 8 B per pixel; rendered tiles are smooth, so each tile's channels
// are stored as differences from the tile's minimum bit pattern at the bit
// width of the largest difference.
//
// Stream (32-bit words): [0, ntiles] the word where tile t's code starts (entry
// ntiles: the stream's end), then per tile 3 header words -- the four channel
// bases (16 bits each, R | G << 16, B | A << 16) and the four widths (5 bits
// each) -- and per channel with width w > 0 the npx differences packed
// little-endian at w bits each (8 w words for a 16 x 16 tile).  Any bit
// pattern round-trips (the differences are of unsigned 16-bit patterns, so
// signs, NaNs and infinities are just patterns).
//
// Three launches: per-tile sizes, one workgroup's scan into the start table,
// and the packing; the decode is one launch.  A wave per tile throughout (64
// lanes over the tile's pixels; the packing reads its pixels from LDS).
#include <algorithm>

#include "cvr_internal.h"

namespace cvr {

namespace {

constexpr int kCodecHeaderWords = 3;
constexpr int kScanThreads = 1024;

__device__ __forceinline__ uint32_t chan(uint2 v, int c) {
  const uint32_t w = (c < 2) ? v.x : v.y;
  return (c & 1) ? (w >> 16) : (w & 0xffffu);
}

__device__ __forceinline__ uint32_t wave_min_u32(uint32_t v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v = min(v, (uint32_t)__shfl_xor((int)v, off, 64));
  return v;
}
__device__ __forceinline__ uint32_t wave_max_u32(uint32_t v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v = max(v, (uint32_t)__shfl_xor((int)v, off, 64));
  return v;
}

// The tile's per-channel bases and widths (every lane of the calling wave gets them;
// a wave codes one tile, so the lane is the thread's index within its wave).
__device__ __forceinline__ void tile_stats(const uint2* __restrict__ px, int npx, uint32_t (&base)[4],
                                           uint32_t (&width)[4]) {
  const int lane = (int)threadIdx.x & 63;
  uint32_t mn[4] = {0xffffu, 0xffffu, 0xffffu, 0xffffu}, mx[4] = {0u, 0u, 0u, 0u};
  for (int p = lane; p < npx; p += 64) {
    const uint2 v = px[p];
#pragma unroll
    for (int c = 0; c < 4; c++) {
      const uint32_t x = chan(v, c);
      mn[c] = min(mn[c], x);
      mx[c] = max(mx[c], x);
    }
  }
#pragma unroll
  for (int c = 0; c < 4; c++) {
    base[c] = wave_min_u32(mn[c]);
    const uint32_t span = wave_max_u32(mx[c]) - base[c];
    width[c] = span ? 32u - (uint32_t)__builtin_clz(span) : 0u;
  }
}

__device__ __forceinline__ uint32_t code_words(int npx, const uint32_t (&width)[4]) {
  uint32_t n = kCodecHeaderWords;
#pragma unroll
  for (int c = 0; c < 4; c++) n += ((uint32_t)npx * width[c] + 31u) >> 5;
  return n;
}

__global__ void __launch_bounds__(64) tile_code_size_kernel(const uint2* __restrict__ tiles, int npx,
                                                            int ntiles, uint32_t* __restrict__ stream) {
  const int t = blockIdx.x;
  if (t >= ntiles) return;
  uint32_t base[4], width[4];
  tile_stats(tiles + (size_t)t * npx, npx, base, width);
  if (threadIdx.x == 0) stream[t] = code_words(npx, width);
}

// In place: stream[0..ntiles) holds the tiles' word counts; afterwards stream[t] =
// (ntiles + 1) + the exclusive sum, stream[ntiles] = the total, *bytes = 4 x total.
__global__ void __launch_bounds__(kScanThreads) tile_code_scan_kernel(uint32_t* __restrict__ stream, int ntiles,
                                                                      unsigned long long* __restrict__ bytes) {
  __shared__ uint32_t part[kScanThreads];
  const int tid = (int)threadIdx.x;
  const int per = (ntiles + kScanThreads - 1) / kScanThreads;
  const int b0 = min(tid * per, ntiles), b1 = min(b0 + per, ntiles);
  uint32_t s = 0;
  for (int i = b0; i < b1; i++) s += stream[i];
  part[tid] = s;
  __syncthreads();
  for (int off = 1; off < kScanThreads; off <<= 1) {   // inclusive scan of the partial sums
    const uint32_t v = tid >= off ? part[tid - off] : 0u;
    __syncthreads();
    part[tid] += v;
    __syncthreads();
  }
  uint32_t run = (uint32_t)(ntiles + 1) + (tid ? part[tid - 1] : 0u);
  for (int i = b0; i < b1; i++) {
    const uint32_t n = stream[i];
    stream[i] = run;
    run += n;
  }
  if (tid == kScanThreads - 1) {
    const uint32_t end = (uint32_t)(ntiles + 1) + part[kScanThreads - 1];
    stream[ntiles] = end;
    *bytes = 4ull * end;
  }
}

__global__ void __launch_bounds__(64) tile_encode_kernel(const uint2* __restrict__ tiles, int npx, int ntiles,
                                                         uint32_t* __restrict__ stream) {
  extern __shared__ uint2 pxl[];
  const int t = blockIdx.x;
  if (t >= ntiles) return;
  const int lane = (int)threadIdx.x;
  const uint2* src = tiles + (size_t)t * npx;
  for (int p = lane; p < npx; p += 64) pxl[p] = src[p];
  __syncthreads();
  uint32_t base[4], width[4];
  tile_stats(pxl, npx, base, width);
  uint32_t* out = stream + stream[t];
  if (lane == 0) {
    out[0] = base[0] | (base[1] << 16);
    out[1] = base[2] | (base[3] << 16);
    out[2] = width[0] | (width[1] << 5) | (width[2] << 10) | (width[3] << 15);
  }
  uint32_t pos = kCodecHeaderWords;
#pragma unroll
  for (int c = 0; c < 4; c++) {
    const uint32_t w = width[c];
    const uint32_t nw = ((uint32_t)npx * w + 31u) >> 5;
    for (uint32_t j = (uint32_t)lane; j < nw; j += 64) {
      const uint32_t bit0 = j << 5;
      const uint32_t p0 = bit0 / w, p1 = min((bit0 + 31u) / w, (uint32_t)npx - 1u);
      uint32_t acc = 0;
      for (uint32_t p = p0; p <= p1; p++) {
        const uint32_t d = chan(pxl[p], c) - base[c];
        const int sh = (int)(p * w) - (int)bit0;   // < 32: p <= (bit0 + 31) / w
        acc |= sh >= 0 ? (d << sh) : (d >> -sh);
      }
      out[pos + j] = acc;
    }
    pos += nw;
  }
}

__global__ void __launch_bounds__(64) tile_decode_kernel(const uint32_t* __restrict__ stream, int npx, int ntiles,
                                                         size_t max_words, uint2* __restrict__ tiles) {
  const int t = blockIdx.x;
  if (t >= ntiles) return;
  // a stream that does not parse is skipped rather than followed past its bound
  const uint32_t t0 = stream[t];
  if ((size_t)t0 + kCodecHeaderWords > max_words) return;
  const uint32_t* in = stream + t0;
  const uint32_t h0 = in[0], h1 = in[1], h2 = in[2];
  const uint32_t base[4] = {h0 & 0xffffu, h0 >> 16, h1 & 0xffffu, h1 >> 16};
  const uint32_t width[4] = {h2 & 31u, (h2 >> 5) & 31u, (h2 >> 10) & 31u, (h2 >> 15) & 31u};
  if (max(max(width[0], width[1]), max(width[2], width[3])) > 16u) return;
  uint32_t start[4];
  uint32_t pos = kCodecHeaderWords;
#pragma unroll
  for (int c = 0; c < 4; c++) {
    start[c] = pos;
    pos += ((uint32_t)npx * width[c] + 31u) >> 5;
  }
  if ((size_t)t0 + pos > max_words) return;
  uint2* dst = tiles + (size_t)t * npx;
  for (int p = (int)threadIdx.x; p < npx; p += 64) {
    uint32_t v[4];
#pragma unroll
    for (int c = 0; c < 4; c++) {
      const uint32_t w = width[c];
      uint32_t d = 0;
      if (w) {
        const uint32_t bit = (uint32_t)p * w, j = bit >> 5, b = bit & 31u;
        uint32_t x = in[start[c] + j] >> b;
        if (b + w > 32u) x |= in[start[c] + j + 1] << (32u - b);
        d = x & ((1u << w) - 1u);
      }
      v[c] = base[c] + d;
    }
    dst[p] = make_uint2(v[0] | (v[1] << 16), v[2] | (v[3] << 16));
  }
}

// ---------------------------------------------------------------------------
// The exchange's form of the code (cvr_comm.cpp): ONE launch per exchange group.
// Tile t of the group is frame f = t / k, the rank's tile i = t % k, read from slot
// f * tpr + i of the packed buffer.  A workgroup codes kEncTiles tiles, one per wave,
// and claims their words with ONE 64-bit atomic on *ctr: the low half counts words
// (the old value is the workgroup's offset, so codes land in claim order, not in t
// order -- the start table makes the order irrelevant to the decode), the high half
// counts tiles, so the claim that completes ntiles knows the total: it zeroes the
// counter for the next launch that uses it and writes the stream's end word and its
// length in bytes (cvr_encode_tiles passes the length itself as the counter).
// Measured forms before this one: an atomic per tile (2048 claims on one address
// serialise, ~20 us per 4-frame share at N = 8), and a __threadfence per workgroup
// (it writes back the XCD's L2 every time, 55-160 us).  No fence is needed: nothing
// in the kernel reads another tile's words, and the kernel's end publishes them.
// Two launches in flight must not share a counter (each exchange buffer set has its
// own).
constexpr int kEncTiles = 8;
__global__ void __launch_bounds__(64 * kEncTiles) exchange_encode_kernel(
    const uint2* __restrict__ packed, int npx, int k, int tpr, int ntiles, uint32_t* __restrict__ dst,
    unsigned long long* ctr, unsigned long long* d_bytes, unsigned long long* h_bytes) {
  extern __shared__ uint2 pxl_all[];
  __shared__ uint32_t s_words[kEncTiles];
  __shared__ uint32_t s_off;
  const int lane = (int)threadIdx.x & 63, wv = (int)threadIdx.x >> 6;
  if (ntiles == 0) {   // a rank without tiles: the empty stream
    if (threadIdx.x == 0) {
      dst[0] = 1u;
      if (d_bytes) *d_bytes = 4ull;
      if (h_bytes) *h_bytes = 4ull;
    }
    return;
  }
  const int tpb = (int)(blockDim.x >> 6);   // tiles (waves) per workgroup, <= kEncTiles
  const int t0 = blockIdx.x * tpb;
  const int nvalid = min(tpb, ntiles - t0);
  const int t = t0 + wv;
  const bool live = wv < nvalid;
  uint2* pxl = pxl_all + (size_t)wv * npx;
  uint32_t base[4] = {0, 0, 0, 0}, width[4] = {0, 0, 0, 0};
  if (live) {
    const int f = t / k, i = t - f * k;
    const uint2* src = packed + ((size_t)f * tpr + i) * npx;
    for (int p = lane; p < npx; p += 64) pxl[p] = src[p];
    // (a wave reads only its own tile from LDS: the wave's own program order suffices)
    __builtin_amdgcn_s_waitcnt(0);
    __builtin_amdgcn_wave_barrier();
    tile_stats(pxl, npx, base, width);
    if (lane == 0) s_words[wv] = code_words(npx, width);
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t tot = 0;
    for (int w = 0; w < nvalid; w++) tot += s_words[w];
    const unsigned long long old = atomicAdd(ctr, ((unsigned long long)nvalid << 32) | tot);
    s_off = (uint32_t)old;
    if ((uint32_t)(old >> 32) + (uint32_t)nvalid == (uint32_t)ntiles) {   // the last claim
      const uint32_t end = (uint32_t)ntiles + 1u + (uint32_t)old + tot;
      atomicExch(ctr, 0ull);
      dst[ntiles] = end;
      if (d_bytes) *d_bytes = 4ull * end;
      if (h_bytes) *h_bytes = 4ull * end;   // mapped host memory: the host reads it after the launch
    }
  }
  __syncthreads();
  if (!live) return;
  uint32_t start = (uint32_t)ntiles + 1u + s_off;
  for (int w = 0; w < wv; w++) start += s_words[w];
  uint32_t* out = dst + start;
  if (lane == 0) {
    dst[t] = start;
    out[0] = base[0] | (base[1] << 16);
    out[1] = base[2] | (base[3] << 16);
    out[2] = width[0] | (width[1] << 5) | (width[2] << 10) | (width[3] << 15);
  }
  uint32_t pos = kCodecHeaderWords;
#pragma unroll
  for (int c = 0; c < 4; c++) {
    const uint32_t w = width[c];
    const uint32_t nw = ((uint32_t)npx * w + 31u) >> 5;
    for (uint32_t j = (uint32_t)lane; j < nw; j += 64) {
      const uint32_t bit0 = j << 5;
      const uint32_t p0 = bit0 / w, p1 = min((bit0 + 31u) / w, (uint32_t)npx - 1u);
      uint32_t acc = 0;
      for (uint32_t p = p0; p <= p1; p++) {
        const uint32_t d = chan(pxl[p], c) - base[c];
        const int sh = (int)(p * w) - (int)bit0;
        acc |= sh >= 0 ? (d << sh) : (d >> -sh);
      }
      out[pos + j] = acc;
    }
    pos += nw;
  }
}

// Rank 0's half, fused: decode every source's stream of the group and write its
// pixels straight into the frames' images (the unpack of unpack_tiles_kernel, the
// tile's screen position from split_tile).  Workgroup = (source r, frame f, slot i)
// over nsrc x nframes x tpr slots; slots past the source's tiles exit.  Source r is
// frame rank r of the split; its stream is at src + r * slot_words, or, for r = 0
// with raw0 set (a rendering root), its raw packed tiles at raw0 (frame f at
// f * raw0_fstride tiles).  A tile's code is staged in LDS (one coalesced read of
// its words) before 64 lanes unpack 4 pixels each.
__global__ void __launch_bounds__(64) exchange_decode_kernel(ExchangeDecode a) {
  extern __shared__ uint32_t code[];
  const int lane = (int)threadIdx.x;
  const int per_src = a.nframes * a.tpr;
  const int r = (int)blockIdx.x / per_src;
  const int rem = (int)blockIdx.x - r * per_src;
  const int f = rem / a.tpr, i = rem - f * a.tpr;
  const int nt = a.tile_grid_n;
  const int k = nt > r ? (nt - r + a.nsplit - 1) / a.nsplit : 0;   // cvr_tiles_for_rank
  if (i >= k) return;
  uint2* __restrict__ img = a.img[f];
  if (!img) return;
  int tx, ty;
  split_tile(r, a.nsplit, i, a.ntx, tx, ty);
  const int npx = a.tile * a.tile;
  const int x0 = tx * a.tile, y0 = ty * a.tile;
  if (r == 0 && a.raw0) {
    const uint2* src = a.raw0 + ((size_t)f * a.raw0_fstride + i) * npx;
    for (int p = lane; p < npx; p += 64) {
      const int px = x0 + p % a.tile, py = y0 + p / a.tile;
      if (px < a.W && py < a.H) img[(size_t)py * a.W + px] = src[p];
    }
    return;
  }
  const uint32_t* in = a.src + (size_t)r * a.slot_words;
  // a stream that does not parse (never produced by the encode) is skipped rather than
  // followed out of its slot: the tile stays as it was
  const uint32_t t0 = in[f * k + i];
  if ((size_t)t0 + kCodecHeaderWords > a.slot_words) return;
  const uint32_t* tc = in + t0;
  const uint32_t h0 = tc[0], h1 = tc[1], h2 = tc[2];
  const uint32_t base[4] = {h0 & 0xffffu, h0 >> 16, h1 & 0xffffu, h1 >> 16};
  const uint32_t width[4] = {h2 & 31u, (h2 >> 5) & 31u, (h2 >> 10) & 31u, (h2 >> 15) & 31u};
  if (max(max(width[0], width[1]), max(width[2], width[3])) > 16u) return;
  uint32_t start[4];
  uint32_t nw = kCodecHeaderWords;
#pragma unroll
  for (int c = 0; c < 4; c++) {
    start[c] = nw;
    nw += ((uint32_t)npx * width[c] + 31u) >> 5;
  }
  if ((size_t)t0 + nw > a.slot_words) return;
  for (uint32_t j = (uint32_t)lane; j < nw; j += 64) code[j] = tc[j];
  code[nw] = 0u;   // the word after the last one a straddling read may touch (weight 0)
  __syncthreads();
  for (int p = lane; p < npx; p += 64) {
    uint32_t v[4];
#pragma unroll
    for (int c = 0; c < 4; c++) {
      const uint32_t w = width[c];
      uint32_t d = 0;
      if (w) {
        const uint32_t bit = (uint32_t)p * w, j = bit >> 5, b = bit & 31u;
        uint32_t x = code[start[c] + j] >> b;
        if (b + w > 32u) x |= code[start[c] + j + 1] << (32u - b);
        d = x & ((1u << w) - 1u);
      }
      v[c] = base[c] + d;
    }
    const int px = x0 + p % a.tile, py = y0 + p / a.tile;
    if (px < a.W && py < a.H) img[(size_t)py * a.W + px] = make_uint2(v[0] | (v[1] << 16), v[2] | (v[3] << 16));
  }
}

}  // namespace

hipError_t launch_exchange_encode(const void* d_packed, int tile, int k, int tpr, int nframes, void* d_dst,
                                  unsigned long long* ctr, unsigned long long* d_bytes, unsigned long long* h_bytes,
                                  hipStream_t s) {
  const int npx = tile * tile;
  const long long nt = (long long)k * nframes;
  if (nt > 0x7fffffffLL || k > tpr) return hipErrorInvalidValue;
  // 16 KB of LDS per workgroup: 8 tiles of 16 x 16, 2 of 32 x 32
  const int tpb = std::max(1, std::min(kEncTiles, 2048 / npx));
  const unsigned nblk = nt > 0 ? (unsigned)((nt + tpb - 1) / tpb) : 1u;
  hipLaunchKernelGGL(exchange_encode_kernel, dim3(nblk), dim3(64 * tpb), (size_t)tpb * npx * sizeof(uint2), s, static_cast<const uint2*>(d_packed), npx, k > 0 ? k : 1,
                     tpr, (int)nt, static_cast<uint32_t*>(d_dst), ctr, d_bytes, h_bytes);
  return hipGetLastError();
}

hipError_t launch_exchange_decode(const ExchangeDecode& a, hipStream_t s) {
  const long long slots = (long long)a.nsrc * a.nframes * a.tpr;
  if (slots <= 0) return hipSuccess;
  if (slots > 0x7fffffffLL) return hipErrorInvalidValue;
  // a tile's words: 3 + 4 channels x (npx x 16 bits) at most, + the guard word
  const size_t lds = 4 * ((size_t)kCodecHeaderWords + 4 * ((size_t)a.tile * a.tile / 2) + 1);
  hipLaunchKernelGGL(exchange_decode_kernel, dim3((unsigned)slots), dim3(64), lds, s, a);
  return hipGetLastError();
}

size_t tile_code_bound_bytes(int tile, int ntiles) {
  const size_t npx = (size_t)tile * tile;
  return 4 * ((size_t)ntiles + 1 + (size_t)ntiles * (kCodecHeaderWords + 4 * ((npx * 16 + 31) / 32)));
}

hipError_t launch_tile_encode(const void* d_tiles, int tile, int ntiles, void* d_stream,
                              unsigned long long* d_bytes, hipStream_t s) {
  const int npx = tile * tile;
  uint32_t* stream = static_cast<uint32_t*>(d_stream);
  const uint2* tiles = static_cast<const uint2*>(d_tiles);
  if (ntiles > 0)
    hipLaunchKernelGGL(tile_code_size_kernel, dim3(ntiles), dim3(64), 0, s, tiles, npx, ntiles, stream);
  hipLaunchKernelGGL(tile_code_scan_kernel, dim3(1), dim3(kScanThreads), 0, s, stream, ntiles, d_bytes);
  if (ntiles > 0)
    hipLaunchKernelGGL(tile_encode_kernel, dim3(ntiles), dim3(64), (size_t)npx * sizeof(uint2), s, tiles, npx,
                       ntiles, stream);
  return hipGetLastError();
}

hipError_t launch_tile_decode(const void* d_stream, int tile, int ntiles, void* d_tiles, hipStream_t s) {
  if (ntiles <= 0) return hipSuccess;
  hipLaunchKernelGGL(tile_decode_kernel, dim3(ntiles), dim3(64), 0, s, static_cast<const uint32_t*>(d_stream),
                     tile * tile, ntiles, tile_code_bound_bytes(tile, ntiles) / 4, static_cast<uint2*>(d_tiles));
  return hipGetLastError();
}

}  // namespace cvr
