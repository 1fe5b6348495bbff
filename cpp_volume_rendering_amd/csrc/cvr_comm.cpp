// cvr_comm.cpp — the screen-tile split's one exchange step:
// rank 0 gathers every rank's packed tiles with one ncclGather (RCCL over xGMI)
// and unpacks them into the frame.  Native, so a frame costs two C calls on the host (render +
// gather) instead of a Python collective: at 8 GPUs a rank's share of a
// 1024^2 frame renders in tens of microseconds.
//
// Pipelining: the gather runs on the context's communication stream after the
// render that produced its tiles; the render stream only waits for the gather
// issued one call earlier.  With two packed buffers used alternately, frame
// n+1 renders while frame n is in flight (cvr.h, cvr_gather_tiles).
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <cstdarg>
#include <cstdio>
#include <cstring>

#include "cvr_internal.h"

using cvr::Ctx;

namespace {

struct Comm {
  ncclComm_t comm = nullptr;
  int nranks = 0, rank = 0;
  hipStream_t stream = nullptr;        // communication stream (gathers + rank-0 unpack)
  hipEvent_t ev_render = nullptr;      // end of the render whose tiles are gathered
  // end of exchange g at ev_gather[g % kRing]: a render stream waits for the
  // exchange that last used the buffer set its next render writes
  static constexpr int kRing = 64;
  hipEvent_t ev_gather[kRing] = {};
  long long ngather = 0;
};

cvr_status cfail(Ctx* c, cvr_status st, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  c->err = buf;
  return st;
}

#define CHIP(ctx, expr)                                                                  \
  do {                                                                                   \
    hipError_t _e = (expr);                                                              \
    if (_e != hipSuccess)                                                                \
      return cfail(ctx, CVR_ERR_HIP, "%s: %s (%s:%d)", #expr, hipGetErrorString(_e),     \
                   __FILE__, __LINE__);                                                  \
  } while (0)

#define CNCCL(ctx, expr)                                                                 \
  do {                                                                                   \
    ncclResult_t _r = (expr);                                                            \
    if (_r != ncclSuccess)                                                               \
      return cfail(ctx, CVR_ERR_HIP, "%s: %s (%s:%d)", #expr, ncclGetErrorString(_r),    \
                   __FILE__, __LINE__);                                                  \
  } while (0)

Comm* comm_of(Ctx* c) { return static_cast<Comm*>(c->comm); }

}  // namespace

namespace cvr {
// called by cvr_destroy
void comm_release(Ctx* c) {
  Comm* m = comm_of(c);
  if (!m) return;
  (void)hipSetDevice(c->device);
  if (m->stream) (void)hipStreamSynchronize(m->stream);
  if (m->comm) (void)ncclCommDestroy(m->comm);
  if (m->ev_render) (void)hipEventDestroy(m->ev_render);
  for (hipEvent_t e : m->ev_gather)
    if (e) (void)hipEventDestroy(e);
  if (m->stream) (void)hipStreamDestroy(m->stream);
  delete m;
  c->comm = nullptr;
}
}  // namespace cvr

#pragma GCC visibility push(default)
extern "C" {

cvr_status cvr_comm_unique_id(unsigned char out_id[CVR_COMM_ID_BYTES]) {
  if (!out_id) return CVR_ERR_ARG;
  static_assert(sizeof(ncclUniqueId) == CVR_COMM_ID_BYTES, "ncclUniqueId size");
  ncclUniqueId id;
  if (ncclGetUniqueId(&id) != ncclSuccess) return CVR_ERR_HIP;
  std::memcpy(out_id, &id, sizeof(id));
  return CVR_OK;
}

cvr_status cvr_comm_init(cvr_ctx* ctx, int nranks, int rank,
                         const unsigned char id[CVR_COMM_ID_BYTES]) {
  Ctx* c = reinterpret_cast<Ctx*>(ctx);
  if (!c) return CVR_ERR_ARG;
  if (!id || nranks < 1 || rank < 0 || rank >= nranks)
    return cfail(c, CVR_ERR_ARG, "cvr_comm_init: bad rank %d of %d", rank, nranks);
  if (c->comm) return cfail(c, CVR_ERR_STATE, "cvr_comm_init: already initialised");
  CHIP(c, hipSetDevice(c->device));
  Comm* m = new Comm();
  c->comm = m;
  m->nranks = nranks;
  m->rank = rank;
  ncclUniqueId uid;
  std::memcpy(&uid, id, sizeof(uid));
  ncclResult_t r = ncclCommInitRank(&m->comm, nranks, uid, rank);
  if (r != ncclSuccess) {
    m->comm = nullptr;
    cvr::comm_release(c);
    return cfail(c, CVR_ERR_HIP, "ncclCommInitRank: %s", ncclGetErrorString(r));
  }
  int lo = 0, hi = 0;
  CHIP(c, hipDeviceGetStreamPriorityRange(&lo, &hi));
  CHIP(c, hipStreamCreateWithPriority(&m->stream, hipStreamNonBlocking, hi));
  CHIP(c, hipEventCreateWithFlags(&m->ev_render, hipEventDisableTiming));
  for (hipEvent_t& e : m->ev_gather) CHIP(c, hipEventCreateWithFlags(&e, hipEventDisableTiming));
  return CVR_OK;
}

cvr_status cvr_comm_destroy(cvr_ctx* ctx) {
  Ctx* c = reinterpret_cast<Ctx*>(ctx);
  if (!c) return CVR_ERR_ARG;
  cvr::comm_release(c);
  return CVR_OK;
}

cvr_status cvr_gather_tiles_n(cvr_ctx* ctx, const cvr_frame* f, int nframes, const void* d_packed,
                              int tpr_max, int format, void* d_gathered, void* const* d_images) {
  Ctx* c = reinterpret_cast<Ctx*>(ctx);
  if (!c) return CVR_ERR_ARG;
  Comm* m = comm_of(c);
  if (!m) return cfail(c, CVR_ERR_STATE, "cvr_gather_tiles: cvr_comm_init not called");
  // gather_root_idle: rank 0 renders nothing; communicator ranks 1..N-1 render the
  // split over N-1 render ranks (frame rank = communicator rank - 1).  An idle
  // root sends nothing, so it needs no packed buffer.
  const bool idle_root = c->gather_root_idle && m->nranks > 2;
  if (!f || (!d_packed && !(idle_root && m->rank == 0)) || nframes < 1 || tpr_max < 0 ||
      (f->nranks > 1 && f->tile_size < 16) ||
      (format != CVR_FORMAT_RGBA32F && format != CVR_FORMAT_RGBA16F))
    return cfail(c, CVR_ERR_ARG, "cvr_gather_tiles: bad arguments");
  const int want_nranks = idle_root ? m->nranks - 1 : m->nranks;
  const int want_rank = idle_root ? m->rank - 1 : m->rank;
  if (f->nranks != want_nranks || (f->rank != want_rank && !(idle_root && m->rank == 0)))
    return cfail(c, CVR_ERR_ARG, "cvr_gather_tiles: frame rank %d/%d, communicator %d/%d%s",
                 f->rank, f->nranks, m->rank, m->nranks, idle_root ? " (idle root)" : "");
  if (m->rank == 0 && (!d_gathered || !d_images))
    return cfail(c, CVR_ERR_ARG, "cvr_gather_tiles: rank 0 needs the gather buffer and images");
  if (m->nranks > 1 && !(idle_root && m->rank == 0) && cvr_tiles_for_rank(f, f->rank) > tpr_max)
    return cfail(c, CVR_ERR_ARG, "cvr_gather_tiles: tiles_per_rank_max too small");
  CHIP(c, hipSetDevice(c->device));
  const size_t px = format == CVR_FORMAT_RGBA16F ? 8 : 16;
  // one rank: the frames were rendered whole (row-major); the "gather" is a copy
  const size_t fbytes = m->nranks == 1 ? (size_t)f->width * f->height * px
                                       : (size_t)tpr_max * f->tile_size * f->tile_size * px;
  const size_t bytes = fbytes * (size_t)nframes;
  hipStream_t s = c->stream;
  CHIP(c, hipEventRecord(m->ev_render, s));
  CHIP(c, hipStreamWaitEvent(m->stream, m->ev_render, 0));
  // One ncclGather (rccl.h:745) for all nframes frames: block r of the gather
  // buffer <- rank r's frames.  Rank 0 renders straight into block 0, which makes
  // its part in place.
  if (m->rank == 0) {
    char* g = static_cast<char*>(d_gathered);
    if (d_packed != d_gathered && !idle_root)
      CHIP(c, hipMemcpyAsync(g, d_packed, bytes, hipMemcpyDeviceToDevice, m->stream));
    CNCCL(c, ncclGather(g, g, bytes, ncclChar, 0, m->comm, m->stream));
    // idle root: block 0 (its own, in place) holds nothing; render rank v's frames
    // are block v + 1
    const char* g0 = idle_root ? g + bytes : g;
    for (int j = 0; j < nframes; j++) {
      void* img = d_images[j];
      if (!img) continue;
      const char* fj = g0 + (size_t)j * fbytes;
      if (m->nranks == 1) {
        if (img != (const void*)fj)
          CHIP(c, hipMemcpyAsync(img, fj, fbytes, hipMemcpyDeviceToDevice, m->stream));
      } else {
        CHIP(c, cvr::launch_unpack_tiles(fj, img, format == CVR_FORMAT_RGBA16F, f->width,
                                         f->height, f->tile_size, f->nranks, tpr_max, m->stream,
                                         (size_t)nframes * tpr_max));
      }
    }
  } else {
    CNCCL(c, ncclGather(d_packed, nullptr, bytes, ncclChar, 0, m->comm, m->stream));
  }
  const long long g = m->ngather;
  CHIP(c, hipEventRecord(m->ev_gather[g % Comm::kRing], m->stream));
  // One render stream and two buffers: the next render reuses the buffers of the
  // previous exchange, so the stream waits for the previous gather (this gather
  // overlaps the next render).  D >= 2 streams rotated with B >= D buffer sets
  // (option "gather_sets", a multiple of D; exchange g uses set g % B on stream
  // g % D): this stream's next render (exchange g + D) writes set (g + D) % B,
  // last used by exchange g + D - B, so the stream waits for that one -- with
  // B = D this exchange, with B = 4D one issued three rounds earlier, which has
  // usually finished, so a slow exchange no longer stalls the render pipeline.
  if (c->split_streams >= 2) {
    const int D = c->split_streams;
    const int B = c->gather_sets > D ? c->gather_sets : D;
    const long long w = g + D - B;
    if (w >= 0) CHIP(c, hipStreamWaitEvent(s, m->ev_gather[w % Comm::kRing], 0));
  } else if (g > 0) {
    CHIP(c, hipStreamWaitEvent(s, m->ev_gather[(g - 1) % Comm::kRing], 0));
  }
  m->ngather++;
  return CVR_OK;
}

cvr_status cvr_gather_tiles(cvr_ctx* ctx, const cvr_frame* f, const void* d_packed,
                            int tpr_max, int format, void* d_gathered, void* d_rgba) {
  void* imgs[1] = {d_rgba};
  return cvr_gather_tiles_n(ctx, f, 1, d_packed, tpr_max, format, d_gathered, imgs);
}

cvr_status cvr_gather_sync(cvr_ctx* ctx) {
  Ctx* c = reinterpret_cast<Ctx*>(ctx);
  if (!c) return CVR_ERR_ARG;
  Comm* m = comm_of(c);
  if (!m) return cfail(c, CVR_ERR_STATE, "cvr_gather_sync: cvr_comm_init not called");
  if (m->ngather == 0) return CVR_OK;
  CHIP(c, hipSetDevice(c->device));
  CHIP(c, hipStreamWaitEvent(c->stream, m->ev_gather[(m->ngather - 1) % Comm::kRing], 0));
  return CVR_OK;
}

}  // extern "C"
#pragma GCC visibility pop
