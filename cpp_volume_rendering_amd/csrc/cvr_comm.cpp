// cvr_comm.cpp — the screen-tile split's one exchange step.
//
// Every exchange moves a group of frames' packed tiles from the render ranks to
// rank 0, which writes them into the frames' images.  Two transports move the
// bytes:
//   * RCCL over xGMI (cvr_comm_init): one process per GPU;
//   * device copies inside one process (cvr_comm_init_local): N contexts, on one
//     device or several (the single-process group of cvr_create_group, and the
//     one-GPU tests of the protocol at world 3 and 8).
// and two forms of the bytes:
//   * raw tiles (RGBA32F, or option exchange_code 0): one ncclGather of
//     tiles_per_rank_max tiles per rank and frame, then the unpack;
//   * the lossless per-tile code (RGBA16F, the default; codec.hip):
//     each render rank encodes its group in ONE launch, only the coded bytes
//     travel (grouped ncclSend / ncclRecv), and rank 0 decodes every rank's
//     stream straight into the images in ONE launch.
//
// The coded exchange has variable sizes.  RCCL has no gatherv and a send's count
// must equal its receive's, so the sizes travel first (the encode writes its
// length to mapped host memory and to the device; an 8-byte ncclGather on a
// second communicator and stream brings them to rank 0) and the data of
// exchange g is posted `lag` exchanges later, when the host reads g's sizes
// (option exchange_lag): by then the sizes have normally long arrived, and the
// render streams hold the groups in between, so the device never waits for the
// host.  A render stream's next group reuses buffers only after the exchange that
// last used them (buffer sets, option gather_sets); if that exchange is still
// unposted the host posts it first (its sizes are waited for).  No capacity is
// guessed and nothing overflows: every receive is posted with its exact size.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <vector>

#include "cvr_internal.h"

using cvr::Ctx;

namespace {

constexpr int kRing = CVR_MAX_GATHER_SETS;   // exchanges whose events are kept

struct LocalHub;

// One exchange, as issued (phase A); its data phase (B) may come later.
struct Pending {
  int set = 0;
  int nframes = 0;
  int tpr = 0;                      // tile slots per frame in the caller's buffers
  int k = 0;                        // this rank's tiles per frame (0: renders nothing)
  bool code = false;
  const void* d_packed = nullptr;   // this rank's tiles (the caller's buffer)
  void* d_gathered = nullptr;       // rank 0: the caller's gather buffer
  cvr_frame f{};                    // the tile layout
  void* images[64] = {};            // rank 0: frame j's image
  size_t fbytes = 0;                // raw bytes per frame and rank
  bool half = false;                // RGBA16F pixels
  size_t recv_slot = 0;             // rank 0, coded: bytes per source slot of the receive set
};

// The coded exchange's buffers of one buffer set.
struct CodeSet {
  void* send = nullptr;                  // this rank's stream
  size_t send_cap = 0;
  unsigned long long* ctr = nullptr;     // the encode's claim counter (left zero)
  unsigned long long* d_size = nullptr;  // [1] this rank's stream bytes
  void* recv = nullptr;                  // rank 0: nsrc slots of recv_slot bytes
  size_t recv_slot = 0, recv_cap = 0;
  unsigned long long* d_sizes = nullptr; // rank 0: [nranks] gathered sizes (RCCL; its own slot stays 0)
  unsigned long long* h_sizes = nullptr; // pinned: rank 0 all sizes, others its own at [0]
  unsigned long long* h_sizes_dev = nullptr;   // the device pointer of h_sizes (mapped)
};

struct Comm {
  ncclComm_t comm = nullptr;        // RCCL: data
  ncclComm_t comm_sz = nullptr;     // RCCL: the coded exchange's sizes (own stream, own order)
  LocalHub* hub = nullptr;          // in-process transport
  int nranks = 0, rank = 0;
  hipStream_t stream = nullptr;     // data: gathers / sends / receives and rank 0's decode
  hipStream_t stream_sz = nullptr;  // sizes
  hipEvent_t ev_render = nullptr;   // end of the render whose tiles are exchanged
  hipEvent_t ev_gather[kRing] = {}; // exchange g done (rank 0: decoded; others: sent)
  hipEvent_t ev_enc[kRing] = {};    // exchange g's tiles ready (encoded, or rendered when raw)
  hipEvent_t ev_sz[kRing] = {};     // rank 0 (RCCL): exchange g's gathered sizes in h_sizes
  long long ngather = 0;            // exchanges issued (phase A)
  long long nposted = 0;            // exchanges whose data phase is issued
  Pending pend[kRing];
  std::vector<CodeSet> sets;
};

struct LocalHub {
  std::vector<Ctx*> ctxs;           // rank -> context
  int refs = 0;
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
      return cfail(ctx, _e == hipErrorOutOfMemory ? CVR_ERR_OOM : CVR_ERR_HIP,           \
                   "%s: %s (%s:%d)", #expr, hipGetErrorString(_e), __FILE__, __LINE__);  \
  } while (0)

#define CNCCL(ctx, expr)                                                                 \
  do {                                                                                   \
    ncclResult_t _r = (expr);                                                            \
    if (_r != ncclSuccess)                                                               \
      return cfail(ctx, CVR_ERR_HIP, "%s: %s (%s:%d)", #expr, ncclGetErrorString(_r),    \
                   __FILE__, __LINE__);                                                  \
  } while (0)

#define CTRY(expr)                      \
  do {                                  \
    cvr_status _s = (expr);             \
    if (_s != CVR_OK) return _s;        \
  } while (0)

Comm* comm_of(const Ctx* c) { return static_cast<Comm*>(c->comm); }

// idle root: communicator rank 0 renders nothing, ranks 1..N-1 are split ranks 0..N-2
bool idle_root(const Ctx* c, const Comm* m) { return c->gather_root_idle && m->nranks > 2; }

int buffer_sets(const Ctx* c) {
  const int D = std::max(c->split_streams, 1);
  return std::max(std::max(c->gather_sets, D), 2);
}

// exchanges the data phase may trail the issue by
int effective_lag(const Ctx* c, const Comm* m) {
  if (c->exchange_lag == 0) return 0;
  const int D = std::max(c->split_streams, 1);
  // a render stream's next group needs exchange g + D - B; the in-process transport
  // also needs rank 0 to have posted it one call earlier (rank 0 calls last)
  int room = buffer_sets(c) - D - (m->hub ? 1 : 0);
  int lag = c->exchange_lag < 0 ? D - 1 : c->exchange_lag;
  return std::max(0, std::min(lag, room));
}

cvr_status grow(Ctx* c, const Comm* m, void** p, size_t* cap, size_t want) {
  if (*cap >= want && *p) return CVR_OK;
  if (*p) {   // in-flight exchanges may still use the old buffer (any member's device)
    if (m->hub)
      for (Ctx* o : m->hub->ctxs)
        if (o && o->device != c->device) {
          CHIP(c, hipSetDevice(o->device));
          CHIP(c, hipDeviceSynchronize());
        }
    CHIP(c, hipSetDevice(c->device));
    CHIP(c, hipDeviceSynchronize());
    (void)hipFree(*p);
    *p = nullptr;
    *cap = 0;
  }
  CHIP(c, hipMalloc(p, want));
  *cap = want;
  return CVR_OK;
}

cvr_status ensure_set(Ctx* c, Comm* m, int set, size_t send_bytes, size_t recv_slot, int nsrc) {
  if ((int)m->sets.size() <= set) m->sets.resize((size_t)set + 1);
  CodeSet& S = m->sets[(size_t)set];
  if (!S.ctr) {
    CHIP(c, hipMalloc((void**)&S.ctr, 2 * sizeof(unsigned long long)));
    CHIP(c, hipMemset(S.ctr, 0, 2 * sizeof(unsigned long long)));
    S.d_size = S.ctr + 1;
    // mapped, coherent: a render rank's encode writes its stream length here itself,
    // so the host reads it after the launch without a copy
    CHIP(c, hipHostMalloc((void**)&S.h_sizes, sizeof(unsigned long long) * (size_t)m->nranks,
                          hipHostMallocMapped | hipHostMallocCoherent));
    std::memset(S.h_sizes, 0, sizeof(unsigned long long) * (size_t)m->nranks);
    CHIP(c, hipHostGetDevicePointer((void**)&S.h_sizes_dev, S.h_sizes, 0));
    if (m->rank == 0 && m->comm_sz) {
      CHIP(c, hipMalloc((void**)&S.d_sizes, sizeof(unsigned long long) * (size_t)m->nranks));
      CHIP(c, hipMemset(S.d_sizes, 0, sizeof(unsigned long long) * (size_t)m->nranks));
    }
  }
  if (send_bytes) CTRY(grow(c, m, &S.send, &S.send_cap, send_bytes));
  if (m->rank == 0 && nsrc > 0) {
    CTRY(grow(c, m, &S.recv, &S.recv_cap, recv_slot * (size_t)nsrc));
    S.recv_slot = recv_slot;
  }
  return CVR_OK;
}

Comm* root_comm(const Comm* m) { return comm_of(m->hub->ctxs[0]); }

// Rank 0's decode of exchange e's coded streams (and raw block 0) into its images:
// one launch for the group, or one per run of frames whose images do not repeat
// (a repeated image must see its frames in order).  Every launch covers the whole
// group's grid; frames outside the run have no image and exit at once.
cvr_status decode_group(Ctx* c, Comm* m, const Pending& P, int nsrc, bool raw0) {
  const cvr_frame& f = P.f;
  const int ntx = (f.width + f.tile_size - 1) / f.tile_size;
  const int nty = (f.height + f.tile_size - 1) / f.tile_size;
  cvr::ExchangeDecode a{};
  a.src = static_cast<const uint32_t*>(m->sets[(size_t)P.set].recv);
  a.slot_words = P.recv_slot / 4;
  a.raw0 = raw0 ? static_cast<const uint2*>(P.d_packed) : nullptr;
  a.raw0_fstride = (size_t)P.tpr;
  a.nsrc = nsrc;
  a.nsplit = f.nranks;
  a.nframes = P.nframes;
  a.tpr = P.tpr;
  a.tile = f.tile_size;
  a.W = f.width;
  a.H = f.height;
  a.ntx = ntx;
  a.tile_grid_n = ntx * nty;
  int j0 = 0;
  while (j0 < P.nframes) {
    int j1 = j0 + 1;
    for (; j1 < P.nframes; j1++) {
      bool dup = false;
      for (int q = j0; q < j1; q++) dup |= P.images[j1] && P.images[q] == P.images[j1];
      if (dup) break;
    }
    for (int q = 0; q < cvr::kMaxLaunchFrames; q++)
      a.img[q] = (q >= j0 && q < j1) ? static_cast<uint2*>(P.images[q]) : nullptr;
    CHIP(c, cvr::launch_exchange_decode(a, m->stream));
    j0 = j1;
  }
  return CVR_OK;
}

// Rank 0 of the raw exchange: unpack every frame of the gathered block.
cvr_status unpack_raw(Ctx* c, Comm* m, const Pending& P, const char* g0, bool half) {
  for (int j = 0; j < P.nframes; j++) {
    void* img = P.images[j];
    if (!img) continue;
    const char* fj = g0 + (size_t)j * P.fbytes;
    if (m->nranks == 1) {
      if (img != (const void*)fj)
        CHIP(c, hipMemcpyAsync(img, fj, P.fbytes, hipMemcpyDeviceToDevice, m->stream));
    } else {
      CHIP(c, cvr::launch_unpack_tiles(fj, img, half, P.f.width, P.f.height, P.f.tile_size,
                                       P.f.nranks, P.tpr, m->stream, (size_t)P.nframes * P.tpr));
    }
  }
  return CVR_OK;
}

// ---------------------------------------------------------------------------
// Phase B: the data of exchange e (its sizes are read on the host first).
// ---------------------------------------------------------------------------
cvr_status post_data(Ctx* c, Comm* m, long long e) {
  Pending& P = m->pend[e % kRing];
  const bool idle = idle_root(c, m);
  const size_t bytes = P.fbytes * (size_t)P.nframes;
  if (m->hub) {
    // in-process transport: rank 0 pulls every rank's bytes (device copies); the
    // other ranks only make sure they issued the exchange (they call first)
    if (m->rank == 0) {
      // its own tiles (raw block 0) come from its own render
      CHIP(c, hipStreamWaitEvent(m->stream, m->ev_enc[e % kRing], 0));
      for (int r = 1; r < m->nranks; r++) {
        const Comm* mr = comm_of(m->hub->ctxs[(size_t)r]);
        if (mr->ngather <= e)
          return cfail(c, CVR_ERR_STATE,
                       "local exchange %lld: rank %d has not issued it (call ranks 1..N-1 "
                       "before rank 0)", e, r);
      }
      if (P.code) {
        const CodeSet& S = m->sets[(size_t)P.set];
        for (int r = 1; r < m->nranks; r++) {
          Ctx* cr = m->hub->ctxs[(size_t)r];
          Comm* mr = comm_of(cr);
          const Pending& Pr = mr->pend[e % kRing];
          const CodeSet& Sr = mr->sets[(size_t)Pr.set];
          CHIP(c, hipEventSynchronize(mr->ev_enc[e % kRing]));   // its encode wrote the length
          const size_t nb = (size_t)Sr.h_sizes[0];
          const int src = idle ? r - 1 : r;
          if (nb > P.recv_slot)
            return cfail(c, CVR_ERR_STATE, "local exchange: stream of %zu B over the slot", nb);
          CHIP(c, hipStreamWaitEvent(m->stream, mr->ev_enc[e % kRing], 0));
          CHIP(c, hipMemcpyAsync(static_cast<char*>(S.recv) + (size_t)src * P.recv_slot, Sr.send,
                                 nb, hipMemcpyDefault, m->stream));
        }
        const int nsrc = idle ? m->nranks - 1 : m->nranks;
        CTRY(decode_group(c, m, P, nsrc, !idle));
      } else {
        char* g = static_cast<char*>(P.d_gathered);
        for (int r = 1; r < m->nranks; r++) {
          Comm* mr = comm_of(m->hub->ctxs[(size_t)r]);
          const Pending& Pr = mr->pend[e % kRing];
          CHIP(c, hipStreamWaitEvent(m->stream, mr->ev_enc[e % kRing], 0));
          CHIP(c, hipMemcpyAsync(g + (size_t)r * bytes, Pr.d_packed, bytes, hipMemcpyDefault,
                                 m->stream));
        }
        if (P.d_packed != P.d_gathered && !idle && P.d_packed)
          CHIP(c, hipMemcpyAsync(g, P.d_packed, bytes, hipMemcpyDeviceToDevice, m->stream));
        CTRY(unpack_raw(c, m, P, idle ? g + bytes : g, P.half));
      }
    }
  } else if (P.code) {
    // RCCL: exact sizes, grouped point-to-point.  Rank 0 has every size once its
    // gather's copy is done; a render rank has its own once its encode is.
    CHIP(c, hipEventSynchronize(m->rank == 0 ? m->ev_sz[e % kRing] : m->ev_enc[e % kRing]));
    const CodeSet& S = m->sets[(size_t)P.set];
    if (m->rank == 0) {
      CNCCL(c, ncclGroupStart());
      for (int r = 1; r < m->nranks; r++) {
        const size_t nb = (size_t)S.h_sizes[r];
        const int src = idle ? r - 1 : r;
        if (nb > P.recv_slot) {
          (void)ncclGroupEnd();
          return cfail(c, CVR_ERR_STATE, "coded exchange: rank %d sent %zu B over the slot", r, nb);
        }
        CNCCL(c, ncclRecv(static_cast<char*>(S.recv) + (size_t)src * P.recv_slot, nb, ncclChar, r,
                          m->comm, m->stream));
      }
      CNCCL(c, ncclGroupEnd());
      CHIP(c, hipStreamWaitEvent(m->stream, m->ev_enc[e % kRing], 0));   // its own raw tiles
      const int nsrc = idle ? m->nranks - 1 : m->nranks;
      CTRY(decode_group(c, m, P, nsrc, !idle));
    } else {
      CHIP(c, hipStreamWaitEvent(m->stream, m->ev_enc[e % kRing], 0));
      CNCCL(c, ncclSend(S.send, (size_t)S.h_sizes[0], ncclChar, 0, m->comm, m->stream));
    }
  } else {
    // RCCL, raw tiles: one ncclGather (rccl.h:745) of every rank's frames
    CHIP(c, hipStreamWaitEvent(m->stream, m->ev_enc[e % kRing], 0));
    if (m->rank == 0) {
      char* g = static_cast<char*>(P.d_gathered);
      if (P.d_packed != P.d_gathered && !idle && P.d_packed)
        CHIP(c, hipMemcpyAsync(g, P.d_packed, bytes, hipMemcpyDeviceToDevice, m->stream));
      if (m->nranks > 1) CNCCL(c, ncclGather(g, g, bytes, ncclChar, 0, m->comm, m->stream));
      CTRY(unpack_raw(c, m, P, idle ? g + bytes : g, P.half));
    } else {
      CNCCL(c, ncclGather(P.d_packed, nullptr, bytes, ncclChar, 0, m->comm, m->stream));
    }
  }
  CHIP(c, hipEventRecord(m->ev_gather[e % kRing], m->stream));
  m->nposted = e + 1;
  return CVR_OK;
}

cvr_status post_through(Ctx* c, Comm* m, long long last) {
  while (m->nposted <= last && m->nposted < m->ngather) CTRY(post_data(c, m, m->nposted));
  return CVR_OK;
}

// The event that marks exchange e done for the reuse of its buffers: rank 0's (it
// reads every rank's buffers) under the in-process transport, else this rank's.
cvr_status reuse_event(Ctx* c, Comm* m, long long e, hipEvent_t* out) {
  if (m->hub && m->rank != 0) {
    const Comm* m0 = root_comm(m);
    if (m0->nposted <= e)
      return cfail(c, CVR_ERR_STATE,
                   "local exchange %lld: rank 0 has not posted it yet (more buffer sets, or "
                   "call rank 0 after the others each round)", e);
    *out = m0->ev_gather[e % kRing];
    return CVR_OK;
  }
  CTRY(post_through(c, m, e));
  *out = m->ev_gather[e % kRing];
  return CVR_OK;
}

cvr_status comm_common_init(Ctx* c, Comm* m) {
  int lo = 0, hi = 0;
  CHIP(c, hipDeviceGetStreamPriorityRange(&lo, &hi));
  CHIP(c, hipStreamCreateWithPriority(&m->stream, hipStreamNonBlocking, hi));
  CHIP(c, hipStreamCreateWithPriority(&m->stream_sz, hipStreamNonBlocking, hi));
  CHIP(c, hipEventCreateWithFlags(&m->ev_render, hipEventDisableTiming));
  for (int i = 0; i < kRing; i++) {
    CHIP(c, hipEventCreateWithFlags(&m->ev_gather[i], hipEventDisableTiming));
    CHIP(c, hipEventCreateWithFlags(&m->ev_enc[i], hipEventDisableTiming));
    CHIP(c, hipEventCreateWithFlags(&m->ev_sz[i], hipEventDisableTiming));
  }
  return CVR_OK;
}

}  // namespace

namespace cvr {
// called by cvr_destroy / cvr_comm_destroy
void comm_release(Ctx* c) {
  Comm* m = comm_of(c);
  if (!m) return;
  (void)hipSetDevice(c->device);
  if (m->stream) (void)hipStreamSynchronize(m->stream);
  if (m->stream_sz) (void)hipStreamSynchronize(m->stream_sz);
  if (m->hub) {
    // the other members' streams may still read this context's buffers
    for (Ctx* o : m->hub->ctxs)
      if (o && o != c && o->comm) {
        (void)hipSetDevice(o->device);
        (void)hipStreamSynchronize(comm_of(o)->stream);
      }
    (void)hipSetDevice(c->device);
    for (Ctx*& o : m->hub->ctxs)
      if (o == c) o = nullptr;
    if (--m->hub->refs == 0) delete m->hub;
  }
  if (m->comm_sz) (void)ncclCommDestroy(m->comm_sz);
  if (m->comm) (void)ncclCommDestroy(m->comm);
  if (m->ev_render) (void)hipEventDestroy(m->ev_render);
  for (int i = 0; i < kRing; i++) {
    if (m->ev_gather[i]) (void)hipEventDestroy(m->ev_gather[i]);
    if (m->ev_enc[i]) (void)hipEventDestroy(m->ev_enc[i]);
    if (m->ev_sz[i]) (void)hipEventDestroy(m->ev_sz[i]);
  }
  for (CodeSet& S : m->sets) {
    if (S.send) (void)hipFree(S.send);
    if (S.ctr) (void)hipFree(S.ctr);
    if (S.recv) (void)hipFree(S.recv);
    if (S.d_sizes) (void)hipFree(S.d_sizes);
    if (S.h_sizes) (void)hipHostFree(S.h_sizes);
  }
  if (m->stream) (void)hipStreamDestroy(m->stream);
  if (m->stream_sz) (void)hipStreamDestroy(m->stream_sz);
  delete m;
  c->comm = nullptr;
}

long long comm_exchanges(const Ctx* c) {
  const Comm* m = comm_of(c);
  return m ? m->ngather : 0;
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
  if (c->group) return cfail(c, CVR_ERR_STATE, "cvr_comm_init: a group context exchanges internally");
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
  // the coded exchange's sizes travel on a communicator of their own, so their
  // gathers (issued right after each encode) never queue behind a data exchange
  if (nranks > 1) {
    r = ncclCommSplit(m->comm, 0, rank, &m->comm_sz, nullptr);
    if (r != ncclSuccess) {
      m->comm_sz = nullptr;
      cvr::comm_release(c);
      return cfail(c, CVR_ERR_HIP, "ncclCommSplit: %s", ncclGetErrorString(r));
    }
  }
  cvr_status st = comm_common_init(c, m);
  if (st != CVR_OK) {
    std::string e = c->err;
    cvr::comm_release(c);
    c->err = e;
  }
  return st;
}

cvr_status cvr_comm_init_local(cvr_ctx* const* ctxs, int n) {
  if (!ctxs || n < 1 || n > 1024) return CVR_ERR_ARG;
  for (int i = 0; i < n; i++) {
    Ctx* c = reinterpret_cast<Ctx*>(ctxs[i]);
    if (!c) return CVR_ERR_ARG;
    if (c->comm) return cfail(c, CVR_ERR_STATE, "cvr_comm_init_local: already initialised");
    if (c->group) return cfail(c, CVR_ERR_STATE, "cvr_comm_init_local: a group context exchanges internally");
    for (int j = 0; j < i; j++)
      if (ctxs[j] == ctxs[i]) return cfail(c, CVR_ERR_ARG, "cvr_comm_init_local: repeated context");
  }
  LocalHub* hub = new LocalHub();
  hub->ctxs.resize((size_t)n);
  for (int i = 0; i < n; i++) hub->ctxs[(size_t)i] = reinterpret_cast<Ctx*>(ctxs[i]);
  for (int i = 0; i < n; i++) {
    Ctx* c = hub->ctxs[(size_t)i];
    Comm* m = new Comm();
    c->comm = m;
    m->nranks = n;
    m->rank = i;
    m->hub = hub;
    hub->refs++;
    cvr_status st = hipSetDevice(c->device) == hipSuccess ? comm_common_init(c, m) : CVR_ERR_HIP;
    if (st != CVR_OK) {
      for (int j = 0; j <= i; j++) cvr::comm_release(hub->ctxs[(size_t)j]);
      return st;
    }
  }
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
  const bool idle = idle_root(c, m);
  const bool root_idle = idle && m->rank == 0;
  if (!f || (!d_packed && !root_idle) || nframes < 1 || nframes > 64 || tpr_max < 0 ||
      (f->nranks > 1 && f->tile_size < 16) ||
      (format != CVR_FORMAT_RGBA32F && format != CVR_FORMAT_RGBA16F))
    return cfail(c, CVR_ERR_ARG, "cvr_gather_tiles: bad arguments");
  const int want_nranks = idle ? m->nranks - 1 : m->nranks;
  const int want_rank = idle ? m->rank - 1 : m->rank;
  if (f->nranks != want_nranks || (f->rank != want_rank && !root_idle))
    return cfail(c, CVR_ERR_ARG, "cvr_gather_tiles: frame rank %d/%d, communicator %d/%d%s",
                 f->rank, f->nranks, m->rank, m->nranks, idle ? " (idle root)" : "");
  if (m->rank == 0 && (!d_gathered || !d_images))
    return cfail(c, CVR_ERR_ARG, "cvr_gather_tiles: rank 0 needs the gather buffer and images");
  const int k = root_idle ? 0 : (m->nranks > 1 ? cvr_tiles_for_rank(f, f->rank) : 0);
  if (m->nranks > 1 && k > tpr_max)
    return cfail(c, CVR_ERR_ARG, "cvr_gather_tiles: tiles_per_rank_max too small");
  CHIP(c, hipSetDevice(c->device));
  const size_t px = format == CVR_FORMAT_RGBA16F ? 8 : 16;
  // one rank: the frames were rendered whole (row-major); the "gather" is a copy
  const size_t fbytes = m->nranks == 1 ? (size_t)f->width * f->height * px
                                       : (size_t)tpr_max * f->tile_size * f->tile_size * px;
  const bool code = c->exchange_code && m->nranks > 1 && format == CVR_FORMAT_RGBA16F &&
                    f->tile_size <= 32;   // (the encode stages 8 tiles in LDS)
  if (code && nframes > cvr::kMaxLaunchFrames)
    return cfail(c, CVR_ERR_ARG, "cvr_gather_tiles: the coded exchange takes at most %d frames",
                 cvr::kMaxLaunchFrames);
  const long long g = m->ngather;
  const int B = buffer_sets(c);
  const int set = (int)(g % B);
  // the ring of pending exchanges must not overrun unposted entries
  if (g - m->nposted >= kRing) CTRY(post_through(c, m, g - kRing));
  Pending& P = m->pend[g % kRing];
  P = Pending();
  P.set = set;
  P.nframes = nframes;
  P.tpr = tpr_max;
  P.k = k;
  P.code = code;
  P.d_packed = d_packed;
  P.d_gathered = d_gathered;
  P.f = *f;
  P.fbytes = fbytes;
  P.half = format == CVR_FORMAT_RGBA16F;
  if (m->rank == 0)
    for (int j = 0; j < nframes; j++) P.images[j] = d_images[j];
  hipStream_t s = c->stream;
  const hipStream_t rs = m->stream_sz;
  const int ki = g % kRing;
  // phase A: this rank's tiles are ready (encoded) and its stream size is on its way
  if (code) {
    const int nsrc = idle ? m->nranks - 1 : m->nranks;
    const size_t bound = cvr::tile_code_bound_bytes(f->tile_size, tpr_max * nframes);
    CTRY(ensure_set(c, m, set, m->rank == 0 ? 0 : bound, bound, nsrc));
    P.recv_slot = bound;
    CodeSet& S = m->sets[(size_t)set];
    if (!(m->rank == 0)) {
      // the length lands in d_size (for the sizes' gather) and in mapped host memory
      CHIP(c, cvr::launch_exchange_encode(d_packed, f->tile_size, k, tpr_max, nframes, S.send, S.ctr,
                                          S.d_size, S.h_sizes_dev, s));
    }
    CHIP(c, hipEventRecord(m->ev_enc[ki], s));
    if (m->comm_sz) {
      CHIP(c, hipStreamWaitEvent(rs, m->ev_enc[ki], 0));
      if (m->rank == 0) {
        // rank 0 contributes its slot's zero (its own tiles, if any, stay raw in block 0)
        CNCCL(c, ncclGather(S.d_sizes, S.d_sizes, sizeof(unsigned long long), ncclChar, 0,
                            m->comm_sz, rs));
        CHIP(c, hipMemcpyAsync(S.h_sizes, S.d_sizes, sizeof(unsigned long long) * (size_t)m->nranks,
                               hipMemcpyDeviceToHost, rs));
        CHIP(c, hipEventRecord(m->ev_sz[ki], rs));
      } else {
        CNCCL(c, ncclGather(S.d_size, nullptr, sizeof(unsigned long long), ncclChar, 0, m->comm_sz,
                            rs));
      }
    }
  } else {
    CHIP(c, hipEventRecord(m->ev_enc[ki], s));
  }
  m->ngather = g + 1;
  // phase B of the exchanges that are `lag` behind
  const int lag = code ? effective_lag(c, m) : 0;
  if (!(m->hub && m->rank != 0)) CTRY(post_through(c, m, g - lag));
  // One render stream and two buffers: the next render reuses the buffers of the
  // previous exchange, so the stream waits for the previous exchange (this one
  // overlaps the next render).  D >= 2 streams rotated with B >= D buffer sets
  // (option "gather_sets", a multiple of D; exchange g uses set g % B on stream
  // g % D): this stream's next render (exchange g + D) writes set (g + D) % B,
  // last used by exchange g + D - B, so the stream waits for that one -- with
  // B = D this exchange, with B = 4D one issued three rounds earlier, which has
  // usually finished, so a slow exchange no longer stalls the render pipeline.
  const int D = std::max(c->split_streams, 1);
  const long long w = g + D - B;
  if (w >= 0) {
    hipEvent_t ev = nullptr;
    CTRY(reuse_event(c, m, w, &ev));
    CHIP(c, hipStreamWaitEvent(s, ev, 0));
  }
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
  hipEvent_t ev = nullptr;
  CTRY(reuse_event(c, m, m->ngather - 1, &ev));
  CHIP(c, hipStreamWaitEvent(c->stream, ev, 0));
  return CVR_OK;
}

}  // extern "C"
#pragma GCC visibility pop
