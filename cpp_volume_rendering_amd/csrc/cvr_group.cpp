// cvr_group.cpp — one context over several GPUs in ONE process (cvr_create_group).
//
// The reference renders from a single GL thread (app_freeglut.cpp:125,174 enter
// glutMainLoop; renderingmanager.cpp:199-208 calls Redraw from it), so a plugin
// that wants the node's GPUs cannot be one process per GPU.  A group context
// holds one member context per device (a device may repeat: the one-GPU tests
// run 3 and 8 members on device 0).  Its state setters fan out to every member,
// and its render calls split the frame into 16 x 16 screen tiles on the diagonal
// lattice (cvr::split_tile), render member i's share on member i's device and
// stream, and exchange the tiles to member 0 over the in-process transport of
// cvr_comm.cpp (device copies over xGMI; RGBA16F frames as the per-tile code,
// decoded straight into the caller's image in one launch).  Per-pixel sample
// counts and the sample total, when asked for, are gathered beside it.
//
// A group render returns with the frame queued on the group's stream, as a
// single context's render does; consecutive group frames do not overlap (each
// member's next render waits for the previous frame's exchange).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <vector>

#include "cvr_internal.h"

using cvr::Ctx;

namespace cvr {

struct Group {
  std::vector<Ctx*> members;
  struct Member {
    void* packed = nullptr;           // its tiles (member 0: unused, it renders into `gathered`)
    size_t packed_cap = 0;
    void* samples = nullptr;          // its per-pixel counts, packed like the tiles
    size_t samples_cap = 0;
    unsigned long long* total = nullptr;
    hipEvent_t ev_done = nullptr;     // its render of the current frame is done
  };
  std::vector<Member> mb;
  void* gathered = nullptr;           // device 0: n blocks of nframes x tpr tiles (block 0 = member 0's)
  size_t gathered_cap = 0;
  void* gsamples = nullptr;           // device 0: the members' counts, gathered
  size_t gsamples_cap = 0;
  unsigned long long* totals = nullptr;   // device 0: [n]
  void* stage = nullptr;              // device 0: images / counts of host outputs
  size_t stage_cap = 0;
  hipEvent_t ev_frame = nullptr;      // the previous group frame is done (device 0)
  bool has_frame = false;
};

namespace {

cvr_status gfail(Ctx* c, cvr_status st, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  c->err = buf;
  return st;
}

#define GHIP(ctx, expr)                                                                  \
  do {                                                                                   \
    hipError_t _e = (expr);                                                              \
    if (_e != hipSuccess)                                                                \
      return gfail(ctx, _e == hipErrorOutOfMemory ? CVR_ERR_OOM : CVR_ERR_HIP,           \
                   "%s: %s (%s:%d)", #expr, hipGetErrorString(_e), __FILE__, __LINE__);  \
  } while (0)

// a member's failure, reported on the group with the member's message
cvr_status member_fail(Ctx* g, int i, cvr_status st) {
  g->err = "group member " + std::to_string(i) + ": " + g->group->members[(size_t)i]->err;
  return st;
}

// every member's device idle (before a buffer is replaced)
cvr_status drain(Ctx* g) {
  for (Ctx* m : g->group->members) {
    GHIP(g, hipSetDevice(m->device));
    GHIP(g, hipDeviceSynchronize());
  }
  GHIP(g, hipSetDevice(g->device));
  GHIP(g, hipDeviceSynchronize());
  return CVR_OK;
}

cvr_status grow_on(Ctx* g, int device, void** p, size_t* cap, size_t want) {
  if (*p && *cap >= want) return CVR_OK;
  if (*p) {
    cvr_status st = drain(g);
    if (st != CVR_OK) return st;
    GHIP(g, hipSetDevice(device));
    (void)hipFree(*p);
    *p = nullptr;
    *cap = 0;
  }
  GHIP(g, hipSetDevice(device));
  GHIP(g, hipMalloc(p, want));
  *cap = want;
  return CVR_OK;
}

__global__ void sum_totals_kernel(const unsigned long long* __restrict__ t, int n,
                                  unsigned long long* __restrict__ out, int add) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  unsigned long long s = 0;
  for (int i = 0; i < n; i++) s += t[i];
  if (add) atomicAdd(out, s);
  else *out = s;
}

}  // namespace

void group_release(Ctx* g) {
  Group* G = g->group;
  if (!G) return;
  (void)drain(g);
  for (size_t i = 0; i < G->members.size(); i++) {
    Ctx* m = G->members[i];
    Group::Member& b = G->mb[i];
    (void)hipSetDevice(m->device);
    if (b.packed) (void)hipFree(b.packed);
    if (b.samples) (void)hipFree(b.samples);
    if (b.total) (void)hipFree(b.total);
    if (b.ev_done) (void)hipEventDestroy(b.ev_done);
  }
  // members release their communicator (and the shared hub) as they go
  for (Ctx* m : G->members) cvr_destroy(reinterpret_cast<cvr_ctx*>(m));
  (void)hipSetDevice(g->device);
  if (G->gathered) (void)hipFree(G->gathered);
  if (G->gsamples) (void)hipFree(G->gsamples);
  if (G->totals) (void)hipFree(G->totals);
  if (G->stage) (void)hipFree(G->stage);
  if (G->ev_frame) (void)hipEventDestroy(G->ev_frame);
  delete G;
  g->group = nullptr;
}

cvr_status group_each(Ctx* g, const std::function<cvr_status(cvr_ctx*)>& fn) {
  Group* G = g->group;
  for (size_t i = 0; i < G->members.size(); i++) {
    cvr_status st = fn(reinterpret_cast<cvr_ctx*>(G->members[i]));
    if (st != CVR_OK) return member_fail(g, (int)i, st);
  }
  return CVR_OK;
}

Ctx* group_root(Ctx* g) {
  Ctx* r = g->group->members[0];
  r->stream = g->stream;
  return r;
}

cvr_status group_call_root(Ctx* g, const std::function<cvr_status(cvr_ctx*)>& fn) {
  Ctx* r = group_root(g);
  cvr_status st = fn(reinterpret_cast<cvr_ctx*>(r));
  return st == CVR_OK ? st : member_fail(g, 0, st);
}

cvr_status group_render(Ctx* g, const cvr_frame* frames, int nf, const cvr_output* outs,
                        const MemberRender& render) {
  Group* G = g->group;
  const int n = (int)G->members.size();
  if (!frames || !outs || nf < 1 || nf > kMaxLaunchFrames)
    return gfail(g, CVR_ERR_ARG, "group render: bad arguments");
  const cvr_frame& f0 = frames[0];
  const cvr_output& o0 = outs[0];
  if (f0.width < 1 || f0.height < 1 || f0.width > 32768 || f0.height > 32768)
    return gfail(g, CVR_ERR_ARG, "group render: bad viewport %dx%d", f0.width, f0.height);
  if (o0.format != CVR_FORMAT_RGBA32F && o0.format != CVR_FORMAT_RGBA16F)
    return gfail(g, CVR_ERR_ARG, "group render: unknown output format %d", o0.format);
  for (int j = 0; j < nf; j++) {
    if (frames[j].nranks > 1)
      return gfail(g, CVR_ERR_ARG, "group render: the group splits the frame itself (nranks must be <= 1)");
    if (frames[j].width != f0.width || frames[j].height != f0.height)
      return gfail(g, CVR_ERR_ARG, "group render: frame %d's viewport differs", j);
    if (!outs[j].rgba || outs[j].format != o0.format || outs[j].on_device != o0.on_device)
      return gfail(g, CVR_ERR_ARG, "group render: output %d differs from output 0", j);
    if (j > 0 && outs[j].total)
      return gfail(g, CVR_ERR_ARG, "group render: only output 0 may carry a total");
  }
  if (nf > 1 && !o0.on_device)
    return gfail(g, CVR_ERR_ARG, "group render: several frames need device outputs");
  const bool half = o0.format == CVR_FORMAT_RGBA16F;
  const size_t px = half ? 8 : 16;
  const int T = 16;
  cvr_frame tmpl = f0;
  tmpl.tile_size = T;
  tmpl.nranks = n;
  tmpl.rank = 0;
  const int tpr = n > 1 ? cvr_tiles_for_rank(&tmpl, 0) : 0;
  const size_t npx_img = (size_t)f0.width * f0.height;
  const size_t frame_tiles_px = n > 1 ? (size_t)tpr * T * T : npx_img;   // pixels per frame and member
  const bool want_samples = std::any_of(outs, outs + nf, [](const cvr_output& o) { return o.samples != nullptr; });
  const bool want_total = o0.total != nullptr;
  // buffers (device 0 unless noted)
  cvr_status st;
  st = grow_on(g, g->device, &G->gathered, &G->gathered_cap, (size_t)n * nf * frame_tiles_px * px);
  if (st != CVR_OK) return st;
  if (want_samples) {
    st = grow_on(g, g->device, &G->gsamples, &G->gsamples_cap, (size_t)n * nf * frame_tiles_px * 4);
    if (st != CVR_OK) return st;
  }
  if (!o0.on_device) {
    st = grow_on(g, g->device, &G->stage, &G->stage_cap, npx_img * (px + (want_samples ? 4 : 0)));
    if (st != CVR_OK) return st;
  }
  if (!G->totals) {
    GHIP(g, hipSetDevice(g->device));
    GHIP(g, hipMalloc((void**)&G->totals, sizeof(unsigned long long) * (size_t)n));
  }
  for (int i = 1; i < n; i++) {
    Group::Member& b = G->mb[(size_t)i];
    const int dev = G->members[(size_t)i]->device;
    st = grow_on(g, dev, &b.packed, &b.packed_cap, (size_t)nf * frame_tiles_px * px);
    if (st != CVR_OK) return st;
    if (want_samples) {
      st = grow_on(g, dev, &b.samples, &b.samples_cap, (size_t)nf * frame_tiles_px * 4);
      if (st != CVR_OK) return st;
    }
  }
  GHIP(g, hipSetDevice(g->device));
  hipStream_t s0 = g->stream;
  // the images the exchange writes: the caller's (device outputs) or the staging area
  void* images[kMaxLaunchFrames] = {};
  uint32_t* smp_dst[kMaxLaunchFrames] = {};
  for (int j = 0; j < nf; j++) {
    if (o0.on_device) {
      images[j] = outs[j].rgba;
      smp_dst[j] = static_cast<uint32_t*>(outs[j].samples);
    } else {   // host outputs: one frame (checked above)
      images[j] = G->stage;
      smp_dst[j] = outs[j].samples ? reinterpret_cast<uint32_t*>(static_cast<char*>(G->stage) + npx_img * px)
                                   : nullptr;
    }
  }
  // Members 1..n-1 first, member 0 last (the in-process transport's order): render
  // the share, then hand its tiles to the exchange.
  for (int q = 1; q <= n; q++) {
    const int i = q % n;
    Ctx* m = G->members[(size_t)i];
    Group::Member& b = G->mb[(size_t)i];
    if (i == 0) m->stream = s0;
    GHIP(g, hipSetDevice(m->device));
    hipStream_t ms = m->stream;
    if (G->has_frame && i != 0) GHIP(g, hipStreamWaitEvent(ms, G->ev_frame, 0));
    cvr_frame mf[kMaxLaunchFrames];
    cvr_output mo[kMaxLaunchFrames];
    char* base = i == 0 ? static_cast<char*>(G->gathered) : static_cast<char*>(b.packed);
    char* sbase = want_samples ? (i == 0 ? static_cast<char*>(G->gsamples) : static_cast<char*>(b.samples))
                               : nullptr;
    if (want_total) {
      if (!b.total) GHIP(g, hipMalloc((void**)&b.total, sizeof(unsigned long long)));
      GHIP(g, hipMemsetAsync(b.total, 0, sizeof(unsigned long long), ms));
    }
    for (int j = 0; j < nf; j++) {
      mf[j] = frames[j];
      if (n > 1) {
        mf[j].tile_size = T;
        mf[j].rank = i;
        mf[j].nranks = n;
      }
      mo[j].rgba = base + (size_t)j * frame_tiles_px * px;
      mo[j].samples = sbase && outs[j].samples ? sbase + (size_t)j * frame_tiles_px * 4 : nullptr;
      mo[j].total = (j == 0 && want_total) ? b.total : nullptr;
      mo[j].on_device = 1;
      mo[j].format = o0.format;
    }
    st = render(reinterpret_cast<cvr_ctx*>(m), mf, nf, mo);
    if (st != CVR_OK) return member_fail(g, i, st);
    GHIP(g, hipSetDevice(m->device));
    if (!b.ev_done) GHIP(g, hipEventCreateWithFlags(&b.ev_done, hipEventDisableTiming));
    GHIP(g, hipEventRecord(b.ev_done, m->stream));
    if (n > 1) {
      st = cvr_gather_tiles_n(reinterpret_cast<cvr_ctx*>(m), &mf[0], nf, base, tpr, o0.format,
                              i == 0 ? G->gathered : nullptr, i == 0 ? images : nullptr);
      if (st != CVR_OK) return member_fail(g, i, st);
    }
  }
  Ctx* r = G->members[0];
  GHIP(g, hipSetDevice(g->device));
  if (n > 1) {
    st = cvr_gather_sync(reinterpret_cast<cvr_ctx*>(r));   // s0 waits for the decode
    if (st != CVR_OK) return member_fail(g, 0, st);
  } else {
    // one member: it rendered whole frames into `gathered`
    for (int j = 0; j < nf; j++)
      GHIP(g, hipMemcpyAsync(images[j], static_cast<char*>(G->gathered) + (size_t)j * npx_img * px,
                             npx_img * px, hipMemcpyDeviceToDevice, s0));
  }
  // counts and totals: pulled from the members after their renders
  if (want_samples || want_total) {
    for (int i = 1; i < n; i++) {
      Group::Member& b = G->mb[(size_t)i];
      GHIP(g, hipStreamWaitEvent(s0, b.ev_done, 0));
      if (want_samples)
        GHIP(g, hipMemcpyAsync(static_cast<char*>(G->gsamples) + (size_t)i * nf * frame_tiles_px * 4, b.samples,
                               (size_t)nf * frame_tiles_px * 4, hipMemcpyDefault, s0));
      if (want_total)
        GHIP(g, hipMemcpyAsync(G->totals + i, b.total, sizeof(unsigned long long), hipMemcpyDefault, s0));
    }
    if (want_total)
      GHIP(g, hipMemcpyAsync(G->totals, G->mb[0].total, sizeof(unsigned long long), hipMemcpyDeviceToDevice, s0));
    if (want_samples) {
      for (int j = 0; j < nf; j++) {
        if (!smp_dst[j]) continue;
        const uint32_t* src = reinterpret_cast<const uint32_t*>(G->gsamples) + (size_t)j * frame_tiles_px;
        if (n > 1) {
          GHIP(g, launch_unpack_tiles_u32(src, smp_dst[j], f0.width, f0.height, T, n, tpr, s0,
                                          (size_t)nf * tpr));
        } else {
          GHIP(g, hipMemcpyAsync(smp_dst[j], src, npx_img * 4, hipMemcpyDeviceToDevice, s0));
        }
      }
    }
  }
  unsigned long long* d_sum = nullptr;
  if (want_total) {
    d_sum = o0.on_device ? static_cast<unsigned long long*>(o0.total) : G->totals + 0;
    if (o0.on_device) {
      hipLaunchKernelGGL(sum_totals_kernel, dim3(1), dim3(64), 0, s0, G->totals, n, d_sum, 1);
    } else {
      // host total: sum in place into totals[0] after reading all of them
      hipLaunchKernelGGL(sum_totals_kernel, dim3(1), dim3(64), 0, s0, G->totals, n, G->totals, 0);
    }
    GHIP(g, hipGetLastError());
  }
  if (!G->ev_frame) GHIP(g, hipEventCreateWithFlags(&G->ev_frame, hipEventDisableTiming));
  GHIP(g, hipEventRecord(G->ev_frame, s0));
  G->has_frame = true;
  if (!o0.on_device) {
    GHIP(g, hipMemcpyAsync(o0.rgba, G->stage, npx_img * px, hipMemcpyDeviceToHost, s0));
    if (o0.samples)
      GHIP(g, hipMemcpyAsync(o0.samples, static_cast<char*>(G->stage) + npx_img * px, npx_img * 4,
                             hipMemcpyDeviceToHost, s0));
    if (want_total)
      GHIP(g, hipMemcpyAsync(o0.total, G->totals, sizeof(unsigned long long), hipMemcpyDeviceToHost, s0));
    GHIP(g, hipStreamSynchronize(s0));
  }
  return CVR_OK;
}

}  // namespace cvr

#pragma GCC visibility push(default)
extern "C" {

cvr_status cvr_create_group(const int* devices, int n, cvr_ctx** out_ctx) {
  if (!out_ctx) return CVR_ERR_ARG;
  *out_ctx = nullptr;
  if (!devices || n < 1 || n > 64) return CVR_ERR_ARG;
  cvr_ctx* gh = nullptr;
  cvr_status st = cvr_create(devices[0], &gh);
  if (st != CVR_OK) return st;
  Ctx* g = reinterpret_cast<Ctx*>(gh);
  g->group = new cvr::Group();
  cvr::Group* G = g->group;
  std::vector<cvr_ctx*> hs;
  for (int i = 0; i < n; i++) {
    cvr_ctx* m = nullptr;
    st = cvr_create(devices[i], &m);
    if (st != CVR_OK) {
      g->err = "cvr_create_group: member " + std::to_string(i) + " on device " +
               std::to_string(devices[i]) + " could not be created";
      cvr_destroy(gh);
      return st;
    }
    G->members.push_back(reinterpret_cast<Ctx*>(m));
    G->mb.emplace_back();   // (kept the same length as members: a failed creation releases both)
    hs.push_back(m);
  }
  // members on other devices write nothing remote, but the exchange's device copies
  // and the counts' gathers use the xGMI path directly when peer access is on
  for (int i = 0; i < n; i++)
    for (int j = 0; j < n; j++) {
      const int a = devices[i], b = devices[j];
      int can = 0;
      if (a != b && hipDeviceCanAccessPeer(&can, a, b) == hipSuccess && can) {
        (void)hipSetDevice(a);
        const hipError_t e = hipDeviceEnablePeerAccess(b, 0);
        if (e != hipSuccess && e != hipErrorPeerAccessAlreadyEnabled) {
          cvr_destroy(gh);
          return CVR_ERR_HIP;
        }
        (void)hipGetLastError();
      }
    }
  (void)hipSetDevice(devices[0]);
  if (n > 1) {
    st = cvr_comm_init_local(hs.data(), n);
    if (st != CVR_OK) {
      cvr_destroy(gh);
      return st;
    }
  }
  // one render stream per member, two buffer sets, the exchange posted at once
  for (cvr_ctx* m : hs) {
    (void)cvr_set_option(m, "split_streams", 1);
    (void)cvr_set_option(m, "gather_sets", 2);
    (void)cvr_set_option(m, "exchange_lag", 0);
  }
  *out_ctx = gh;
  return CVR_OK;
}

int cvr_group_size(const cvr_ctx* ctx) {
  const Ctx* c = reinterpret_cast<const Ctx*>(ctx);
  if (!c) return 0;
  return c->group ? (int)c->group->members.size() : 1;
}

cvr_ctx* cvr_group_member(cvr_ctx* ctx, int i) {
  Ctx* c = reinterpret_cast<Ctx*>(ctx);
  if (!c || !c->group || i < 0 || i >= (int)c->group->members.size()) return nullptr;
  return reinterpret_cast<cvr_ctx*>(c->group->members[(size_t)i]);
}

}  // extern "C"
#pragma GCC visibility pop
