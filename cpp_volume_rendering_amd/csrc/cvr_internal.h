// cvr_internal.h — context state and kernel launch parameters shared by the
// C-ABI implementation (cvr_api.cpp) and the gfx950 kernels (raymarch.hip).
#pragma once

#include <hip/hip_runtime.h>
#include <cstdint>
#include <functional>
#include <string>
#include <vector>

#include "../../include/cvr.h"

namespace cvr {

// Padded-cell volume layout ("cell8"): cell (a,b,c), a in [0, N], holds the 8
// corner values that GL trilinear filtering reads for texel coordinate
// x in [a-1, a): corners clamp(a-1) and clamp(a) per axis (CLAMP_TO_EDGE).
// One sample = one 16-byte (fp16 corners) load.  Cells are x-fastest (a 4x4x4
// bricked order measured 6-18 % slower on the headline frame and was dropped).
struct CellGrid {
  int cx, cy, cz;           // cells per axis = N + 1
  int pitch_y, pitch_z;     // cx, cx*cy
  long long linear_origin;  // index of cell (1,1,1) = texel (0,0,0)
  int bpitch_y, bpitch_z;   // the pitches in bytes (16 B per cell)
  uint32_t borigin;         // linear_origin * 16, mod 2^32 (byte offsets of buffer loads)
};

// Screen-tile split: which TxT tile is rank r's k-th.  Tiles
// are numbered in a virtual row-major order in which tile row ty is rotated by
// s*ty tiles, and virtual tile v belongs to rank v mod N.  When N divides the
// tiles per row, rank(tx, ty) = (tx + s*ty) mod N: a diagonal lattice instead
// of the columns plain t mod N gives (tools/split_balance.py, samples max/mean
// over ranks on four reference camera views at 1024^2, 16^2 tiles, N = 8:
// columns up to 1.21, s = 3 at most 1.014).  Any s keeps the per-rank counts of
// t mod N (cvr_tiles_for_rank).
__host__ __device__ inline int split_shift(int nranks) { return nranks >= 4 ? 3 : 1; }
__host__ __device__ inline void split_tile(int rank, int nranks, int k, int ntx, int& tx, int& ty) {
  const int v = rank + k * nranks;
  ty = v / ntx;
  const int xv = v - ty * ntx;
  tx = xv - (int)(((long long)split_shift(nranks) * ty) % ntx);
  if (tx < 0) tx += ntx;
}

// Per-frame constants of the rc1pass kernel (passed by value).
struct Rc1passArgs {
  // ray generation (ray_marching_1p.comp:87-99)
  float eye[3];
  float col0[3], col1[3], col2[3];   // columns of mat3(View)
  float tan_half_fovy, aspect;
  float inv_w, inv_h;                // unused: exact division by W/H is used
  int W, H;
  // volume grid (rc1prenderer.cpp:233-258)
  float half_grid[3];                // VolumeGridSize / 2
  float n_over_g[3];                 // N / VolumeGridSize  (texel space)
  float nm1[3];                      // N - 1 (float)
  int N[3];
  CellGrid cells;
  float step;
  int tf_n;
  int exp_fast;                      // 1: every -(alpha*h) lies in [-86, 0] (no exp range checks)
  int exp_native;                    // tolerance mode (option native_exp): v_exp_f32, not CVR-SPEC
  // Blinn-Phong (ray_marching_1p.comp:48-81)
  float ka, kd, ks, shininess;
  float ispec[3];
  float light[3];
  // screen-tile split (cvr_frame)
  int tile, rank, nranks, ntx, my_tiles;
  int packed;
  int interleave;                    // no launch order: tile t on block t (XCD t % 8) instead of XCD bands
  int out_half;                      // 1: store RGBA16F (uint2 per pixel), 0: float4
  int ntiles;                        // 8x8 wave tiles of this launch
  unsigned long long* tile_stats;    // diagnostics (tile_stats option) or null
  unsigned long long* shade_ctr;     // measurement (shade_counters): [0] += shaded samples (Phong),
                                     // [1] += samples the cell skip stepped over without a load
  int cost_time;                     // LPT cost = measured tile time (1) or longest ray (0)
  // empty-space skipping: occupancy byte per macro cell (null = off)
  const uint8_t* occ;
  int mdim[3];                       // macro cells per axis
  int mshift;                        // macro cell = 2^mshift texels a side
  // GL texture-unit filter mode (option "filter_bits"): 0 = exact float weights
  // (CVR-SPEC), 8 = every GL_LINEAR weight (volume, gradient, TF) rounded to 8
  // fraction bits, as GPU texture units filter (CVR-SPEC-8)
  int filter_bits;
  // per-cell skip (march_common.h cell_empty): 0 off, 1 empty-sample flags,
  // 2 flags + distance skip; inv_step = 1 / step (the full-step bound)
  int cell_skip;
  float inv_step;
};

constexpr int kMaxTfLds = 4096;          // TF entries a kernel stages into LDS
constexpr int kMaxExtLevels = 16;        // extinction mip levels (up to 32768^3)

// One level of the extinction pyramid as the cone fetches address it.
struct ExtLevel {
  int off;                           // first cell8 texel of the level
  int dx, dy, dz;                    // dimensions
  float sx, sy, sz;                  // d / G: texel coordinate = fma(p, d/G, -0.5)
  float mx, my, mz;                  // d - 1 (clamp-to-edge bound)
  int pad[2];
};

// Directional-occlusion shading (dos.hip): one cone's tables on the device.
// Early exit of a cone stage (dos.hip cone_stage): per stage, the sections where
// the border scale 2^-(2 floor(mip) + 1) changes ("runs": first section, its
// tap distance `track`, the scale) and the track after the stage's last section,
// all by the kernel's own float recurrence on the fp16-rounded table.
constexpr int kMaxConeRuns = 12;
struct ConeStageExit {
  int nruns;                         // 0: no exit test for this stage
  int end_s;                         // first section after the stage
  float end_track;                   // track after the stage's last section
  int run_first[kMaxConeRuns];
  float run_t[kMaxConeRuns], run_inv[kMaxConeRuns];
};

struct DosCone {
  int counts[3];                     // sections of 1, 3, 7 rays
  float initial_step, ray7w, ui_weight;
  float axes[30];                    // 3-ray then 7-ray axes (x, y, z)
  const float4* sections;            // (interval, mip, d_integral, amplitude), fp16-rounded
  ConeStageExit exit[3];
};

struct DosArgs {
  Rc1passArgs a;                     // ray, volume, TF, Blinn-Phong constants, tiles
  float G[3];                        // VolumeScaledSizes
  int ext_levels;
  const struct ExtLevel* levels;     // per level, device memory (read by scalar loads)
  int apply_occlusion, apply_shadow, shadow_type, phong;
  float ka, kd, ks;                  // Kambient if occlusion, Kdiffuse/Kspecular if shadow, else 0
  float lfwd[3], lup[3], lright[3];  // light camera vectors (RenderingParameters)
  float spot_cos;                    // SpotLightMaxAngle uniform
  int zero_skip;                     // every pyramid value finite: taps with a 0 border factor are 0
  int count_taps;                    // shade_counters: count the taps fetched (measurement)
  DosCone occ, sdw;
};

// Extinction-based shading (ebs.hip): the SAT and the shader's uniforms.
struct EbsArgs {
  Rc1passArgs a;                     // ray, volume, TF, Blinn-Phong constants, tiles
  float S[3], G[3];                  // VolumeScales, VolumeScaledSizes
  float inv_vs[3];                   // 1 / (G + 2 S)
  float nsat[3], nsat_m1[3];         // SAT dims as float, and dims - 1
  int sat_dims[3];
  uint32_t sat_pz;                   // texels per SAT plane (the cell4 layout's z + 1 plane offset)
  float min_sat[3], max_sat[3];      // S / 2, G + 1.5 S
  int apply_occlusion, occ_shells;
  float occ_radius;
  // 1 / r^2 of shell i (r = R*(i+1)) and W_A = 1 / (R*shells)^2, computed on the host
  // with the shader's float expressions (the divisions are the same for every sample)
  static constexpr int kMaxAoShells = 64;
  float ao_w[kMaxAoShells];
  float ao_wa;
  int apply_shadow, shadow_type, phong;
  float p_cs, p_sn, n_cs, n_sn;      // cos / sin of +-DirSdwConeAngle
  int recip_cone;                    // cone angle <= 44 deg: cone-edge divisions by reciprocal (ebs.hip cone_div)
  float interval, initial_step, ui_weight, max_distance;
  float lfwd[3];
  float ka, kd, ks;                  // Kambient if occlusion, Kdiffuse/Kspecular if shadow, else 0
};

// Isosurface ray-casters with block skipping (iso.hip): the shaders' uniforms.
struct IsoArgs {
  Rc1passArgs a;                     // ray, volume, Blinn-Phong constants, tiles
  float G[3];                        // VolumeGridSize
  float nb[3];                       // numBlocks (vec3 uniform)
  int nbi[3];                        // the same as int (table addressing, REPEAT wrap)
  float iso, step_small, step_large, step_range;
  float half_block_len;              // length(G / numBlocks) * 0.5 (variant 1)
  float bs[3];                       // G / numBlocks (getBlockBounds' blockSize)
  float nhg[3];                      // -G * 0.5
  float inv_g[3];                    // 1 / G (the block index fast path, verified)
  float color[4];
};

// Several frames in one ray-march launch (cvr_render_rc1pass_frames): frame f
// takes workgroups [f * grid, (f + 1) * grid) and differs from frame 0 only in
// its view (camera) and its outputs.  grid is a multiple of 8 whenever the
// single-frame grid is, so workgroup b keeps XCD b % 8's share of the frame.
// interleave (under a launch order, grid a multiple of 8): workgroup
// 8 (n e + f) + x runs entry e of XCD band x of frame f, so the dispatcher hands
// out entry e of every frame before entry e + 1 of any -- each band's longest
// tiles of ALL frames start first (LPT over the launch, not per frame).
constexpr int kMaxLaunchFrames = 16;
struct FrameView {
  float eye[3];
  float col0[3], col1[3], col2[3];   // columns of mat3(View)
  float tan_half_fovy, aspect;
};
struct LaunchFrames {
  int n;                             // frames in the launch (1: a plain launch, the rest unused)
  int grid;                          // workgroups per frame
  int interleave;                    // 1: the frames' entries interleaved by launch-order entry (below)
  FrameView view[kMaxLaunchFrames];
  float4* out[kMaxLaunchFrames];
  uint32_t* samples[kMaxLaunchFrames];
};

// How one frame is cut into work: one 8x8 wave tile per workgroup.
struct RenderPlan {
  int ntiles;                        // 8x8 wave tiles (one workgroup each)
  int order_slots;                   // grid size under an LPT order (8 x entries per band)
  int boost;                         // per band, the first `boost` entries run at priority 2
  int quad_pct;                      // per band, this % of the longest tiles march 4 lanes/ray
  int keep;                          // diagnostics: >0 keeps only the first `keep` entries per band
  int max_seg;                       // most tiles one (work-balanced) band may take
  int epi_stop;                      // diagnostics: the epilogue stops after phase k (0 = full)
  const LaunchFrames* frames;        // null: one frame; else frames->n frames in one launch
};

constexpr int kMaxBandTiles = 8192;


// Flat shading of the DOS/EBS renderers (option "shade_flat", shaded_march.h):
// one frame's shading jobs in a single global list, shaded by a grid of their own
// and folded into the pixels afterwards.  Buffers grow on demand, one set per context.
// One set of flat-shading buffers (shaded_march.h launch_shaded_flat).  Each
// render stream gets its own set (Ctx::flat), so DOS/EBS frames on different
// streams pipeline; a set is sized from the totals of its earlier frames, read
// back without blocking (ev_read), and a frame whose list would not fit renders
// through the per-wave kernel instead, decided on the device (flag).
struct FlatJobs {
  uint32_t* tile_off = nullptr;             // jobs per 8x8 tile, scanned in place to offsets [tiles + 1]
  uint32_t* tile_roff = nullptr;            // march rounds with a job per tile, scanned likewise
  unsigned long long* masks = nullptr;      // per such round: the lanes that made a job (ballot)
  unsigned long long* total = nullptr;      // [3]: the frame's jobs, rounds, overflow flag (device)
  unsigned long long* h_total = nullptr;    // pinned host copy of an earlier frame's [3]
  float4* cam = nullptr;                    // the ray's camera direction per pixel slot
  float4* jobs = nullptr;                   // 2 float4 per job (+1 with Phong)
  float4* res = nullptr;                    // shaded rgb * alpha, alpha, per job
  int tiles = 0;                            // allocated 8x8 tiles
  size_t cap = 0;                           // allocated jobs (float4 units: cap * 3)
  size_t rcap = 0;                          // allocated round masks
  // host side of the set
  hipEvent_t ev_read = nullptr;             // h_total holds the totals of the frame recorded last
  hipEvent_t ev_done = nullptr;             // the set's last frame is done with its buffers
  bool pending_read = false;
  size_t want_jobs = 0, want_rounds = 0;    // the largest totals read back so far
  hipStream_t stream = nullptr;             // the render stream the set serves
  bool owned = false;
  long long last_use = -1;
};    // the epilogue sorts a band in LDS (32 KiB + group prefixes)

struct Ctx {
  int device = 0;
  hipStream_t own_stream = nullptr;
  hipStream_t stream = nullptr;
  std::string err;
  // volume
  int N[3] = {0, 0, 0};
  float scale[3] = {1, 1, 1};
  int bpv = 0;
  void* d_vox = nullptr;          // raw voxels (u8/u16), kept for gradient/precompute
  size_t vox_bytes = 0;
  void* d_cells = nullptr;        // cell8 fp16 layout
  size_t cells_bytes = 0;
  CellGrid cells{};
  uint16_t* d_lut = nullptr;      // raw value -> R16F bits (GetNormalizedSample)
  // empty-space skipping (option "macro": log2 of the macro cell, 0 = off)
  int macro_shift = 3;
  int mm_shift = -1;              // shift the macro min/max below was built for
  int mdim[3] = {0, 0, 0};
  uint32_t* d_macro_minmax = nullptr;
  uint8_t* d_occ = nullptr;
  int occ_valid = 0;              // occupancy matches the current volume, TF and shift
  float occ_empty = 0.0f;         // fraction of empty macro cells
  int skip_min_pct = 15;          // skipping is compiled in when >= this % of cells are empty
  int* d_tf_prefix = nullptr;     // count of padded TF entries with alpha > 0 before k
  // per-cell skip flags in the cells' sign bits (march_common.h cell_empty /
  // cell_skip_q; option "cell_skip": 0 off, 1 empty-sample flags, 2 flags + the
  // distance skip per lane, 3 (default) when every marching lane can, 4 by the
  // lanes that can; raymarch.hip march_ray); rebuilt lazily after the volume or TF changes
  int cell_skip = 3;
  int cell_flags_valid = 0;       // the cells' flags match the current TF
  int cell_flags_set = 0;         // the cells carry flags (of some TF)
  int cell_flags_oom = 0;         // the last flag build ran out of memory (retried after a volume / TF change)
  int debug_flags_oom = 0;        // tests (option "debug_cell_flags_oom"): the flag build reports OOM
  // transfer function (RGBA16F values as float)
  float* d_tf = nullptr;
  int tf_n = 0;
  float tf_max_alpha = 0.0f;         // largest (fp16-rounded) TF opacity; NaN if any is not finite
  // gradient (4 x fp16 per voxel, x-fastest)
  void* d_grad = nullptr;          // gradient cell8: 3 uint4 (x, y, z fp16 pairs) per volume cell
  size_t grad_bytes = 0;
  int grad_mode = 0;
  // march tuning: samples fetched per batch (2, 4; 0 = auto: 4, or 2 with Phong
  // shading, whose extra registers make occupancy worth more than a deeper batch)
  int batch = 0;
  int cost_time = 0;               // option "tile_cost": 0 longest ray, 1 measured time (worse)
  int max_waves_cu = 0;            // experiment (option "max_waves_cu"): cap residency via LDS
  int epi_stop = 0;                // diagnostics (option "debug_epi_stop")
  int debug_keep = 0;              // diagnostics (option "debug_keep"): render only the longest entries
  int band_cap_pct = 130;           // option "band_cap": most tiles a work-balanced XCD band may take, % of 1/8
  int boost_pct = 5;               // % of every band's longest entries run at raised priority
  int filter_bits = 0;             // GL_LINEAR weights at this many fraction bits (0 = exact; rc1pass)
  int quad_pct = 0;                // % of every band's longest tiles marched 4 lanes per ray
  int shade_counters = 0;          // DOS/EBS: count shaded and shadow-lit samples
  int shade_flat = 1;              // DOS/EBS: 1 = flat job list (FlatJobs), 0 = per-wave batches
  int flat_group = 8;              // flat shading: 64-job chunks per XCD turn (XCD-aware order)
  int debug_flat_limit = 0;        // tests: a frame with more jobs takes the per-wave fallback
  static constexpr int kFlatSets = 16;    // flat-shading buffer sets, one per render stream
  mutable FlatJobs flat[kFlatSets];
  mutable long long flat_clock = 0;
  unsigned long long* d_shade = nullptr;   // [3]: shaded, lit, secondary fetches (last frame)
  int tile_stats = 0;              // record per-tile timing (diagnostics)
  unsigned long long* d_tile_stats = nullptr;
  int tile_stats_n = 0;
  // kernel_timing option: HIP events around every frame's ray-march launch (ring)
  std::vector<hipEvent_t> ev_start, ev_stop;
  long long timed_frames = 0;
  int use_order = 1;               // 1: longest-first (LPT) from an earlier frame's costs;
                                   // 0: screen order in XCD bands; 2: screen order interleaved over XCDs
  // The LPT order is built off the critical path: frame i's costs are sorted
  // on a side stream while frames i+1, i+2 render, and frame i+3 uses the
  // result (kOrderSlots slots in rotation; frame i uses and refills slot
  // i % kOrderSlots).  With two slots the sort, which only gets CUs in the
  // next frame's tail, still held up the frame after (~11 us per frame).
  struct OrderSlot {
    int* d_order = nullptr;        // launch order (8 x slots per band)
    uint32_t* d_cost = nullptr;    // per-wave-tile critical path, written by the frame
    int units = 0;                 // order entries allocated
    int ntiles = 0;                // cost entries allocated
    int key = -1;                  // plan signature of the order in d_order
    int valid = 0;
    hipEvent_t done = nullptr;     // the side-stream sort of this slot has finished
    bool pending = false;
    hipStream_t stream = nullptr;  // render stream that owns the slot (async_order 0)
    bool owned = false;
    long long frames = 0;          // frames rendered with this slot
    float view[7] = {0};           // eye, unit forward, tan(fovy/2) of the frame the order came from
    bool has_view = false;
    float last_view[7] = {0};      // the previous frame's view on this slot
    bool has_last = false;
  };
  int stale_deg = 5;               // option "stale_deg": an order learned on a view more than this
                                   // far away (degrees / 1/12 of the eye distance) is not used
  static constexpr int kOrderSlots = 32;  // one per render stream (async_order uses the first 3)
  int async_order = 0;             // option "async_order": 1 = sort on a side stream (lag 3)
  int order_interval = 8;          // option "order_interval": rebuild the order every n-th frame
  OrderSlot oslot[kOrderSlots];
  int slot_rr = 0;                 // next slot handed to a new render stream
  long long frame_no = 0;
  hipStream_t side = nullptr;      // high-priority stream for the order builds
  hipEvent_t ev_frame = nullptr;   // end of a frame's ray-march (the side stream waits on it)
  int num_cus = 0;
  // extinction-coefficient mip volume (directional occlusion)
  uint16_t* d_ext = nullptr;       // fp16 levels, concatenated (x-fastest)
  uint4* d_ext_cells = nullptr;    // the same levels as cell8 (8 fp16 corners per texel)
  ExtLevel* d_ext_levels = nullptr;  // [kMaxExtLevels] addressing of the levels
  // extinction-based shading: the float SAT of (N+2) cells per axis
  int sat_chunk = 32;                // z planes per SAT work item (option "sat_chunk")
  int sat_build_us = 0;              // GPU time of the last SAT build (option "sat_build_us")
  float* d_sat = nullptr;
  float4* d_sat_cells = nullptr;   // the same SAT as cell4 texels (4 float corners of a plane, sat.hip)
  int sat_layout = 0;              // option "sat_layout": the frame reads 0 = cell4 copy, 1 = the plain SAT
  int sat_keep_scratch = 0;        // option "sat_keep_scratch": 1 keeps the double build grid for rebuilds
  void* d_sat_scratch = nullptr;   // the double grid of the build (kept for rebuilds)
  int sat_dims[3] = {0, 0, 0};
  int ext_res[3] = {0, 0, 0};
  int ext_levels = 0;
  int ext_finite = 0;                // every TF opacity < 1: the pyramid's extinctions are finite
  long long ext_off[kMaxExtLevels + 1] = {};
  float ext_sigma0 = 1.0f;
  // cone tables on the device (occlusion, shadow), rebuilt when their params change
  float4* d_cones = nullptr;
  cvr_cone_params cone_key[2] = {};
  int cone_valid = 0;
  cvr_cone_tables* cone_tab = nullptr;   // host copies [2]
  unsigned long long* d_tile_samples = nullptr;   // per-wave-tile sample counts (zeroed)
  int tile_samples_n = 0;
  // d_tile_samples and d_shade are one set per context: a frame that uses them on
  // another stream than the previous user waits for that frame (counters_guard)
  hipStream_t counters_stream = nullptr;
  hipEvent_t ev_counters = nullptr;
  // isosurface block table (float2 min/max per block), built for iso_nb
  float2* d_iso_mm = nullptr;
  int iso_nb[3] = {0, 0, 0};
  int iso_valid = 0;               // matches the current volume and iso_nb
  // multi-GPU gather (cvr_comm.cpp): RCCL communicator, its stream and events
  void* comm = nullptr;
  int split_streams = 1;           // option "split_streams": render streams the caller rotates
  int gather_sets = 0;             // option "gather_sets": buffer sets the caller rotates (>= split_streams)
  int launch_interleave = 1;       // option "launch_interleave": multi-frame launches deal the frames'
                                   // launch-order entries interleaved (LaunchFrames::interleave)
  int gather_root_idle = 0;        // option "gather_root_idle": rank 0 only gathers (renders nothing)
  int exchange_code = 1;           // option "exchange_code": RGBA16F exchanges move the per-tile code
  int native_exp = 0;               // option "native_exp": tolerance mode (v_exp_f32 in the EA composite)
  int encode_onepass = 0;          // option "encode_onepass": cvr_encode_tiles uses the exchange's
                                   // one-launch encode (tiles in claim order)
  int exchange_lag = -1;           // option "exchange_lag": data phase trails by this many exchanges
                                   // (-1 = split_streams - 1, bounded by the buffer sets)
  // single-process group (cvr_create_group, cvr_group.cpp): the members this context fans out to
  struct Group* group = nullptr;
  // scratch
  unsigned long long* d_total = nullptr;
  void* d_scratch = nullptr;      // host-output staging
  size_t scratch_bytes = 0;
};

void comm_release(Ctx* c);   // cvr_comm.cpp
// cvr_group.cpp: a group context's members
struct Group;
using MemberRender = std::function<cvr_status(cvr_ctx*, const cvr_frame*, int, const cvr_output*)>;
void group_release(Ctx* g);
cvr_status group_each(Ctx* g, const std::function<cvr_status(cvr_ctx*)>& fn);
cvr_status group_call_root(Ctx* g, const std::function<cvr_status(cvr_ctx*)>& fn);
Ctx* group_root(Ctx* g);
cvr_status group_render(Ctx* g, const cvr_frame* frames, int nf, const cvr_output* outs,
                        const MemberRender& render);
void flat_release(FlatJobs& J);   // flat.hip

// postpass.hip: multiscaling filters (mode 1-3, kernel 0-5) and the screenshot
hipError_t launch_multiscale(int mode, int kernel, void* frame, int fw, int fh, void* screen, int sw,
                             int sh, hipStream_t s);
hipError_t launch_screenshot(const void* frame, int half, int w, int h, uint8_t* rgb,
                             hipStream_t s);

// kernels / launchers (raymarch.hip)
hipError_t launch_build_cells_impl(const void* vox, int bpv, const uint16_t* lut, const int N[3],
                                   const CellGrid& g, void* cells, hipStream_t s);
hipError_t launch_gradient(const Ctx& c, int mode, uint2* tmp, hipStream_t s);
hipError_t launch_selftest_arith(int e_rcp_lo, int e_rcp_n, int e_sqrt_lo, int e_sqrt_n,
                                 unsigned long long* bad, hipStream_t s);
// plan.frames: null for one frame, else plan.frames->n frames in one launch
// (out / samples: frame 0's)
hipError_t launch_rc1pass(const Ctx& c, const Rc1passArgs& a, bool phong, float4* out,
                          uint32_t* samples, unsigned long long* tile_samples, const int* order,
                          uint32_t* tile_cost, const RenderPlan& plan, hipStream_t s);
// after a frame: sums tile_samples into *total and/or builds the next LPT order
hipError_t launch_tile_epilogue(uint32_t* tile_cost, unsigned long long* tile_samples,
                                unsigned long long* total, const RenderPlan& plan, int* order,
                                hipStream_t s);
hipError_t launch_macro_minmax(const Ctx& c, int shift, const int mdim[3], uint32_t* out,
                               hipStream_t s);
hipError_t launch_occupancy(const uint32_t* minmax, int n_macro, const uint16_t* lut,
                            const int* prefix, int tf_n, uint8_t* occ, unsigned int* n_empty,
                            hipStream_t s);
// skip flags of the density cells for the current TF (clear: strip them); t0, t1
// are two scratch bytes per cell
hipError_t launch_cell_flags(const Ctx& c, bool clear, uint8_t* t0, uint8_t* t1, hipStream_t s);
hipError_t launch_ext_volume(const Ctx& c, const float4* d_tf_rgba, int tf_n, const int res[3],
                             float sigma0, int nlevels, const long long* off, uint16_t* d_ext,
                             uint4* d_ext_cells,
                             hipStream_t s);
hipError_t launch_sat_build(const Ctx& c, const float* d_lut, double* d_sd, float* d_sf,
                            hipStream_t s);
hipError_t launch_sat_cells(const Ctx& c, const float* d_sf, float4* d_cells, hipStream_t s);
size_t sat_cells_float4s(int w, int h, int d);   // the size of that layout, in float4
hipError_t launch_ebs(const Ctx& c, const EbsArgs& q, float4* out, uint32_t* samples,
                      unsigned long long* shade, unsigned long long* tile_samples, hipStream_t s);
hipError_t launch_dos(const Ctx& c, const DosArgs& q, float4* out, uint32_t* samples,
                      unsigned long long* shade,
                      unsigned long long* tile_samples, hipStream_t s);
// iso.hip: raw per-block extremes (uint2), and the isosurface march (variant 0/1)
hipError_t launch_block_minmax(const void* vox, int bpv, const int N[3], const int nb[3], uint2* out,
                               hipStream_t s);
hipError_t launch_iso(const Ctx& c, const IsoArgs& q, int variant, bool phong, const float2* mm,
                      float4* out, uint32_t* samples, unsigned long long* tile_samples,
                      hipStream_t s);
// codec.hip: the lossless per-tile code of RGBA16F tiles (cvr_encode_tiles)
size_t tile_code_bound_bytes(int tile, int ntiles);
hipError_t launch_tile_encode(const void* d_tiles, int tile, int ntiles, void* d_stream,
                              unsigned long long* d_bytes, hipStream_t s);
hipError_t launch_tile_decode(const void* d_stream, int tile, int ntiles, void* d_tiles, hipStream_t s);
hipError_t launch_unpack_tiles(const void* packed, void* out, int half, int W, int H, int tile,
                               int nranks, int tpr_max, hipStream_t s, size_t rank_stride = 0);
hipError_t launch_unpack_tiles_u32(const uint32_t* packed, uint32_t* out, int W, int H, int tile,
                                   int nranks, int tpr_max, hipStream_t s, size_t rank_stride);
// the exchange's one-launch encode of a group (nframes x k tiles at slot stride tpr)
// into d_dst; ctr: a zeroed 64-bit counter on this device that no other launch in
// flight uses, left zero (it may be d_bytes itself); h_bytes (may be null): the same
// length into mapped host memory (its device pointer)
hipError_t launch_exchange_encode(const void* d_packed, int tile, int k, int tpr, int nframes, void* d_dst,
                                  unsigned long long* ctr, unsigned long long* d_bytes, unsigned long long* h_bytes,
                                  hipStream_t s);
// rank 0: every source's stream (or raw tiles) of a group decoded into the frames' images
struct ExchangeDecode {
  const uint32_t* src;               // source r's stream at src + r * slot_words
  size_t slot_words;
  const uint2* raw0;                 // source 0 as raw packed tiles (a rendering root), or null
  size_t raw0_fstride;               // tiles between frames of raw0
  int nsrc;                          // sources = the split's ranks
  int nsplit;                        // the split's nranks (split_tile)
  int nframes, tpr;                  // frames of the group, tile slots per frame and source
  int tile, W, H, ntx, tile_grid_n;  // tile size, image, tiles per row, tiles per frame
  uint2* img[kMaxLaunchFrames];      // frame f's RGBA16F image (null: skipped)
};
hipError_t launch_exchange_decode(const ExchangeDecode& a, hipStream_t s);

inline CellGrid make_cell_grid(const int N[3]) {
  CellGrid g;
  g.cx = N[0] + 1; g.cy = N[1] + 1; g.cz = N[2] + 1;
  g.pitch_y = g.cx;
  g.pitch_z = g.cx * g.cy;
  g.linear_origin = 1 + (long long)g.pitch_y + (long long)g.pitch_z;
  g.bpitch_y = (int)((long long)g.pitch_y * 16 < (1ll << 31) ? g.pitch_y * 16 : 0);
  g.bpitch_z = (int)((long long)g.pitch_z * 16 < (1ll << 31) ? (long long)g.pitch_z * 16 : 0);
  g.borigin = (uint32_t)((unsigned long long)g.linear_origin * 16ull);
  return g;
}

inline size_t cell_count(const CellGrid& g) { return (size_t)g.cx * g.cy * g.cz; }

// ---------------------------------------------------------------------------
// Addressing of a SAT fetch (ebs.hip), shared by the kernels and the host check
// cvr_sat_layout_check.  The texel (tx, ty, tz) is clamped to [0, dims - 1]; its
// element index (tz * h + ty) * w + tx is formed with 24-bit products (both
// operands < 2^24, the result < 2^32: checked on the host).  A fetch reads:
//  * layout 0 (cell4, float4 per texel): elements idx and idx + w*h;
//  * layout 1 (plain float SAT): the float pairs at idx, idx + w, idx + w*h and
//    idx + w*h + w (x, x + 1 of rows y, y + 1 of planes z, z + 1).  A clamped
//    texel's +1 neighbours have weight 0 but are still read; at the far corner
//    (w-1, h-1, d-1) the last one is element w*h*d + w*h + w, so the buffer
//    carries kSatPlainPadPlanes planes of zeros after the SAT.  (Round 3's
//    variant padded one plane: that read ran w + 1 floats past its allocation,
//    4108 B at 1026^3 — always into the next 4 KiB page — and faulted there.)
// ---------------------------------------------------------------------------
constexpr int kSatPlainPadPlanes = 2;

__host__ __device__ inline uint32_t sat_texel_index(uint32_t tx, uint32_t ty, uint32_t tz, uint32_t w,
                                                    uint32_t h) {
#ifdef __HIP_DEVICE_COMPILE__
  return __umul24(__umul24(tz, h) + ty, w) + tx;
#else
  return ((tz * h + ty) & 0xffffffu) * w + tx;   // the 24-bit product's operand, as the device
#endif
}

// floats the plain layout allocates for a w x h x d SAT
inline size_t sat_plain_floats(int w, int h, int d) {
  return (size_t)w * h * (size_t)(d + kSatPlainPadPlanes);
}

}  // namespace cvr
