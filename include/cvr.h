/*
 * cvr.h — C-ABI of the MI355X-native structured volume ray-caster.
 *
 * This is the drop-in boundary for cppvolrend's renderer-plugin path
 * (k2683/cpp_volume_rendering).  A reference-side adapter class
 * (`HipRayCasting1Pass : BaseVolumeRenderer`) forwards the
 * plugin calls to these functions; no GL object and no torch type crosses the
 * boundary, only plain pointers, sizes and POD structs.
 *
 * Mapping to the reference interface (paths relative to the reference root):
 *
 *   cvr_create / cvr_destroy     <- BaseVolumeRenderer ctor / Clean()
 *                                   cppvolrend/volrenderbase.cpp:5-29
 *   cvr_set_volume               <- DataManager::GenerateStructuredVolumeTexture +
 *                                   vis::GenerateRTexture (u8/255 -> float -> GL_R16F)
 *                                   libs/volvis_utils/datamanager.cpp:311-330,
 *                                   libs/volvis_utils/utils.cpp:20-56
 *   cvr_set_transfer_function    <- TransferFunction1D::GenerateTexture_1D_RGBt
 *                                   (256 x RGBA16F, alpha already converted to extinction)
 *                                   libs/volvis_utils/transferfunction1d.cpp:89-118
 *   cvr_set_gradient             <- DataManager::GenerateStructuredGradientTexture
 *                                   libs/volvis_utils/datamanager.cpp:332-352,
 *                                   libs/volvis_utils/utils.cpp:146-284 (finite differences)
 *   cvr_render_rc1pass           <- RayCasting1Pass::Update + Redraw
 *                                   cppvolrend/structured/rc1pass/rc1prenderer.cpp:72-151
 *                                   (the dispatch of ray_marching_1p.comp:85-179)
 *   cvr_set_extinction_volume    <- ExtinctionCoefficientVolume::BuildMipMappedTexture (extcoefvolumegenerator.cpp:20-40)
 *                                   (Gaussian mip pyramid of TF opacity -> extinction)
 *                                   cppvolrend/structured/rc1pdosct/extcoefvolumegenerator.cpp:230-408
 *   cvr_render_dosct             <- RC1PConeTracingDirOcclusionShading::Update + Redraw
 *                                   cppvolrend/structured/rc1pdosct/dosrcrenderer.cpp:134-260
 *                                   (the dispatch of ray_bbox_marching.comp:658-734)
 *   cvr_set_extinction_sat       <- RC1PExtinctionBasedShading::GenerateExtinctionSAT3DTex +
 *                                   SummedAreaTable3D<double>::BuildSAT
 *                                   cppvolrend/structured/rc1pextbsd/ebsrenderer.cpp:624-716,
 *                                   libs/vis_utils/summedareatable.h:218-278
 *   cvr_render_extbsd            <- RC1PExtinctionBasedShading::Update + Redraw
 *                                   cppvolrend/structured/rc1pextbsd/ebsrenderer.cpp:125-260
 *                                   (the dispatch of ebs_ray_bbox_marching.comp)
 *   cvr_status (never exit())    <- gl::ExitOnGLError  libs/gl_utils/utils.cpp:11-30
 *
 * Threading: one context per device, externally synchronised (the reference
 * renderer runs on the single GLUT thread, app_freeglut.cpp:172-175).
 * Ownership: the context owns every device allocation; no caller pointer is
 * retained after a call returns.
 */
#ifndef CVR_H
#define CVR_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Bumped whenever a public struct's layout or an entry point's meaning changes
 * (2: cvr_frame gained use_view/view).  Callers compare cvr_abi_version() with
 * the CVR_ABI_VERSION they were compiled against before the first call that
 * passes a struct. */
#define CVR_ABI_VERSION 2

typedef enum cvr_status {
  CVR_OK = 0,
  CVR_ERR_ARG = 1,    /* invalid argument (null pointer, bad size, bad enum)   */
  CVR_ERR_HIP = 2,    /* a HIP runtime call failed                              */
  CVR_ERR_OOM = 3,    /* device allocation failed                               */
  CVR_ERR_STATE = 4,  /* call out of order (e.g. render before set_volume);
                         mirrors RayCasting1Pass::Init returning false when the
                         volume texture is missing, rc1prenderer.cpp:54          */
  CVR_ERR_IO = 5      /* a reader could not open / parse its file              */
} cvr_status;

typedef struct cvr_ctx cvr_ctx;

/* ----------------------------------------------------------------------------
 * Frame description: vis::Camera state + viewport + optional screen-tile split.
 * -------------------------------------------------------------------------- */
typedef struct cvr_camera {
  float eye[3];     /* Camera::GetEye                       camera.cpp:340   */
  float center[3];  /* look-at target                       camera.cpp:281   */
  float up[3];      /* up vector                            camera.cpp:281   */
  float fovy_deg;   /* 45 by default                        camera.cpp:25,44 */
  float aspect;     /* <= 0: width / height                 camera.cpp:307   */
} cvr_camera;

typedef struct cvr_frame {
  cvr_camera camera;
  int width;        /* viewport (RenderingParameters::GetScreenWidth)         */
  int height;
  /* Screen-tile split (multi-GPU): nranks <= 1 renders the whole W x H image
   * row-major.  nranks > 1: the image is cut into tile_size^2 tiles (a multiple
   * of 16; 16 recommended) on a diagonal lattice: with ntx tiles per row, this
   * rank's k-th tile is virtual tile v = rank + k*nranks, at row ty = v / ntx
   * and column tx = (v % ntx - s*ty) mod ntx, s = 3 for nranks >= 4 else 1
   * (when nranks divides ntx: rank (tx + s*ty) % nranks).  It is written packed
   * at offset k*tile_size*tile_size pixels, row-major inside the tile.  Every
   * rank gets cvr_tiles_for_rank tiles, as with plain t % nranks.  (ABI 2.)  */
  int tile_size;
  int rank;
  int nranks;
  /* use_view = 1: `view` is the column-major view matrix the reference uploads
   * as u_CameraLookAt (vis::Camera::LookAt, camera.cpp:281-284, which keeps the
   * look-at centre private) and camera.center is ignored; camera.eye is still
   * CameraEye.  use_view = 0: view = glm::lookAt(eye, center, up).          */
  int use_view;
  float view[16];
} cvr_frame;

/* Output buffers.  rgba: premultiplied RGBA, W*H pixels (or the packed tile
 * buffer), in `format`: CVR_FORMAT_RGBA32F (0, 16 B/pixel, the exact
 * composite) or CVR_FORMAT_RGBA16F (1, 8 B/pixel: binary16 rounded to nearest
 * even, the reference's own framebuffer, imageStore into the RGBA16F
 * OutputFrag image, ray_marching_1p.comp:174-176 / renderoutputframe.cpp:64-87).
 * samples (optional): per-pixel loop-iteration count of
 * ray_marching_1p.comp:124-172 (transparent samples included, stopping at the
 * ERT break).  total (optional): the sum of all iteration counts (uint64).
 * on_device = 1: all three are device pointers and the call is asynchronous
 * on the context stream; the frame's count is atomically ADDED to *total, so
 * the caller zeroes it (one counter can accumulate many frames).
 * on_device = 0: host pointers, *total is overwritten, the call blocks.      */
#define CVR_FORMAT_RGBA32F 0
#define CVR_FORMAT_RGBA16F 1
typedef struct cvr_output {
  void* rgba;
  void* samples;
  void* total;
  int on_device;
  int format;       /* CVR_FORMAT_RGBA32F | CVR_FORMAT_RGBA16F */
} cvr_output;

/* ----------------------------------------------------------------------------
 * Renderer parameters
 * -------------------------------------------------------------------------- */

/* RayCasting1Pass ("1-Pass - Ray Casting", s_1rc): rc1prenderer.cpp:18-138. */
typedef struct cvr_rc1pass_params {
  float step;                  /* <= 0: 0.5/sqrt(3)*|scale|, rc1prenderer.cpp:62-63 */
  int   apply_gradient_shading;/* Blinn-Phong with the gradient volume, :112        */
  float ka, kd, ks, shininess; /* renderingparameters.cpp:23-26 (0.5,0.5,0.8,30)     */
  float ispecular[3];          /* light specular colour, lightsourcelist.cpp:24      */
  float light_pos[3];          /* RenderingParameters::GetBlinnPhongLightingPosition */
} cvr_rc1pass_params;

/* Isosurface ray-casters with block empty-space skipping:
 *   variant 0: CustomRayCasting1PassIsoAdapt ("1-Pass - Custom Isosurface
 *              Raycaster Adaptive", rc1pisocustom/rc1custompisoadaptrenderer.cpp),
 *              4^3 blocks, the block chord as the skip distance;
 *   variant 1: CustomRayCasting1PassIsodfsAdapt ("Empty Sapce Skipping V2",
 *              rc1pisodfscustom/rc1custompisoadaptdfsrenderer.cpp), 32^3 blocks,
 *              the block exit distance and a tolerance of 0.001;
 *   variant 2: RayCasting1PassIsoAdapt ("1-Pass - Isosurface Raycaster
 *              Adaptive", rc1pisoadapt/rc1pisoadaptrenderer.cpp), no blocks.
 * Defaults (cvr_iso_params_default): rc1custompisoadaptrenderer.cpp:119-127. */
typedef struct cvr_iso_params {
  int   variant;               /* 0, 1 or 2                                            */
  int   num_blocks[3];         /* <= 0: 4^3 (variant 0) / 32^3 (variant 1), :190       */
  float isovalue;              /* m_u_isovalue 0.5                                     */
  float step_small;            /* m_u_step_size_small 0.05                             */
  float step_large;            /* m_u_step_size_large 1.0                              */
  float step_range;            /* m_u_step_size_range 0.1                              */
  float color[4];              /* m_u_color (0.66, 0.6, 0.05, 1.0)                     */
  int   apply_gradient_shading;/* m_apply_gradient_shading (default 0; needs gradient) */
  float ka, kd, ks, shininess; /* Blinn-Phong constants (renderingparameters.cpp:23-26) */
  float ispecular[3];          /* BlinnPhongIspecular                                  */
  float light_pos[3];          /* LightSourcePosition                                  */
} cvr_iso_params;

/* Directional-occlusion cones (RC1PConeTracingDirOcclusionShading,
 * cppvolrend/structured/rc1pdosct): the parameters of one ConeGaussianSampler
 * (conegaussiansampler.h) and the tables the renderer uploads from it. */
#define CVR_MAX_CONE_SECTIONS 1024
typedef struct cvr_cone_params {
  float half_angle_deg;    /* SetConeHalfAngle (clamped to [0.5, 89.5]); occlusion 20, shadow 0.5 */
  int   max_packing;       /* SetMaxGaussianPacking: 0 = 1 ray, 1 = 3 rays, 2 = 7 rays
                              (occlusion 1, shadow 0; dosrcrenderer.cpp:47-58)            */
  float covered_distance;  /* SetCoveredDistance (>= 10); <= 0 at render: diagonal * 0.50
                              (occlusion) / 0.75 (shadow), dosrcrenderer.cpp:112-113      */
  float ui_weight;         /* SetUIWeightPercentage; occlusion 0.35, shadow 1.0           */
  float initial_step;      /* <= 0: 3.0 (the sampler's default)                           */
} cvr_cone_params;

typedef struct cvr_cone_tables {
  int   n_sections;        /* sections below                                            */
  int   counts[3];         /* gaussian_samples_1 / _3 / _7                               */
  float initial_step;      /* Occ/SdwInitialStep                                         */
  float ray7_adj_weight;   /* (float)GetRay7AdjacentWeight                               */
  float ui_weight;         /* Occ/SdwUIWeight                                            */
  float axes[10][3];       /* Get3ConeRayID(0..2), Get7ConeRayID(0..6)                   */
  float sections[CVR_MAX_CONE_SECTIONS][4];
                           /* per section (interval distance, mip level, d_integral,
                              amplitude) as floats, before the RGBA16F upload
                              (GetConeSectionsInfoTex, conegaussiansampler.cpp:179-205) */
} cvr_cone_tables;

/* One light source of a #list_light_sources file (vis::LightSourceData,
 * lightsourcelist.cpp:97-140) as RenderingParameters hands it to the shaders:
 * WorldLightingPos, LightCamForward/Up/Right, SpotLightMaxAngle (degrees). */
typedef struct cvr_light {
  float position[3];
  float forward[3];
  float up[3];
  float right[3];
  float spot_angle_deg;
} cvr_light;

/* RC1PConeTracingDirOcclusionShading ("1-Pass - Dir. Occlusion Shading",
 * s_1rcdosct): dosrcrenderer.cpp:24-60, 134-260. */
typedef struct cvr_dos_params {
  float step;                  /* <= 0: 0.5/sqrt(3)*|scale| (dosrcrenderer.cpp:124-125) */
  int   apply_gradient_shading;/* ApplyPhongShading (needs cvr_set_gradient)           */
  float ka, kd, ks, shininess; /* Blinn-Phong constants (renderingparameters.cpp:23-26) */
  float ispecular[3];          /* Ispecular                                             */
  cvr_light light;             /* the current light source                              */
  int   apply_occlusion;       /* ApplyOcclusion (default 1)                            */
  int   apply_shadow;          /* ApplyShadow (default 0)                               */
  int   shadow_type;           /* TypeOfShadow: 0 point, 1 spot, 2 directional          */
  cvr_cone_params occlusion;   /* sampler_occlusion: 20 deg, packing 1, weight 0.35     */
  cvr_cone_params shadow;      /* sampler_shadow:    0.5 deg, packing 0, weight 1.0     */
} cvr_dos_params;

/* RC1PExtinctionBasedShading ("1-Pass - Extinction Based Shading", s_1rcebs):
 * ebsrenderer.cpp:19-55, 125-260. */
typedef struct cvr_ebs_params {
  float step;                  /* <= 0: 0.5/sqrt(3)*|scale| (ebsrenderer.cpp:116-117)   */
  int   apply_gradient_shading;/* ApplyPhongShading (needs cvr_set_gradient)           */
  float ka, kd, ks, shininess; /* Blinn-Phong constants (renderingparameters.cpp:23-26) */
  float ispecular[3];          /* Ispecular                                             */
  float light_pos[3];          /* WorldLightingPos (point light)                        */
  float light_forward[3];      /* LightCamForward (directional light)                   */
  int   apply_occlusion;       /* apply_ambient_occlusion (default 1)                   */
  int   occlusion_shells;      /* ambient_occlusion_shells (15)                         */
  float occlusion_radius;      /* ambient_occlusion_radius (1.0, in voxels)             */
  int   apply_shadow;          /* apply_directional_shadows (default 1)                 */
  int   shadow_type;           /* type_of_shadow: 0 point light, 1 directional          */
  float shadow_cone_angle_deg; /* dir_shadow_cone_angle (1.0)                           */
  float shadow_sample_interval;/* dir_shadow_sample_interval (2.0 voxels)               */
  float shadow_initial_step;   /* dir_shadow_initial_step (2.0 voxels)                  */
  float shadow_ui_weight;      /* dir_shadow_user_interface_weight (1.0)                */
  float shadow_max_distance;   /* <= 0: 0.75 * volume diagonal (ebsrenderer.cpp:98-105) */
} cvr_ebs_params;

/* ----------------------------------------------------------------------------
 * Context
 * -------------------------------------------------------------------------- */
int         cvr_abi_version(void);
const char* cvr_status_string(cvr_status s);
cvr_status  cvr_create(int device, cvr_ctx** out_ctx);
void        cvr_destroy(cvr_ctx* ctx);
const char* cvr_last_error(const cvr_ctx* ctx);
/* Launch stream (a hipStream_t); NULL = the legacy default (null) stream.
 * A new context starts on a private non-blocking stream of its own. */
cvr_status  cvr_set_stream(cvr_ctx* ctx, void* hip_stream);
/* Tuning options (results are identical for every setting):
 *   "batch"      samples addressed + fetched per batch of the march (2 or 4; default 0 =
 *                auto: 4, or 2 with gradient shading — measured 8 % faster there)
 *   "tile_order" 1: each XCD takes the tiles of its screen band longest-first (LPT),
 *                using the previous frame's per-tile critical paths (default);
 *                0: screen order, one contiguous band per XCD; 2: screen order
 *                interleaved over the XCDs (tile t on XCD t mod 8)
 *   "stale_deg"  with tile_order 1: an order learned on a view more than this many
 *                degrees away (view direction; eye moved by that chord of its
 *                distance to the volume centre; fovy changed by that fraction) is
 *                not used, the frame runs in interleaved screen order and the
 *                order is relearned (default 5; 0 = always use it)
 *   "boost"      percent of each band's longest entries launched at raised wave
 *                priority (with tile_order 1; default 5)
 *   "band_cap"   most tiles a work-balanced XCD band may take, in percent of an
 *                even eighth (100..200, default 130); the launch has 8 x that many
 *                slots, the ones past a band's tiles exit at once
 *   "quad"       percent of each band's longest tiles marched sample-parallel, four
 *                lanes per ray (with tile_order 1; default 0)
 *   "order_interval" rebuild the LPT order every n-th frame (default 8; costs
 *                drift slowly, a rebuild costs ~15 us on the frame's stream)
 *   "async_order" 1: rebuild it on a side stream instead, used 3 frames later
 *                (default 0: cross-stream events cost more than they save)
 *   "macro"      empty-space skipping: log2 of the macro cell (2..6, default 3;
 *                0 off); compiled in only when >= "skip_min_pct" % (default 15)
 *                of the macro cells are empty for the current volume and TF
 *   "tile_stats" 1: record per-tile timing of every frame (diagnostics)
 *   "kernel_timing" N > 0: time the ray-march kernel of the last N frames
 *                (cvr_read_kernel_times); 0 off (default)
 *   "cell_skip"  per-cell skip flags kept in the density cells' fp16 sign bits
 *                (rebuilt after a volume or TF change): 0 off; 1 a sample in an
 *                EMPTY cell (no density its corners interpolate to has tau > 0) skips
 *                its classification; 2 also steps over the next samples that stay
 *                within the cell's chessboard distance to non-empty cells, per lane;
 *                3 (default) the same when every marching lane of the wave can;
 *                4 the fewest steps any lane may, for the lanes that can
 *   "sat_chunk"  z planes per work item of the EBS SAT build (1..64, default 32)
 *   "sat_layout" EBS: 0 (default) = frames read a cell4 copy of the SAT (4 float
 *                corners of a plane per texel, 16 B per texel more); 1 = frames read
 *                the plain float SAT (no copy; slower)
 *   "sat_keep_scratch" EBS: 1 keeps the SAT build's double grid (8 B per texel)
 *                allocated for rebuilds; 0 (default) frees it after each build
 *   "shade_counters" 1: count shaded / shadow-lit samples of cvr_render_dosct
 *                and cvr_render_extbsd (cvr_read_shade_counters; one atomic per wave)
 *   "shade_flat" cvr_render_dosct / cvr_render_extbsd: 1 (default) = the frame's
 *                shading jobs in one list, shaded by a grid of their own and folded
 *                per pixel; one list per render stream, sized from earlier frames'
 *                totals (read back without blocking); a frame whose list would not
 *                fit renders through the per-wave kernel, decided on the device;
 *                0 = per-wave deferred shading inside the march
 *   "flat_group" flat shading: consecutive 64-job chunks per XCD turn (default 8)
 *   "debug_flat_limit" tests: a smaller job-list capacity, to exercise the fallback
 *   "split_streams" screen-tile split: render streams the caller rotates over its
 *                cvr_gather_tiles_n calls (1..32, default 1)
 *   "gather_sets" buffer sets the caller rotates over those calls (a multiple of
 *                split_streams; 0 = one per stream): exchange g uses set g % B on
 *                stream g % D, and the stream's next render waits for exchange
 *                g + D - B, the last user of the set it writes next
 *                (0..CVR_MAX_GATHER_SETS)
 *   "gather_root_idle" 1 (communicators of N >= 3 ranks): rank 0 renders nothing and
 *                only gathers and unpacks; ranks 1..N-1 render the split over N-1
 *                render ranks (their cvr_frame: rank = communicator rank - 1,
 *                nranks = N - 1; rank 0 passes a frame of that geometry).  Rank 0's
 *                block of the gather buffer stays unused.  
 *   "launch_interleave" cvr_render_rc1pass_frames under a launch order (tile_order
 *                1/2): 1 (default) = the launch deals entry e of every frame's XCD
 *                bands before entry e + 1 of any (the longest tiles of all frames
 *                first); 0 = frame after frame.  Images identical either way.
 *   "native_exp" 1: TOLERANCE MODE, not bit-exact: the emission-absorption march
 *                (cvr_render_rc1pass[_frames] with cell_skip 3, buffer addressing)
 *                takes alpha = 1 - exp through the hardware v_exp_f32 instead of the
 *                CVR-SPEC polynomial; parity is SURVEY §8(c)'s gate (|dRGBA| <= 2e-3 for
 *                99.9 % of pixels, max 2e-2, SSIM >= 0.99), measured in DESIGN §5‴.
 *                cvr_render_dosct likewise takes the CONSIDER_BORDERS attenuation of
 *                an outside cone tap through v_exp_f32 (its march, counts and ERT
 *                stay bit-exact).  Default 0.
 * One option changes the arithmetic (and so the image) rather than the speed:
 *   "filter_bits" 0: exact float GL_LINEAR weights (CVR-SPEC, the default);
 *                8: every GL_LINEAR weight (volume, gradient, TF; ray_marching_1p.comp:133,
 *                :138; the DOS extinction pyramid, ray_bbox_marching.comp:92-112; the
 *                EBS SAT, ebs_ray_bbox_marching.comp:77-83) rounded to 8 fraction
 *                bits, the fixed-point weights of GPU texture units (CVR-SPEC-8).
 *                cvr_render_extbsd needs sat_layout 0 for it. */
cvr_status  cvr_set_option(cvr_ctx* ctx, const char* key, int value);
int         cvr_get_option(const cvr_ctx* ctx, const char* key);
cvr_status  cvr_synchronize(cvr_ctx* ctx);

/* State setters (cvr_set_volume*, cvr_set_transfer_function, cvr_set_gradient,
 * cvr_set_extinction_volume, cvr_set_extinction_sat, and the cone-table upload
 * inside cvr_render_dosct when its cone parameters change) first drain the
 * WHOLE device (hipDeviceSynchronize): frames already issued on any stream --
 * the caller may rotate several non-blocking streams -- finish with the old
 * state, and frames issued after the call see the new one (the ordering GL
 * gives the reference's Init after a TF change, renderingmanager.cpp:1050-1127).
 * The per-cell skip flags a new volume or TF needs are rebuilt lazily by the
 * next frame; if their scratch (2 B per cell) cannot be allocated, that frame
 * and the following ones render without the skip (the same pixels) until the
 * next state change. */

/* Volume: x-fastest voxels (i + j*w + k*w*h), 1 byte (u8) or 2 bytes (u16)
 * per voxel, normalised as v/255 or v/65535 (structuredgridvolume.cpp:121-151)
 * and stored with GL_R16F semantics.  The data is copied (host pointer). */
cvr_status  cvr_set_volume(cvr_ctx* ctx, const void* voxels, int bytes_per_voxel,
                           int w, int h, int d, const float scale[3]);
/* Same, from a device pointer that stays owned by the caller. */
cvr_status  cvr_set_volume_device(cvr_ctx* ctx, const void* d_voxels, int bytes_per_voxel,
                                  int w, int h, int d, const float scale[3]);

/* Transfer function as n entries of (r, g, b, extinction) floats, i.e. the
 * data GenerateTexture_1D_RGBt uploads; stored with GL_RGBA16F semantics and
 * sampled linearly at x = v*n - 0.5, clamp-to-edge. */
cvr_status  cvr_set_transfer_function(cvr_ctx* ctx, const float* rgbt, int n);

/* Gradient volume for Blinn-Phong.  0 = none, 1 = finite differences
 * (GenerateGradientTexture defaults: sample size 1, no filter, normalised),
 * 2 = Sobel-Feldman (GenerateSobelFeldmanGradientTexture, unnormalised). */
#define CVR_GRADIENT_NONE 0
#define CVR_GRADIENT_FINITE_DIFFERENCES 1
#define CVR_GRADIENT_SOBEL_FELDMAN 2
cvr_status  cvr_set_gradient(cvr_ctx* ctx, int mode);

/* Device bytes held by the context (volume layouts, TF, gradient, ...). */
size_t      cvr_device_bytes(const cvr_ctx* ctx);

/* Copy the volume's cell grid back (diagnostics and tests): (W+1)(H+1)(D+1)
 * cells, x-fastest, 16 B each = the 8 R16F corners GL_LINEAR reads for a
 * sample in the cell.  The corners' sign bits carry the per-cell skip flags of
 * the current TF (option "cell_skip").  No reference counterpart:
 * the reference keeps the volume in a GL_R16F texture (utils.cpp:20-56). */
cvr_status  cvr_copy_cells(cvr_ctx* ctx, void* out, size_t capacity);

/* ----------------------------------------------------------------------------
 * Rendering
 * -------------------------------------------------------------------------- */
/* Number of tiles rank `rank` owns under the split described by `frame`. */
int         cvr_tiles_for_rank(const cvr_frame* frame, int rank);

cvr_status  cvr_render_rc1pass(cvr_ctx* ctx, const cvr_frame* frame,
                               const cvr_rc1pass_params* params, const cvr_output* out);

/* nframes frames (1..16) in ONE ray-march launch: frames[i] is rendered into
 * outs[i] exactly as nframes calls of cvr_render_rc1pass would render it (same
 * pixels, same per-pixel counts).  The frames share the viewport and the screen
 * split (width, height, tile_size, rank, nranks) and may differ in camera; the
 * outputs are device buffers of one format.  outs[0].total (if set) receives the
 * samples of all the frames; the other totals must be NULL.  One launch holds
 * nframes x the waves of a frame, so the tail of one frame's longest rays
 * overlaps the next frame's, and the host pays one call.  The
 * launch order learned on frame 0's view is used when every frame is within
 * "stale_deg" of it.  No reference counterpart: the reference draws one frame
 * per Redraw (rc1prenderer.cpp:100-151); this is the batch form of that call. */
cvr_status  cvr_render_rc1pass_frames(cvr_ctx* ctx, const cvr_frame* frames, int nframes,
                                      const cvr_rc1pass_params* params, const cvr_output* outs);

/* Extinction-coefficient mip pyramid of the current volume for the DOS
 * renderer (ExtinctionCoefficientVolume, extcoefvolumegenerator.cpp:230-408): level 0 at
 * res (NULL: 128^3) is a 7^3 Gaussian (sigma0, default 1) of the opacity TF
 * over the volume, level L the sigma 2^L Gaussian of level L-1 at res >> L,
 * each stored R16F and converted to tau = -log(1 - opacity).  tf_rgba is the
 * RGBA TF (GenerateTexture_1D_RGBA, alpha = opacity), n entries. */
cvr_status  cvr_set_extinction_volume(cvr_ctx* ctx, const float* tf_rgba, int n,
                                      const int res[3], float sigma0);
/* Copy level `level` back as float (NULL out: dims / level count only). */
cvr_status  cvr_copy_extinction_level(cvr_ctx* ctx, int level, float* out, int dims[3],
                                      int* n_levels);

/* One directional-occlusion frame: the ray-march of cvr_render_rc1pass with
 * each sample shaded by cone-traced ambient occlusion and/or a cone shadow
 * toward the light.  Needs cvr_set_extinction_volume. */
cvr_status  cvr_render_dosct(cvr_ctx* ctx, const cvr_frame* frame,
                             const cvr_dos_params* params, const cvr_output* out);

/* Extinction summed-area table of the current volume for the EBS renderer
 * (GenerateExtinctionSAT3DTex, ebsrenderer.cpp:624-716): a (W+2)(H+2)(D+2)
 * grid, zero on its border, holding ext_lut[voxel] inside, summed in double
 * exactly as SummedAreaTable3D<double>::BuildSAT and stored as float.
 * ext_lut: GetExtN(v / (2^bits - 1)) for every voxel value v (256 entries for
 * 8-bit volumes, 65536 for 16-bit; cvr_tf1d_ext_lut builds it). */
cvr_status  cvr_set_extinction_sat(cvr_ctx* ctx, const float* ext_lut, int lut_n);
/* Copy the float SAT back (x-fastest); out = NULL: dims only. */
cvr_status  cvr_copy_extinction_sat(cvr_ctx* ctx, float* out, size_t capacity, int dims[3]);

/* Host check of the SAT fetch addressing (no device work): for a SAT of
 * sat_dims = (W+2, H+2, D+2) texels in `layout` (0 = cell4 copy, 1 = the plain
 * float SAT; option "sat_layout"), evaluates every load of a fetch at every
 * clamped corner texel with the kernels' own index arithmetic and reports
 * out[0] = one past the last byte read, out[1] = bytes the library allocates
 * for that layout, out[2] = 1 if any 24-bit operand or 32-bit index would
 * wrap, out[3] = 1 if the addressing is safe (out[0] <= out[1] and no wrap).
 * pad_planes < 0 = the library's padding; >= 0 evaluates another padding (the
 * round-3 variant's one plane: tests/test_ebs.py).  No reference counterpart:
 * the reference samples the SAT through a GL texture (ebsrenderer.cpp:700-716). */
cvr_status  cvr_sat_layout_check(const int sat_dims[3], int layout, int pad_planes,
                                 unsigned long long out[4]);

/* One extinction-based shading frame: the ray-march with each sample shaded by
 * a SAT ambient occlusion and a SAT box-chain shadow.  Needs
 * cvr_set_extinction_sat. */
cvr_status  cvr_render_extbsd(cvr_ctx* ctx, const cvr_frame* frame,
                              const cvr_ebs_params* params, const cvr_output* out);

/* The reference renderers' default parameters for `variant`. */
void        cvr_iso_params_default(int variant, cvr_iso_params* out);
/* One isosurface frame (first hits composited front to back with Color).  The
 * block min/max table (ComputeBlocksFromVolume, rc1custompisoadaptrenderer.cpp
 * :20-117) is built on the GPU when the volume or num_blocks changes. */
cvr_status  cvr_render_iso(cvr_ctx* ctx, const cvr_frame* frame, const cvr_iso_params* params,
                           const cvr_output* out);
/* Copy the current block table back (x-fastest, num_blocks of the last build);
 * builds it first for `num_blocks` when needed.  Empty blocks hold (FLT_MAX,
 * -FLT_MAX) as in the reference. */
cvr_status  cvr_iso_block_ranges(cvr_ctx* ctx, const int num_blocks[3], float* out_min,
                                 float* out_max);

/* Rank-0 side of the screen-tile split: `d_packed` holds nranks consecutive
 * blocks of `tiles_per_rank_max` packed tiles (rank r's block at offset
 * r*tiles_per_rank_max*tile_size^2 pixels); scatter them into the W x H
 * device image `d_rgba`.  Both buffers hold pixels of `format`
 * (CVR_FORMAT_RGBA32F or CVR_FORMAT_RGBA16F).  Asynchronous on the context
 * stream. */
cvr_status  cvr_unpack_tiles_device(cvr_ctx* ctx, const cvr_frame* frame,
                                    const void* d_packed, int tiles_per_rank_max,
                                    int format, void* d_rgba);

/* The same for frame `frame_index` of a grouped exchange: `d_gathered` holds
 * nranks blocks of nframes * tiles_per_rank_max tiles (rank r's frame j at
 * tile slot (r * nframes + j) * tiles_per_rank_max), as cvr_gather_tiles_n
 * leaves it. */
cvr_status  cvr_unpack_tiles_device_n(cvr_ctx* ctx, const cvr_frame* frame,
                                      const void* d_gathered, int tiles_per_rank_max,
                                      int nframes, int frame_index, int format, void* d_rgba);

/* Lossless per-tile code of RGBA16F screen tiles (every world
 * size was bound by rank 0's inbound bytes, and a rendered tile's channels span few
 * bits; the exchange moves this code since round 6).  d_tiles: ntiles tiles of
 * tile x tile RGBA16F pixels, each row-major (the packed layout of a screen-tile
 * share).  The stream, 32-bit words: ntiles + 1 tile starts (the last = the
 * stream's end), then per tile 3 header words (four 16-bit channel bases, four
 * 5-bit widths) and each channel's differences from its base at its width.
 * Every bit pattern round-trips.  cvr_tile_code_bound: the largest stream
 * (bytes) for these sizes (tile 16..64, a multiple of 16; 0 = invalid);
 * cvr_encode_tiles writes the stream and its length (bytes, a device u64) on
 * the context stream; cvr_decode_tiles restores the tiles.  Option "encode_onepass"
 * 1: cvr_encode_tiles runs the exchange's ONE-launch encode instead of three (each
 * tile claims its words with an atomic, so the codes follow in claim order, not
 * tile order; the start table says where each is, the length and the decode are
 * the same).  The multi-rank exchange uses the code (option exchange_code). */
size_t      cvr_tile_code_bound(int tile, int ntiles);
cvr_status  cvr_encode_tiles(cvr_ctx* ctx, const void* d_tiles, int tile, int ntiles,
                             void* d_stream, unsigned long long* d_bytes);
cvr_status  cvr_decode_tiles(cvr_ctx* ctx, const void* d_stream, int tile, int ntiles, void* d_tiles);

/* ----------------------------------------------------------------------------
 * After the march: pixel multiscaling and the screenshot
 * (libs/vis_utils/renderoutputframe.cpp:89-146, 265-539 and its
 * shader/renderoutputframe/ compute shaders; renderingmanager.cpp:103-112,
 * 476-492)
 * -------------------------------------------------------------------------- */

/* BaseVolumeRenderer multiscaling modes (volrenderbase.h:28-33) */
#define CVR_SINGLE_RAY_PER_PIXEL    0
#define CVR_MULTIPLE_RAYS_PER_PIXEL 1
#define CVR_DOWN_SCALING_RENDER     2
#define CVR_UP_SCALING_RENDER       3
/* vis::IMAGE_FILTER_KERNEL (libs/vis_utils/filters/utils.hpp:8-15); K2_HAT is
 * RenderFrameToScreen's default (renderoutputframe.cpp:34) */
#define CVR_FILTER_BOX                0
#define CVR_FILTER_HAT                1
#define CVR_FILTER_CATMULL_ROM        2
#define CVR_FILTER_MITCHELL_NETRAVALI 3
#define CVR_FILTER_CARDINAL_BSPLINE_3 4
#define CVR_FILTER_CARDINAL_OMOMS3    5

/* Render resolution of a mode at screen size (w, h): 2w x 2h for modes 1-2,
 * w/2 x h/2 for mode 3 (UpdateScreenResolutionMultiScaling with the 2 x 2
 * multiplier of cppvolrend/defines.h:16-17). */
cvr_status  cvr_multiscale_resolution(int mode, int screen_w, int screen_h, int* render_w,
                                      int* render_h);

/* Filter a rendered RGBA16F frame (fw x fh, device) to the RGBA16F screen
 * image (sw x sh, device): mode 1 = multisample_filter (bilinear), 2 = kernel
 * downscale (+ the digital filter over the result for the cardinal kernels),
 * 3 = kernel upscale (the cardinal kernels' digital prefilter runs IN PLACE on
 * d_frame first, as the reference does).  Asynchronous on the context stream. */
cvr_status  cvr_multiscale_filter(cvr_ctx* ctx, int mode, int kernel, void* d_frame, int fw,
                                  int fh, void* d_screen, int sw, int sh);

/* Screenshot: the frame (device, CVR_FORMAT_*) blended over the white clear
 * colour with SRC_ALPHA / ONE_MINUS_SRC_ALPHA and stored as RGB8, row 0 =
 * bottom as glReadPixels returns it (w*h*3 bytes, device).  Asynchronous. */
cvr_status  cvr_screenshot_rgb8(cvr_ctx* ctx, const void* d_frame, int format, int w, int h,
                                void* d_rgb);

/* ----------------------------------------------------------------------------
 * Multi-GPU: the screen-tile split's gather, native RCCL over xGMI
 * (the reference renders on one GPU, so this has no reference
 * counterpart beyond the Redraw it feeds, rc1prenderer.cpp:140-151).
 * One context per GPU, one process (or thread) per context.
 * -------------------------------------------------------------------------- */

#define CVR_COMM_ID_BYTES 128
/* The most exchange buffer sets (option "gather_sets"): the library keeps the
 * end events of the last 64 exchanges. */
#define CVR_MAX_GATHER_SETS 64

/* Rank 0 creates the communicator id (ncclGetUniqueId) and hands it to every
 * rank out of band (e.g. torch.distributed broadcast). */
cvr_status  cvr_comm_unique_id(unsigned char out_id[CVR_COMM_ID_BYTES]);

/* Collective over the nranks contexts: joins this context to the communicator. */
cvr_status  cvr_comm_init(cvr_ctx* ctx, int nranks, int rank,
                          const unsigned char id[CVR_COMM_ID_BYTES]);
cvr_status  cvr_comm_destroy(cvr_ctx* ctx);

/* The same protocol without RCCL, for n contexts of THIS process (rank i =
 * ctxs[i]; the devices may repeat, e.g. n contexts on one GPU): the bytes move
 * as device copies (over xGMI between GPUs).  Every exchange call
 * (cvr_gather_tiles_n) must be made by ranks 1..n-1 before rank 0 makes it, and
 * the buffer sets must exceed the render streams (gather_sets > split_streams):
 * a rank's next render waits for rank 0's completed exchange of its buffers.
 * cvr_create_group uses it; tests use it to run the multi-rank exchange on one
 * GPU (RCCL refuses several ranks per device). */
cvr_status  cvr_comm_init_local(cvr_ctx* const* ctxs, int n);

/* Gather one frame's packed tiles on rank 0 (one ncclGather) and unpack them
 * into the image.
 * Every rank calls it right after rendering its tiles (frame->rank/nranks
 * must match the communicator) into `d_packed` (tiles_per_rank_max tiles,
 * padding allowed).  Rank 0 also passes `d_gathered` (nranks blocks of
 * tiles_per_rank_max tiles; when d_packed == d_gathered, rank 0 rendered
 * straight into its block 0 and no copy is made) and the W x H image `d_rgba`.
 * Asynchronous: the gather and unpack run on the context's communication
 * stream after the render.  Callers alternate two packed (and, on rank 0, two
 * gather) buffers, frame n using buffer n % 2 (see split_streams for more).  With option split_streams = 1
 * (default) the context stream then waits only for the PREVIOUS gather, so the
 * next render overlaps this gather.  With split_streams = D >= 2 the caller
 * rotates D streams and D buffer sets (frame n on stream n % D, cvr_set_stream
 * before each render) and the stream waits for THIS gather, so D consecutive
 * frames overlap on the device as well.
 * Frames on different streams each use their own LPT order state; frames that
 * count samples (cvr_output.total) must not overlap.  Before reading the image
 * on the context stream, call cvr_gather_sync.  With a one-rank communicator
 * the frame is rendered whole (nranks 1) and the gather copies it to d_rgba. */
cvr_status  cvr_gather_tiles(cvr_ctx* ctx, const cvr_frame* frame, const void* d_packed,
                             int tiles_per_rank_max, int format, void* d_gathered,
                             void* d_rgba);

/* The same for `nframes` frames rendered by this rank one after another on the
 * context stream into consecutive blocks of `d_packed` (frame j at j *
 * tiles_per_rank_max tiles), exchanged in ONE ncclGather (fewer, larger
 * collectives: a gather's host and launch cost is shared by nframes frames).
 * `frame` gives the tile layout (the camera is not used).  Rank 0's
 * `d_gathered` holds nranks blocks of nframes * tiles_per_rank_max tiles, and
 * frame j is unpacked into d_images[j] (in frame order; NULL skips it). */
cvr_status  cvr_gather_tiles_n(cvr_ctx* ctx, const cvr_frame* frame, int nframes,
                               const void* d_packed, int tiles_per_rank_max, int format,
                               void* d_gathered, void* const* d_images);

/* The context stream waits for every gather issued so far (posting any whose
 * data phase still trails, see exchange_lag). */
cvr_status  cvr_gather_sync(cvr_ctx* ctx);

/* Exchange form (options, set on every rank alike):
 *   "exchange_code" 1 (default): RGBA16F exchanges of N > 1 ranks move the lossless
 *                per-tile code (cvr_encode_tiles' stream, encoded in one launch per
 *                exchange on the render stream) instead of raw tiles, and rank 0
 *                decodes every rank's stream straight into the images in one
 *                launch; 0: raw tiles (one ncclGather, then the unpack).  RGBA32F
 *                always moves raw tiles.  The images are identical either way.
 *   "exchange_lag" the coded exchange's sizes vary, so they travel first (an 8-byte
 *                gather on a second communicator, right after the encode) and
 *                exchange g's data is posted when a later call reads g's sizes on
 *                the host: at most this many exchanges later (-1, the default:
 *                split_streams - 1; bounded by gather_sets - split_streams so a
 *                render stream never waits for an unposted exchange; 0: at once,
 *                which blocks the host until this rank's encode is done). */

/* ----------------------------------------------------------------------------
 * One context over several GPUs of this process (SURVEY.md §8b threading row:
 * multi-GPU inside cvr_render when ndev > 1).  The reference app is one GLUT
 * process with one GL thread (app_freeglut.cpp:125,174), so its plugin cannot be
 * one process per GPU.  cvr_create_group returns a context whose state setters
 * (volume, TF, gradient, extinction pyramid, SAT, options) apply to one member
 * context per device, and whose render calls (rc1pass, rc1pass_frames, dosct,
 * extbsd, iso; whole frames, nranks <= 1) split the frame into 16 x 16 screen
 * tiles on the diagonal lattice over the members, render every share on its own
 * device concurrently, and gather the tiles on devices[0] (the in-process
 * transport of cvr_comm_init_local; RGBA16F as the per-tile code) into the
 * caller's outputs, which live on devices[0] (or the host).  Same pixels, counts
 * and totals as one context.  Devices may repeat.  The group's stream
 * (cvr_set_stream) is devices[0]'s; member 0 renders on it.  Host outputs block;
 * device outputs are queued on the group's stream.  Options split_streams,
 * gather_sets, gather_root_idle and exchange_lag belong to the group's own
 * exchange and are refused. */
cvr_status  cvr_create_group(const int* devices, int n, cvr_ctx** out_ctx);
/* Members of a group (1 for a plain context) and member i's context (NULL if none;
 * owned by the group: for inspection, not for cvr_destroy). */
int         cvr_group_size(const cvr_ctx* ctx);
cvr_ctx*    cvr_group_member(cvr_ctx* ctx, int i);

/* Diagnostics (tile_stats option): for each 8x8 tile of the last frame, four
 * uint64: start and end stamp (s_memrealtime, 100 MHz), its longest ray's
 * iteration count, (workgroup << 32 | HW_ID).  out = NULL queries *out_tiles. */
cvr_status  cvr_copy_tile_stats(cvr_ctx* ctx, uint64_t* out, int max_tiles, int* out_tiles);

/* Measurement (kernel_timing option = ring of N frames): milliseconds of the
 * ray-march kernel alone (HIP events recorded on the context stream around its
 * launch) for the most recent min(N, frames since the last read, max_frames)
 * frames, oldest first.  Waits for those frames; resets the frame count. */
cvr_status  cvr_read_kernel_times(cvr_ctx* ctx, float* ms, int max_frames, int* out_frames);

/* Self-check of the device arithmetic the kernels take shortcuts with
 * (cvr_device.h), exhaustive over every significand: out[0] = floats b with
 * |b| in [2^-100, 2^100) whose rcp_cr(b) differs from the IEEE 1.0f / b,
 * out[1] = floats x in [2^-96, 2^126) whose sqrt_cr_normal(x) differs from the
 * correctly rounded sqrtf(x), out[2] = (x, y) pairs (every positive normal
 * x < 4 at five exponents y, and the special arguments) whose branch-free
 * cvr_powf_nb differs from cvr_powf.  All must be 0; synchronous (~1 s). */
cvr_status  cvr_selftest_arith(cvr_ctx* ctx, uint64_t out[3]);

/* Measurement (shade_counters option), for the last shaded frame
 * (cvr_render_dosct / cvr_render_extbsd; cvr_render_rc1pass: out[0] the
 * Blinn-Phong shaded samples, out[1] the samples the per-cell skip stepped over
 * without a load, out[2] (emission-absorption, cell_skip > 0) the waves' march
 * rounds, each K = 4 cell loads per wave): out[0] samples that ran the shading
 * (alpha > 0), out[1] those whose shadow was traced (spot cut-off excluded),
 * out[2] the secondary trilinear fetches actually issued (extinction pyramid /
 * SAT): the secondary traffic of the roofline.  For DOS the reference's own tap
 * count is out[0] * (n1 + 3 n3 + 7 n7)_occlusion + out[1] * (...)_shadow; out[2]
 * leaves out the taps whose CONSIDER_BORDERS factor is exactly 0 (not fetched). */
cvr_status  cvr_read_shade_counters(cvr_ctx* ctx, uint64_t out[3]);

/* ----------------------------------------------------------------------------
 * Host-side helpers (native replacements for the reference's MSVC-only
 * readers and its CPU table builders).  They touch no device.
 * -------------------------------------------------------------------------- */
/* ConeGaussianSampler::ComputeConeIntegrationSteps + ComputeAdditionalInfo
 * (conegaussiansampler.cpp:212-414) for one cone; sigma0 = the extinction
 * volume's base Gaussian sigma (ExtinctionCoefficientVolume default 1). */
cvr_status  cvr_build_cone_tables(const cvr_cone_params* params, float sigma0,
                                  cvr_cone_tables* out);

/* Derived render constants, exposed for testing: the view matrix the ray
 * generator uses (glm::lookAt, column-major 4x4) and tan(fovy/2). */
cvr_status  cvr_camera_lookat(const cvr_camera* cam, float out_view[16], float* out_tan_half_fovy);
/* Default integration step for a voxel scale: 0.5/sqrt(3)*|scale|. */
float       cvr_default_step(const float scale[3]);

/* TransferFunction1D built from control points (BuildLinear,
 * transferfunction1d.cpp:319-358) and converted like GenerateTexture_1D_RGBt
 * (:89-118).  rgb_cp: n_rgb x (r, g, b, isovalue); a_cp: n_a x (a, isovalue).
 * out_rgbt receives (max_density+1) x 4 floats. */
cvr_status  cvr_tf1d_build_rgbt(const double* rgb_cp, int n_rgb, const double* a_cp, int n_a,
                                int max_density, int extinction_input, float* out_rgbt);

/* TransferFunction1D::GetExtN (transferfunction1d.cpp:132-157, 189-197) of
 * every voxel value v / (2^bits - 1), bits = 8 * bytes_per_voxel: the cell
 * values of the EBS SAT.  out_lut receives 256 or 65536 floats. */
cvr_status  cvr_tf1d_ext_lut(const double* rgb_cp, int n_rgb, const double* a_cp, int n_a,
                             int max_density, int extinction_input, int bytes_per_voxel,
                             float* out_lut);

/* .tf1d reader (TransferFunctionReader::readtf1d, reader.cpp:744-814) and the
 * built table.  out_rgbt must hold 4*(max_density+1) floats; pass NULL to
 * query *out_n first. */
cvr_status  cvr_read_tf1d(const char* path, float* out_rgbt, int* out_n);

/* .raw reader: dims and bytes per voxel parsed from "name.<bytes>.<W>x<H>x<D>.raw"
 * (VolumeReader::readraw, reader.cpp:162-225).  Pass voxels = NULL to query. */
cvr_status  cvr_read_raw(const char* path, void* voxels, size_t capacity,
                         int* out_w, int* out_h, int* out_d, int* out_bytes_per_voxel);

/* .pvm reader (VolumeReader::readpvm, reader.cpp:100-159; DDSV3 decoder,
 * libs/file_utils/pvm.cpp:191-620): plain or DDS-compressed PVM/PVM2/PVM3,
 * 1 component -> u8, 2 -> u16 (data[2i] + 256*data[2i+1], as Pvm::PostProcessData).
 * out_scale (may be NULL) receives the PVM2/3 voxel spacing.  voxels = NULL queries. */
cvr_status  cvr_read_pvm(const char* path, void* voxels, size_t capacity, int* out_w,
                         int* out_h, int* out_d, int* out_bytes_per_voxel, float out_scale[3]);

/* .syn reader (VolumeReader::readsyn, reader.cpp:283-371); u8 voxels. */
cvr_status  cvr_read_syn(const char* path, uint8_t* voxels, size_t capacity,
                         int* out_w, int* out_h, int* out_d);

/* #list_camera_states (CameraStateList::ReadCameraStates, camerastatelist.cpp:26-87):
 * returns the index-th ARCBALL state. */
cvr_status  cvr_read_camera_state(const char* path, int index, cvr_camera* out_cam,
                                  char* out_name, int name_capacity, int* out_count);

/* #list_light_sources (LightSourceList::ReadLightSourceLists, lightsourcelist.cpp:81-148):
 * position of light `light` of list `list`. */
cvr_status  cvr_read_light_position(const char* path, int list, int light, float out_pos[3],
                                    int* out_count);
/* The same light with its camera frame and spot angle (forward = -z_axis). */
cvr_status  cvr_read_light(const char* path, int list, int light, cvr_light* out,
                           int* out_count);

#ifdef __cplusplus
}
#endif

#endif /* CVR_H */
