/**
 * MI355X drop-ins for the reference's structured single-pass renderers, each a
 * BaseVolumeRenderer (cppvolrend/volrenderbase.h:25-96) that forwards to libcvr.so:
 *
 *   HipRayCasting1Pass               <- RayCasting1Pass        (rc1pass/rc1prenderer.h:31-76)
 *   HipDirOcclusionShading           <- RC1PConeTracingDirOcclusionShading
 *                                                              (rc1pdosct/dosrcrenderer.h:40-120)
 *   HipExtinctionBasedShading        <- RC1PExtinctionBasedShading
 *                                                              (rc1pextbsd/ebsrenderer.h:47-123)
 *   HipRayCasting1PassIsoAdapt       <- RayCasting1PassIsoAdapt (rc1pisoadapt/rc1pisoadaptrenderer.h)
 *   HipCustomRayCasting1PassIsoAdapt <- CustomRayCasting1PassIsoAdapt (rc1pisocustom/...)
 *   HipCustomRayCasting1PassIsodfsAdapt <- CustomRayCasting1PassIsodfsAdapt (rc1pisodfscustom/...)
 *
 * Parameters keep the reference's member names and defaults; the GLSL uniforms
 * they fed become the plain structs of include/cvr.h.
 */
#ifndef CVR_HIP_RENDERERS_H
#define CVR_HIP_RENDERERS_H

#include "hip_renderer_base.h"

class HipRayCasting1Pass : public HipRendererBase
{
public:
  HipRayCasting1Pass ();
  const char* GetName () override { return "1-Pass - Ray Casting (HIP, MI355X)"; }
  const char* GetAbbreviationName () override { return "s_1rc_hip"; }
  bool Init (int shader_width, int shader_height) override;
  bool Update (vis::Camera* camera) override;
  void FillParameterSpace (ParameterSpace& pspace) override;

  float m_u_step_size;                 // rc1prenderer.h:63
  bool m_apply_gradient_shading;

protected:
  cvr_status RenderFrame (const cvr_output* out) override;
  cvr_rc1pass_params m_params;
};

class HipDirOcclusionShading : public HipRendererBase
{
public:
  HipDirOcclusionShading ();
  const char* GetName () override { return "1-Pass - Ray Casting - Dir. Occlusion Shading (HIP, MI355X)"; }
  const char* GetAbbreviationName () override { return "s_1rc_dos_hip"; }
  bool Init (int shader_width, int shader_height) override;
  bool Update (vis::Camera* camera) override;

  // dosrcrenderer.cpp:29-60
  bool glsl_apply_occlusion;
  bool glsl_apply_shadow;
  int type_of_shadow;                  // 0 point, 1 spot, 2 directional
  cvr_cone_params sampler_occlusion;   // ConeGaussianSampler settings
  cvr_cone_params sampler_shadow;
  float m_u_step_size;
  bool m_apply_gradient_shading;

protected:
  cvr_status RenderFrame (const cvr_output* out) override;
  cvr_dos_params m_params;
};

class HipExtinctionBasedShading : public HipRendererBase
{
public:
  HipExtinctionBasedShading ();
  const char* GetName () override { return "1-Pass - Ray Casting - Extinction-based (HIP, MI355X)"; }
  const char* GetAbbreviationName () override { return "s_1rc_eb_hip"; }
  bool Init (int shader_width, int shader_height) override;
  bool Update (vis::Camera* camera) override;

  // ebsrenderer.cpp:18-51
  float m_u_step_size;
  bool m_apply_gradient_shading;
  bool apply_ambient_occlusion;
  int ambient_occlusion_shells;
  float ambient_occlusion_radius;
  bool apply_directional_shadows;
  float dir_shadow_cone_angle;
  float dir_shadow_sample_interval;
  float dir_shadow_initial_step;
  float dir_shadow_user_interface_weight;
  float dir_cone_max_distance;
  int type_of_shadow;                  // 0 point, 1 directional

protected:
  cvr_status RenderFrame (const cvr_output* out) override;
  bool UploadExtinctionSAT ();         // GenerateExtinctionSAT3DTex (:624-723), on the GPU
  cvr_ebs_params m_params;
};

// The three single-pass isosurface ray-casters share one library entry point
// (cvr_render_iso) and differ in `variant`: 2 = no blocks, 0 = 4^3 block chords,
// 1 = 32^3 block exit distances.
class HipIsoRayCasterBase : public HipRendererBase
{
public:
  explicit HipIsoRayCasterBase (int variant);
  bool Init (int shader_width, int shader_height) override;
  bool Update (vis::Camera* camera) override;
  void FillParameterSpace (ParameterSpace& pspace) override;

  float m_u_isovalue;
  float m_u_step_size_small;
  float m_u_step_size_large;
  float m_u_step_size_range;
  glm::vec4 m_u_color;
  bool m_apply_gradient_shading;

protected:
  cvr_status RenderFrame (const cvr_output* out) override;
  cvr_iso_params m_params;
};

class HipRayCasting1PassIsoAdapt : public HipIsoRayCasterBase
{
public:
  HipRayCasting1PassIsoAdapt () : HipIsoRayCasterBase(2) {}
  const char* GetName () override { return "1-Pass - Isosurface Raycaster Adaptive (HIP, MI355X)"; }
  const char* GetAbbreviationName () override { return "iso_hip"; }
};

class HipCustomRayCasting1PassIsoAdapt : public HipIsoRayCasterBase
{
public:
  HipCustomRayCasting1PassIsoAdapt () : HipIsoRayCasterBase(0) {}
  const char* GetName () override { return "1-Pass - Custom Isosurface Raycaster Adaptive (HIP, MI355X)"; }
  const char* GetAbbreviationName () override { return "iso_hip"; }
};

class HipCustomRayCasting1PassIsodfsAdapt : public HipIsoRayCasterBase
{
public:
  HipCustomRayCasting1PassIsodfsAdapt () : HipIsoRayCasterBase(1) {}
  const char* GetName () override { return "Empty Space Skipping V2 (HIP, MI355X)"; }
  const char* GetAbbreviationName () override { return "iso_hip"; }
};

// Adds every HIP renderer to the RenderingManager (register_hip_renderers.cpp;
// call it next to main.cpp:65).
void RegisterHipRenderers ();

#endif
