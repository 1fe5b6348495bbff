#include "hip_renderers.h"

#include "../../utils/parameterspace.h"

#include <volvis_utils/structuredgridvolume.h>
#include <volvis_utils/transferfunction.h>

#include <vector>

// Blinn-Phong constants and the light of RenderingParameters
// (renderingparameters.h:45-74), as every Update uploads them.
template <typename P>
static void fill_phong (P* p, vis::RenderingParameters* rp)
{
  p->ka = rp->GetBlinnPhongKambient();
  p->kd = rp->GetBlinnPhongKdiffuse();
  p->ks = rp->GetBlinnPhongKspecular();
  p->shininess = rp->GetBlinnPhongNshininess();
  const glm::vec3 is = rp->GetLightSourceSpecular();
  for (int i = 0; i < 3; i++) p->ispecular[i] = is[i];
}

static void copy3 (float* dst, const glm::vec3& v)
{
  dst[0] = v.x; dst[1] = v.y; dst[2] = v.z;
}

////////////////////////////////////////////////////////////////////////////////
// RayCasting1Pass (rc1prenderer.cpp:18-151)
////////////////////////////////////////////////////////////////////////////////
HipRayCasting1Pass::HipRayCasting1Pass ()
  : m_u_step_size(0.5f)
  , m_apply_gradient_shading(false)
  , m_params()
{
}

bool HipRayCasting1Pass::Init (int swidth, int sheight)
{
  if (IsBuilt()) Clean();
  if (m_ext_data_manager->GetCurrentVolumeTexture() == nullptr) return false;   // :54
  if (!UploadVolume() || !UploadTransferFunction() || !UploadGradient(m_apply_gradient_shading))
    return false;
  m_u_step_size = DefaultStep();                                                // :62-63
  Reshape(swidth, sheight);
  SetBuilt(true);
  SetOutdated();
  return true;
}

bool HipRayCasting1Pass::Update (vis::Camera* camera)
{
  FillFrame(camera);
  m_params.step = m_u_step_size;
  m_params.apply_gradient_shading =
      (m_apply_gradient_shading && m_ext_data_manager->GetCurrentGradientTexture()) ? 1 : 0;
  fill_phong(&m_params, m_ext_rendering_parameters);
  copy3(m_params.light_pos, m_ext_rendering_parameters->GetBlinnPhongLightingPosition());
  return true;
}

cvr_status HipRayCasting1Pass::RenderFrame (const cvr_output* out)
{
  return cvr_render_rc1pass(m_cvr, &frame_, &m_params, out);
}

// rc1prenderer.cpp:225-229: the evaluation sweep over StepSize
void HipRayCasting1Pass::FillParameterSpace (ParameterSpace& pspace)
{
  pspace.ClearParameterDimensions();
  pspace.AddParameterDimension(new ParameterRangeFloat("StepSize", &m_u_step_size, 0.2, 2.0, 0.1));
}

////////////////////////////////////////////////////////////////////////////////
// RC1PConeTracingDirOcclusionShading (dosrcrenderer.cpp:29-260)
////////////////////////////////////////////////////////////////////////////////
HipDirOcclusionShading::HipDirOcclusionShading ()
  : glsl_apply_occlusion(true)
  , glsl_apply_shadow(false)
  , type_of_shadow(0)
  , m_u_step_size(0.5f)
  , m_apply_gradient_shading(false)
  , m_params()
{
  // ConeGaussianSampler settings of the constructor (:47-58); the covered
  // distances are set from the volume diagonal in Init (:110-113)
  sampler_occlusion.half_angle_deg = 20.0f;
  sampler_occlusion.max_packing = 1;           // CONEPACKING::_3
  sampler_occlusion.covered_distance = 0.0f;
  sampler_occlusion.ui_weight = 0.35f;
  sampler_occlusion.initial_step = 0.0f;       // the sampler's default
  sampler_shadow.half_angle_deg = 0.5f;
  sampler_shadow.max_packing = 0;              // CONEPACKING::_1
  sampler_shadow.covered_distance = 0.0f;
  sampler_shadow.ui_weight = 1.0f;
  sampler_shadow.initial_step = 0.0f;
}

bool HipDirOcclusionShading::Init (int swidth, int sheight)
{
  if (IsBuilt()) Clean();
  if (m_ext_data_manager->GetCurrentVolumeTexture() == nullptr) return false;
  if (!UploadVolume() || !UploadTransferFunction() || !UploadGradient(m_apply_gradient_shading))
    return false;
  vis::StructuredGridVolume* vol = m_ext_data_manager->GetCurrentStructuredVolume();
  sampler_occlusion.covered_distance = (float)(vol->GetDiagonal() * 0.50f);
  sampler_shadow.covered_distance = (float)(vol->GetDiagonal() * 0.75f);
  // GenerateExtCoefVolume (:745-764): the Gaussian pyramid of the RGBA (opacity) TF
  // at ExtinctionCoefficientVolume's defaults (128^3, sigma0 1)
  std::vector<float> rgba;
  int n = 0;
  if (!ReadTransferFunctionRGBA(&rgba, &n)) return false;
  if (cvr_set_extinction_volume(m_cvr, rgba.data(), n, nullptr, 1.0f) != CVR_OK)
    return Fail("cvr_set_extinction_volume");
  m_u_step_size = DefaultStep();
  Reshape(swidth, sheight);
  SetBuilt(true);
  SetOutdated();
  return true;
}

bool HipDirOcclusionShading::Update (vis::Camera* camera)
{
  vis::RenderingParameters* rp = m_ext_rendering_parameters;
  FillFrame(camera);
  m_params.step = m_u_step_size;
  m_params.apply_gradient_shading =
      (m_apply_gradient_shading && m_ext_data_manager->GetCurrentGradientTexture()) ? 1 : 0;
  fill_phong(&m_params, rp);
  copy3(m_params.light.position, rp->GetBlinnPhongLightingPosition());
  copy3(m_params.light.forward, rp->GetBlinnPhongLightSourceCameraForward());
  copy3(m_params.light.up, rp->GetBlinnPhongLightSourceCameraUp());
  copy3(m_params.light.right, rp->GetBlinnPhongLightSourceCameraRight());
  m_params.light.spot_angle_deg = rp->GetSpotLightMaxAngle();
  m_params.apply_occlusion = glsl_apply_occlusion ? 1 : 0;
  m_params.apply_shadow = glsl_apply_shadow ? 1 : 0;
  m_params.shadow_type = type_of_shadow;
  m_params.occlusion = sampler_occlusion;
  m_params.shadow = sampler_shadow;
  return true;
}

cvr_status HipDirOcclusionShading::RenderFrame (const cvr_output* out)
{
  return cvr_render_dosct(m_cvr, &frame_, &m_params, out);
}

////////////////////////////////////////////////////////////////////////////////
// RC1PExtinctionBasedShading (ebsrenderer.cpp:18-260, 624-723)
////////////////////////////////////////////////////////////////////////////////
HipExtinctionBasedShading::HipExtinctionBasedShading ()
  : m_u_step_size(0.5f)
  , m_apply_gradient_shading(false)
  , apply_ambient_occlusion(true)
  , ambient_occlusion_shells(15)
  , ambient_occlusion_radius(1.0f)
  , apply_directional_shadows(true)
  , dir_shadow_cone_angle(1.0f)
  , dir_shadow_sample_interval(2.0f)
  , dir_shadow_initial_step(2.0f)
  , dir_shadow_user_interface_weight(1.0f)
  , dir_cone_max_distance(0.0f)
  , type_of_shadow(0)
  , m_params()
{
}

// The SAT cells are GetExtN(value / max) of the CPU transfer function
// (ebsrenderer.cpp:636-662); the library sums them on the GPU with the
// reference's double recurrence (SummedAreaTable3D<double>::BuildSAT).
bool HipExtinctionBasedShading::UploadExtinctionSAT ()
{
  vis::StructuredGridVolume* v = m_ext_data_manager->GetCurrentStructuredVolume();
  vis::TransferFunction* tf = m_ext_data_manager->GetCurrentTransferFunction();
  const bool u16 = v->m_data_storage_size == vis::DataStorageSize::_16_BITS;
  const double vmax = u16 ? 65535.0 : 255.0;
  std::vector<float> lut(u16 ? 65536 : 256);
  for (size_t i = 0; i < lut.size(); i++) lut[i] = tf->GetExtN((double)i / vmax);
  if (cvr_set_extinction_sat(m_cvr, lut.data(), (int)lut.size()) != CVR_OK)
    return Fail("cvr_set_extinction_sat");
  return true;
}

bool HipExtinctionBasedShading::Init (int swidth, int sheight)
{
  if (IsBuilt()) Clean();
  if (m_ext_data_manager->GetCurrentVolumeTexture() == nullptr) return false;
  if (!UploadVolume() || !UploadTransferFunction() || !UploadGradient(m_apply_gradient_shading) ||
      !UploadExtinctionSAT())
    return false;
  vis::StructuredGridVolume* vold = m_ext_data_manager->GetCurrentStructuredVolume();
  float v_w = vold->GetWidth() * vold->GetScaleX();                            // :98-105
  float v_h = vold->GetHeight() * vold->GetScaleY();
  float v_d = vold->GetDepth() * vold->GetScaleZ();
  dir_cone_max_distance = 0.75f * glm::sqrt(v_w * v_w + v_h * v_h + v_d * v_d);
  m_u_step_size = DefaultStep();
  Reshape(swidth, sheight);
  SetBuilt(true);
  SetOutdated();
  return true;
}

bool HipExtinctionBasedShading::Update (vis::Camera* camera)
{
  vis::RenderingParameters* rp = m_ext_rendering_parameters;
  FillFrame(camera);
  m_params.step = m_u_step_size;
  m_params.apply_gradient_shading =
      (m_apply_gradient_shading && m_ext_data_manager->GetCurrentGradientTexture()) ? 1 : 0;
  fill_phong(&m_params, rp);
  copy3(m_params.light_pos, rp->GetBlinnPhongLightingPosition());
  copy3(m_params.light_forward, rp->GetBlinnPhongLightSourceCameraForward());
  m_params.apply_occlusion = apply_ambient_occlusion ? 1 : 0;
  m_params.occlusion_shells = ambient_occlusion_shells;
  m_params.occlusion_radius = ambient_occlusion_radius;
  m_params.apply_shadow = apply_directional_shadows ? 1 : 0;
  m_params.shadow_type = type_of_shadow;
  m_params.shadow_cone_angle_deg = dir_shadow_cone_angle;
  m_params.shadow_sample_interval = dir_shadow_sample_interval;
  m_params.shadow_initial_step = dir_shadow_initial_step;
  m_params.shadow_ui_weight = dir_shadow_user_interface_weight;
  m_params.shadow_max_distance = dir_cone_max_distance;
  return true;
}

cvr_status HipExtinctionBasedShading::RenderFrame (const cvr_output* out)
{
  return cvr_render_extbsd(m_cvr, &frame_, &m_params, out);
}

////////////////////////////////////////////////////////////////////////////////
// The isosurface ray-casters (rc1pisoadapt, rc1pisocustom, rc1pisodfscustom)
////////////////////////////////////////////////////////////////////////////////
HipIsoRayCasterBase::HipIsoRayCasterBase (int variant)
  : m_u_isovalue(0.5f)                 // rc1custompisoadaptrenderer.cpp:121-126
  , m_u_step_size_small(0.05f)
  , m_u_step_size_large(1.0f)
  , m_u_step_size_range(0.1f)
  , m_u_color(0.66f, 0.6f, 0.05f, 1.0f)
  , m_apply_gradient_shading(false)
  , m_params()
{
  cvr_iso_params_default(variant, &m_params);
}

// No transfer function: the block min/max table ComputeBlocksFromVolume builds on
// the CPU (rc1custompisoadaptrenderer.cpp:20-117) is built by the library on the GPU.
bool HipIsoRayCasterBase::Init (int swidth, int sheight)
{
  if (IsBuilt()) Clean();
  if (m_ext_data_manager->GetCurrentVolumeTexture() == nullptr) return false;
  if (!UploadVolume() || !UploadGradient(m_apply_gradient_shading)) return false;
  Reshape(swidth, sheight);
  SetBuilt(true);
  SetOutdated();
  return true;
}

bool HipIsoRayCasterBase::Update (vis::Camera* camera)
{
  FillFrame(camera);
  m_params.isovalue = m_u_isovalue;
  m_params.step_small = m_u_step_size_small;
  m_params.step_large = m_u_step_size_large;
  m_params.step_range = m_u_step_size_range;
  for (int i = 0; i < 4; i++) m_params.color[i] = m_u_color[i];
  m_params.apply_gradient_shading =
      (m_apply_gradient_shading && m_ext_data_manager->GetCurrentGradientTexture()) ? 1 : 0;
  fill_phong(&m_params, m_ext_rendering_parameters);
  copy3(m_params.light_pos, m_ext_rendering_parameters->GetBlinnPhongLightingPosition());
  return true;
}

cvr_status HipIsoRayCasterBase::RenderFrame (const cvr_output* out)
{
  return cvr_render_iso(m_cvr, &frame_, &m_params, out);
}

// rc1custompisoadaptrenderer.cpp:349-355
void HipIsoRayCasterBase::FillParameterSpace (ParameterSpace& pspace)
{
  pspace.ClearParameterDimensions();
  pspace.AddParameterDimension(new ParameterRangeFloat("StepSizeSmall", &m_u_step_size_small, 0.01f, 0.25f, 0.05f));
  pspace.AddParameterDimension(new ParameterRangeFloat("StepSizeLarge", &m_u_step_size_large, 0.25f, 2.0f, 0.25f));
  pspace.AddParameterDimension(new ParameterRangeFloat("StepSizeRange", &m_u_step_size_range, 0.05f, 0.26f, 0.05f));
}
