#include "hip_renderer_base.h"

#include <gl_utils/texture1d.h>
#include <gl_utils/texture2d.h>
#include <volvis_utils/structuredgridvolume.h>
#include <volvis_utils/transferfunction.h>

#include <glm/gtc/type_ptr.hpp>

#include <cmath>
#include <cstdio>

HipRendererBase::HipRendererBase (int hip_device)
  : m_cvr(nullptr)
  , frame_()
  , m_gl_interop(true)
  , m_stream(nullptr)
  , m_gl_res(nullptr)
  , m_gl_tex(0)
  , m_gl_w(0)
  , m_gl_h(0)
  , m_dev_rgba16f(nullptr)
{
  // One GL thread drives the renderer (app_freeglut.cpp:125,174), so the node's GPUs
  // are used from this process: with more than one visible device (and no device
  // named) the context is a group over all of them (cvr_create_group), which splits
  // every frame into screen tiles over the GPUs and gathers it on device 0.
  int ndev = 0;
  if (hip_device < 0 && hipGetDeviceCount(&ndev) == hipSuccess && ndev > 1) {
    std::vector<int> devs((size_t)ndev);
    for (int i = 0; i < ndev; i++) devs[(size_t)i] = i;
    if (cvr_create_group(devs.data(), ndev, &m_cvr) != CVR_OK) m_cvr = nullptr;
  } else if (cvr_create(hip_device < 0 ? 0 : hip_device, &m_cvr) != CVR_OK) {
    m_cvr = nullptr;
  }
#ifdef MULTISAMPLE_AVAILABLE
  vr_pixel_multiscaling_support = true;        // as the GLSL renderers (rc1prenderer.cpp:27-29)
#endif
}

HipRendererBase::~HipRendererBase ()
{
  Clean();
  if (m_cvr) cvr_destroy(m_cvr);
  m_cvr = nullptr;
  if (m_stream) (void)hipStreamDestroy(m_stream);
  m_stream = nullptr;
}

void HipRendererBase::Clean ()
{
  DetachScreenTexture();
  m_rgba16f.clear();
  m_rgba16f.shrink_to_fit();
  BaseVolumeRenderer::Clean();
}

void HipRendererBase::ReloadShaders ()
{
  m_rdr_frame_to_screen.ClearShaders();
}

bool HipRendererBase::Fail (const char* where)
{
  fprintf(stderr, "%s: %s\n", where, m_cvr ? cvr_last_error(m_cvr) : "no HIP device context");
  return false;
}

// The raw x-fastest voxels and the voxel scale of the current structured volume
// (the data GenerateRTexture uploads, utils.cpp:20-56).  u8 and u16 volumes only,
// the storage sizes GetNormalizedSample reads (structuredgridvolume.cpp:121-151).
bool HipRendererBase::UploadVolume ()
{
  if (!m_cvr) return Fail("HIP renderer");
  vis::StructuredGridVolume* v = m_ext_data_manager->GetCurrentStructuredVolume();
  if (v == nullptr || v->GetArrayData() == nullptr) return false;
  int bpv = 0;
  if (v->m_data_storage_size == vis::DataStorageSize::_8_BITS) bpv = 1;
  else if (v->m_data_storage_size == vis::DataStorageSize::_16_BITS) bpv = 2;
  else return false;
  const float scale[3] = {(float)v->GetScaleX(), (float)v->GetScaleY(), (float)v->GetScaleZ()};
  if (cvr_set_volume(m_cvr, v->GetArrayData(), bpv, (int)v->GetWidth(), (int)v->GetHeight(),
                     (int)v->GetDepth(), scale) != CVR_OK)
    return Fail("cvr_set_volume");
  return true;
}

bool HipRendererBase::ReadTexture1D (gl::Texture1D* tex, std::vector<float>* rgba, int* n)
{
  if (tex == nullptr) return false;
  GLint w = 0;
  glBindTexture(GL_TEXTURE_1D, tex->GetTextureID());
  glGetTexLevelParameteriv(GL_TEXTURE_1D, 0, GL_TEXTURE_WIDTH, &w);
  rgba->assign((size_t)w * 4, 0.0f);
  glGetTexImage(GL_TEXTURE_1D, 0, GL_RGBA, GL_FLOAT, rgba->data());
  glBindTexture(GL_TEXTURE_1D, 0);
  *n = (int)w;
  return w > 1;
}

// The table RayCasting1Pass samples: GenerateTexture_1D_RGBt (RGB + extinction,
// transferfunction1d.cpp:89-118), read back from its RGBA16F texture.
bool HipRendererBase::UploadTransferFunction ()
{
  vis::TransferFunction* tf = m_ext_data_manager->GetCurrentTransferFunction();
  if (tf == nullptr) return false;
  gl::Texture1D* t = tf->GenerateTexture_1D_RGBt();
  std::vector<float> rgbt;
  int n = 0;
  const bool ok = ReadTexture1D(t, &rgbt, &n);
  delete t;
  if (!ok) return false;
  if (cvr_set_transfer_function(m_cvr, rgbt.data(), n) != CVR_OK)
    return Fail("cvr_set_transfer_function");
  return true;
}

// GenerateTexture_1D_RGBA (alpha = opacity, transferfunction1d.cpp:58-87): the
// table the DOS extinction pyramid filters (dosrcrenderer.cpp:745-764).
bool HipRendererBase::ReadTransferFunctionRGBA (std::vector<float>* rgba, int* n)
{
  vis::TransferFunction* tf = m_ext_data_manager->GetCurrentTransferFunction();
  if (tf == nullptr) return false;
  gl::Texture1D* t = tf->GenerateTexture_1D_RGBA();
  const bool ok = ReadTexture1D(t, rgba, n);
  delete t;
  return ok;
}

// DataManager's gradient model (datamanager.h:63-68) -> the library's precompute.
bool HipRendererBase::UploadGradient (bool wanted)
{
  int mode = CVR_GRADIENT_NONE;
  if (wanted && m_ext_data_manager->GetCurrentGradientTexture()) {
    switch (m_ext_data_manager->GetCurrentGradientGenerationTypeID()) {
      case vis::DataManager::FINITE_DIFERENCES: mode = CVR_GRADIENT_FINITE_DIFFERENCES; break;
      case vis::DataManager::SOBEL_FELDMAN_FILTER:
      case vis::DataManager::COMPUTE_SHADER_SOBEL: mode = CVR_GRADIENT_SOBEL_FELDMAN; break;
      default: mode = CVR_GRADIENT_NONE; break;
    }
  }
  if (cvr_set_gradient(m_cvr, mode) != CVR_OK) return Fail("cvr_set_gradient");
  return true;
}

// rc1prenderer.cpp:62-63 (the same expression, evaluated as the reference does)
float HipRendererBase::DefaultStep ()
{
  glm::dvec3 sv = m_ext_data_manager->GetCurrentStructuredVolume()->GetScale();
  return float((0.5f / glm::sqrt(3.0f)) * glm::sqrt(sv.x * sv.x + sv.y * sv.y + sv.z * sv.z));
}

// CameraEye + u_CameraLookAt + u_TanCameraFovY + u_CameraAspectRatio
// (rc1prenderer.cpp:91-101); the dispatch size of Update (:76-87).
void HipRendererBase::FillFrame (vis::Camera* camera)
{
  const glm::vec3 e = camera->GetEye();
  const glm::vec3 d = camera->GetDir();
  const glm::vec3 u = camera->GetUp();
  const glm::mat4 view = camera->LookAt();
  frame_ = cvr_frame();
  for (int i = 0; i < 3; i++) {
    frame_.camera.eye[i] = e[i];
    frame_.camera.center[i] = e[i] + d[i];      // unused: use_view carries the exact matrix
    frame_.camera.up[i] = u[i];
  }
  frame_.camera.fovy_deg = camera->GetFovY();
  frame_.camera.aspect = camera->GetAspectRatio();
  frame_.use_view = 1;
  const float* m = glm::value_ptr(view);       // column-major, as glUniformMatrix4fv
  for (int i = 0; i < 16; i++) frame_.view[i] = m[i];
  if (IsPixelMultiScalingSupported() && GetCurrentMultiScalingMode() > 0) {
    frame_.width = m_rdr_frame_to_screen.GetWidth();
    frame_.height = m_rdr_frame_to_screen.GetHeight();
  } else {
    frame_.width = m_ext_rendering_parameters->GetScreenWidth();
    frame_.height = m_ext_rendering_parameters->GetScreenHeight();
  }
  frame_.tile_size = 0;
  frame_.rank = 0;
  frame_.nranks = 1;
}

// (Re)registers RenderFrameToScreen's RGBA16F output texture with HIP when its
// GL name or size changed (Update re-creates it on a viewport change).  Any
// failure switches the interop path off for the rest of this object's life.
bool HipRendererBase::AttachScreenTexture (gl::Texture2D* t)
{
  if (!m_gl_interop || t == nullptr) return false;
  const GLuint id = t->GetTextureID();
  if (m_gl_res != nullptr && id == m_gl_tex && frame_.width == m_gl_w && frame_.height == m_gl_h)
    return true;
  DetachScreenTexture();
  hipGraphicsResource_t res = nullptr;
  if (hipGraphicsGLRegisterImage(&res, id, GL_TEXTURE_2D, hipGraphicsRegisterFlagsWriteDiscard) != hipSuccess) {
    m_gl_interop = false;
    return false;
  }
  const size_t bytes = (size_t)frame_.width * frame_.height * 8;
  if (hipMalloc(&m_dev_rgba16f, bytes) != hipSuccess) {
    (void)hipGraphicsUnregisterResource(res);
    m_dev_rgba16f = nullptr;
    m_gl_interop = false;
    return false;
  }
  m_gl_res = res;
  m_gl_tex = id;
  m_gl_w = frame_.width;
  m_gl_h = frame_.height;
  return true;
}

void HipRendererBase::DetachScreenTexture ()
{
  if (m_stream) (void)hipStreamSynchronize(m_stream);
  if (m_gl_res) (void)hipGraphicsUnregisterResource(m_gl_res);
  if (m_dev_rgba16f) (void)hipFree(m_dev_rgba16f);
  m_gl_res = nullptr;
  m_dev_rgba16f = nullptr;
  m_gl_tex = 0;
  m_gl_w = m_gl_h = 0;
}

// Device-resident handoff, the counterpart of the compute shader's imageStore into
// the RGBA16F screen texture (renderoutputframe.cpp:197-202): map the registered
// texture, render into a device RGBA16F buffer on the context stream, copy it into
// the texture's array (device to device, 8 B per pixel), unmap.  Map and unmap
// order the HIP work against GL's use of the texture; nothing crosses PCIe.
bool HipRendererBase::RenderToMappedTexture (gl::Texture2D* t)
{
  if (!AttachScreenTexture(t)) return false;
  if (hipGraphicsMapResources(1, &m_gl_res, m_stream) != hipSuccess) {
    DetachScreenTexture();
    m_gl_interop = false;
    return false;
  }
  bool ok = false;
  hipArray_t arr = nullptr;
  if (hipGraphicsSubResourceGetMappedArray(&arr, m_gl_res, 0, 0) == hipSuccess) {
    cvr_output out;
    out.rgba = m_dev_rgba16f;
    out.samples = nullptr;
    out.total = nullptr;
    out.on_device = 1;
    out.format = CVR_FORMAT_RGBA16F;
    const size_t row = (size_t)frame_.width * 8;
    if (RenderFrame(&out) == CVR_OK)
      ok = hipMemcpy2DToArrayAsync(arr, 0, 0, m_dev_rgba16f, row, row, frame_.height,
                                   hipMemcpyDeviceToDevice, m_stream) == hipSuccess;
    else
      Fail(GetName());
  }
  if (hipGraphicsUnmapResources(1, &m_gl_res, m_stream) != hipSuccess) ok = false;
  return ok;
}

// One frame into RenderFrameToScreen's output texture (the image the compute
// shader's imageStore fills; row 0 = bottom): through HIP-GL interop when the
// texture registers, else rendered into a host RGBA16F buffer and uploaded with
// glTexSubImage2D (one PCIe copy of 8 B per pixel).
bool HipRendererBase::RenderToScreenTexture ()
{
  if (!m_cvr || frame_.width <= 0 || frame_.height <= 0) return false;
  gl::Texture2D* screen = m_rdr_frame_to_screen.GetScreenOutputTexture();
  if (m_gl_interop) {
    if (m_stream == nullptr) {
      if (hipStreamCreateWithFlags(&m_stream, hipStreamNonBlocking) != hipSuccess ||
          cvr_set_stream(m_cvr, m_stream) != CVR_OK)
        m_gl_interop = false;
    }
    if (m_gl_interop && RenderToMappedTexture(screen)) return true;
  }
  m_rgba16f.resize((size_t)frame_.width * frame_.height * 4);
  cvr_output out;
  out.rgba = m_rgba16f.data();
  out.samples = nullptr;
  out.total = nullptr;
  out.on_device = 0;
  out.format = CVR_FORMAT_RGBA16F;
  if (RenderFrame(&out) != CVR_OK) return Fail(GetName());
  glBindTexture(GL_TEXTURE_2D, screen->GetTextureID());
  glTexSubImage2D(GL_TEXTURE_2D, 0, 0, 0, frame_.width, frame_.height, GL_RGBA, GL_HALF_FLOAT,
                  m_rgba16f.data());
  glBindTexture(GL_TEXTURE_2D, 0);
  return true;
}

void HipRendererBase::Redraw ()
{
  if (RenderToScreenTexture()) m_rdr_frame_to_screen.Draw();
}

void HipRendererBase::MultiSampleRedraw ()
{
  if (RenderToScreenTexture()) m_rdr_frame_to_screen.DrawMultiSampleHigherResolutionMode();
}

void HipRendererBase::DownScalingRedraw ()
{
  if (RenderToScreenTexture()) m_rdr_frame_to_screen.DrawHigherResolutionWithDownScale();
}

void HipRendererBase::UpScalingRedraw ()
{
  if (RenderToScreenTexture()) m_rdr_frame_to_screen.DrawLowerResolutionWithUpScale();
}
