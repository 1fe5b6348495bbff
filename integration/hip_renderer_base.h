/**
 * Reference-side adapters: cppvolrend renderer plugins that forward to libcvr.so
 * (include/cvr.h).  These files are meant to be dropped into the reference tree
 * (e.g. cppvolrend/structured/hip/) and registered next to the existing renderers
 * in cppvolrend/main.cpp:62-79 (see register_hip_renderers.cpp).
 *
 * HipRendererBase holds what every adapter shares:
 *   - the cvr context (one per renderer object): every visible GPU by default -- a
 *     group context (cvr_create_group) that splits each frame over the GPUs of this
 *     process and gathers it on device 0 -- or the one device it is given;
 *   - the upload of the current structured volume (DataManager, datamanager.h:82-84;
 *     StructuredGridVolume::GetArrayData / m_data_storage_size, structuredgridvolume.h:67-76)
 *     and of the transfer function tables GenerateTexture_1D_RGBt / _RGBA build
 *     (transferfunction.h:62-63), read back from their GL textures so the library
 *     samples exactly the table the GLSL renderer samples;
 *   - the frame: the camera's eye and its LookAt() matrix (camera.cpp:281-284) as
 *     the reference uploads them (CameraEye, u_CameraLookAt, rc1prenderer.cpp:91-95);
 *     the viewport as Update chooses it (rc1prenderer.cpp:76-87);
 *   - Redraw and the three multiscaling redraws: RenderFrameToScreen's own RGBA16F
 *     texture is registered with HIP-GL interop (hipGraphicsGLRegisterImage), the
 *     library renders into a device RGBA16F buffer and a device-to-device copy
 *     fills the mapped texture, as the compute shader's imageStore does
 *     (renderoutputframe.cpp:197-202); if the texture does not register, the frame
 *     comes back to a host buffer and glTexSubImage2D uploads it.  The reference's
 *     Draw* functions then draw it (renderoutputframe.h:38-51), as
 *     rc1prenderer.cpp:140-189 does after its dispatch.
 * Errors: a non-OK cvr_status becomes Init() == false (rc1prenderer.cpp:54) or a
 * printed message; the library never calls exit().
 */
#ifndef CVR_HIP_RENDERER_BASE_H
#define CVR_HIP_RENDERER_BASE_H

#include "../../volrenderbase.h"

#include <cvr.h>

#include <hip/hip_runtime_api.h>
#include <hip/hip_gl_interop.h>

#include <cstdint>
#include <vector>

class HipRendererBase : public BaseVolumeRenderer
{
public:
  // hip_device >= 0: that GPU; -1 (default): every visible GPU (a cvr_create_group
  // context when there are several, SURVEY.md §8b threading row)
  explicit HipRendererBase (int hip_device = -1);
  virtual ~HipRendererBase ();

  vis::GRID_VOLUME_DATA_TYPE GetDataTypeSupport () override
  {
    return vis::GRID_VOLUME_DATA_TYPE::STRUCTURED;
  }

  void Clean () override;
  void ReloadShaders () override;       // compiled kernels: only the screen shaders reload
  void Redraw () override;
  void MultiSampleRedraw () override;
  void DownScalingRedraw () override;
  void UpScalingRedraw () override;

protected:
  // One frame of this renderer into `out` (host RGBA16F, frame_'s viewport).
  virtual cvr_status RenderFrame (const cvr_output* out) = 0;

  bool UploadVolume ();                          // cvr_set_volume
  bool UploadTransferFunction ();                // cvr_set_transfer_function (RGBt)
  bool ReadTransferFunctionRGBA (std::vector<float>* rgba, int* n);   // opacity TF
  bool UploadGradient (bool wanted);             // cvr_set_gradient from the DataManager's type
  float DefaultStep ();                          // rc1prenderer.cpp:62-63
  void FillFrame (vis::Camera* camera);          // frame_ from the camera + viewport
  bool Fail (const char* where);

  cvr_ctx* m_cvr;
  cvr_frame frame_;

private:
  bool RenderToScreenTexture ();
  bool AttachScreenTexture (gl::Texture2D* t);    // hipGraphicsGLRegisterImage
  void DetachScreenTexture ();
  bool RenderToMappedTexture (gl::Texture2D* t);  // map, render, D2D copy, unmap
  static bool ReadTexture1D (gl::Texture1D* tex, std::vector<float>* rgba, int* n);
  std::vector<uint16_t> m_rgba16f;               // host fallback frame

  bool m_gl_interop;                              // off after the first interop failure
  hipStream_t m_stream;                           // the context stream (interop path)
  hipGraphicsResource_t m_gl_res;                 // the registered screen texture
  GLuint m_gl_tex;
  int m_gl_w, m_gl_h;
  void* m_dev_rgba16f;                            // device frame, 8 B per pixel
};

#endif
