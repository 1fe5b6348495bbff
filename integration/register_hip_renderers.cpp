// Registration of the HIP renderers, called from main() next to the GLSL
// renderers (cppvolrend/main.cpp:62-79):
//
//   #include "structured/hip/hip_renderers.h"
//   ...
//   RenderingManager::Instance()->AddVolumeRenderer(new RayCasting1Pass());
//   RegisterHipRenderers();
//
// Not part of `make syntax`: renderingmanager.h includes defines.h, which
// hard-defines USING_FREEGLUT, and freeglut_std.h includes <GL/glu.h>, which this
// image does not have (no stand-in headers are written for it).
#include "hip_renderers.h"

#include "../../renderingmanager.h"

void RegisterHipRenderers ()
{
  RenderingManager::Instance()->AddVolumeRenderer(new HipRayCasting1Pass());
  RenderingManager::Instance()->AddVolumeRenderer(new HipDirOcclusionShading());
  RenderingManager::Instance()->AddVolumeRenderer(new HipExtinctionBasedShading());
  RenderingManager::Instance()->AddVolumeRenderer(new HipRayCasting1PassIsoAdapt());
  RenderingManager::Instance()->AddVolumeRenderer(new HipCustomRayCasting1PassIsoAdapt());
  RenderingManager::Instance()->AddVolumeRenderer(new HipCustomRayCasting1PassIsodfsAdapt());
}
