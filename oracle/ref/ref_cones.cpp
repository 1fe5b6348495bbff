// ref_cones.cpp — golden cone-section tables from the reference's OWN
// ConeGaussianSampler (cppvolrend/structured/rc1pdosct/conegaussiansampler.cpp)
// and RodriguesRotation (libs/math_utils/utils.cpp), compiled where they lie
// under /root/reference with clang's MSVC-compatibility mode (see Makefile).
//
// For each configuration it prints what RC1PConeTracingDirOcclusionShading
// uploads (dosrcrenderer.cpp:823-985 and GetConeSectionsInfoTex,
// conegaussiansampler.cpp:179-205): per section (interval distance, mip level,
// d_integral, amplitude) as floats (before the RGBA16F upload), the 3- and 7-ray
// axes, the per-packing section counts, the initial step and the 7-ray weight.
// The interval distance is private to the sampler; it is recovered exactly as
// 2 * d_integral of the next section (ComputeAdditionalInfo sets
// d_integral[i] = interval[i-1] * 0.5), and the last interval is 0 (:365-367).
#include "cppvolrend/structured/rc1pdosct/conegaussiansampler.h"

#include <cmath>
#include <cstdio>
#include <vector>

namespace {

void emit(const char* name, float half_angle, int packing, float covered, float ui_weight,
          bool last) {
  ConeGaussianSampler s;
  s.SetUIWeightPercentage(ui_weight);
  s.SetConeHalfAngle(half_angle);
  s.SetMaxGaussianPacking(packing);
  s.SetCoveredDistance(covered);
  s.ComputeConeIntegrationSteps(1.0f);   // ExtinctionCoefficientVolume base sigma0 = 1
  std::vector<ConeGaussianSampler::SectionInfo> sec = s.GetConeSectionsInfoVec();
  std::printf("\"%s\": {\"half_angle\": %.9g, \"packing\": %d, \"covered\": %.9g, "
              "\"ui_weight\": %.9g,\n", name, half_angle, packing, covered, ui_weight);
  std::printf("  \"counts\": [%d, %d, %d], \"initial_step\": %.9g, \"ray7_adj_weight\": %.17g,\n",
              s.gaussian_samples_1, s.gaussian_samples_3, s.gaussian_samples_7,
              (double)s.GetInitialStep(), s.GetRay7AdjacentWeight());
  std::printf("  \"axes\": [");
  for (int i = 0; i < 10; i++) {
    glm::vec3 a = i < 3 ? s.Get3ConeRayID(i) : s.Get7ConeRayID(i - 3);
    std::printf("%s%.9g,%.9g,%.9g", i ? "," : "", a.x, a.y, a.z);
  }
  std::printf("],\n  \"sections\": [");
  for (size_t i = 0; i < sec.size(); i++) {
    const double interval = i + 1 < sec.size() ? 2.0 * sec[i + 1].d_integral : 0.0;
    std::printf("%s%.9g,%.9g,%.9g,%.9g", i ? "," : "", (float)interval,
                (float)sec[i].mip_map_level, (float)sec[i].d_integral, (float)sec[i].amplitude);
  }
  std::printf("]}%s\n", last ? "" : ",");
}

}  // namespace

int main() {
  // GetDiagonal (structuredgridvolume.cpp:96-102) of the configs' volumes, scale 512/N
  const double diag512 = std::sqrt(3.0 * 512.0 * 512.0);
  const double diag64 = std::sqrt(3.0 * 64.0 * 64.0);
  std::printf("{\n");
  // dosrcrenderer.cpp:47-58 defaults; covered distance = diag * 0.50 / 0.75 (:112-113)
  emit("occ_512", 20.0f, 1, (float)(diag512 * 0.50f), 0.35f, false);
  emit("sdw_512", 0.5f, 0, (float)(diag512 * 0.75f), 1.0f, false);
  emit("occ_64", 20.0f, 1, (float)(diag64 * 0.50f), 0.35f, false);
  emit("sdw_64", 0.5f, 0, (float)(diag64 * 0.75f), 1.0f, false);
  // wider cones exercise the 7-ray packing and the 3 -> 7 split
  emit("occ7_30", 30.0f, 2, 300.0f, 0.35f, false);
  emit("occ7_45", 45.0f, 2, 600.0f, 0.5f, true);
  std::printf("}\n");
  return 0;
}
