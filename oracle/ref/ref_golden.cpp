// ref_golden.cpp — golden-vector generator linked against the reference's OWN
// CPU sources, compiled where they lie under /root/reference (see Makefile):
//
//   libs/volvis_utils/transferfunction1d.cpp, transferfunction.cpp   (TF build, Get, GetExtN)
//   libs/volvis_utils/structuredgridvolume.cpp, gridvolume.cpp       (GetNormalizedSample)
//   libs/vis_utils/summedareatable.h                                  (SummedAreaTable3D<double>)
//   include/glm (vendored glm 0.9.5)                                  (lookAt)
//   cppvolrend/structured/rc1pdosct/conegaussiansampler.cpp           (cone section tables)
//   libs/math_utils/utils.cpp                                         (RodriguesRotation)
//
// Only this driver is ours: it feeds inputs to those functions and prints
// their outputs as JSON.  GL-only members (GenerateTexture_*) are never called;
// their GL symbols stay unresolved at link time.  Output: oracle/_ref/ (binary),
// tests/golden/ref_vectors.json (data, via make_golden.py).
#include <volvis_utils/transferfunction1d.h>
#include <volvis_utils/structuredgridvolume.h>
#include <vis_utils/summedareatable.h>

#include <glm/glm.hpp>
#include <glm/gtc/matrix_transform.hpp>
#include <glm/gtc/constants.hpp>

#include <cmath>
#include <cstdio>
#include <fstream>
#include <string>
#include <vector>

namespace {

void print_floats(const char* key, const std::vector<double>& v, bool last = false) {
  std::printf("\"%s\": [", key);
  for (size_t i = 0; i < v.size(); i++) std::printf(i ? ",%.17g" : "%.17g", v[i]);
  std::printf("]%s\n", last ? "" : ",");
}

// Parses a .tf1d with the grammar of TransferFunctionReader::readtf1d and feeds the
// control points to the reference TransferFunction1D.
vis::TransferFunction1D* load_tf(const char* path) {
  std::ifstream f(path);
  std::string interp;
  std::getline(f, interp);
  int init;
  f >> init;
  vis::TransferFunction1D* tf = new vis::TransferFunction1D();
  int n;
  f >> n;
  for (int i = 0; i < n; i++) {
    double r, g, b; int iso;
    f >> r >> g >> b >> iso;
    tf->AddRGBControlPoint(vis::TransferControlPoint(r, g, b, iso));
  }
  f >> n;
  for (int i = 0; i < n; i++) {
    double a; int iso;
    f >> a >> iso;
    tf->AddAlphaControlPoint(vis::TransferControlPoint(a, iso));
  }
  tf->Build();
  return tf;
}

}  // namespace

int main(int argc, char** argv) {
  if (argc < 3) {
    std::fprintf(stderr, "usage: ref_golden <tf1d> <camera_states>\n");
    return 2;
  }
  vis::TransferFunction1D* tf = load_tf(argv[1]);
  std::printf("{\n");
  // ---- TF table as GenerateTexture_1D_RGBt builds it (transferfunction1d.cpp:89-118):
  // Get(i) at integer i returns m_transferfunction[i] (t = 0), alpha -> extinction.
  std::vector<double> rgba, rgbt;
  for (int i = 0; i <= 255; i++) {
    glm::vec4 v = tf->Get((double)i);
    for (int c = 0; c < 4; c++) rgba.push_back(v[c]);
    rgbt.push_back(v.r); rgbt.push_back(v.g); rgbt.push_back(v.b);
    rgbt.push_back((float)tf->MaterialOpacityToExtinction(v.a));
  }
  print_floats("tf_bonsai_rgba", rgba);
  print_floats("tf_bonsai_rgbt", rgbt);
  // ---- Get / GetExtN at fractional inputs (the CPU mapping used by the EBS SAT)
  std::vector<double> gets, extn;
  for (int k = 0; k <= 64; k++) {
    double u = k / 64.0;
    glm::vec4 v = tf->Get(u, 1.0);
    gets.push_back(u);
    for (int c = 0; c < 4; c++) gets.push_back(v[c]);
    extn.push_back(u);
    extn.push_back(tf->GetExtN(u));
  }
  print_floats("tf_bonsai_get_norm", gets);
  print_floats("tf_bonsai_getextn", extn);

  // ---- GetNormalizedSample + EBS SAT (ebsrenderer.cpp:624-716) on a small u8 volume
  const int w = 6, h = 5, d = 4;
  static unsigned char vox[w * h * d];
  for (int i = 0; i < w * h * d; i++) vox[i] = (unsigned char)((i * 37 + 11) % 256);
  vis::StructuredGridVolume vol("golden", w, h, d);
  vol.SetArrayData(vox, vis::DataStorageSize::_8_BITS);
  std::vector<double> vox_d, norm;
  for (int i = 0; i < w * h * d; i++) vox_d.push_back(vox[i]);
  for (int z = -1; z <= d; z++)
    for (int y = -1; y <= h; y++)
      for (int x = -1; x <= w; x++) norm.push_back(vol.GetNormalizedSample(x, y, z));
  std::printf("\"sat_dims\": [%d, %d, %d],\n", w, h, d);
  print_floats("sat_volume_u8", vox_d);
  print_floats("norm_samples_padded", norm);
  int sw = w + 2, sh = h + 2, sd = d + 2;
  vis::SummedAreaTable3D<double> sat(sw, sh, sd);
  for (int x = 0; x < sw; x++)
    for (int y = 0; y < sh; y++)
      for (int z = 0; z < sd; z++) {
        double val;
        if (x == 0 || y == 0 || z == 0 || x == sw - 1 || y == sh - 1 || z == sd - 1)
          val = 0.0f;
        else
          val = tf->GetExtN(vol.GetNormalizedSample(x - 1, y - 1, z - 1));
        sat.SetValue(val, x, y, z);
      }
  sat.BuildSAT();
  std::vector<double> satf;
  double* sd_ = sat.GetData();
  for (int i = 0; i < sw * sh * sd; i++) satf.push_back((float)sd_[i]);
  print_floats("sat_float", satf);
  vol.SetArrayData(nullptr, vis::DataStorageSize::UNKNOWN);

  // ---- glm 0.9.5 lookAt for every "#list_camera_states" ARCBALL entry + tan(fovy/2)
  std::ifstream cf(argv[2]);
  std::vector<double> views;
  std::string line;
  int ncam = 0;
  while (!cf.eof()) {
    std::getline(cf, line);
    std::getline(cf, line);
    if (line.rfind("ARCBALL", 0) != 0) break;
    glm::vec3 e, c, u;
    cf >> e.x >> e.y >> e.z >> c.x >> c.y >> c.z >> u.x >> u.y >> u.z;
    std::getline(cf, line);
    glm::mat4 V = glm::lookAt(e, c, u);
    for (int i = 0; i < 3; i++) views.push_back(e[i]);
    for (int i = 0; i < 3; i++) views.push_back(c[i]);
    for (int i = 0; i < 3; i++) views.push_back(u[i]);
    for (int col = 0; col < 4; col++)
      for (int row = 0; row < 4; row++) views.push_back(V[col][row]);
    ncam++;
  }
  std::printf("\"camera_count\": %d,\n", ncam);
  print_floats("camera_eye_center_up_view", views);
  // (float)tan(DEGREE_TO_RADIANS(45.0f) / 2.0), rc1prenderer.cpp:97
  double fov = 45.0f;
  std::printf("\"tan_half_fovy_45\": %.17g\n", (double)(float)std::tan((fov * (glm::pi<double>() / 180.0)) / 2.0));
  std::printf("}\n");
  return 0;
}
