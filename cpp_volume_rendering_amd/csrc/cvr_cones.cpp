// cvr_cones.cpp — cone-section tables of the directional-occlusion renderer
// (host side, no device).  Restates ConeGaussianSampler
// (cppvolrend/structured/rc1pdosct/conegaussiansampler.cpp) with the same
// arithmetic: the section placement, sigma doubling and integrals in double
// (:212-285, :318-414, :418-498), the cone-ray axes with the float
// RodriguesRotation of libs/math_utils/utils.cpp:149-156 (glm 0.9.5 vector
// semantics: dot = (x+y)+z, normalize = v * (1/sqrt(dot(v,v)))).  The tables
// are pinned against the reference's own sampler compiled under oracle/ref
// (tests/golden/ref_vectors.json "cones").
#include <cmath>
#include <cstring>
#include <vector>

#include "cvr_internal.h"

namespace {

struct V3 { float x, y, z; };
inline V3 operator*(V3 a, float s) { return {a.x * s, a.y * s, a.z * s}; }
inline V3 operator+(V3 a, V3 b) { return {a.x + b.x, a.y + b.y, a.z + b.z}; }
inline float dotv(V3 a, V3 b) {
  V3 t{a.x * b.x, a.y * b.y, a.z * b.z};
  return t.x + t.y + t.z;
}
inline V3 crossv(V3 a, V3 b) {
  return {a.y * b.z - b.y * a.z, a.z * b.x - b.z * a.x, a.x * b.y - b.x * a.y};
}
inline V3 normalizev(V3 v) { return v * (1.0f / std::sqrt(dotv(v, v))); }

// RodriguesRotation(glm::vec3, float, glm::vec3): the float overload is the
// one the sampler's (vec3, double, vec3) calls resolve to.
V3 rodrigues(V3 v, float teta, V3 k) {
  const float c = std::cos(teta), s = std::sin(teta);
  V3 r = v * c + crossv(k, v) * s + (k * dotv(k, v)) * (1.0f - c);
  return normalizev(r);
}

constexpr double kPi = 3.14159265358979323846;
const double kDiv3 = 1.0 + (2.0 / std::sqrt(3.0));            // D_HEMISPHERE_CONE_DIV_3
constexpr double kDiv7 = 3.010000;                           // D_HEMISPHERE_CONE_DIV_7

struct Section {
  int n;
  double pos, radius, sigma;
  double d_integral, amplitude, mip;
};

struct Sampler {
  float half_angle;
  int packing;        // 0: _1, 1: _3, 2: _7
  float covered;
  float d_sigma = 1.25f, r_sigma = 2.0f;
  std::vector<Section> sec;
  std::vector<double> interval;   // s_distance per interval

  bool add7(double pos, double sg, int* ng) {
    *ng = 7;
    const double rad = (half_angle / kDiv7) * kPi / 180.0;
    const double r = pos * std::tan(rad);
    if (r > r_sigma * sg) return false;
    sec.push_back({7, pos, r, sg, 0, 0, 0});
    return true;
  }
  bool add3(double pos, double sg, int* ng) {
    if (*ng > 3) return add7(pos, sg, ng);
    *ng = 3;
    const double rad = (half_angle / kDiv3) * kPi / 180.0;
    const double r = pos * std::tan(rad);
    if (r > r_sigma * sg) return packing > 1 ? add7(pos, sg, ng) : false;
    sec.push_back({3, pos, r, sg, 0, 0, 0});
    return true;
  }
  bool add(double pos, double sg, int* ng) {
    if (*ng > 1) return add3(pos, sg, ng);
    *ng = 1;
    const double rad = half_angle * kPi / 180.0;
    const double r = pos * std::tan(rad);
    if (r > r_sigma * sg) return packing > 0 ? add3(pos, sg, ng) : false;
    sec.push_back({1, pos, r, sg, 0, 0, 0});
    return true;
  }
};

double gaussian_eval(double x, double sig) {
  return (1.0 / (std::sqrt(2.0 * kPi) * sig)) * std::exp(-(x * x) / (2.0 * sig * sig));
}

double integrate_gaussian(double sdev, double cone_radius) {
  const double t = (2.0 * cone_radius) / 0.05;
  const int nt = (int)std::ceil(t);
  const double segment = (2.0 * cone_radius) / double(nt);
  const double s0 = -cone_radius + segment * 0.5;
  double S = 0.0;
  for (int i = 0; i < nt; i++) S += gaussian_eval(s0 + segment * double(i), sdev) * segment;
  return S;
}

}  // namespace

extern "C" {
#pragma GCC visibility push(default)

cvr_status cvr_build_cone_tables(const cvr_cone_params* p, float sigma0, cvr_cone_tables* out) {
  if (!p || !out || !(sigma0 > 0.0f)) return CVR_ERR_ARG;
  if (p->max_packing < 0 || p->max_packing > 2) return CVR_ERR_ARG;
  std::memset(out, 0, sizeof(*out));
  Sampler s;
  // SetConeHalfAngle clamps to [0.5, 89.5]; SetCoveredDistance to >= 10 (:61-64, :167-170)
  s.half_angle = std::fmin(std::fmax(p->half_angle_deg, 0.5f), 89.5f);
  s.packing = p->max_packing;
  s.covered = p->covered_distance > 10.0f ? p->covered_distance : 10.0f;
  const float initial_step = p->initial_step > 0.0f ? p->initial_step : 3.0f;

  // 3- and 7-ray axes (:221-251)
  V3 r3[3], r7[7];
  {
    const double adj = s.half_angle / kDiv3;
    const double t1 = (s.half_angle - adj) * kPi / 180.0;
    r3[0] = rodrigues(V3{0, 0, 1}, (float)t1, V3{0, 1, 0});
    r3[0] = rodrigues(r3[0], (float)(30.0 * kPi / 180.0), V3{0, 0, 1});
    const double at = 120.0 * kPi / 180.0;
    r3[1] = rodrigues(r3[0], (float)at, V3{0, 0, 1});
    r3[2] = rodrigues(r3[1], (float)at, V3{0, 0, 1});
  }
  {
    r7[0] = V3{0, 0, 1};
    const double adj = s.half_angle / kDiv7;
    const double t1 = (s.half_angle - adj) * kPi / 180.0;
    r7[1] = rodrigues(r7[0], (float)t1, V3{0, 1, 0});
    const double at = 60.0 * kPi / 180.0;
    for (int i = 2; i < 7; i++) r7[i] = rodrigues(r7[i - 1], (float)at, V3{0, 0, 1});
  }

  // section placement (:253-282)
  int ng = 1;
  double curr = initial_step;
  double sg = sigma0;
  while (!s.add(curr, sg, &ng)) sg *= 2.0;
  while (curr < s.covered) {
    double si = (double)s.d_sigma * sg;
    while (!s.add(curr + si + ((double)s.d_sigma * sg), sg, &ng)) sg *= 2.0;
    si += (double)s.d_sigma * sg;
    s.interval.push_back(si);
    curr += si;
    if (s.sec.size() > (size_t)CVR_MAX_CONE_SECTIONS) return CVR_ERR_ARG;
  }
  // ComputeAdditionalInfo (:318-414)
  if (s.sec.size() != s.interval.size() + 1 || s.sec.size() > (size_t)CVR_MAX_CONE_SECTIONS)
    return CVR_ERR_ARG;
  for (size_t i = 0; i + 1 < s.sec.size(); i++)
    if (!(s.sec[i].n <= s.sec[i + 1].n)) return CVR_ERR_ARG;
  s.interval.push_back(0.0);
  const double min_sg = sigma0;
  for (size_t i = 0; i < s.sec.size(); i++) {
    Section& e = s.sec[i];
    if (e.n == 1) out->counts[0]++;
    else if (e.n == 3) out->counts[1]++;
    else out->counts[2]++;
    if (i == 0) e.d_integral = e.sigma * std::sqrt(2.0 * kPi) * 0.5;
    else e.d_integral = s.interval[i - 1] * 0.5;
    const double pr = integrate_gaussian(e.sigma, e.radius);
    const double Ac = kPi * e.radius * e.radius;
    const double Ig = e.sigma * std::sqrt(2.0 * kPi);
    e.amplitude = ((pr * pr) * (Ig * Ig)) / Ac;
    e.mip = std::log2(e.sigma / min_sg);
    out->sections[i][0] = (float)s.interval[i];
    out->sections[i][1] = (float)e.mip;
    out->sections[i][2] = (float)e.d_integral;
    out->sections[i][3] = (float)e.amplitude;
  }
  out->n_sections = (int)s.sec.size();
  out->initial_step = initial_step;
  out->ray7_adj_weight = (float)(double)dotv(V3{0, 0, 1}, r7[1]);
  out->ui_weight = p->ui_weight;
  for (int i = 0; i < 3; i++) { out->axes[i][0] = r3[i].x; out->axes[i][1] = r3[i].y; out->axes[i][2] = r3[i].z; }
  for (int i = 0; i < 7; i++) {
    out->axes[3 + i][0] = r7[i].x; out->axes[3 + i][1] = r7[i].y; out->axes[3 + i][2] = r7[i].z;
  }
  return CVR_OK;
}

#pragma GCC visibility pop
}  // extern "C"
