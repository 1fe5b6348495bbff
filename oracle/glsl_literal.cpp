/*
 * glsl_literal.cpp — a second, LITERAL reading of the reference shaders.
 * TEST INFRASTRUCTURE ONLY (tests/, never the product).
 *
 * cvr_oracle.cpp restates the shaders under CVR-SPEC, the arithmetic contract the
 * HIP kernels reproduce bit for bit (fma where the kernels use one, a texel-space
 * ray, a polynomial exp).  This file reads the same GLSL text the plain way, to
 * measure how far CVR-SPEC sits from the shader as written:
 *   - every expression in the shader's own order, left to right, no fused
 *     multiply-add (IEEE float, -ffp-contract=off);
 *   - positions as the shader forms them: tex_pos + dir * (s + h * 0.5), then the
 *     texture coordinate u = p / G (ray_marching_1p.comp:129-133) or
 *     p * (1 / G) (ray_bbox_marching.comp:701-708, ebs_ray_bbox_marching.comp:601-604);
 *   - GL_LINEAR filtering as the GL specification defines it (4.6 §8.14.2): texel
 *     coordinate u*N - 1/2, i0 = floor, alpha = frac, CLAMP_TO_EDGE on the texel
 *     indices, tau = sum of the 2^d corners weighted by products of (1-alpha)/alpha;
 *     optionally with the weights quantised to `wbits` fraction bits (GPU texture
 *     units use fixed-point weights; 8 is the common width), 0 = exact float;
 *     wbits < 0 (diagnostics) = CVR-SPEC's filter arithmetic inside an otherwise
 *     literal shader, to separate the filter's share of a difference;
 *   - libm expf / powf / sqrtf, normalize(v) = v / length(v), dot left to right.
 * Inputs are the same fp16-rounded tables the CVR-SPEC oracle consumes.
 *
 * Shader line references (reference root, read-only):
 *   rc1pass ........ cppvolrend/structured/rc1pass/ray_marching_1p.comp:48-179
 *   slab test ...... cppvolrend/structured/_common_shaders/ray_bbox_intersection.comp:18-52
 *   DOS ............ cppvolrend/structured/rc1pdosct/ray_bbox_marching.comp:92-734
 *   EBS ............ cppvolrend/structured/rc1pextbsd/ebs_ray_bbox_marching.comp:63-627
 */
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <vector>

#ifdef _OPENMP
#include <omp.h>
#endif

#include "oracle_types.h"

#define ORACLE_API extern "C" __attribute__((visibility("default")))

extern "C" void oracle_lookat(const float eye_[3], const float center_[3], const float up_[3],
                              float fovy_deg, float out_view[16], float* out_tan);

namespace {

struct vec3 { float x, y, z; };
inline vec3 V(float x, float y, float z) { return vec3{x, y, z}; }
inline vec3 operator+(vec3 a, vec3 b) { return V(a.x + b.x, a.y + b.y, a.z + b.z); }
inline vec3 operator-(vec3 a, vec3 b) { return V(a.x - b.x, a.y - b.y, a.z - b.z); }
inline vec3 operator-(vec3 a) { return V(-a.x, -a.y, -a.z); }
inline vec3 operator*(vec3 a, vec3 b) { return V(a.x * b.x, a.y * b.y, a.z * b.z); }
inline vec3 operator*(vec3 a, float s) { return V(a.x * s, a.y * s, a.z * s); }
inline vec3 operator*(float s, vec3 a) { return V(s * a.x, s * a.y, s * a.z); }
inline vec3 operator/(vec3 a, vec3 b) { return V(a.x / b.x, a.y / b.y, a.z / b.z); }
inline vec3 operator/(float s, vec3 a) { return V(s / a.x, s / a.y, s / a.z); }
inline vec3 operator/(vec3 a, float s) { return V(a.x / s, a.y / s, a.z / s); }
inline float dot(vec3 a, vec3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
inline float length(vec3 v) { return std::sqrt(dot(v, v)); }
inline vec3 normalize(vec3 v) { const float l = length(v); return V(v.x / l, v.y / l, v.z / l); }
inline vec3 cross(vec3 x, vec3 y) {
  return V(x.y * y.z - y.y * x.z, x.z * y.x - y.z * x.x, x.x * y.y - y.x * x.y);
}
inline vec3 vmin(vec3 a, vec3 b) { return V(std::fmin(a.x, b.x), std::fmin(a.y, b.y), std::fmin(a.z, b.z)); }
inline vec3 vmax(vec3 a, vec3 b) { return V(std::fmax(a.x, b.x), std::fmax(a.y, b.y), std::fmax(a.z, b.z)); }
inline vec3 clamp(vec3 v, vec3 lo, vec3 hi) { return vmin(vmax(v, lo), hi); }
inline vec3 vabs(vec3 v) { return V(std::fabs(v.x), std::fabs(v.y), std::fabs(v.z)); }
inline vec3 P3(const float* p) { return V(p[0], p[1], p[2]); }

// GL_LINEAR weights (GL 4.6 §8.14.2), optionally quantised to wbits fraction bits.
inline float weight(float a, int wbits) {
  if (wbits <= 0) return a;
  const float s = std::ldexp(1.0f, wbits);
  return std::nearbyint(a * s) / s;
}

// texture(sampler3D, u), comps channels, CLAMP_TO_EDGE: x-fastest float texels.
void tex3d(const float* v, const int N[3], int comps, vec3 u, int wbits, float* out) {
  const float tx = u.x * (float)N[0] - 0.5f, ty = u.y * (float)N[1] - 0.5f,
              tz = u.z * (float)N[2] - 0.5f;
  const float fx = std::floor(tx), fy = std::floor(ty), fz = std::floor(tz);
  const float a = weight(tx - fx, wbits), b = weight(ty - fy, wbits), g = weight(tz - fz, wbits);
  auto cl = [](float f, int n) { return std::min(std::max((int)f, 0), n - 1); };
  const int i0 = cl(fx, N[0]), i1 = cl(fx + 1.0f, N[0]);
  const int j0 = cl(fy, N[1]), j1 = cl(fy + 1.0f, N[1]);
  const int k0 = cl(fz, N[2]), k1 = cl(fz + 1.0f, N[2]);
  auto at = [&](int i, int j, int k, int c) {
    return v[(((int64_t)k * N[1] + j) * N[0] + i) * comps + c];
  };
  if (wbits < 0) {   // diagnostics: CVR-SPEC's filter arithmetic (fma texel coordinate, lerps)
    const float x = std::fmaf(u.x, (float)N[0], -0.5f), y = std::fmaf(u.y, (float)N[1], -0.5f),
                z = std::fmaf(u.z, (float)N[2], -0.5f);
    const float ex = std::floor(x), ey = std::floor(y), ez = std::floor(z);
    const float ax = x - ex, ay = y - ey, az = z - ez;
    const int p0 = cl(ex, N[0]), p1 = cl(ex + 1.0f, N[0]), q0 = cl(ey, N[1]), q1 = cl(ey + 1.0f, N[1]);
    const int r0 = cl(ez, N[2]), r1 = cl(ez + 1.0f, N[2]);
    auto lp = [](float x0, float x1, float t) { return std::fmaf(t, x1 - x0, x0); };
    for (int c = 0; c < comps; c++) {
      const float c00 = lp(at(p0, q0, r0, c), at(p1, q0, r0, c), ax);
      const float c10 = lp(at(p0, q1, r0, c), at(p1, q1, r0, c), ax);
      const float c01 = lp(at(p0, q0, r1, c), at(p1, q0, r1, c), ax);
      const float c11 = lp(at(p0, q1, r1, c), at(p1, q1, r1, c), ax);
      out[c] = lp(lp(c00, c10, ay), lp(c01, c11, ay), az);
    }
    return;
  }
  const float wa = 1.0f - a, wb = 1.0f - b, wg = 1.0f - g;
  for (int c = 0; c < comps; c++)
    out[c] = wa * wb * wg * at(i0, j0, k0, c) + a * wb * wg * at(i1, j0, k0, c) +
             wa * b * wg * at(i0, j1, k0, c) + a * b * wg * at(i1, j1, k0, c) +
             wa * wb * g * at(i0, j0, k1, c) + a * wb * g * at(i1, j0, k1, c) +
             wa * b * g * at(i0, j1, k1, c) + a * b * g * at(i1, j1, k1, c);
}

// texture(sampler1D, u) of an RGBA table, CLAMP_TO_EDGE.
void tex1d(const float* t, int n, float u, int wbits, float out[4]) {
  const float x = u * (float)n - 0.5f;
  const float f = std::floor(x);
  const float a = weight(x - f, wbits);
  const int i0 = std::min(std::max((int)f, 0), n - 1), i1 = std::min(std::max((int)f + 1, 0), n - 1);
  for (int c = 0; c < 4; c++) out[c] = (1.0f - a) * t[i0 * 4 + c] + a * t[i1 * 4 + c];
}

struct Cam {
  float View[16], tanf, aspect;
  vec3 eye;
};

Cam camera(const OracleRc1pass& P) {
  Cam c;
  oracle_lookat(P.eye, P.center, P.up, P.fovy_deg, c.View, &c.tanf);
  c.aspect = P.aspect > 0 ? P.aspect : (float)P.W / (float)P.H;
  c.eye = P3(P.eye);
  return c;
}

// vec3(VerPos.x * tan * aspect, VerPos.y * tan, -1.0) * mat3(View): component j is
// the dot product with column j (GLSL vector-times-matrix).
vec3 camera_dir(const Cam& C, int px, int py, int W, int H) {
  const float fx = (float)px + 0.5f, fy = (float)py + 0.5f;
  const float vx = (fx / (float)W) * 2.0f - 1.0f, vy = (fy / (float)H) * 2.0f - 1.0f;
  const vec3 c = V(vx * C.tanf * C.aspect, vy * C.tanf, -1.0f);
  const float* M = C.View;
  return V(dot(c, V(M[0], M[1], M[2])), dot(c, V(M[4], M[5], M[6])), dot(c, V(M[8], M[9], M[10])));
}

// IntersectBox / RayAABBIntersection (ray_bbox_intersection.comp:18-52)
bool ray_aabb(vec3 eye, vec3 vert_dir, vec3 G, vec3& dir, float& tnear, float& tfar) {
  const vec3 aabbmin = -G * 0.5f, aabbmax = G * 0.5f;
  dir = normalize(vert_dir);
  const vec3 invR = 1.0f / dir;
  const vec3 tbbmin = invR * (aabbmin - eye), tbbmax = invR * (aabbmax - eye);
  const vec3 tmin = vmin(tbbmin, tbbmax), tmax = vmax(tbbmin, tbbmax);
  tnear = std::fmax(std::fmax(tmin.x, tmin.y), tmin.z);
  tfar = std::fmin(std::fmin(tmax.x, tmax.y), tmax.z);
  const bool hit = tfar > tnear;
  tnear = std::fmax(tnear, 0.0f);
  return hit;
}

// ShadeBlinnPhong (ray_marching_1p.comp:48-81)
vec3 blinn_phong(const OracleRc1pass& P, vec3 G, vec3 Tpos, vec3 clr, int wbits) {
  float g[3];
  tex3d(P.grad, P.N, 3, Tpos / G, wbits, g);
  vec3 n = V(g[0], g[1], g[2]);
  if (n.x == 0.0f && n.y == 0.0f && n.z == 0.0f) return clr;
  const vec3 Wpos = Tpos - (G * 0.5f);
  n = normalize(n);
  const vec3 L = normalize(P3(P.light) - Wpos);
  const vec3 E = normalize(P3(P.eye) - Wpos);
  const vec3 Hv = normalize(E + L);
  const float dd = std::fmax(0.0f, dot(n, L));
  const float ds = std::fmax(0.0f, dot(Hv, n));
  const float pw = std::pow(ds, P.shininess);
  return (clr * (P.ka + P.kd * dd)) + P3(P.ispec) * P.ks * pw;
}

// The front-to-back loop shared by the three shaders: sample position from `pos_of`,
// density from `density_of`, shading `shade` for src.a > 0.
template <class Pos, class Dens, class Shade>
void march(const OracleRc1pass& P, float D, float step, const Pos& pos_of, const Dens& density_of,
           const Shade& shade, int wbits, float dst[4], uint32_t& cnt) {
  for (float s = 0.0f; s < D;) {
    const float h = std::fmin(step, D - s);
    const vec3 tp = pos_of(s, h);
    float src[4];
    tex1d(P.tf, P.tf_n, density_of(tp), wbits, src);
    cnt++;
    if (src[3] > 0.0f) {
      vec3 rgb = shade(tp, V(src[0], src[1], src[2]));
      float a = 1.0f - std::exp(-src[3] * h);
      rgb = rgb * a;
      const float om = 1.0f - dst[3];
      dst[0] = dst[0] + om * rgb.x;
      dst[1] = dst[1] + om * rgb.y;
      dst[2] = dst[2] + om * rgb.z;
      dst[3] = dst[3] + om * a;
      if (dst[3] > 0.99f) break;
    }
    s = s + h;
  }
}

// ---------------------------------------------------------------------------
// DOS: GetGaussianExtinction and the cones (ray_bbox_marching.comp:92-562)
// ---------------------------------------------------------------------------
struct Ext {
  const float* v; int res[3]; int nl; vec3 G; std::vector<int64_t> off; int wbits;
  float gge(vec3 tex_pos, float mip) const {
    int L = std::min(std::max((int)mip, 0), nl - 1);
    int d[3];
    for (int i = 0; i < 3; i++) d[i] = std::max(1, res[i] >> L);
    float rg;
    tex3d(v + off[L], d, 1, tex_pos / G, wbits, &rg);
    if (tex_pos.x < 0.0f || tex_pos.x > G.x || tex_pos.y < 0.0f || tex_pos.y > G.y ||
        tex_pos.z < 0.0f || tex_pos.z > G.z) {
      const float sg = std::pow(2.0f, mip);
      const vec3 c = clamp(tex_pos, V(0, 0, 0), G) - tex_pos;
      const float dist = c.x * c.x + c.y * c.y + c.z * c.z;
      rg = rg * std::exp(-(dist) / (2.0f * sg * sg));
    }
    return rg;
  }
};

// Cone1/3/7 Ray{Occlusion,Shadow}: the same accumulation, the split at the end of
// each stage; amptau = Tau_s * gaussian_amp.
float cone(const Ext& E, const OracleDosCone& C, vec3 pos, vec3 k, vec3 u, vec3 v) {
  float rays[7], last[7];
  float track = C.initial_step;
  rays[0] = 0.0f;
  last[0] = 0.0f;
  int s = 0;
  auto axis = [&](int a) {
    const float* A = C.axes + 3 * a;
    return k * A[2] + u * A[1] + v * A[0];
  };
  for (int i = 0; i < C.counts[0]; i++, s++) {
    const float* sec = C.sections + 4 * s;
    const float amptau = E.gge(pos + k * track, sec[1]) * sec[3];
    rays[0] += (last[0] + amptau) * sec[2] * C.ui_weight;
    last[0] = amptau;
    track += sec[0];
  }
  if (C.counts[1] + C.counts[2] == 0) return std::exp(-rays[0]);
  rays[2] = rays[0]; rays[1] = rays[0];
  last[2] = last[0]; last[1] = last[0];
  vec3 vk[7];
  for (int j = 0; j < 3; j++) vk[j] = axis(j);
  for (int i = 0; i < C.counts[1]; i++, s++) {
    const float* sec = C.sections + 4 * s;
    for (int j = 0; j < 3; j++) {
      const float amptau = E.gge(pos + vk[j] * track, sec[1]) * sec[3];
      rays[j] += (last[j] + amptau) * sec[2] * C.ui_weight;
      last[j] = amptau;
    }
    track += sec[0];
  }
  if (C.counts[2] == 0) return (std::exp(-rays[0]) + std::exp(-rays[1]) + std::exp(-rays[2])) / 3.0f;
  rays[6] = rays[5] = rays[2];
  rays[4] = rays[3] = rays[1];
  const float avg = (rays[2] + rays[1] + rays[0]) / 3.0f;
  rays[2] = rays[1] = rays[0];
  rays[0] = avg;
  last[6] = last[5] = last[2];
  last[4] = last[3] = last[1];
  const float avgt = (last[2] + last[1] + last[0]) / 3.0f;
  last[2] = last[1] = last[0];
  last[0] = avgt;
  for (int j = 0; j < 7; j++) vk[j] = axis(3 + j);
  for (int i = 0; i < C.counts[2]; i++, s++) {
    const float* sec = C.sections + 4 * s;
    for (int j = 0; j < 7; j++) {
      const float amptau = E.gge(pos + vk[j] * track, sec[1]) * sec[3];
      rays[j] += (last[j] + amptau) * sec[2] * C.ui_weight;
      last[j] = amptau;
    }
    track += sec[0];
  }
  return (std::exp(-rays[0]) + (std::exp(-rays[1]) + std::exp(-rays[2]) + std::exp(-rays[3]) +
                                std::exp(-rays[4]) + std::exp(-rays[5]) + std::exp(-rays[6])) *
                                   C.ray7w) /
         (1.0f + C.ray7w * 6.0f);
}

// ---------------------------------------------------------------------------
// EBS: the SAT fetches and the box chains (ebs_ray_bbox_marching.comp:63-481)
// ---------------------------------------------------------------------------
struct Sat {
  const float* v; int dims[3]; vec3 S, G, inv_vs, min_sat, max_sat; int wbits;
  float f(float x, float y, float z) const {   // GetSummed3Density
    float r;
    tex3d(v, dims, 1, V(x, y, z) * inv_vs, wbits, &r);
    return r;
  }
  float box(vec3 p1, vec3 p2) const {          // EvaluateSAT3D
    const float V1 = f(p2.x, p2.y, p2.z), V2 = f(p1.x, p2.y, p2.z);
    const float V3 = f(p2.x, p2.y, p1.z), V4 = f(p1.x, p2.y, p1.z);
    const float V5 = f(p2.x, p1.y, p2.z), V6 = f(p1.x, p1.y, p2.z);
    const float V7 = f(p2.x, p1.y, p1.z), V8 = f(p1.x, p1.y, p1.z);
    return (V1 - V2 - V3 + V4 - V5 + V6 + V7 - V8);
  }
  float ao_box(vec3 p1, vec3 p2) const {       // EvaluateAmbientOcclusionSAT3D
    return box(clamp(p1 + S, min_sat, max_sat), clamp(p2 + S, min_sat, max_sat));
  }
  float shadow_box(vec3 p1, vec3 p2, float uiw) const {   // EvaluateShadowSAT3D (texture path)
    const float volquery = ((std::fabs(p1.x - p2.x) / S.x)) * ((std::fabs(p1.y - p2.y) / S.y)) *
                           ((std::fabs(p1.z - p2.z) / S.z));
    p1 = clamp(p1 + S, min_sat, max_sat);
    p2 = clamp(p2 + S, min_sat, max_sat);
    return ((box(p1, p2) / volquery)) * uiw;
  }
};

float ebs_ao(const Sat& T, vec3 tx, int shells, float R) {   // ExtinctionAmbientOcclusion
  const float SAT_Sh0 = T.ao_box(tx - R * T.S, tx + R * T.S);
  const float rsh0 = R;
  const float tSh0 = SAT_Sh0 * (1.0f / (rsh0 * rsh0));
  float SAT_Shi = SAT_Sh0, tshi = tSh0;
  for (int i = 1; i < shells; i++) {
    const float r1 = R * (float)(i + 1);
    const float SAT_Shi_1 = T.ao_box(tx - r1 * T.S, tx + r1 * T.S);
    tshi = tshi + (SAT_Shi_1 - SAT_Shi) * (1.0f / (r1 * r1));
    SAT_Shi = SAT_Shi_1;
  }
  const float rshi = R * (float)shells;
  const float W_A = 1.0f / (rshi * rshi);
  return std::exp(-(W_A * tshi));
}

struct ConeCS { float p_cs, p_sn, n_cs, n_sn; };

float cone_z(const Sat& T, const OracleEbs& Q, const ConeCS& c, vec3 pos, vec3 cv) {
  float Stau = 0.0f;
  float signal = 1.0f;
  if (cv.z < 0) signal = -1.0f;
  const vec3 proj_y = normalize(V(0.0f, cv.y, cv.z));
  const vec3 proj_x = normalize(V(cv.x, 0.0f, cv.z));
  const vec3 pj_x1 = normalize(V(proj_x.x * c.n_cs - proj_x.z * c.n_sn, 0.0f, proj_x.x * c.n_sn + proj_x.z * c.n_cs));
  const vec3 pj_x2 = normalize(V(proj_x.x * c.p_cs - proj_x.z * c.p_sn, 0.0f, proj_x.x * c.p_sn + proj_x.z * c.p_cs));
  const vec3 pj_y1 = normalize(V(0.0f, proj_y.y * c.n_cs - proj_y.z * c.n_sn, proj_y.y * c.n_sn + proj_y.z * c.n_cs));
  const vec3 pj_y2 = normalize(V(0.0f, proj_y.y * c.p_cs - proj_y.z * c.p_sn, proj_y.y * c.p_sn + proj_y.z * c.p_cs));
  const float si = Q.interval * signal * T.S.z;
  float z_pos = Q.initial_step * signal * T.S.z;
  const float vmn = T.S.z * 0.5f, vmx = T.G.z - T.S.z * 0.5f;
  while ((z_pos / cv.z) < Q.max_distance && (pos.z + (z_pos + si) > vmn && pos.z + (z_pos + si) < vmx)) {
    const float z_mean = std::fabs(z_pos + si * 0.5f);
    const float p_x1 = pj_x1.x * (z_mean / std::fabs(pj_x1.z)), p_x2 = pj_x2.x * (z_mean / std::fabs(pj_x2.z));
    const float p_y1 = pj_y1.y * (z_mean / std::fabs(pj_y1.z)), p_y2 = pj_y2.y * (z_mean / std::fabs(pj_y2.z));
    float x1 = std::fmin(p_x1, p_x2), x2 = std::fmax(p_x1, p_x2);
    float y1 = std::fmin(p_y1, p_y2), y2 = std::fmax(p_y1, p_y2);
    const float xdiff = std::fabs(x2 - x1), ydiff = std::fabs(y2 - y1);
    const float xs = (std::ceil(xdiff / T.S.x) - (xdiff / T.S.x)) * 0.5f;
    const float ys = (std::ceil(ydiff / T.S.y) - (ydiff / T.S.y)) * 0.5f;
    x1 = x1 - xs * T.S.x; x2 = x2 + xs * T.S.x;
    y1 = y1 - ys * T.S.y; y2 = y2 + ys * T.S.y;
    const float z1 = std::fmin(z_pos, z_pos + si), z2 = std::fmax(z_pos, z_pos + si);
    Stau += T.shadow_box(pos + V(x1, y1, z1), pos + V(x2, y2, z2), Q.ui_weight);
    z_pos = z_pos + si;
  }
  return Stau;
}

float cone_y(const Sat& T, const OracleEbs& Q, const ConeCS& c, vec3 pos, vec3 cv) {
  float Stau = 0.0f;
  float signal = 1.0f;
  if (cv.y < 0) signal = -1.0f;
  const vec3 proj_x = normalize(V(cv.x, cv.y, 0.0f));
  const vec3 proj_z = normalize(V(0.0f, cv.y, cv.z));
  const vec3 pj_x1 = normalize(V(proj_x.x * c.n_cs - proj_x.y * c.n_sn, proj_x.x * c.n_sn + proj_x.y * c.n_cs, 0.0f));
  const vec3 pj_x2 = normalize(V(proj_x.x * c.p_cs - proj_x.y * c.p_sn, proj_x.x * c.p_sn + proj_x.y * c.p_cs, 0.0f));
  const vec3 pj_z1 = normalize(V(0.0f, proj_z.z * c.n_sn + proj_z.y * c.n_cs, proj_z.z * c.n_cs - proj_z.y * c.n_sn));
  const vec3 pj_z2 = normalize(V(0.0f, proj_z.z * c.p_sn + proj_z.y * c.p_cs, proj_z.z * c.p_cs - proj_z.y * c.p_sn));
  const float si = Q.interval * signal * T.S.y;
  float y_pos = Q.initial_step * signal * T.S.y;
  const float vmn = T.S.y * 0.5f, vmx = T.G.y - T.S.y * 0.5f;
  while ((y_pos / cv.y) < Q.max_distance && (pos.y + (y_pos + si) > vmn && pos.y + (y_pos + si) < vmx)) {
    const float y_mean = std::fabs(y_pos + si * 0.5f);
    const float p_x1 = pj_x1.x * (y_mean / std::fabs(pj_x1.y)), p_x2 = pj_x2.x * (y_mean / std::fabs(pj_x2.y));
    const float p_z1 = pj_z1.z * (y_mean / std::fabs(pj_z1.y)), p_z2 = pj_z2.z * (y_mean / std::fabs(pj_z2.y));
    float x1 = std::fmin(p_x1, p_x2), x2 = std::fmax(p_x1, p_x2);
    float z1 = std::fmin(p_z1, p_z2), z2 = std::fmax(p_z1, p_z2);
    const float xdiff = std::fabs(x2 - x1), zdiff = std::fabs(z2 - z1);
    const float xs = (std::ceil(xdiff / T.S.x) - (xdiff / T.S.x)) * 0.5f;
    const float zs = (std::ceil(zdiff / T.S.z) - (zdiff / T.S.z)) * 0.5f;
    x1 = x1 - xs * T.S.x; x2 = x2 + xs * T.S.x;
    z1 = z1 - zs * T.S.z; z2 = z2 + zs * T.S.z;
    const float y1 = std::fmin(y_pos, y_pos + si), y2 = std::fmax(y_pos, y_pos + si);
    Stau += T.shadow_box(pos + V(x1, y1, z1), pos + V(x2, y2, z2), Q.ui_weight);
    y_pos = y_pos + si;
  }
  return Stau;
}

float cone_x(const Sat& T, const OracleEbs& Q, const ConeCS& c, vec3 pos, vec3 cv) {
  float Stau = 0.0f;
  float signal = 1.0f;
  if (cv.x < 0) signal = -1.0f;
  const vec3 proj_y = normalize(V(cv.x, cv.y, 0.0f));
  const vec3 proj_z = normalize(V(cv.x, 0.0f, cv.z));
  const vec3 pj_y1 = normalize(V(proj_y.y * c.n_sn + proj_y.x * c.n_cs, proj_y.y * c.n_cs - proj_y.x * c.n_sn, 0.0f));
  const vec3 pj_y2 = normalize(V(proj_y.y * c.p_sn + proj_y.x * c.p_cs, proj_y.y * c.p_cs - proj_y.x * c.p_sn, 0.0f));
  const vec3 pj_z1 = normalize(V(proj_z.z * c.n_sn + proj_z.x * c.n_cs, 0.0f, proj_z.z * c.n_cs - proj_z.x * c.n_sn));
  const vec3 pj_z2 = normalize(V(proj_z.z * c.p_sn + proj_z.x * c.p_cs, 0.0f, proj_z.z * c.p_cs - proj_z.x * c.p_sn));
  const float si = Q.interval * signal * T.S.x;
  float x_pos = Q.initial_step * signal * T.S.x;
  const float vmn = T.S.x * 0.5f, vmx = T.G.x - T.S.x * 0.5f;
  while ((x_pos / cv.x) < Q.max_distance && (pos.x + (x_pos + si) > vmn && pos.x + (x_pos + si) < vmx)) {
    const float x_mean = std::fabs(x_pos + si * 0.5f);
    const float p_y1 = pj_y1.y * (x_mean / std::fabs(pj_y1.x)), p_y2 = pj_y2.y * (x_mean / std::fabs(pj_y2.x));
    const float p_z1 = pj_z1.z * (x_mean / std::fabs(pj_z1.x)), p_z2 = pj_z2.z * (x_mean / std::fabs(pj_z2.x));
    float y1 = std::fmin(p_y1, p_y2), y2 = std::fmax(p_y1, p_y2);
    float z1 = std::fmin(p_z1, p_z2), z2 = std::fmax(p_z1, p_z2);
    const float ydiff = std::fabs(y2 - y1), zdiff = std::fabs(z2 - z1);
    const float ys = (std::ceil(ydiff / T.S.y) - (ydiff / T.S.y)) * 0.5f;
    const float zs = (std::ceil(zdiff / T.S.z) - (zdiff / T.S.z)) * 0.5f;
    y1 = y1 - ys * T.S.y; y2 = y2 + ys * T.S.y;
    z1 = z1 - zs * T.S.z; z2 = z2 + zs * T.S.z;
    const float x1 = std::fmin(x_pos, x_pos + si), x2 = std::fmax(x_pos, x_pos + si);
    Stau += T.shadow_box(pos + V(x1, y1, z1), pos + V(x2, y2, z2), Q.ui_weight);
    x_pos = x_pos + si;
  }
  return Stau;
}

// Rows [y0, y1): the per-pixel driver of the three mains.  `kind` 0 = rc1pass
// (u = p / G), 1 = DOS/EBS (u = p * (1 / G)); shade(tx_pos, rgb, cam_dir, dir).
template <class Shade>
uint64_t rows_loop(const OracleRc1pass& P, int kind, int y0, int y1, float* out, uint32_t* counts,
                   int nthreads, int wbits, const Shade& shade) {
  const Cam C = camera(P);
  const vec3 G = V((float)P.N[0] * P.scale[0], (float)P.N[1] * P.scale[1], (float)P.N[2] * P.scale[2]);
  const vec3 invG = 1.0f / G;
#ifdef _OPENMP
  if (nthreads > 0) omp_set_num_threads(nthreads);
#endif
  y0 = std::max(0, y0);
  y1 = std::min(P.H, y1);
  uint64_t total = 0;
#pragma omp parallel for schedule(dynamic, 1) reduction(+ : total)
  for (int py = y0; py < y1; py++) {
    for (int px = 0; px < P.W; px++) {
      const int64_t pix = (int64_t)py * P.W + px;
      float dst[4] = {0, 0, 0, 0};
      uint32_t cnt = 0;
      // camera_dir = normalize(vec3(...) * mat3(View)) in all three mains
      const vec3 cd = normalize(camera_dir(C, px, py, P.W, P.H));
      vec3 dir;
      float tnear, tfar;
      if (ray_aabb(C.eye, cd, G, dir, tnear, tfar)) {
        const float D = std::fabs(tfar - tnear);
        const vec3 tex_pos = (C.eye + dir * tnear) + (G * 0.5f);
        auto pos_of = [&](float s, float h) { return tex_pos + dir * (s + h * 0.5f); };
        auto dens = [&](vec3 tp) {
          float d;
          tex3d(P.vol, P.N, 1, kind == 0 ? tp / G : tp * invG, wbits, &d);
          return d;
        };
        auto sh = [&](vec3 tp, vec3 rgb) { return shade(tp, rgb, cd, dir); };
        march(P, D, P.step, pos_of, dens, sh, wbits, dst, cnt);
      }
      if (out) for (int k = 0; k < 4; k++) out[pix * 4 + k] = dst[k];
      if (counts) counts[pix] = cnt;
      total += cnt;
    }
  }
  return total;
}

}  // namespace

// ray_marching_1p.comp read literally (EA, or Blinn-Phong with P.phong).
ORACLE_API uint64_t oracle_render_rc1pass_literal(const OracleRc1pass* P, int y0, int y1,
                                                  float* out_rgba, uint32_t* out_counts,
                                                  int nthreads, int wbits) {
  const vec3 G = V((float)P->N[0] * P->scale[0], (float)P->N[1] * P->scale[1],
                   (float)P->N[2] * P->scale[2]);
  auto shade = [&](vec3 tp, vec3 rgb, vec3, vec3) {
    return (P->phong && P->grad) ? blinn_phong(*P, G, tp, rgb, wbits) : rgb;
  };
  return rows_loop(*P, 0, y0, y1, out_rgba, out_counts, nthreads, wbits, shade);
}

// ray_bbox_marching.comp read literally.
ORACLE_API uint64_t oracle_render_dos_literal(const OracleDos* Q, int y0, int y1, float* out_rgba,
                                              uint32_t* out_counts, int nthreads, int wbits) {
  const OracleRc1pass& P = Q->base;
  const vec3 G = V((float)P.N[0] * P.scale[0], (float)P.N[1] * P.scale[1], (float)P.N[2] * P.scale[2]);
  Ext E{Q->ext, {Q->ext_res[0], Q->ext_res[1], Q->ext_res[2]}, Q->ext_levels, G, {}, wbits};
  E.off.assign(E.nl + 1, 0);
  for (int L = 0; L < E.nl; L++) {
    int64_t n = 1;
    for (int i = 0; i < 3; i++) n *= std::max(1, E.res[i] >> L);
    E.off[L + 1] = E.off[L] + n;
  }
  const float spot_cos = std::cos(3.14159265358979323846f * Q->spot_angle_deg / 180.0f);
  const vec3 light = P3(P.light), lfwd = P3(Q->light_forward), lup = P3(Q->light_up),
             lright = P3(Q->light_right), eye = P3(P.eye);
  auto shade = [&](vec3 tx, vec3 rgb, vec3 camera_dir, vec3) {
    const vec3 v_right = normalize(cross(camera_dir, V(0, 1, 0)));
    const vec3 v_up = normalize(cross(-camera_dir, v_right));
    float ka = 0.0f, kd = 0.0f, ks = 0.0f, iocc = 0.0f, isdw = 0.0f;
    if (Q->apply_occlusion) {   // OcclusionEvaluationKernel
      ka = P.ka;
      const vec3 k = normalize(eye - (tx - (G * 0.5f)));
      iocc = cone(E, Q->occ, tx, k, v_up, v_right);
    }
    if (Q->apply_shadow) {      // ShadowEvaluationKernel; Cone1RayShadow(pos, k, u, v)
      kd = P.kd;
      ks = P.ks;
      vec3 k, u, v;
      bool lit = true;
      if (Q->shadow_type == 2) {
        k = lfwd; v = lup; u = lright;
      } else {
        const vec3 cv = normalize(light - (tx - (G / 2.0f)));
        k = cv;
        u = normalize(cross(k, lright));
        v = normalize(cross(k, u));
        if (Q->shadow_type == 1 && dot(cv, lfwd) < spot_cos) lit = false;
      }
      isdw = lit ? cone(E, Q->sdw, tx, k, v, u) : 0.0f;
    }
    if (P.phong && P.grad) {
      const vec3 Wpos = tx - (G * 0.5f);
      float g[3];
      tex3d(P.grad, P.N, 3, tx / G, wbits, g);
      vec3 n = V(g[0], g[1], g[2]);
      if (n.x != 0.0f || n.y != 0.0f || n.z != 0.0f) {
        n = normalize(n);
        const vec3 L = normalize(light - Wpos), Ed = normalize(eye - Wpos);
        const vec3 Hv = normalize(Ed + L);
        const float dd = std::fmax(0.0f, dot(n, L)), ds = std::fmax(0.0f, dot(Hv, n));
        return rgb * ((1.0f / (ka + kd)) * (iocc * ka + isdw * kd * dd)) +
               P3(P.ispec) * (isdw * ks * std::pow(ds, P.shininess));
      }
      return rgb;
    }
    return (1.0f / (ka + kd)) * (rgb * iocc * ka + rgb * isdw * kd);
  };
  return rows_loop(P, 1, y0, y1, out_rgba, out_counts, nthreads, wbits, shade);
}

// ebs_ray_bbox_marching.comp read literally.
ORACLE_API uint64_t oracle_render_ebs_literal(const OracleEbs* Q, int y0, int y1, float* out_rgba,
                                              uint32_t* out_counts, int nthreads, int wbits) {
  const OracleRc1pass& P = Q->base;
  Sat T;
  T.v = Q->sat;
  for (int i = 0; i < 3; i++) T.dims[i] = Q->sat_dims[i];
  T.S = P3(P.scale);
  T.G = V((float)P.N[0] * P.scale[0], (float)P.N[1] * P.scale[1], (float)P.N[2] * P.scale[2]);
  T.inv_vs = 1.0f / (T.G + T.S * 2.0f);
  T.min_sat = T.S * 0.5f;
  T.max_sat = T.G + T.S * 1.5f;
  T.wbits = wbits;
  const ConeCS cs{std::cos(Q->cone_angle), std::sin(Q->cone_angle), std::cos(-Q->cone_angle),
                  std::sin(-Q->cone_angle)};
  const vec3 light = P3(P.light), eye = P3(P.eye), lfwd = P3(Q->light_forward);
  auto shade = [&](vec3 tx, vec3 rgb, vec3, vec3) {
    float ka = 0.0f, kd = 0.0f, ks = 0.0f, iocc = 0.0f, isdw = 0.0f;
    if (Q->apply_occlusion) {
      ka = P.ka;
      iocc = ebs_ao(T, tx, Q->occ_shells, Q->occ_radius);
    }
    if (Q->apply_shadow) {   // ExtinctionDirectionalShadows
      kd = P.kd;
      ks = P.ks;
      const vec3 realpos = tx - (T.G * 0.5f);
      const vec3 cv = Q->shadow_type == 0 ? normalize(light - realpos) : normalize(lfwd);
      const vec3 ac = vabs(cv);
      float Stau;
      if (ac.z > ac.x && ac.z > ac.y) Stau = cone_z(T, *Q, cs, tx, cv);
      else if (ac.y > ac.x) Stau = cone_y(T, *Q, cs, tx, cv);
      else Stau = cone_x(T, *Q, cs, tx, cv);
      isdw = std::exp(-Stau);
    }
    if (P.phong && P.grad) {
      const vec3 Wpos = tx - (T.G * 0.5f);
      float g[3];
      tex3d(P.grad, P.N, 3, tx / T.G, wbits, g);
      vec3 n = V(g[0], g[1], g[2]);
      if (n.x != 0.0f || n.y != 0.0f || n.z != 0.0f) {
        n = normalize(n);
        const vec3 L = normalize(light - Wpos), Ed = normalize(eye - Wpos);
        const vec3 Hv = normalize(Ed + L);
        const float dd = std::fmax(0.0f, dot(n, L)), ds = std::fmax(0.0f, dot(Hv, n));
        return (1.0f / (ka + kd)) * (rgb * iocc * ka + isdw * (rgb * kd * dd)) +
               isdw * (ks * P3(P.ispec) * std::pow(ds, P.shininess));
      }
      return rgb;
    }
    return (1.0f / (ka + kd)) * (rgb * iocc * ka + rgb * isdw * kd);
  };
  return rows_loop(P, 1, y0, y1, out_rgba, out_counts, nthreads, wbits, shade);
}
