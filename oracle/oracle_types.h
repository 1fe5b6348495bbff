// oracle_types.h — parameter blocks of the CPU oracle (TEST INFRASTRUCTURE ONLY:
// tests/, smoke() and bench.py's CPU leg load liboracle.so; the product never does).
// Shared by the CVR-SPEC restatement (cvr_oracle.cpp) and the literal GLSL reading
// (glsl_literal.cpp).
#pragma once
#include <cstdint>

struct OracleRc1pass {
  // volume (float values of the stored halves), x-fastest
  const float* vol; int N[3]; float scale[3];
  const float* tf; int tf_n;           // tf_n x (r,g,b,tau), half-rounded
  const float* grad;                   // N voxels x 3, or null
  // camera
  float eye[3], center[3], up[3], fovy_deg, aspect;
  int W, H;
  float step;
  int phong; float ka, kd, ks, shininess; float ispec[3]; float light[3];
  int filter_bits;                     // GL_LINEAR weights at this many fraction bits (0: exact): every fetch of rc1pass, DOS, EBS
};

struct OracleDosCone {
  const float* sections; int counts[3];   // n x 4 (interval, mip, d_integral, amplitude)
  float axes[30]; float initial_step, ray7w, ui_weight;
};

struct OracleDos {
  OracleRc1pass base;                     // volume, TF (RGBt), camera, step, Blinn-Phong
  const float* ext; int ext_res[3]; int ext_levels;
  int apply_occlusion, apply_shadow, shadow_type;
  float light_forward[3], light_up[3], light_right[3], spot_angle_deg;
  OracleDosCone occ, sdw;
};

struct OracleEbs {
  OracleRc1pass base;
  const float* sat; int sat_dims[3];   // the float SAT (W+2)(H+2)(D+2), x-fastest
  int apply_occlusion, occ_shells; float occ_radius;
  int apply_shadow, shadow_type;       // 0: point light, 1: LightCamForward
  float cone_angle;                    // DirSdwConeAngle (radians, float)
  float interval, initial_step, ui_weight, max_distance;
  float light_forward[3];
};
