// dos.hip — directional-occlusion shading (cppvolrend rc1pdosct) on gfx950.
//
//  * the extinction-coefficient mip volume (ExtinctionCoefficientVolume, custom
//    resolution path: extcoefvolumegenerator.cpp:230-408 and glslextgen/*.comp):
//    level 0 = 7^3-tap Gaussian of the TF opacity over the volume, level L = the
//    same Gaussian (sigma 2^L) over level L-1, then tau = -log(1 - opacity);
//    every level stored as fp16 (GL_R16F), x-fastest, levels concatenated;
//  * the ray-march of ray_bbox_marching.comp:658-734 with ShadeSample (:607-656):
//    for every sample with alpha > 0, a cone-traced ambient occlusion toward the
//    eye (Cone1/3/7RayOcclusion, :116-333) and a cone-traced shadow toward the
//    light (Cone1/3/7RayShadow, :337-562), each a trapezoid accumulation of
//    Gaussian-filtered extinctions along 1 -> 3 -> 7 rays.
//
// Arithmetic follows CVR-SPEC exactly as oracle/cvr_oracle.cpp (oracle_ext_volume,
// oracle_render_dos) so results are bit-identical.  Compiled -ffp-contract=off.
#include <hip/hip_runtime.h>
#include <cstdint>

#include "cvr_device.h"
#include "march_common.h"

namespace cvr {

// ---------------------------------------------------------------------------
// fp16 level sampling (trilinear, clamp-to-edge, texel-centre convention)
// ---------------------------------------------------------------------------

__device__ __forceinline__ float h2f(uint16_t h) { return (float)__builtin_bit_cast(_Float16, h); }

// float -> binary16, round to nearest even (v_cvt_f16_f32)
__device__ __forceinline__ uint16_t f2h_rne(float f) { return __builtin_bit_cast(uint16_t, (_Float16)f); }

// x, y, z in texel space of a d[0] x d[1] x d[2] level.  Clamping to [0, d-1]
// gives the same values as GL's CLAMP_TO_EDGE on [-1, d-1] (see sample_pos).
__device__ __forceinline__ float sample_level(const uint16_t* __restrict__ lv, const int d[3],
                                              float x, float y, float z) {
  x = __builtin_amdgcn_fmed3f(x, 0.0f, (float)(d[0] - 1));
  y = __builtin_amdgcn_fmed3f(y, 0.0f, (float)(d[1] - 1));
  z = __builtin_amdgcn_fmed3f(z, 0.0f, (float)(d[2] - 1));
  const int ix = (int)x, iy = (int)y, iz = (int)z;
  const float ax = __builtin_amdgcn_fractf(x), ay = __builtin_amdgcn_fractf(y),
              az = __builtin_amdgcn_fractf(z);
  const int x1 = min(ix + 1, d[0] - 1), y1 = min(iy + 1, d[1] - 1), z1 = min(iz + 1, d[2] - 1);
  const long long sy = d[0], sz = (long long)d[0] * d[1];
  const long long r00 = iz * sz + iy * sy, r10 = iz * sz + y1 * sy;
  const long long r01 = z1 * sz + iy * sy, r11 = z1 * sz + y1 * sy;
  const float c00 = lerpf(h2f(lv[r00 + ix]), h2f(lv[r00 + x1]), ax);
  const float c10 = lerpf(h2f(lv[r10 + ix]), h2f(lv[r10 + x1]), ax);
  const float c01 = lerpf(h2f(lv[r01 + ix]), h2f(lv[r01 + x1]), ax);
  const float c11 = lerpf(h2f(lv[r11 + ix]), h2f(lv[r11 + x1]), ax);
  return lerpf(lerpf(c00, c10, ay), lerpf(c01, c11, ay), az);
}

// ---------------------------------------------------------------------------
// Extinction-coefficient volume
// ---------------------------------------------------------------------------

struct ExtBuildArgs {
  // the volume (cell8 layout, see sample_pos) and the opacity TF
  CellGrid cells;
  float nm1[3];
  int N[3];
  float G[3];                 // VolumeGridSize
  int tf_n;
  // this level
  int L;
  int d[3], pd[3];            // this level's and the previous level's dimensions
  float S;                    // sigma0 * 2^L
  float vs[3];                // G / d (voxel size)
};

// One thread per voxel of level L (gen_extcoefvol_anysize.comp:36-76 for L = 0,
// gen_extcoefvol_anysize_mmlevel.comp:35-78 for L >= 1).  The 343 tap weights are
// shared by the block (LDS).  L = 0 samples the volume cells and the opacity TF
// (padded alpha table in LDS); L >= 1 samples level L-1 (`prev`).
__global__ void __launch_bounds__(256)
ext_level_kernel(ExtBuildArgs E, const uint4* __restrict__ cells, const float4* __restrict__ tf,
                 const uint16_t* __restrict__ prev, uint16_t* __restrict__ out) {
  __shared__ float w_lds[343];
  __shared__ float a_lds[kMaxTfLds + 2];
  const float S = E.S, S3 = (S * S) * S, den = (2.0f * S) * S;
  for (int t = threadIdx.x; t < 343; t += blockDim.x) {
    const int tx = t / 49 - 3, ty = (t / 7) % 7 - 3, tz = t % 7 - 3;
    const float fx = (float)tx * S, fy = (float)ty * S, fz = (float)tz * S;
    w_lds[t] = S3 * cvr_expf(-((fx * fx + fy * fy) + fz * fz) / den);
  }
  if (E.L == 0)
    for (int i = threadIdx.x; i < E.tf_n + 2; i += blockDim.x)
      a_lds[i] = tf[min(max(i - 1, 0), E.tf_n - 1)].w;
  __syncthreads();
  const long long nv = (long long)E.d[0] * E.d[1] * E.d[2];
  const long long v = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (v >= nv) return;
  const int i = (int)(v % E.d[0]), j = (int)((v / E.d[0]) % E.d[1]),
            k = (int)(v / ((long long)E.d[0] * E.d[1]));
  const float gx = ((float)i + 0.5f) * E.vs[0], gy = ((float)j + 0.5f) * E.vs[1],
              gz = ((float)k + 0.5f) * E.vs[2];
  const float fn = (float)E.tf_n;
  float swc = 0.0f, sw = 0.0f;
  int t = 0;
  for (int tx = -3; tx <= 3; tx++)
    for (int ty = -3; ty <= 3; ty++)
      for (int tz = -3; tz <= 3; tz++, t++) {
        const float w = w_lds[t];
        const float px = gx + (float)tx * S, py = gy + (float)ty * S, pz = gz + (float)tz * S;
        const float ux = px / E.G[0], uy = py / E.G[1], uz = pz / E.G[2];
        float c = 0.0f;
        if (!(ux < 0.0f || uy < 0.0f || uz < 0.0f || ux > 1.0f || uy > 1.0f || uz > 1.0f)) {
          if (E.L == 0) {
            Rc1passArgs A;   // sample_pos reads only nm1 and the cell pitches
            A.nm1[0] = E.nm1[0]; A.nm1[1] = E.nm1[1]; A.nm1[2] = E.nm1[2];
            A.cells = E.cells;
            const SamplePos sp = sample_pos(fmaf(ux, (float)E.N[0], -0.5f),
                                            fmaf(uy, (float)E.N[1], -0.5f),
                                            fmaf(uz, (float)E.N[2], -0.5f), A);
            const float dens = trilerp_cell(cells[sp.idx], sp.ax, sp.ay, sp.az);
            // texture(TF, d).a: padded table, x = d*n - 0.5
            const float xt = fmaf(dens, fn, -0.5f);
            const float fl = floorf(xt);
            const int ti = (int)fl + 1;
            c = lerpf(a_lds[ti], a_lds[ti + 1], xt - fl);
          } else {
            c = sample_level(prev, E.pd, fmaf(ux, (float)E.pd[0], -0.5f),
                             fmaf(uy, (float)E.pd[1], -0.5f), fmaf(uz, (float)E.pd[2], -0.5f));
          }
        }
        swc = swc + w * c;
        sw = sw + w;
      }
  out[v] = f2h_rne(swc / sw);
}

// backtotau.comp:11-34: tau = -1 * log(1 - opacity), in place over all levels.
__global__ void ext_to_tau_kernel(uint16_t* __restrict__ lv, long long n) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) lv[i] = f2h_rne(-1.0f * cvr_logf(1.0f - h2f(lv[i])));
}

hipError_t launch_ext_volume(const Ctx& c, const float4* d_tf_rgba, int tf_n, const int res[3],
                             float sigma0, int nlevels, const long long* off, uint16_t* d_ext,
                             hipStream_t s) {
  if (tf_n > kMaxTfLds) return hipErrorInvalidValue;
  ExtBuildArgs E{};
  E.cells = c.cells;
  for (int i = 0; i < 3; i++) {
    E.N[i] = c.N[i];
    E.nm1[i] = (float)(c.N[i] - 1);
    E.G[i] = (float)c.N[i] * c.scale[i];
  }
  E.tf_n = tf_n;
  const uint4* cells = (const uint4*)c.d_cells + c.cells.linear_origin;
  for (int L = 0; L < nlevels; L++) {
    E.L = L;
    for (int i = 0; i < 3; i++) {
      E.d[i] = res[i] >> L > 1 ? res[i] >> L : 1;
      E.pd[i] = L == 0 ? 1 : (res[i] >> (L - 1) > 1 ? res[i] >> (L - 1) : 1);
      E.vs[i] = E.G[i] / (float)E.d[i];
    }
    E.S = L == 0 ? sigma0 : sigma0 * (float)(1 << L);
    const long long nv = (long long)E.d[0] * E.d[1] * E.d[2];
    hipLaunchKernelGGL(ext_level_kernel, dim3((unsigned)((nv + 255) / 256)), dim3(256), 0, s, E,
                       cells, d_tf_rgba, L == 0 ? nullptr : d_ext + off[L - 1], d_ext + off[L]);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
  }
  const long long n = off[nlevels];
  hipLaunchKernelGGL(ext_to_tau_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, d_ext, n);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------
// Cone tracing
// ---------------------------------------------------------------------------

// GetGaussianExtinction (:92-112): textureLod at an integer level (clamped to the
// pyramid), plus the CONSIDER_BORDERS attenuation outside the volume box.
__device__ __forceinline__ float gge(const DosArgs& Q, const uint16_t* __restrict__ ext, f3 p,
                                     float mip) {
  int L = (int)mip;
  L = min(max(L, 0), Q.ext_levels - 1);
  const int* d = Q.ext_dim[L];
  const float ux = p.x / Q.G[0], uy = p.y / Q.G[1], uz = p.z / Q.G[2];
  float rg = sample_level(ext + Q.ext_off[L], d, fmaf(ux, (float)d[0], -0.5f),
                          fmaf(uy, (float)d[1], -0.5f), fmaf(uz, (float)d[2], -0.5f));
  if (p.x < 0.0f || p.x > Q.G[0] || p.y < 0.0f || p.y > Q.G[1] || p.z < 0.0f || p.z > Q.G[2]) {
    const float sg = ldexpf(1.0f, (int)mip);   // pow(2.0, mip) of an integer level
    const float cx = fminf(fmaxf(p.x, 0.0f), Q.G[0]) - p.x;
    const float cy = fminf(fmaxf(p.y, 0.0f), Q.G[1]) - p.y;
    const float cz = fminf(fmaxf(p.z, 0.0f), Q.G[2]) - p.z;
    const float dist = (cx * cx + cy * cy) + cz * cz;
    rg = rg * cvr_expf(-(dist) / ((2.0f * sg) * sg));
  }
  return rg;
}

__device__ __forceinline__ f3 vmad(f3 d, float t, f3 p) {
  return f3{fmaf(d.x, t, p.x), fmaf(d.y, t, p.y), fmaf(d.z, t, p.z)};
}
__device__ __forceinline__ f3 cone_axis(const float* a, f3 k, f3 u, f3 v) {
  return f3{fmaf(v.x, a[0], fmaf(u.x, a[1], k.x * a[2])), fmaf(v.y, a[0], fmaf(u.y, a[1], k.y * a[2])),
            fmaf(v.z, a[0], fmaf(u.z, a[1], k.z * a[2]))};
}
__device__ __forceinline__ f3 cross3(f3 x, f3 y) {   // glm / GLSL cross, no fma
  return f3{x.y * y.z - y.y * x.z, x.z * y.x - y.z * x.x, x.x * y.y - y.x * x.y};
}

// Cone1/3/7 RayOcclusion and Cone1/3/7 RayShadow (the same accumulation): the
// visibility exp(-sum) of a cone from `pos` along k, split 1 -> 3 -> 7 rays.
__device__ float cone_trace(const DosArgs& Q, const DosCone& C, const uint16_t* __restrict__ ext,
                            f3 pos, f3 k, f3 u, f3 v) {
  float rays[7], last[7];
  float track = C.initial_step;
  rays[0] = 0.0f;
  last[0] = 0.0f;
  const float4* sec = C.sections;
  int s = 0;
  for (int i = 0; i < C.counts[0]; i++, s++) {
    const float4 e = sec[s];
    const float amptau = gge(Q, ext, vmad(k, track, pos), e.y) * e.w;
    rays[0] += ((last[0] + amptau) * e.z) * C.ui_weight;
    last[0] = amptau;
    track += e.x;
  }
  if (C.counts[1] + C.counts[2] == 0) return cvr_expf(-rays[0]);
  rays[2] = rays[0]; rays[1] = rays[0];
  last[2] = last[0]; last[1] = last[0];
  {
    f3 vk[3];
#pragma unroll
    for (int j = 0; j < 3; j++) vk[j] = cone_axis(C.axes + 3 * j, k, u, v);
    for (int i = 0; i < C.counts[1]; i++, s++) {
      const float4 e = sec[s];
#pragma unroll
      for (int j = 0; j < 3; j++) {
        const float amptau = gge(Q, ext, vmad(vk[j], track, pos), e.y) * e.w;
        rays[j] += ((last[j] + amptau) * e.z) * C.ui_weight;
        last[j] = amptau;
      }
      track += e.x;
    }
  }
  if (C.counts[2] == 0)
    return ((cvr_expf(-rays[0]) + cvr_expf(-rays[1])) + cvr_expf(-rays[2])) / 3.0f;
  // transform 3 to 7 (:127-139)
  rays[6] = rays[5] = rays[2];
  rays[4] = rays[3] = rays[1];
  const float avg = ((rays[2] + rays[1]) + rays[0]) / 3.0f;
  rays[2] = rays[1] = rays[0];
  rays[0] = avg;
  last[6] = last[5] = last[2];
  last[4] = last[3] = last[1];
  const float avgt = ((last[2] + last[1]) + last[0]) / 3.0f;
  last[2] = last[1] = last[0];
  last[0] = avgt;
  f3 vk[7];
#pragma unroll
  for (int j = 0; j < 7; j++) vk[j] = cone_axis(C.axes + 3 * (3 + j), k, u, v);
  for (int i = 0; i < C.counts[2]; i++, s++) {
    const float4 e = sec[s];
#pragma unroll
    for (int j = 0; j < 7; j++) {
      const float amptau = gge(Q, ext, vmad(vk[j], track, pos), e.y) * e.w;
      rays[j] += ((last[j] + amptau) * e.z) * C.ui_weight;
      last[j] = amptau;
    }
    track += e.x;
  }
  float side = cvr_expf(-rays[1]);
#pragma unroll
  for (int j = 2; j < 7; j++) side = side + cvr_expf(-rays[j]);
  return (cvr_expf(-rays[0]) + side * C.ray7w) / (1.0f + C.ray7w * 6.0f);
}

// ---------------------------------------------------------------------------
// The march
// ---------------------------------------------------------------------------

// One wave = one 8x8 tile (XCD b%8 takes a contiguous band of tiles).
__global__ void __launch_bounds__(64)
dos_tile_kernel(DosArgs Q, const uint4* __restrict__ cells, const uint2* __restrict__ grad,
                const float4* __restrict__ tf_g, const uint16_t* __restrict__ ext,
                float4* __restrict__ out, uint32_t* __restrict__ samples,
                unsigned long long* __restrict__ tile_samples) {
  extern __shared__ float4 tfp[];
  load_tf_lds(tfp, tf_g, Q.a.tf_n);
  const Rc1passArgs& A = Q.a;
  const int b = blockIdx.x, nt = A.ntiles;
  const int t = (nt & 7) == 0 ? (b & 7) * (nt >> 3) + (b >> 3) : b;
  const int lane = threadIdx.x;
  int px, py;
  long long oidx;
  tile_pixel(A, t, lane & 7, lane >> 3, px, py, oidx);
  const bool inside = px < A.W && py < A.H;
  float4 dst = make_float4(0.f, 0.f, 0.f, 0.f);
  uint32_t cnt = 0;
  Ray r;
  if (inside && ray_setup(A, px, py, r)) {
    const f3 eye{A.eye[0], A.eye[1], A.eye[2]};
    const f3 hg{A.half_grid[0], A.half_grid[1], A.half_grid[2]};
    const f3 light{A.light[0], A.light[1], A.light[2]};
    const f3 v_right = normalize3(cross3(r.cam, f3{0.0f, 1.0f, 0.0f}));
    const f3 v_up = normalize3(cross3(f3{-r.cam.x, -r.cam.y, -r.cam.z}, v_right));
    const float step = A.step, D = r.D, fn = (float)A.tf_n;
    const float inv_k = 1.0f / (Q.ka + Q.kd);
    float s = 0.0f;
    while (s < D) {
      const float h = fminf(step, D - s);
      const float tt = fmaf(h, 0.5f, s);
      const SamplePos sp = sample_pos(fmaf(r.dt.x, tt, r.o.x), fmaf(r.dt.y, tt, r.o.y),
                                      fmaf(r.dt.z, tt, r.o.z), A);
      float4 sc = classify(tfp, fn, trilerp_cell(cells[sp.idx], sp.ax, sp.ay, sp.az));
      cnt++;
      if (sc.w > 0.0f) {
        const f3 tx = vmad(r.dir, tt, r.tpos);        // tx_pos, box at [0, G]
        const f3 wp{tx.x - hg.x, tx.y - hg.y, tx.z - hg.z};
        float iocc = 0.0f, isdw = 0.0f;
        if (Q.apply_occlusion) {
          const f3 k = normalize3(f3{eye.x - wp.x, eye.y - wp.y, eye.z - wp.z});
          iocc = cone_trace(Q, Q.occ, ext, tx, k, v_up, v_right);
        }
        if (Q.apply_shadow) {
          f3 k, u, v;
          bool lit = true;
          const f3 lf{Q.lfwd[0], Q.lfwd[1], Q.lfwd[2]};
          if (Q.shadow_type == 2) {
            k = lf;
            v = f3{Q.lup[0], Q.lup[1], Q.lup[2]};
            u = f3{Q.lright[0], Q.lright[1], Q.lright[2]};
          } else {
            k = normalize3(f3{light.x - wp.x, light.y - wp.y, light.z - wp.z});
            u = normalize3(cross3(k, f3{Q.lright[0], Q.lright[1], Q.lright[2]}));
            v = normalize3(cross3(k, u));
            if (Q.shadow_type == 1 && dot3(k, lf) < Q.spot_cos) lit = false;
          }
          // Cone1RayShadow(pos, k, v, u) is called as (pos, k, u, v): swapped (:559-561)
          isdw = lit ? cone_trace(Q, Q.sdw, ext, tx, k, v, u) : 0.0f;
        }
        if (Q.phong) {
          Texel txl;
          txl.ix = sp.ix; txl.iy = sp.iy; txl.iz = sp.iz;
          txl.ax = sp.ax; txl.ay = sp.ay; txl.az = sp.az;
          const f3 g = sample_gradient(grad, A.N, txl);
          if (g.x != 0.0f || g.y != 0.0f || g.z != 0.0f) {
            const f3 n = normalize3(g);
            const f3 L = normalize3(f3{light.x - wp.x, light.y - wp.y, light.z - wp.z});
            const f3 Ve = normalize3(f3{eye.x - wp.x, eye.y - wp.y, eye.z - wp.z});
            const f3 Hv = normalize3(f3{Ve.x + L.x, Ve.y + L.y, Ve.z + L.z});
            const float dd = fmaxf(0.0f, dot3(n, L));
            const float ds = fmaxf(0.0f, dot3(Hv, n));
            const float diff = inv_k * (iocc * Q.ka + (isdw * Q.kd) * dd);
            const float spec = (isdw * Q.ks) * cvr_powf(ds, A.shininess);
            sc.x = fmaf(A.ispec[0], spec, sc.x * diff);
            sc.y = fmaf(A.ispec[1], spec, sc.y * diff);
            sc.z = fmaf(A.ispec[2], spec, sc.z * diff);
          }
        } else {
          sc.x = inv_k * ((sc.x * iocc) * Q.ka + (sc.x * isdw) * Q.kd);
          sc.y = inv_k * ((sc.y * iocc) * Q.ka + (sc.y * isdw) * Q.kd);
          sc.z = inv_k * ((sc.z * iocc) * Q.ka + (sc.z * isdw) * Q.kd);
        }
        const float a = 1.0f - cvr_expf(-(sc.w * h));
        const float om = 1.0f - dst.w;
        dst.x = fmaf(om, sc.x * a, dst.x);
        dst.y = fmaf(om, sc.y * a, dst.y);
        dst.z = fmaf(om, sc.z * a, dst.z);
        dst.w = fmaf(om, a, dst.w);
        if (dst.w > 0.99f) break;
      }
      s = s + h;
    }
  }
  if (inside || A.packed) {
    out[oidx] = dst;
    if (samples) samples[oidx] = cnt;
  }
  if (tile_samples) {
    const unsigned long long v = wave_sum(cnt);
    if (lane == 0) tile_samples[t] = v;
  }
}

hipError_t launch_dos(const Ctx& c, const DosArgs& q, float4* out, uint32_t* samples,
                      unsigned long long* tile_samples, hipStream_t s) {
  if (q.a.ntiles <= 0) return hipSuccess;
  if (q.a.tf_n > kMaxTfLds) return hipErrorInvalidValue;
  const size_t lds = (size_t)(q.a.tf_n + 2) * sizeof(float4);
  const uint4* cells = (const uint4*)c.d_cells + c.cells.linear_origin;
  hipLaunchKernelGGL(dos_tile_kernel, dim3(q.a.ntiles), dim3(64), lds, s, q, cells,
                     (const uint2*)c.d_grad, (const float4*)c.d_tf, (const uint16_t*)c.d_ext, out,
                     samples, tile_samples);
  return hipGetLastError();
}

}  // namespace cvr
