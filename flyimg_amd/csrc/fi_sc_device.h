// fi_sc_device.h -- smartcrop per-pixel device functions shared by the
// generic (fi_kernels.hip) and fused (fi_smartcrop.hip) kernels, so both
// paths compute the same bits.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "fi_internal.h"

namespace fi {

// Pillow ImagingConvertMatrix L = R*0.2126 + G*0.7152 + B*0.0722 (smartcrop.py:94):
// float sum in order (no FMA: -ffp-contract=off), +0.5 in double, CLIPF.
__device__ __forceinline__ uint32_t sc_luma(uint32_t r, uint32_t g, uint32_t b) {
  float v = 0.2126f * (float)r + 0.7152f * (float)g;
  v = v + 0.0722f * (float)b;
  v = v + 0.0f;
  v = (float)((double)v + 0.5);
  return v <= 0.0f ? 0u : v >= 255.0f ? 255u : (uint32_t)v;
}

// Pillow Resample.c clip8 of a 22-bit fixed-point accumulator
__device__ __forceinline__ uint8_t pil_clip8(int32_t v) {
  v >>= 22;
  return (uint8_t)(v < 0 ? 0 : v > 255 ? 255 : v);
}

__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// detect_skin (smartcrop.py:250-274) and saturation()/detect_saturation
// (:16-27, :234-248) of one pixel, f64 as numpy: the skin and the saturation
// byte (0 when below the threshold or outside the brightness range)
__device__ __forceinline__ uint32_t sc_skin_f64(double rd_, double gd_, double bd_, const ScParamsDev &P) {
  double rd = -P.skin_color[0], gd = -P.skin_color[1], bd = -P.skin_color[2];
  const double mag = sqrt(rd_ * rd_ + gd_ * gd_ + bd_ * bd_);
  if (!(fabs(mag) < 1e-6)) {
    rd = rd_ / mag - P.skin_color[0];
    gd = gd_ / mag - P.skin_color[1];
    bd = bd_ / mag - P.skin_color[2];
  }
  const double skin = 1 - sqrt(rd * rd + gd * gd + bd * bd);
  return skin > P.skin_threshold ? (uint32_t)(uint8_t)(int)((skin - P.skin_threshold) * (255 / (1 - P.skin_threshold)))
                                 : 0u;
}
__device__ __forceinline__ uint32_t sc_sat_f64(double rd_, double gd_, double bd_, const ScParamsDev &P) {
  const double mx = fmax(fmax(rd_, gd_), bd_), mn = fmin(fmin(rd_, gd_), bd_);
  double s = (mx + mn) / 255, d = (mx - mn) / 255;
  if (mx == mn) {
    d = 0;
    s = 1;
  }
  if (s > 1) s = 2 - d;
  const double sat = d / s;
  const double thr = P.saturation_threshold;
  return sat > thr ? (uint32_t)(uint8_t)(int)((sat - thr) * (255 / (1 - thr))) : 0u;
}
// packed skin | sat << 16
__device__ __forceinline__ uint32_t sc_skin_sat(uint32_t r, uint32_t g, uint32_t b, uint32_t L,
                                                const ScParamsDev &P) {
  const double Ld = (double)L;
  uint32_t S = 0, T = 0;
  if (Ld >= P.skin_brightness_min * 255 && Ld <= P.skin_brightness_max * 255) S = sc_skin_f64(r, g, b, P);
  if (Ld >= P.saturation_brightness_min * 255 && Ld <= P.saturation_brightness_max * 255) T = sc_sat_f64(r, g, b, P);
  return S | (T << 16);
}
// Cheap exact skin / saturation for most pixels (k_sc_fd's maps pass):
// sc_skin_sat_est returns true with the packed bytes when f32 arithmetic with
// an error margin decides them, false when the caller must take the exact
// value (k_sc_skinsat's table, or sc_skin_sat):
//  * brightness: L >= min * 255 <=> L >= ceil(min * 255) for an integer L, so
//    the reference's f64 compares become integer compares;
//  * skin: q = sum (rgb / |rgb| - c)^2 = 1 + |c|^2 - 2 c.rgb / |rgb|; skin =
//    1 - sqrt(q) > thr needs q < (1 - thr)^2.  The f32 q is within ~1e-6 of the
//    exact one (|c| <= 4), far inside the margin q > (1 - thr)^2 + 1e-4 that
//    rejects (skin byte 0); every other pixel in range is a candidate;
//  * saturation: sat = (mx - mn) / (mx + mn), or (mx - mn) / (510 - mx + mn)
//    when mx + mn > 255 (the reference's (mx + mn) / 255 > 1, exact on
//    integers); v = (sat - thr) * K with K = fl(255 / (1 - thr)) is within
//    E = 1e-6 K + 1e-4 of the f64 chain (each f32 step adds a few 2^-24
//    relative; sat <= 1, 0 <= thr <= 0.99), so v + E < 0 gives byte 0, and an interval
//    [v - E, v + E] above 0 with no integer in it gives (int) v.
// k_sc_skinsat builds its table through this function (f64 where it returns
// false), and the all-colours test compares that table with the oracle.
struct ScFast {
  float c0, c1, c2, cc, Q, thr, K, E;
  int32_t slo, shi, tlo, thi;  // brightness bounds (inclusive) on the integer luma
  int32_t skin_est, sat_est;   // the estimates apply to these parameters
};
__host__ __device__ __forceinline__ int32_t sc_lbound(double a) {  // L >= a <=> L >= ceil(a)
  return a <= 0 ? 0 : a > 256 ? 256 : (int32_t)ceil(a);
}
__host__ __device__ __forceinline__ int32_t sc_ubound(double b) {  // L <= b <=> L <= floor(b)
  return b < 0 ? -1 : b >= 255 ? 255 : (int32_t)floor(b);
}
__host__ __device__ __forceinline__ ScFast sc_fast_params(const ScParamsDev &P) {
  ScFast F;
  F.c0 = (float)P.skin_color[0];
  F.c1 = (float)P.skin_color[1];
  F.c2 = (float)P.skin_color[2];
  F.cc = F.c0 * F.c0 + F.c1 * F.c1 + F.c2 * F.c2;
  const double st = P.skin_threshold;
  F.skin_est = fabs(P.skin_color[0]) + fabs(P.skin_color[1]) + fabs(P.skin_color[2]) <= 4.0 && st < 0.9999;
  F.Q = (float)((1.0 - st) * (1.0 - st) + 1e-4);  // q > (1 - thr)^2 + 1e-4: skin < thr certainly
  const double tt = P.saturation_threshold;
  F.thr = (float)tt;
  F.K = (float)(255 / (1 - tt));
  F.E = 1e-6f * F.K + 1e-4f;
  F.sat_est = tt >= 0.0 && tt <= 0.99;
  F.slo = sc_lbound(P.skin_brightness_min * 255);
  F.shi = sc_ubound(P.skin_brightness_max * 255);
  F.tlo = sc_lbound(P.saturation_brightness_min * 255);
  F.thi = sc_ubound(P.saturation_brightness_max * 255);
  return F;
}
__device__ __forceinline__ bool sc_skin_sat_est(const ScFast &F, uint32_t r, uint32_t g, uint32_t b, uint32_t L,
                                                uint32_t &st) {
  const int32_t Li = (int32_t)L;
  uint32_t T = 0;
  if (Li >= F.slo && Li <= F.shi) {
    const uint32_t m2 = r * r + g * g + b * b;
    if (!F.skin_est || m2 == 0) return false;
    const float q = 1.0f + F.cc -
                    2.0f * (F.c0 * (float)r + F.c1 * (float)g + F.c2 * (float)b) * __builtin_amdgcn_rsqf((float)m2);
    if (!(q > F.Q)) return false;  // a skin candidate
  }
  if (Li >= F.tlo && Li <= F.thi) {
    const uint32_t mx = max(max(r, g), b), mn = min(min(r, g), b);
    if (!F.sat_est) return false;
    const uint32_t den = mx + mn > 255 ? 510 - (mx - mn) : mx + mn;
    const float sat = mx == mn ? 0.0f : (float)(mx - mn) * __builtin_amdgcn_rcpf((float)den);
    const float v = (sat - F.thr) * F.K;
    if (!(v + F.E < 0.0f)) {
      if (!(v - F.E > 0.0f) || floorf(v - F.E) != floorf(v + F.E)) return false;
      T = (uint32_t)(uint8_t)(int)v;
    }
  }
  st = T << 16;
  return true;
}

}  // namespace fi
