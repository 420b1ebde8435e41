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
// (:16-27, :234-248) of one pixel, f64 as numpy; packed skin | sat << 16.
__device__ __forceinline__ uint32_t sc_skin_sat(uint32_t r, uint32_t g, uint32_t b, uint32_t L,
                                                const ScParamsDev &P) {
  const double rd_ = (double)r, gd_ = (double)g, bd_ = (double)b;
  uint32_t S = 0;
  {
    double rd = -P.skin_color[0], gd = -P.skin_color[1], bd = -P.skin_color[2];
    const double mag = sqrt(rd_ * rd_ + gd_ * gd_ + bd_ * bd_);
    if (!(fabs(mag) < 1e-6)) {
      rd = rd_ / mag - P.skin_color[0];
      gd = gd_ / mag - P.skin_color[1];
      bd = bd_ / mag - P.skin_color[2];
    }
    const double skin = 1 - sqrt(rd * rd + gd * gd + bd * bd);
    if ((skin > P.skin_threshold) && ((double)L >= P.skin_brightness_min * 255) &&
        ((double)L <= P.skin_brightness_max * 255))
      S = (uint32_t)(uint8_t)(int)((skin - P.skin_threshold) * (255 / (1 - P.skin_threshold)));
  }
  uint32_t T = 0;
  {
    const double mx = fmax(fmax(rd_, gd_), bd_), mn = fmin(fmin(rd_, gd_), bd_);
    double s = (mx + mn) / 255, d = (mx - mn) / 255;
    if (mx == mn) {
      d = 0;
      s = 1;
    }
    if (s > 1) s = 2 - d;
    const double sat = d / s;
    const double thr = P.saturation_threshold;
    if ((sat > thr) && ((double)L >= P.saturation_brightness_min * 255) &&
        ((double)L <= P.saturation_brightness_max * 255))
      T = (uint32_t)(uint8_t)(int)((sat - thr) * (255 / (1 - thr)));
  }
  return S | (T << 16);
}

}  // namespace fi
