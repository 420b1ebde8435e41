// fi_pixelate.hip -- flyimg's face-blur pixelation (FaceDetectProcessor.php:58-74):
//   mogrify -gravity NorthWest -region WxH+X+Y -scale 10% -scale 1000% <out>
// per face box, on the 8-bit output image.  IM 6.9 mogrify's -region crops
// the box (clipped to the image), runs the two -scale operators on the crop
// and composites the result back at (X, Y) (an opaque source replaces the
// destination, clipped to the canvas).  -scale is ScaleImage (resize.c): per
// output sample a list of (source index, weight) contributions along each
// axis -- rows accumulated first, into the column value the x pass then
// weighs -- with one ClampToQuantum per pass (host lists: fi_plan.cpp
// im_scale_rows / im_scale_cols, the same additions in the same order as
// the oracle's literal loops, so the result is bit-exact vs or_im_scale_q16).
//
// Two launches per box, boxes in order (each face is its own mogrify run, so
// overlapping boxes see the earlier ones' pixels):
//   k_pix_down  crop -> 10% : Q16 of the 8-bit crop (x 257) -> Q16 scratch
//   k_pix_up    10% -> 1000%: Q16 scratch -> ScaleQuantumToChar -> the image
// Both are latency-bound and tiny next to the resample (a face box is a few
// hundred KB); one thread per output pixel (all channels).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "fi_internal.h"

namespace fi {

namespace {
__device__ __forceinline__ uint16_t pix_clamp_q16(double v) {  // ClampToQuantum (Q16)
  if (v <= 0.0) return 0;
  if (v >= 65535.0) return 65535;
  return (uint16_t)(v + 0.5);
}
}  // namespace

// MODE 0: src = 8-bit crop (value x 257), dst = Q16 (dst16, pitch ow * C).
// MODE 1: src = Q16 (src16), dst = 8-bit image rows (dst8, dstride) with the
//         output clipped to clip_w x clip_h (the canvas beyond (X, Y)).
template <int MODE>
__global__ __launch_bounds__(256) void k_pix(const PixPass P, const int32_t *__restrict__ ai,
                                             const double *__restrict__ ad) {
  const int o = blockIdx.x * 256 + threadIdx.x;
  if (o >= P.ow * P.oh) return;
  const int oy = o / P.ow, ox = o - oy * P.ow;
  if (MODE == 1 && (ox >= P.clip_w || oy >= P.clip_h)) return;
  const int C = P.C;
  const int32_t *yoff = ai + P.yoff, *yidx = ai + P.yidx, *xoff = ai + P.xoff, *xidx = ai + P.xidx;
  const double *yw = ad + P.yw, *xw = ad + P.xw;
  double acc[4] = {0.0, 0.0, 0.0, 0.0};
  for (int kx = xoff[ox]; kx < xoff[ox + 1]; kx++) {
    const int sx = xidx[kx];
    double col[4] = {0.0, 0.0, 0.0, 0.0};  // ScaleImage's scanline[sx]: the rows' sum
    for (int ky = yoff[oy]; ky < yoff[oy + 1]; ky++) {
      const int sy = yidx[ky];
      const double w = yw[ky];
      for (int c = 0; c < C; c++) {
        const double v = MODE == 0 ? (double)(257u * P.src8[(int64_t)sy * P.sstride + (int64_t)sx * C + c])
                                   : (double)P.src16[((int64_t)sy * P.iw + sx) * C + c];
        col[c] = col[c] + w * v;
      }
    }
    const double w = xw[kx];
    for (int c = 0; c < C; c++) acc[c] = acc[c] + w * col[c];
  }
  for (int c = 0; c < C; c++) {
    const uint32_t q = pix_clamp_q16(acc[c]);
    if (MODE == 0)
      P.dst16[((int64_t)oy * P.ow + ox) * C + c] = (uint16_t)q;
    else
      P.dst8[(int64_t)oy * P.dstride + (int64_t)ox * C + c] = (uint8_t)(((q + 128u) - ((q + 128u) >> 8)) >> 8);
  }
}

int launch_pix(hipStream_t s, int mode, const PixPass &P, const int32_t *ai, const double *ad) {
  const int n = P.ow * P.oh;
  if (n <= 0) return 0;
  if (mode == 0)
    hipLaunchKernelGGL(k_pix<0>, dim3((n + 255) / 256), dim3(256), 0, s, P, ai, ad);
  else
    hipLaunchKernelGGL(k_pix<1>, dim3((n + 255) / 256), dim3(256), 0, s, P, ai, ad);
  return 0;
}

}  // namespace fi
