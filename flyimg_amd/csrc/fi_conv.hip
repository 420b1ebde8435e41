// fi_conv.hip -- the forwarded convolution operators of ImageProcessor
// (-unsharp, -sharpen, -blur; src/Core/Processor/ImageProcessor.php:303-315,
// applied after -rotate in that order) on the rotated Q16 image the resample
// epilogue leaves in the workspace (ResizeDesc::q16out).
//
// IM 6.9 semantics, restated in oracle/fi_oracle.c (or_im_convolve_ops):
//   -blur      MorphologyApply(Convolve, "blur:RxS;blur:RxS+90"): a horizontal
//              then a vertical 1-D pass with the KernelRank-3 Gaussian,
//              ClampToQuantum between them;
//   -sharpen   one 2-D convolution (negated Gaussian, centre -2 * sum, normalised);
//   -unsharp   blur, then d = p - b: |2 d| < QuantumRange * threshold ? p : p + gain * d.
// Edge virtual pixels (clamped coordinates); f64 sums from bias 0 over the
// kernel in IM's order (kernel walked backwards, pixels forwards), so the
// results are bit-identical to the oracle on identical Q16 input.
//
// One workgroup per (image, output row), threads over the row's W * C values
// (the kernel values come from the f64 table heap, L1/L2 resident).  These
// are latency-bound helpers off the BASELINE configurations' path.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "fi_internal.h"

namespace fi {

__device__ __forceinline__ uint32_t cv_clamp_q16(double v) {  // ClampToQuantum
  if (!(v > 0.0)) return 0u;
  if (v >= 65535.0) return 65535u;
  return (uint32_t)(v + 0.5);
}
__device__ __forceinline__ int cv_find(const int32_t *prefix, int n, int t) {
  int lo = 0, hi = n;
  while (hi - lo > 1) {
    const int mid = (lo + hi) >> 1;
    if (prefix[mid] <= t)
      lo = mid;
    else
      hi = mid;
  }
  return lo;
}

template <int MODE>
__global__ __launch_bounds__(256) void k_conv(const ConvStep *__restrict__ steps, const int32_t *__restrict__ prefix,
                                              int n, const double *__restrict__ ad) {
  const int t = blockIdx.x;
  const int i = cv_find(prefix, n, t);
  const ConvStep &S = steps[i];
  const int y = t - prefix[i];
  const int W = S.W, H = S.H, C = S.C;
  const int64_t rs = (int64_t)W * C;  // row stride (elements)
  const double *k = ad + S.k;
  for (int e = threadIdx.x; e < W * C; e += 256) {
    const int x = e / C, c = e - x * C;
    if (MODE == 4) {
      const uint32_t q = S.in[(int64_t)y * rs + e];
      S.dst8[(int64_t)y * S.dst_stride + e] = (uint8_t)(((q + 128u) - ((q + 128u) >> 8)) >> 8);
      continue;
    }
    double r = 0.0;  // bias
    if (MODE == 0) {
      const int ox = (S.kw - 1) / 2;
      const uint16_t *row = S.in + (int64_t)y * rs;
      for (int u = 0; u < S.kw; u++) {
        const int sx = min(max(x + u - ox, 0), W - 1);
        r += k[S.kw - 1 - u] * (double)row[(int64_t)sx * C + c];
      }
    } else if (MODE == 1 || MODE == 2) {
      const int oy = (S.kh - 1) / 2;
      for (int v = 0; v < S.kh; v++) {
        const int sy = min(max(y + v - oy, 0), H - 1);
        r += k[S.kh - 1 - v] * (double)S.in[(int64_t)sy * rs + e];
      }
    } else {  // 2-D
      const int ox = (S.kw - 1) / 2, oy = (S.kh - 1) / 2;
      const double *kk = k + S.kw * S.kh - 1;
      for (int v = 0; v < S.kh; v++) {
        const uint16_t *row = S.in + (int64_t)min(max(y + v - oy, 0), H - 1) * rs;
        for (int u = 0; u < S.kw; u++, kk--) r += (*kk) * (double)row[(int64_t)min(max(x + u - ox, 0), W - 1) * C + c];
      }
    }
    uint32_t q = cv_clamp_q16(r);
    if (MODE == 2) {  // UnsharpMaskImage: p - blur, thresholded gain
      const double p = (double)S.orig[(int64_t)y * rs + e];
      double d = p - (double)q;
      if (fabs(2.0 * d) < S.thr)
        d = p;
      else
        d = p + (d * S.gain);
      q = cv_clamp_q16(d);
    }
    S.out[(int64_t)y * rs + e] = (uint16_t)q;
  }
}

int launch_conv(hipStream_t s, int mode, const ConvStep *steps, const int32_t *prefix, int n, int tiles,
                const double *ad) {
  if (n <= 0 || tiles <= 0) return 0;
  switch (mode) {
    case 0: hipLaunchKernelGGL(k_conv<0>, dim3(tiles), dim3(256), 0, s, steps, prefix, n, ad); break;
    case 1: hipLaunchKernelGGL(k_conv<1>, dim3(tiles), dim3(256), 0, s, steps, prefix, n, ad); break;
    case 2: hipLaunchKernelGGL(k_conv<2>, dim3(tiles), dim3(256), 0, s, steps, prefix, n, ad); break;
    case 3: hipLaunchKernelGGL(k_conv<3>, dim3(tiles), dim3(256), 0, s, steps, prefix, n, ad); break;
    default: hipLaunchKernelGGL(k_conv<4>, dim3(tiles), dim3(256), 0, s, steps, prefix, n, ad); break;
  }
  return 0;
}

}  // namespace fi
