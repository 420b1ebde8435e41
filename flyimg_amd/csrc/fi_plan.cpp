// fi_plan.cpp -- host planner.  Every floating-point expression mirrors the
// reference's evaluation order (built with -ffp-contract=off):
//   * ImageMagick 6.9 geometry.c ParseMetaGeometry / GravityAdjustGeometry,
//     resize.c ThumbnailImage / SampleImage / ResizeImage contribution lists
//     (flyimg emits them from ImageProcessor.php:66-110);
//   * Pillow 12.2 Image.thumbnail/resize/reduce (PIL/Image.py:2831-2915,
//     :2328-2470) and Resample.c precompute_coeffs, used by
//     python/smartcrop.py:157-172;
//   * smartcrop.py crop() geometry (:137-191), crops() (:193-229) and
//     importance()/thirds() (:276-298, :30-34).
#include "fi_plan.h"

#include <math.h>

#include <cmath>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <map>

namespace fi {

static constexpr double kImEpsilon = 1.0e-12;  // MagickEpsilon

// ---------------------------------------------------------------------------
// ImageMagick geometry
// ---------------------------------------------------------------------------
static void meta_geometry(int W, int H, int tw, int th, bool fill, bool shrink, int *ow, int *oh) {
  double scale;
  const bool has_w = tw > 0, has_h = th > 0;
  if (has_w && has_h) {
    scale = (double)tw / (double)W;
    if (!fill) {
      if (scale > ((double)th / (double)H)) scale = (double)th / (double)H;
    } else if (scale < ((double)th / (double)H)) {
      scale = (double)th / (double)H;
    }
  } else if (has_w) {
    scale = (double)tw / (double)W;
    if (fill && scale < ((double)tw / (double)H)) scale = (double)tw / (double)H;
  } else {
    scale = (double)th / (double)H;
    if (fill && scale < ((double)th / (double)W)) scale = (double)th / (double)W;
  }
  long w = (long)floor(scale * W + 0.5), h = (long)floor(scale * H + 0.5);
  if (w < 1) w = 1;
  if (h < 1) h = 1;
  if (shrink) {
    if (W < w) w = W;
    if (H < h) h = H;
  }
  *ow = (int)w;
  *oh = (int)h;
}

static void gravity_offset(int W, int H, int ew, int eh, int gravity, int *x, int *y) {
  long ox = 0, oy = 0;
  switch (gravity) {
    case FI_GRAVITY_NORTHEAST: case FI_GRAVITY_EAST: case FI_GRAVITY_SOUTHEAST:
      ox = (long)((unsigned long)W - (unsigned long)ew);
      break;
    case FI_GRAVITY_NORTH: case FI_GRAVITY_SOUTH: case FI_GRAVITY_CENTER:
      ox = (long)((unsigned long)W / 2 - (unsigned long)ew / 2);
      break;
    default: break;
  }
  switch (gravity) {
    case FI_GRAVITY_SOUTHWEST: case FI_GRAVITY_SOUTH: case FI_GRAVITY_SOUTHEAST:
      oy = (long)((unsigned long)H - (unsigned long)eh);
      break;
    case FI_GRAVITY_EAST: case FI_GRAVITY_WEST: case FI_GRAVITY_CENTER:
      oy = (long)((unsigned long)H / 2 - (unsigned long)eh / 2);
      break;
    default: break;
  }
  *x = (int)ox;
  *y = (int)oy;
}

int plan_im(const fi_image &img, ImPlan *p) {
  *p = ImPlan();
  p->W = img.src_w;
  p->H = img.src_h;
  p->C = img.src_channels;
  auto fail = [&](int code, const char *m) {
    p->status = code;
    p->err = m;
    return code;
  };
  if (img.src_w <= 0 || img.src_h <= 0) return fail(FI_EINVAL, "source dimensions must be positive");
  // RGB8, or RGBA8 (straight alpha, a PNG with an alpha channel: IM's matte
  // image -- Mitchell filter, alpha-weighted resample)
  if (img.src_channels != 3 && img.src_channels != 4)
    return fail(FI_EUNSUPPORTED, "only RGB8 / RGBA8 sources (src_channels 3 or 4) are supported");
  if ((int64_t)img.src_stride < (int64_t)img.src_w * img.src_channels) return fail(FI_EINVAL, "src_stride < C*src_w");
  const bool matte = img.src_channels == 4;
  const uint32_t f = img.flags;
  if ((f & FI_OP_THUMBNAIL) && (f & FI_OP_RESIZE)) return fail(FI_EINVAL, "both -thumbnail and -resize");
  const bool has_geom = img.target_w > 0 || img.target_h > 0;
  p->tw = p->W;
  p->th = p->H;
  if (has_geom) {
    if (!(f & (FI_OP_THUMBNAIL | FI_OP_RESIZE))) return fail(FI_EINVAL, "geometry without a resize operator");
    meta_geometry(p->W, p->H, img.target_w, img.target_h, f & FI_GEOM_FILL, f & FI_GEOM_SHRINK_ONLY, &p->tw,
                  &p->th);
  }
  p->resize = (p->tw != p->W || p->th != p->H);
  p->sw = p->W;
  p->sh = p->H;
  if (p->resize && (f & FI_OP_THUMBNAIL)) {
    // ThumbnailImage: area factor <= 0.1 and 5*w, 5*h >= 128 -> SampleImage
    const double xf = (double)p->tw / (double)p->W, yf = (double)p->th / (double)p->H;
    if (!((xf * yf) > 0.1) && !((5 * p->tw) < 128 || (5 * p->th) < 128)) {
      p->sample = true;
      p->sw = 5 * p->tw;
      p->sh = 5 * p->th;
    }
  }
  if (p->resize) {
    p->xf = (double)p->tw / (double)p->sw;
    p->yf = (double)p->th / (double)p->sh;
    // ResizeImage with the default filter (resize.c): Mitchell for PseudoClass
    // (palette / gray) and matte (alpha) sources and for enlargements, Lanczos otherwise
    const bool pseudo = (f & FI_SRC_PSEUDOCLASS) != 0;
    p->filter = (matte || pseudo || (p->xf * p->yf) > 1.0) ? kFilterMitchell : kFilterLanczos;
    p->hfirst = p->xf > p->yf;
  }
  p->ex0 = p->ey0 = 0;
  p->ew = p->tw;
  p->eh = p->th;
  if (f & FI_OP_EXTENT) {
    const int ew = img.target_w > 0 ? img.target_w : p->tw;
    const int eh = img.target_h > 0 ? img.target_h : p->th;
    int gx, gy;
    gravity_offset(p->tw, p->th, ew, eh, img.gravity ? img.gravity : FI_GRAVITY_CENTER, &gx, &gy);
    if (gx < 0 || gy < 0 || gx + ew > p->tw || gy + eh > p->th)
      return fail(FI_EUNSUPPORTED, "-extent larger than the resized image (background fill) is not supported");
    p->ex0 = gx;
    p->ey0 = gy;
    p->ew = ew;
    p->eh = eh;
  }
  // -monochrome (ImageProcessor.php:90-92) converts to GRAY first (SetImageType Bilevel)
  p->mono = (f & FI_OP_MONOCHROME) != 0;
  p->gray = (f & FI_OP_GRAY) != 0 || p->mono;
  p->rot = 0;
  if (f & FI_OP_ROTATE) {
    if (img.rotate % 90) return fail(FI_EUNSUPPORTED, "only -rotate by multiples of 90 (IntegralRotateImage)");
    p->rot = ((img.rotate % 360) + 360) % 360;
  }
  if (matte && p->mono) return fail(FI_EUNSUPPORTED, "-monochrome of an RGBA source is not on the GPU path");
  if (matte && (f & FI_OP_SMARTCROP))
    return fail(FI_EUNSUPPORTED, "smartcrop of an RGBA image: smartcrop.py fails on RGBA (split(), smartcrop.py:17)");
  p->out_c = matte ? (p->gray ? 2 : 4) : (p->gray ? 1 : 3);
  p->conv = ((f & FI_OP_UNSHARP) ? 1u : 0u) | ((f & FI_OP_SHARPEN) ? 2u : 0u) | ((f & FI_OP_BLUR) ? 4u : 0u);
  if (p->conv) {
    if (matte || p->mono)
      return fail(FI_EUNSUPPORTED, "-unsharp/-sharpen/-blur of an RGBA or -monochrome image are not on the GPU path");
    for (int k = 0; k < 4; k++) p->cv[k] = img.unsharp[k];
    p->cv[4] = img.sharpen[0];
    p->cv[5] = img.sharpen[1];
    p->cv[6] = img.blur[0];
    p->cv[7] = img.blur[1];
    for (double v : p->cv)
      if (!std::isfinite(v) || fabs(v) > 1e6) return fail(FI_EINVAL, "convolution parameter out of range");
    std::vector<double> kk;
    if ((p->conv & 1) && im_blur_kernel(p->cv[0], p->cv[1], &kk) < 0)
      return fail(FI_EUNSUPPORTED, "-unsharp kernel wider than the GPU path supports");
    if ((p->conv & 2) && im_sharpen_kernel(p->cv[4], p->cv[5], &kk) < 0)
      return fail(FI_EUNSUPPORTED, "-sharpen kernel wider than the GPU path supports");
    if ((p->conv & 4) && im_blur_kernel(p->cv[6], p->cv[7], &kk) < 0)
      return fail(FI_EUNSUPPORTED, "-blur kernel wider than the GPU path supports");
  }
  const bool swap = p->rot == 90 || p->rot == 270;
  p->out_w = swap ? p->eh : p->ew;
  p->out_h = swap ? p->ew : p->eh;
  return FI_OK;
}

// --- forwarded convolution kernels (IM 6.9 gem.c / morphology.c / effect.c) ----
static double conv_reciprocal(double x) {  // PerceptibleReciprocal
  const double sign = x < 0.0 ? -1.0 : 1.0;
  if ((sign * x) >= kImEpsilon) return 1.0 / x;
  return sign / kImEpsilon;
}
static constexpr double kSq2Pi = 2.50662827463100024161235523934010416269302368164062;  // MagickSQ2PI
static constexpr double k2Pi = 6.283185307179586476925286766559005768394338798750211641949;  // Magick2PI
static int kernel_width_1d(double radius, double sigma) {  // GetOptimalKernelWidth1D
  if (radius > kImEpsilon) return (int)(2.0 * ceil(radius) + 1.0);
  const double gamma = fabs(sigma);
  if (gamma <= kImEpsilon) return 3;
  const double alpha = conv_reciprocal(2.0 * gamma * gamma), beta = conv_reciprocal(kSq2Pi * gamma);
  int width;
  for (width = 5; width < 4 * kConvMaxBlur;) {
    double normalize = 0.0;
    const int j = (width - 1) / 2;
    for (int i = -j; i <= j; i++) normalize += exp(-((double)(i * i)) * alpha) * beta;
    const double value = exp(-((double)(j * j)) * alpha) * beta / normalize;
    if ((value < 1.0 / 65535.0) || (value < kImEpsilon)) break;
    width += 2;
  }
  return width - 2;
}
static int kernel_width_2d(double radius, double sigma) {  // GetOptimalKernelWidth2D
  if (radius > kImEpsilon) return (int)(2.0 * ceil(radius) + 1.0);
  const double gamma = fabs(sigma);
  if (gamma <= kImEpsilon) return 3;
  const double alpha = conv_reciprocal(2.0 * gamma * gamma), beta = conv_reciprocal(k2Pi * gamma * gamma);
  int width;
  for (width = 5; width < 4 * kConvMaxSharpen;) {
    double normalize = 0.0;
    const int j = (width - 1) / 2;
    for (int v = -j; v <= j; v++)
      for (int u = -j; u <= j; u++) normalize += exp(-((double)(u * u + v * v)) * alpha) * beta;
    const double value = exp(-((double)(j * j)) * alpha) * beta / normalize;
    if ((value < 1.0 / 65535.0) || (value < kImEpsilon)) break;
    width += 2;
  }
  return width - 2;
}
int im_blur_kernel(double radius, double sigma, std::vector<double> *k) {
  sigma = fabs(sigma);
  const int width = radius >= 1.0 ? (int)radius * 2 + 1 : kernel_width_1d(radius, sigma);
  if (width < 1 || width > kConvMaxBlur) return -1;
  k->assign(width, 0.0);
  const int x = (width - 1) / 2;
  if (sigma > kImEpsilon) {  // KernelRank 3: a Gaussian 3x as wide, binned
    const int v = (width * 3 - 1) / 2;
    const double s3 = sigma * 3.0;
    const double alpha = 1.0 / (2.0 * s3 * s3), beta = 1.0 / (kSq2Pi * s3);
    for (int u = -v; u <= v; u++) (*k)[(u + v) / 3] += exp(-((double)(u * u)) * alpha) * beta;
  } else {
    (*k)[x] = 1.0;
  }
  double pos = 0.0;  // ScaleKernelInfo(1.0, CorrelateNormalizeValue): 1 / positive range
  for (double v : *k)
    if (v > 0.0) pos += v;
  const double scale = 1.0 / (fabs(pos) >= kImEpsilon ? pos : 1.0);
  for (double &v : *k) v *= scale;
  return width;
}
int im_sharpen_kernel(double radius, double sigma, std::vector<double> *k) {
  const int width = kernel_width_2d(radius, sigma);
  if (width < 1 || width > kConvMaxSharpen) return -1;
  k->assign((size_t)width * width, 0.0);
  const double ms = fabs(sigma) < kImEpsilon ? kImEpsilon : sigma;  // MagickSigma
  const int j = (width - 1) / 2;
  double normalize = 0.0;
  int i = 0;
  for (int v = -j; v <= j; v++)
    for (int u = -j; u <= j; u++) {
      (*k)[i] = -exp(-((double)u * u + v * v) / (2.0 * ms * ms)) /
                (2.0 * 3.14159265358979323846264338327950288419716939937510 * ms * ms);
      normalize += (*k)[i];
      i++;
    }
  (*k)[i / 2] = (-2.0) * normalize;
  normalize = 0.0;
  for (double v : *k) normalize += v;
  const double gamma = conv_reciprocal(normalize);
  for (double &v : *k) v *= gamma;
  return width;
}

// --- resize.c filters --------------------------------------------------------
static double sinc(double x) {
  if (x != 0.0) {
    const double alpha = 3.14159265358979323846264338327950288419716939937510 * x;
    return sin(alpha) / alpha;
  }
  return 1.0;
}
static double sincfast(double x) {
  if (x > 4.0) return sinc(x);
  const double xx = x * x;
  const double c0 = 0.173611107357320220183368594093166520811e-2;
  const double c1 = -0.384240921114946632192116762889211361285e-3;
  const double c2 = 0.394201182359318128221229891724947048771e-4;
  const double c3 = -0.250963301609117217660068889165550534856e-5;
  const double c4 = 0.111902032818095784414237782071368805120e-6;
  const double c5 = -0.372895101408779549368465614321137048875e-8;
  const double c6 = 0.957694196677572570319816780188718518330e-10;
  const double c7 = -0.187208577776590710853865174371617338991e-11;
  const double c8 = 0.253524321426864752676094495396308636823e-13;
  const double c9 = -0.177084805010701112639035485248501049364e-15;
  const double p =
      c0 + xx * (c1 + xx * (c2 + xx * (c3 + xx * (c4 + xx * (c5 + xx * (c6 + xx * (c7 + xx * (c8 + xx * c9))))))));
  return (xx - 1.0) * (xx - 4.0) * (xx - 9.0) * (xx - 16.0) * p;
}
static double mitchell(double x) {
  const double B = 1.0 / 3.0, C = 1.0 / 3.0, twoB = B + B;
  const double k0 = 1.0 - (1.0 / 3.0) * B, k1 = -3.0 + twoB + C, k2 = 2.0 - 1.5 * B - C;
  const double k3 = (4.0 / 3.0) * B + 4.0 * C, k4 = -8.0 * C - twoB, k5 = B + 5.0 * C,
               k6 = (-1.0 / 6.0) * B - C;
  if (x < 1.0) return k0 + x * (x * (k1 + x * k2));
  if (x < 2.0) return k3 + x * (k4 + x * (k5 + x * k6));
  return 0.0;
}
static double filter_weight(int filter, double x) {
  const double xb = fabs(x) / 1.0;
  if (filter == kFilterLanczos) {
    const double scale = 1.0 / 3.0;
    const double win = sincfast(xb * scale);
    return win * sincfast(xb);
  }
  return 1.0 * mitchell(xb);
}
static double perceptible_reciprocal(double x) {
  const double sign = x < 0.0 ? -1.0 : 1.0;
  if ((sign * x) >= kImEpsilon) return 1.0 / x;
  return sign / kImEpsilon;
}

void build_axis(int filter, double factor, int in_sampled, int out_size, int o0, int o1, bool sample,
                int in_src, AxisTable *t) {
  (void)out_size;
  *t = AxisTable();
  double scale = fmax(1.0 / factor + kImEpsilon, 1.0);
  double support = scale * (filter == kFilterLanczos ? 3.0 : 2.0);
  if (support < 0.5) {
    support = 0.5;
    scale = 1.0;
  }
  scale = perceptible_reciprocal(scale);
  std::vector<double> w;
  std::vector<double> merged;
  t->src_lo = 1 << 30;
  t->src_hi = 0;
  for (int o = o0; o < o1; o++) {
    const double bisect = (double)(o + 0.5) / factor + kImEpsilon;
    const long s = (long)fmax(bisect - support + 0.5, 0.0);
    const long e = (long)fmin(bisect + support + 0.5, (double)in_sampled);
    const int n = (int)(e - s);
    w.assign(n > 0 ? n : 0, 0.0);
    double density = 0.0;
    for (int i = 0; i < n; i++) {
      w[i] = filter_weight(filter, scale * ((double)(s + i) - bisect + 0.5));
      density += w[i];
    }
    if (density != 0.0 && density != 1.0) {
      density = perceptible_reciprocal(density);
      for (int i = 0; i < n; i++) w[i] *= density;
    }
    // map sampled taps to source indices (SampleImage offsets) and merge
    auto src_of = [&](long j) -> long {
      if (!sample) return j;
      return (long)((((double)j + (0.5 - kImEpsilon)) * in_src) / in_sampled);
    };
    const long m0 = n > 0 ? src_of(s) : 0;
    const long m1 = n > 0 ? src_of(s + n - 1) : -1;
    const int cnt = (int)(m1 - m0 + 1);
    merged.assign(cnt > 0 ? cnt : 0, 0.0);
    for (int i = 0; i < n; i++) merged[src_of(s + i) - m0] += w[i];
    t->start.push_back((int32_t)m0);
    t->count.push_back(cnt);
    t->woff.push_back((int32_t)t->w.size());
    for (int i = 0; i < cnt; i++) {
      t->w.push_back((float)merged[i]);
      t->wd.push_back(merged[i]);
    }
    t->maxtaps = std::max(t->maxtaps, cnt);
    t->src_lo = std::min<int32_t>(t->src_lo, (int32_t)m0);
    t->src_hi = std::max<int32_t>(t->src_hi, (int32_t)(m0 + cnt));
  }
  if (o1 <= o0) t->src_lo = 0;
  // source indices carrying a non-zero weight (SampleImage skips some when it decimates)
  std::vector<uint8_t> used(std::max(t->src_hi - t->src_lo, 0), 0);
  for (size_t o = 0; o < t->start.size(); o++)
    for (int j = 0; j < t->count[o]; j++)
      if (t->w[t->woff[o] + j] != 0.0f) used[t->start[o] + j - t->src_lo] = 1;
  t->touched = 0;
  for (uint8_t u : used) t->touched += u;
}

// ---------------------------------------------------------------------------
// MFMA resample tables
// ---------------------------------------------------------------------------
static void limbs3(int32_t k, int32_t l[3]) {
  l[0] = ((k + 128) & 255) - 128;
  const int32_t k1 = (k - l[0]) / 256;
  l[1] = ((k1 + 128) & 255) - 128;
  l[2] = (k1 - l[1]) / 256;
}
static int32_t quant_w(float w) { return (int32_t)lrint((double)w * (double)(1 << kMfmaWBits)); }
static void limbs2(int32_t k, int32_t l[2]) {
  // W = hi * 256 + lo, both signed bytes
  l[0] = ((k + 128) & 255) - 128;
  l[1] = (k - l[0]) / 256;
}
static void put_frag2(std::vector<int32_t> &frag, size_t base, int lane, int j, const int32_t limb[2]) {
  for (int q = 0; q < 2; q++)
    reinterpret_cast<uint8_t *>(&frag[base + (size_t)q * 256])[lane * 16 + j] = (uint8_t)(int8_t)limb[q];
}
// W = rint(w * 2^shift) per tap, then per output the |d| taps whose rounding
// residual points furthest the needed way move by one so that sum(W) =
// 2^shift: IM's weights are normalised to sum 1, and a
// quantised row that keeps its sum reproduces a flat region exactly (rounding
// each tap alone leaves a bias that repeats on every output at integral
// factors: 98.5 % exact at 1/10 against 99.98 % with the sum kept)
static void quant_axis(const AxisTable &t, int shift, std::vector<int32_t> *wq) {
  wq->assign(t.w.size(), 0);
  const double sc = (double)(1 << shift);
  std::vector<int> ord;
  for (size_t o = 0; o < t.start.size(); o++) {
    const int n = t.count[o], w0 = t.woff[o];
    double sx = 0.0;
    int64_t sq = 0;
    for (int j = 0; j < n; j++) {
      const double x = (double)t.w[w0 + j] * sc;
      sx += x;
      (*wq)[w0 + j] = (int32_t)lrint(x);
      sq += (*wq)[w0 + j];
    }
    // IM normalises every row to sum 1 (resize.c density): the target is 2^shift,
    // not the float-rounded sum of the float weights
    int64_t d = (n > 0 ? ((int64_t)1 << shift) : 0) - sq;
    (void)sx;
    if (d == 0) continue;
    const int dir = d > 0 ? 1 : -1;
    ord.clear();
    for (int j = 0; j < n; j++)
      if (t.w[w0 + j] != 0.0f) ord.push_back(j);
    std::stable_sort(ord.begin(), ord.end(), [&](int a, int b) {
      const double ra = ((double)t.w[w0 + a] * sc - (*wq)[w0 + a]) * dir;
      const double rb = ((double)t.w[w0 + b] * sc - (*wq)[w0 + b]) * dir;
      return ra > rb;
    });
    for (size_t k = 0; d != 0 && !ord.empty(); k = (k + 1) % ord.size(), d -= dir) (*wq)[w0 + ord[k]] += dir;
  }
}
int vr_quant(const AxisTable &t, std::vector<int32_t> *wq) {
  for (int s = kVrMaxShift; s >= kVrMinShift; s--) {
    quant_axis(t, s, wq);
    bool ok = true;
    for (int32_t q : *wq)
      if (q < -32896 || q > 32639) {
        ok = false;
        break;
      }
    if (ok) return s;
  }
  wq->clear();
  return 0;
}

// touched indices (non-zero weight) of an axis, ascending, and their list index
static void touched_list(const AxisTable &t, std::vector<int32_t> *list, std::vector<int32_t> *idx) {
  const int span = std::max(t.src_hi - t.src_lo, 0);
  idx->assign(span, -1);
  for (size_t o = 0; o < t.start.size(); o++)
    for (int j = 0; j < t.count[o]; j++)
      if (t.w[t.woff[o] + j] != 0.0f) (*idx)[t.start[o] + j - t.src_lo] = 1;
  list->clear();
  for (int r = 0; r < span; r++)
    if ((*idx)[r] >= 0) {
      (*idx)[r] = (int32_t)list->size();
      list->push_back(t.src_lo + r);
    }
}
// list-index range [lo, hi] of output o's non-zero taps (lo > hi: none)
static void tap_range(const AxisTable &t, const std::vector<int32_t> &idx, int o, int *lo, int *hi) {
  *lo = 1 << 30;
  *hi = -1;
  for (int j = 0; j < t.count[o]; j++)
    if (t.w[t.woff[o] + j] != 0.0f) {
      const int li = idx[t.start[o] + j - t.src_lo];
      *lo = std::min(*lo, li);
      *hi = std::max(*hi, li);
    }
}
// The 2^22-scaled weights of k_rs_vm (and k_sc-independent: AxisTable::w
// order): k_rs_vr's two-limb weights (vr_quant, shift s) times 2^(22 - s) when
// the axis has them, else rint(w 2^22).  k_rs_vm's float conversions then see
// k_rs_vr's integer sums times a power of two, so the two kernels give the
// same pixels bit for bit and an image's output does not depend on which of
// them its batch ran (the choice is per batch: classes, ring fit).
int axis_q22(const AxisTable &t, std::vector<int32_t> *q) {
  std::vector<int32_t> wq;
  const int s = vr_quant(t, &wq);
  q->resize(t.w.size());
  for (size_t i = 0; i < t.w.size(); i++) (*q)[i] = s > 0 ? wq[i] * (1 << (kMfmaWBits - s)) : quant_w(t.w[i]);
  return s > 0 ? s : kMfmaWBits;
}
// quantized weight of output o at list index li (0 if not a tap)
static int32_t tap_w(const AxisTable &t, const std::vector<int32_t> &q22, const std::vector<int32_t> &list, int o,
                     int li) {
  if (li < 0 || li >= (int)list.size()) return 0;
  const int j = list[li] - t.start[o];
  if (j < 0 || j >= t.count[o]) return 0;
  return q22[t.woff[o] + j];
}
static int32_t tap_wq(const AxisTable &t, const std::vector<int32_t> &wq, const std::vector<int32_t> &list, int o,
                      int li) {
  if (li < 0 || li >= (int)list.size()) return 0;
  const int j = list[li] - t.start[o];
  if (j < 0 || j >= t.count[o]) return 0;
  return wq[t.woff[o] + j];
}
static void put_frag(std::vector<int32_t> &frag, size_t base, int lane, int j, const int32_t limb[3]) {
  for (int q = 0; q < 3; q++)
    reinterpret_cast<uint8_t *>(&frag[base + (size_t)q * 256])[lane * 16 + j] = (uint8_t)(int8_t)limb[q];
}

bool build_mfma_h(const AxisTable &h, MfmaH *m, int max_nx) {
  *m = MfmaH();
  const int nx = (int)h.start.size();
  if (nx == 0) return false;
  std::vector<int32_t> idx;
  touched_list(h, &m->cols, &idx);
  std::vector<int32_t> lo(nx), hi(nx);
  for (int x = 0; x < nx; x++) {
    tap_range(h, idx, x, &lo[x], &hi[x]);
    if (hi[x] < lo[x]) return false;  // an output px without taps
    if (x > 0 && (lo[x] < lo[x - 1] || hi[x] < hi[x - 1])) return false;  // not monotone
  }
  std::vector<int32_t> q22;
  axis_q22(h, &q22);
  m->wsum.assign(nx, 0);
  for (int x = 0; x < nx; x++)
    for (int j = 0; j < h.count[x]; j++) m->wsum[x] += q22[h.woff[x] + j];
  std::vector<int32_t> wq2;
  m->shift2 = vr_quant(h, &wq2);
  m->wsum2.assign(nx, 0);
  if (m->shift2 > 0)
    for (int x = 0; x < nx; x++)
      for (int j = 0; j < h.count[x]; j++) m->wsum2[x] += wq2[h.woff[x] + j];
  auto bytes_of = [&](int x0, int x1, int *b0) {
    *b0 = (3 * m->cols[lo[x0]]) / 16 * 16;
    const int be = (3 * (m->cols[hi[x1 - 1]] + 1) + 15) / 16 * 16;
    return be - *b0;
  };
  for (int x0 = 0; x0 < nx;) {
    int x1 = x0 + 1, b0;
    if (bytes_of(x0, x1, &b0) > kMfmaStripBytes) return false;
    while (x1 < nx && x1 - x0 < max_nx && bytes_of(x0, x1 + 1, &b0) <= kMfmaStripBytes) x1++;
    // strips end on multiples of 4 px (the last one at nx): every strip's output
    // segment then starts 12-byte aligned in its row, so with a dword-aligned
    // destination row the stores are whole dwords / 8-byte units, no byte stores
    if (x1 < nx && (x1 & ~3) > x0) x1 &= ~3;
    MfmaStrip S{};
    S.x0 = x0;
    S.x1 = x1;
    S.nbytes = bytes_of(x0, x1, &S.b0);
    S.c_lo = lo[x0];
    S.ncols = hi[x1 - 1] + 1 - S.c_lo;
    S.nocb = (x1 - x0 + 15) / 16;
    S.ks = 1;
    S.s0 = m->s0.size();
    // per 16-px output block: window start (8-B aligned for the two 8-byte
    // fragment reads) and its own k-steps; s0 holds (w0, ks) pairs
    int pitch = S.ncols;
    for (int ob = 0; ob < S.nocb; ob++) {
      const int xa = x0 + 16 * ob, xb = std::min(x1, xa + 16);
      const int w0 = (lo[xa] - S.c_lo) / 8 * 8;
      const int ks = (hi[xb - 1] - S.c_lo + 1 - w0 + 63) / 64;
      S.ks = std::max(S.ks, ks);
      m->s0.push_back(w0);
      m->s0.push_back(ks);
      pitch = std::max(pitch, w0 + 64 * ks);
    }
    if (S.ks > 2) return false;
    // plane pitch = 8 (mod 32) bytes: the fold's byte writes of rows 4 apart and the
    // fragment reads of rows 1 apart spread over the LDS banks
    S.pitch = pitch + ((8 - pitch % 32) + 32) % 32;
    if (S.pitch > kMfmaMaxPitch) return false;
    S.vpitch = (pitch + 15) / 16 * 16;
    S.lut_px0 = S.b0 / 3;
    S.lut_n = (S.b0 + S.nbytes + 2) / 3 - S.lut_px0;
    S.lut = m->lut.size();
    for (int k = 0; k < S.lut_n; k++) {
      const int px = S.lut_px0 + k;
      int ci = -1;
      if (px >= h.src_lo && px < h.src_hi && idx[px - h.src_lo] >= 0) ci = idx[px - h.src_lo] - S.c_lo;
      m->lut.push_back(ci >= 0 && ci < S.ncols ? ci : -1);
    }
    while (m->lut.size() % 4) m->lut.push_back(-1);  // 16-byte rows: k_rs_vr stages the LUT by LDS-DMA
    S.frag = m->frag.size();
    m->frag.resize(m->frag.size() + (size_t)S.nocb * S.ks * 3 * 256, 0);
    for (int ob = 0; ob < S.nocb; ob++)
      for (int t = 0; t < S.ks; t++)
        for (int l = 0; l < 64; l++)
          for (int j = 0; j < 16; j++) {
            const int x = x0 + 16 * ob + (l & 15);
            const int li = S.c_lo + m->s0[S.s0 + 2 * ob] + 64 * t + mfma_i8_k(l, j);
            int32_t limb[3];
            limbs3(x < x1 ? tap_w(h, q22, m->cols, x, li) : 0, limb);
            put_frag(m->frag, S.frag + (size_t)(ob * S.ks + t) * 3 * 256, l, j, limb);
          }
    S.frag2 = m->frag2.size();
    if (m->shift2 > 0) {
      m->frag2.resize(m->frag2.size() + (size_t)S.nocb * S.ks * 2 * 256, 0);
      for (int ob = 0; ob < S.nocb; ob++)
        for (int t = 0; t < S.ks; t++)
          for (int l = 0; l < 64; l++)
            for (int j = 0; j < 16; j++) {
              const int x = x0 + 16 * ob + (l & 15);
              const int li = S.c_lo + m->s0[S.s0 + 2 * ob] + 64 * t + mfma_i8_k(l, j);
              int32_t limb[2];
              limbs2(x < x1 ? tap_wq(h, wq2, m->cols, x, li) : 0, limb);
              put_frag2(m->frag2, S.frag2 + (size_t)(ob * S.ks + t) * 2 * 256, l, j, limb);
            }
    }
    m->strips.push_back(S);
    x0 = x1;
  }
  return true;
}

bool build_vm_v(const AxisTable &v, VmV *m) {
  *m = VmV();
  const int ny = (int)v.start.size();
  if (ny == 0) return false;
  std::vector<int32_t> q22;
  axis_q22(v, &q22);
  std::vector<int32_t> idx;
  touched_list(v, &m->rows, &idx);
  const int nl = (int)m->rows.size();
  if (nl == 0) return false;
  m->nblk = (ny + 15) / 16;
  std::vector<int> L(m->nblk), R(m->nblk);
  for (int b = 0; b < m->nblk; b++) {
    int lo = 1 << 30, hi = -1;
    for (int y = 16 * b; y < std::min(ny, 16 * b + 16); y++) {
      int a, e;
      tap_range(v, idx, y, &a, &e);
      if (e < a) return false;  // an output row without taps
      lo = std::min(lo, a);
      hi = std::max(hi, e);
    }
    L[b] = lo;
    R[b] = hi + 1;
    if (b > 0 && (L[b] < L[b - 1] || R[b] < R[b - 1])) return false;  // not monotone
  }
  // pieces: block b owns [R(b-1), R(b)), R(-1) = L(0)
  std::vector<int> pstart(m->nblk + 1);  // first piece of block b
  for (int b = 0; b < m->nblk; b++) {
    pstart[b] = (int)m->plo.size();
    const int a = b == 0 ? L[0] : R[b - 1], e = R[b];
    // the taps of block b must lie in the pieces of blocks b - 1 and b
    const int own_lo = b == 0 ? L[0] : (b == 1 ? L[0] : R[b - 2]);
    if (L[b] < own_lo) return false;
    int k = a;
    do {
      const int n = std::min(64, e - k);
      m->plo.push_back(k);
      m->pn.push_back(std::max(n, 0));
      m->pblk.push_back(b);
      m->plast.push_back(0);
      k += std::max(n, 0);
    } while (k < e);
    m->plast.back() = 1;
  }
  pstart[m->nblk] = (int)m->plo.size();
  const int np = (int)m->plo.size();
  m->frag.assign((size_t)np * 6 * 256, 0);
  for (int p = 0; p < np; p++)
    for (int s = 0; s < 2; s++) {
      const int bb = m->pblk[p] + s;
      if (bb >= m->nblk) continue;
      for (int l = 0; l < 64; l++)
        for (int j = 0; j < 16; j++) {
          const int y = 16 * bb + (l & 15), k = mfma_i8_k(l, j);
          int32_t limb[3];
          limbs3(y < ny && k < m->pn[p] ? tap_w(v, q22, m->rows, y, m->plo[p] + k) : 0, limb);
          put_frag(m->frag, (size_t)(p * 2 + s) * 3 * 256, l, j, limb);
        }
    }
  // every tap is covered exactly once by (its block's pieces) U (previous block's pieces)
  for (int y = 0; y < ny; y++) {
    const int b = y / 16;
    const int lo_list = b == 0 ? L[0] : m->plo[pstart[b - 1]];
    for (int j = 0; j < v.count[y]; j++) {
      if (v.w[v.woff[y] + j] == 0.0f) continue;
      const int li = idx[v.start[y] + j - v.src_lo];
      if (li < lo_list || li >= R[b]) return false;
    }
  }
  m->w128.assign((size_t)16 * (m->nblk + 2), 0);  // two zero blocks: k_rs_vm loads block b + 2 unconditionally
  for (int y = 0; y < ny; y++)
    for (int j = 0; j < v.count[y]; j++) m->w128[y] += 128 * q22[v.woff[y] + j];
  m->row0 = m->rows[0];
  m->rstep = nl > 1 ? m->rows[1] - m->rows[0] : 1;
  for (int k = 1; k < nl && m->rstep > 0; k++)
    if (m->rows[k] != m->row0 + m->rstep * k) m->rstep = 0;
  return true;
}

bool build_vr_v(const AxisTable &v, VrV *m) {
  *m = VrV();
  const int ny = (int)v.start.size();
  if (ny == 0) return false;
  std::vector<int32_t> idx;
  touched_list(v, &m->rows, &idx);
  const int nl = (int)m->rows.size();
  if (nl == 0) return false;
  m->nblk = (ny + 15) / 16;
  std::vector<int32_t> wq;
  m->shift = vr_quant(v, &wq);
  if (m->shift == 0) return false;
  m->frag.assign((size_t)m->nblk * 4 * 256, 0);
  m->w128.assign((size_t)16 * m->nblk, 0);
  int pK0 = 0, pR = 0;
  for (int b = 0; b < m->nblk; b++) {
    int lo = 1 << 30, hi = -1;
    for (int y = 16 * b; y < std::min(ny, 16 * b + 16); y++) {
      int a, e;
      tap_range(v, idx, y, &a, &e);
      if (e < a) return false;  // an output row without taps
      lo = std::min(lo, a);
      hi = std::max(hi, e);
    }
    const int K0 = lo / 16 * 16, R = hi + 1;
    const int ks = (R - K0 + 63) / 64;
    if (ks > 2) return false;
    if (b > 0 && (K0 < pK0 || R < pR)) return false;  // not monotone
    pK0 = K0;
    pR = R;
    m->bmeta.insert(m->bmeta.end(), {K0, ks, R, 0});
    for (int t = 0; t < ks; t++)
      for (int l = 0; l < 64; l++)
        for (int j = 0; j < 16; j++) {
          const int y = 16 * b + (l & 15), k = K0 + 64 * t + mfma_i8_k(l, j);
          int32_t limb[2];
          limbs2(y < ny ? tap_wq(v, wq, m->rows, y, k) : 0, limb);
          put_frag2(m->frag, (size_t)(b * 2 + t) * 2 * 256, l, j, limb);
        }
  }
  for (int y = 0; y < ny; y++)
    for (int j = 0; j < v.count[y]; j++) m->w128[y] += 128 * wq[v.woff[y] + j];
  // k_rs_vr's MFMA bias is the constant 128 * 2^shift: every row must sum to 2^shift
  for (int y = 0; y < ny; y++)
    if (m->w128[y] != (128 << m->shift)) return false;
  m->row0 = m->rows[0];
  m->rstep = nl > 1 ? m->rows[1] - m->rows[0] : 1;
  for (int k = 1; k < nl && m->rstep > 0; k++)
    if (m->rows[k] != m->row0 + m->rstep * k) m->rstep = 0;
  // unevenly spaced rows (ThumbnailImage sampling, e.g. cfg1's 2000 -> 1250)
  // stream from the touched-row list (fi_vr.hip issue_rows)
  for (int k = 1; k < nl; k++) m->maxgap = std::max(m->maxgap, m->rows[k] - m->rows[k - 1]);
  return true;
}

// source-index range [a, e] of output o's non-zero taps (false: none)
static bool src_range(const AxisTable &t, int o, int *a, int *e) {
  *a = 1 << 30;
  *e = -1;
  for (int j = 0; j < t.count[o]; j++)
    if (t.w[t.woff[o] + j] != 0.0f) {
      *a = std::min(*a, t.start[o] + j);
      *e = std::max(*e, t.start[o] + j);
    }
  return *e >= *a;
}
// quantized weight of output o at source index s (0 if not a tap)
static int32_t tap_w_src(const AxisTable &t, int o, int s) {
  const int j = s - t.start[o];
  return (j < 0 || j >= t.count[o]) ? 0 : quant_w(t.w[t.woff[o] + j]);
}
// per-output tap ranges, monotone in o (false otherwise)
static bool monotone_ranges(const AxisTable &t, std::vector<int> *lo, std::vector<int> *hi) {
  const int n = (int)t.start.size();
  lo->resize(n);
  hi->resize(n);
  for (int o = 0; o < n; o++) {
    if (!src_range(t, o, &(*lo)[o], &(*hi)[o])) return false;
    if (o > 0 && ((*lo)[o] < (*lo)[o - 1] || (*hi)[o] < (*hi)[o - 1])) return false;
  }
  return true;
}

bool build_hv_h(const AxisTable &h, HvH *m) {
  *m = HvH();
  const int nx = (int)h.start.size();
  std::vector<int> lo, hi;
  if (nx == 0 || !monotone_ranges(h, &lo, &hi)) return false;
  m->w128.assign(nx, 0);
  for (int x = 0; x < nx; x++)
    for (int j = 0; j < h.count[x]; j++) m->w128[x] += 128 * quant_w(h.w[h.woff[x] + j]);
  m->col0 = lo[0];
  // strip [x0, x1): window starts / k-steps per 16-px block (false: a block
  // needs more than 2 k-steps or the window more than kHvMaxPP px)
  auto try_strip = [&](int x0, int x1, HvStrip *S, std::vector<int32_t> *s0) {
    S->x0 = x0;
    S->x1 = x1;
    S->px0 = lo[x0] / 16 * 16;
    S->nocb = (x1 - x0 + 15) / 16;
    int pp = 0;
    s0->clear();
    for (int ob = 0; ob < S->nocb; ob++) {
      const int xa = x0 + 16 * ob, xb = std::min(x1, xa + 16);
      const int w0 = (lo[xa] - S->px0) / 8 * 8;
      const int ks = (hi[xb - 1] + 1 - S->px0 - w0 + 63) / 64;
      if (ks > 2) return false;
      s0->push_back(w0);
      s0->push_back(ks);
      pp = std::max(pp, w0 + 64 * ks);
    }
    S->pp = (pp + 15) / 16 * 16;
    return S->pp <= kHvMaxPP;
  };
  for (int x0 = 0; x0 < nx;) {
    HvStrip S{};
    std::vector<int32_t> s0;
    int x1 = std::min(nx, x0 + kHvMaxNx);
    while (!try_strip(x0, x1, &S, &s0)) {
      if (x1 - x0 <= 16) return false;
      x1 = x0 + (x1 - x0 - 1) / 16 * 16;
    }
    S.s0 = m->s0.size();
    m->s0.insert(m->s0.end(), s0.begin(), s0.end());
    S.frag = m->frag.size();
    m->frag.resize(m->frag.size() + (size_t)S.nocb * 2 * 3 * 256, 0);
    for (int ob = 0; ob < S.nocb; ob++)
      for (int t = 0; t < 2; t++)
        for (int l = 0; l < 64; l++)
          for (int j = 0; j < 16; j++) {
            const int x = x0 + 16 * ob + (l & 15);
            const int s = S.px0 + s0[2 * ob] + 64 * t + mfma_i8_k(l, j);
            int32_t limb[3];
            limbs3(t < s0[2 * ob + 1] && x < x1 ? tap_w_src(h, x, s) : 0, limb);
            put_frag(m->frag, S.frag + (size_t)(ob * 2 + t) * 3 * 256, l, j, limb);
          }
    m->strips.push_back(S);
    x0 = x1;
  }
  return true;
}

bool build_hv_v(const AxisTable &v, HvV *m) {
  *m = HvV();
  const int ny = (int)v.start.size();
  std::vector<int> lo, hi;
  if (ny == 0 || !monotone_ranges(v, &lo, &hi)) return false;
  m->row0 = lo[0];
  m->nrows = hi[ny - 1] + 1 - m->row0;
  m->nblk = (ny + 15) / 16;
  m->frag.assign((size_t)m->nblk * 2 * 3 * 256, 0);
  m->wsum.assign((size_t)16 * m->nblk, 0);
  for (int b = 0; b < m->nblk; b++) {
    const int ye = std::min(ny, 16 * b + 16);
    const int K0 = lo[16 * b] - m->row0;
    const int ks = (hi[ye - 1] + 1 - m->row0 - K0 + 63) / 64;
    if (ks > 2) return false;
    m->k0ks.push_back(K0);
    m->k0ks.push_back(ks);
    for (int t = 0; t < ks; t++)
      for (int l = 0; l < 64; l++)
        for (int j = 0; j < 16; j++) {
          const int y = 16 * b + (l & 15);
          const int s = m->row0 + K0 + 64 * t + mfma_i8_k(l, j);
          int32_t limb[3];
          limbs3(y < ny ? tap_w_src(v, y, s) : 0, limb);
          put_frag(m->frag, (size_t)(b * 2 + t) * 3 * 256, l, j, limb);
        }
  }
  for (int y = 0; y < ny; y++)
    for (int j = 0; j < v.count[y]; j++) m->wsum[y] += quant_w(v.w[v.woff[y] + j]);
  return true;
}



// ---------------------------------------------------------------------------
// Pillow
// ---------------------------------------------------------------------------
static double pil_sinc(double x) {
  if (x == 0.0) return 1.0;
  x = x * M_PI;
  return sin(x) / x;
}
static double pil_lanczos(double x) {
  if (-3.0 <= x && x < 3.0) return pil_sinc(x) * pil_sinc(x / 3);
  return 0.0;
}

int pil_coeffs(int in_size, float in0, float in1, int out_size, std::vector<int32_t> *bounds,
               std::vector<int32_t> *kk) {
  double scale, filterscale;
  filterscale = scale = (double)(in1 - in0) / out_size;
  if (filterscale < 1.0) filterscale = 1.0;
  const double support = 3.0 * filterscale;
  const int ksize = (int)ceil(support) * 2 + 1;
  std::vector<double> k(ksize);
  bounds->assign((size_t)out_size * 2, 0);
  kk->assign((size_t)out_size * ksize, 0);
  for (int xx = 0; xx < out_size; xx++) {
    const double center = in0 + (xx + 0.5) * scale;
    double ww = 0.0;
    const double ss = 1.0 / filterscale;
    int xmin = (int)(center - support + 0.5);
    if (xmin < 0) xmin = 0;
    int xmax = (int)(center + support + 0.5);
    if (xmax > in_size) xmax = in_size;
    xmax -= xmin;
    int x;
    for (x = 0; x < xmax; x++) {
      const double w = pil_lanczos((x + xmin - center + 0.5) * ss);
      k[x] = w;
      ww += w;
    }
    for (x = 0; x < xmax; x++)
      if (ww != 0.0) k[x] /= ww;
    for (; x < ksize; x++) k[x] = 0;
    for (x = 0; x < ksize; x++)
      (*kk)[(size_t)xx * ksize + x] =
          k[x] < 0 ? (int32_t)(-0.5 + k[x] * (1 << 22)) : (int32_t)(0.5 + k[x] * (1 << 22));
    (*bounds)[xx * 2 + 0] = xmin;
    (*bounds)[xx * 2 + 1] = xmax;
  }
  return ksize;
}

// Image.thumbnail preserve_aspect_ratio (PIL/Image.py:2878-2893)
static int pil_thumbnail_size(int W, int H, int x, int y, int *tw, int *th) {
  if (x >= W && y >= H) return 1;
  if (y == 0) return FI_EINVAL;  // ZeroDivisionError in x / y
  const double aspect = (double)W / (double)H;
  if ((double)x / (double)y >= aspect) {
    const double num = y * aspect, f = floor(num), c = ceil(num);
    const double kf = fabs(aspect - f / y), kc = fabs(aspect - c / y);
    const double r = (kc < kf) ? c : f;
    x = r < 1 ? 1 : (int)r;
  } else {
    const double num = x / aspect, f = floor(num), c = ceil(num);
    if (f == 0 && c == 0) {
      y = 1;
    } else {
      const double kf = (f == 0) ? 0 : fabs(aspect - x / f), kc = (c == 0) ? 0 : fabs(aspect - x / c);
      const double r = (kc < kf) ? c : f;
      y = r < 1 ? 1 : (int)r;
    }
  }
  *tw = x;
  *th = y;
  return 0;
}

// ---------------------------------------------------------------------------
// smartcrop.py geometry
// ---------------------------------------------------------------------------
int plan_sc(int W, int H, int width, int height, const fi_smartcrop_options &o, ScPlan *p) {
  *p = ScPlan();
  p->W = W;
  p->H = H;
  auto fail = [&](int code, const char *m) {
    p->status = code;
    p->err = m;
    return code;
  };
  if (W <= 0 || H <= 0 || width <= 0 || height <= 0) return fail(FI_EINVAL, "smartcrop: bad dimensions");
  const double sw = (double)W / width, sh = (double)H / height;
  const double scale = (sh < sw) ? sh : sw;  // min(a, b)
  int cw = (int)floor(width * scale), ch = (int)floor(height * scale);
  double min_scale = o.min_scale;
  {
    const double inv = 1 / scale;
    const double m = (min_scale > inv) ? min_scale : inv;          // max(1/scale, min_scale)
    min_scale = (m < o.max_scale) ? m : o.max_scale;                // min(max_scale, .)
  }
  double pre = 1;
  int aw = W, ah = H;
  if (o.prescale) {
    pre = 1 / scale / min_scale;
    if (pre < 1) {
      const int tx = (int)(W * pre), ty = (int)(H * pre);
      int tw = W, th = H;
      const int r = pil_thumbnail_size(W, H, tx, ty, &tw, &th);
      if (r < 0) return fail(FI_EINVAL, "smartcrop: thumbnail size division by zero");
      if (r == 1) {
        tw = W;
        th = H;
      }
      if (tw != W || th != H) {
        p->thumb = true;
        // Image.resize(reducing_gap=2.0)
        const int fx = (int)((double)W / tw / 2.0), fy = (int)((double)H / th / 2.0);
        p->fx = fx ? fx : 1;
        p->fy = fy ? fy : 1;
        float bx1 = (float)W, by1 = (float)H;
        int iw = W, ih = H;
        if (p->fx > 1 || p->fy > 1) {
          iw = (W + p->fx - 1) / p->fx;
          ih = (H + p->fy - 1) / p->fy;
          bx1 = (float)((double)W / p->fx);
          by1 = (float)((double)H / p->fy);
        }
        p->rw = iw;
        p->rh = ih;
        p->need_h = tw != iw || bx1 != (float)iw;
        p->need_v = th != ih || by1 != (float)ih;
        p->ksh = pil_coeffs(iw, 0.0f, bx1, tw, &p->hb, &p->hk);
        p->ksv = pil_coeffs(ih, 0.0f, by1, th, &p->vb, &p->vk);
        p->ybox_first = p->vb[0];
        const int ybox_last = p->vb[th * 2 - 2] + p->vb[th * 2 - 1];
        if (p->need_h) {
          for (int i = 0; i < th; i++) p->vb[i * 2] -= p->ybox_first;
          p->hrows = ybox_last - p->ybox_first;
        } else {
          p->hrows = 0;
        }
      }
      aw = tw;
      ah = th;
      cw = (int)floor(cw * pre);
      ch = (int)floor(ch * pre);
    } else {
      pre = 1;
    }
  }
  if (!p->thumb) {
    p->rw = W;
    p->rh = H;
  }
  p->prescale = pre;
  p->aw = aw;
  p->ah = ah;
  p->cw = cw;
  p->ch = ch;
  // crops() (smartcrop.py:193-229)
  const int i0 = (int)(o.max_scale * 100), i1 = (int)((min_scale - o.scale_step) * 100);
  const int di = -(int)(o.scale_step * 100);
  if (di >= 0 || o.step <= 0) return fail(FI_EINVAL, "smartcrop: bad scale_step/step");
  for (int i = i0; i > i1; i += di) {
    const double s = i / 100.0;
    for (int y = 0; y < ah; y += o.step) {
      if (!(y + ch * s <= ah)) break;
      for (int x = 0; x < aw; x += o.step) {
        if (!(x + cw * s <= aw)) break;
        CropHost c;
        c.fx = x;
        c.fy = y;
        c.fw = cw * s;
        c.fh = ch * s;
        c.x0 = x;
        c.y0 = y;
        c.nin_x = std::min(aw - x, (int)ceil(x + c.fw) - x);
        c.nin_y = std::min(ah - y, (int)ceil(y + c.fh) - y);
        if (c.nin_x < 0) c.nin_x = 0;
        if (c.nin_y < 0) c.nin_y = 0;
        c.rx = (int32_t)floor(c.fx / pre);
        c.ry = (int32_t)floor(c.fy / pre);
        c.rw = (int32_t)floor(c.fw / pre);
        c.rh = (int32_t)floor(c.fh / pre);
        p->crops.push_back(c);
      }
    }
  }
  if (p->crops.empty()) return fail(FI_ENOCROP, "smartcrop: no crop windows (smartcrop.py:227-228 ValueError)");
  plan_sc_prep(p);
  return FI_OK;
}

// k_sc_hrows / k_sc_vmaps launch geometry (fi_smartcrop.hip): row chunks and
// the LDS each needs (transposed H coefficients + staged source rows; staged
// H-stage rows + prescaled rows of an output chunk with its one-row halo).
// Exact-integer MFMA form of Pillow's horizontal pass (k_sc_hmfma): for each
// block of 16 output columns, the banded coefficient matrix over a window of
// 64 * ks source columns, split into three signed-byte limbs
// (k = L0 + 256 L1 + 65536 L2), laid out in the MFMA B-fragment order.
static void plan_sc_hmfma(ScPlan *p, int sw) {
  p->hm_ok = false;
  const int aw = p->aw, nb = (aw + 15) / 16;
  int ks = 1, maxend = sw;
  std::vector<int32_t> s0(nb);
  for (int b = 0; b < nb; b++) {
    int lo = 1 << 30, hi = 0;
    for (int x = 16 * b; x < std::min(aw, 16 * b + 16); x++) {
      lo = std::min(lo, p->hb[2 * x]);
      hi = std::max(hi, p->hb[2 * x] + p->hb[2 * x + 1]);
    }
    s0[b] = lo / 8 * 8;  // fragment reads are two 8-byte LDS reads: 8-B aligned
    ks = std::max(ks, (hi - s0[b] + 63) / 64);
  }
  for (int b = 0; b < nb; b++) maxend = std::max(maxend, s0[b] + 64 * ks);
  const int pitch = (maxend + 15) / 16 * 16;
  int rows = 32;
  while (rows >= 16 && (int64_t)3 * rows * pitch > kHmMaxLds) rows -= 16;
  if (rows < 16 || ks > 2) return;
  p->hm_ks = ks;
  p->hm_pitch = pitch;
  p->hm_rows = rows;
  p->hm_nb = nb;
  p->hm_lds = 3 * rows * pitch;
  p->hm_chunks = (p->hrows + rows - 1) / rows;
  p->hmS0 = s0;
  p->hmC.assign(aw, 0);
  for (int x = 0; x < aw; x++) {
    int64_t sum = 0;
    for (int j = 0; j < p->hb[2 * x + 1]; j++) sum += p->hk[(size_t)x * p->ksh + j];
    p->hmC[x] = (int32_t)((1 << 21) + 128 * sum);
  }
  p->hmB.assign((size_t)nb * ks * 3 * 256, 0);
  for (int b = 0; b < nb; b++)
    for (int t = 0; t < ks; t++)
      for (int l = 0; l < 64; l++)
        for (int j = 0; j < 16; j++) {
          const int x = 16 * b + (l & 15), s = s0[b] + 64 * t + mfma_i8_k(l, j);
          int32_t k = 0;
          if (x < aw) {
            const int xmin = p->hb[2 * x], cnt = p->hb[2 * x + 1];
            if (s >= xmin && s < xmin + cnt) k = p->hk[(size_t)x * p->ksh + (s - xmin)];
          }
          const int32_t l0 = ((k + 128) & 255) - 128;
          const int32_t k1 = (k - l0) / 256;
          const int32_t l1 = ((k1 + 128) & 255) - 128;
          const int32_t l2 = (k1 - l1) / 256;
          const int32_t limb[3] = {l0, l1, l2};
          for (int q = 0; q < 3; q++) {
            uint8_t *frag = reinterpret_cast<uint8_t *>(&p->hmB[((size_t)(b * ks + t) * 3 + q) * 256]);
            frag[l * 16 + j] = (uint8_t)(int8_t)limb[q];
          }
        }
  p->hm_ok = true;
}

// k_sc_vq tables: per chunk of kVqRows analysed rows, the 16 prescaled rows
// [pa, pa + 16) (pa = y0 - 1 clamped) as one MFMA block over a window of <= 64
// H-stage rows starting at vqK0; coefficients as three signed-byte limbs.
static void plan_sc_vq(ScPlan *p) {
  p->vq_ok = false;
  if (!(p->thumb && p->need_h && p->need_v)) return;
  const int ah = p->ah, chunks = (ah + kVqRows - 1) / kVqRows;
  p->vqC.assign(ah, 0);  // (k_sc_vx's bias too, whether or not k_sc_vq's windows fit)
  for (int y = 0; y < ah; y++) {
    int64_t sum = 0;
    for (int j = 0; j < p->vb[2 * y + 1]; j++) sum += p->vk[(size_t)y * p->ksv + j];
    p->vqC[y] = (int32_t)((1 << 21) + 128 * sum);
  }
  p->vqK0.assign(chunks, 0);
  p->vqA.assign((size_t)chunks * 3 * 256, 0);
  for (int c = 0; c < chunks; c++) {
    const int y0 = kVqRows * c, pa = std::max(0, y0 - 1), pe = std::min(ah, pa + 16);
    const int k0 = p->vb[2 * pa];
    for (int y = pa; y < pe; y++)
      if (p->vb[2 * y] < k0 || p->vb[2 * y] + p->vb[2 * y + 1] - k0 > 64) return;
    p->vqK0[c] = k0;
    for (int l = 0; l < 64; l++)
      for (int j = 0; j < 16; j++) {
        const int y = pa + (l & 15), k = k0 + mfma_i8_k(l, j);
        int32_t w = 0;
        if (y < pe && k >= p->vb[2 * y] && k < p->vb[2 * y] + p->vb[2 * y + 1])
          w = p->vk[(size_t)y * p->ksv + (k - p->vb[2 * y])];
        int32_t limb[3];
        limbs3(w, limb);
        for (int q = 0; q < 3; q++)
          reinterpret_cast<uint8_t *>(&p->vqA[((size_t)c * 3 + q) * 256])[l * 16 + j] = (uint8_t)(int8_t)limb[q];
      }
  }
  const int apitch = (p->aw * 3 + 15) / 16 * 16;
  p->vq_lds = 64 * apitch + 16 * apitch + 16 * ((p->aw + 3) / 4 * 4);
  if (p->vq_lds > kPrepMaxLds) return;
  p->vq_chunks = chunks;
  p->vq_ok = true;
}

// k_sc_hx / k_sc_vx tables (fi_plan.h ScPlan::cx_*): per chunk of kVqRows
// analysed rows, the 16 prescaled rows [pa, pa + 16) over the H-stage rows
// [K0, K0 + 64 kv), K0 = the chunk's first tap rounded down to a multiple of 4,
// coefficients as three signed-byte limbs in A-fragment order (row pa + (l & 15),
// K slot mfma_i8_k(l, j) of k-step t).  Needs k_sc_hmfma's horizontal tables.
static void plan_sc_cx(ScPlan *p) {
  p->cx_ok = false;
  p->cxA.clear();
  p->cxK0.clear();
  if (!p->hm_ok || !(p->thumb && p->need_h && p->need_v) || (int)p->vqC.size() != p->ah) return;
  const int ah = p->ah, chunks = (ah + kVqRows - 1) / kVqRows;
  int kv = 1, tp = p->hrows;
  p->cxK0.assign(chunks, 0);
  for (int c = 0; c < chunks; c++) {
    const int y0 = kVqRows * c, pa = std::max(0, y0 - 1), pe = std::min(ah, pa + 16);
    int lo = 1 << 30, hi = 0;
    for (int y = pa; y < pe; y++) {
      lo = std::min(lo, p->vb[2 * y]);
      hi = std::max(hi, p->vb[2 * y] + p->vb[2 * y + 1]);
    }
    p->cxK0[c] = lo & ~3;
    kv = std::max(kv, (hi - p->cxK0[c] + 63) / 64);
  }
  if (kv > 2) return;
  for (int c = 0; c < chunks; c++) tp = std::max(tp, p->cxK0[c] + 64 * kv);
  p->cx_tp = (tp + 15) / 16 * 16 + 16;  // + one row block: the V pass's 16-B reads straddle two
  p->cx_kv = kv;
  p->cxA.assign((size_t)chunks * kv * 3 * 256, 0);
  for (int c = 0; c < chunks; c++) {
    const int y0 = kVqRows * c, pa = std::max(0, y0 - 1), pe = std::min(ah, pa + 16);
    for (int t = 0; t < kv; t++)
      for (int l = 0; l < 64; l++)
        for (int j = 0; j < 16; j++) {
          const int y = pa + (l & 15), k = p->cxK0[c] + 64 * t + mfma_i8_k(l, j);
          int32_t w = 0;
          if (y < pe && k >= p->vb[2 * y] && k < p->vb[2 * y] + p->vb[2 * y + 1])
            w = p->vk[(size_t)y * p->ksv + (k - p->vb[2 * y])];
          int32_t limb[3];
          limbs3(w, limb);
          for (int q = 0; q < 3; q++)
            reinterpret_cast<uint8_t *>(&p->cxA[(((size_t)c * kv + t) * 3 + q) * 256])[l * 16 + j] =
                (uint8_t)(int8_t)limb[q];
        }
  }
  p->cx_ok = true;
}

void plan_sc_prep(ScPlan *p) {
  p->prep_ok = false;
  p->hkT.clear();
  const bool reduced = p->fx > 1 || p->fy > 1;
  const int sw = reduced ? p->rw : p->W;
  const int64_t apitch = (p->aw * 3 + 15) / 16 * 16, spitch = (sw * 3 + 15) / 16 * 16;
  p->h_chunks = 0;
  p->h_lds = 0;
  if (p->thumb && p->need_h) {
    p->hkT.assign((size_t)p->ksh * p->aw, 0);
    for (int x = 0; x < p->aw; x++)
      for (int j = 0; j < p->ksh; j++) p->hkT[(size_t)j * p->aw + x] = p->hk[(size_t)x * p->ksh + j];
    p->h_chunks = (p->hrows + kPrepRows - 1) / kPrepRows;
    const int64_t lds = ((int64_t)p->ksh * p->aw * 4 + 15) / 16 * 16 + kPrepRows * spitch;
    if (lds > kPrepMaxLds) return;
    p->h_lds = (int)lds;
    plan_sc_hmfma(p, sw);
  }
  p->v_chunks = (p->ah + kPrepRows - 1) / kPrepRows;
  int64_t vmax = 0;
  const bool need_v = p->thumb && p->need_v;
  for (int c = 0; c < p->v_chunks; c++) {
    const int y0 = c * kPrepRows, y1 = std::min(y0 + kPrepRows, p->ah);
    const int pa = std::max(0, y0 - 1), pb = std::min(p->ah, y1 + 1);
    int lo = pa, hi = pb;
    if (need_v) {
      lo = p->vb[2 * pa];
      hi = 0;
      for (int y = pa; y < pb; y++) {
        if (p->vb[2 * y] < lo) return;  // kernel stages from the first row's window start
        hi = std::max(hi, p->vb[2 * y] + p->vb[2 * y + 1]);
      }
    }
    vmax = std::max(vmax, (int64_t)(hi - lo) * apitch + (int64_t)(pb - pa) * apitch);
  }
  if (vmax > kPrepMaxLds) return;
  p->v_lds = (int)vmax;
  p->prep_ok = true;
  plan_sc_vq(p);
  // k_sc_fz: both MFMA passes in one per-image workgroup (no reduce step; the
  // source block's items fit the kernel's 4 register slots per thread)
  p->fz_ok = false;
  if (p->hm_ok && p->vq_ok && !reduced && p->hm_pitch <= 1024) {
    const int64_t lpitch = (p->aw + 3) / 4 * 4;
    const int64_t lds = 80 * apitch + std::max<int64_t>(3 * 16 * (int64_t)p->hm_pitch, 16 * apitch + 16 * lpitch);
    if (lds <= kFzMaxLds) {
      p->fz_lds = (int)lds;
      p->fz_ok = true;
    }
  }
  if (!reduced) plan_sc_cx(p);
}

static double thirds(double x) {
  x = (fmod(x + 2.0 / 3.0, 2.0) * 0.5 - 0.5) * 16;
  const double v = 1 - x * x;
  return (0 > v) ? 0.0 : v;
}

void sc_importance_table(const fi_smartcrop_params &P, double fw, double fh, int nx, int ny,
                         std::vector<double> *out) {
  out->assign((size_t)nx * ny, 0.0);
  for (int dy = 0; dy < ny; dy++)
    for (int dx = 0; dx < nx; dx++) {
      const double xr = dx / fw, yr = dy / fh;
      const double px = fabs(0.5 - xr) * 2, py = fabs(0.5 - yr) * 2;
      double ddx = px - 1 + P.edge_radius, ddy = py - 1 + P.edge_radius;
      if (0 > ddx) ddx = 0;
      if (0 > ddy) ddy = 0;
      const double d = (ddx * ddx + ddy * ddy) * P.edge_weight;
      double s = 1.41 - sqrt(px * px + py * py);
      if (P.rule_of_thirds) {
        double m = s + d + 0.5;
        if (0 > m) m = 0;
        s += (m * 1.2) * (thirds(px) + thirds(py));
      }
      (*out)[(size_t)dy * nx + dx] = s + d;
    }
}

// k_sc_score3's B fragments (fi_internal.h ScGroup, v_mfma_i32_16x16x64_i8:
// lane l holds B[k = mfma_i8_k(l, j)][n = l & 15]).  Column n = digit n % 5 of
// slot n / 5.  Tq is formed exactly: imp 2^q and oi 2^q are doubles scaled by
// a power of two, their difference is exact in long double (|.| < 2^44 with
// no bit below 2^-10), then rounded once, so |Tq 2^-q - (imp - oi)| <= 2^-q-1.
void sc_score_btab(const std::vector<double> &imp, int nx, int ny, double oi, int nslot, int step, ScoreBTab *out) {
  *out = ScoreBTab();
  if (nx <= 0 || ny <= 0 || nslot < 1 || nslot > kSgSlots) return;
  double m = 0;
  for (double v : imp) m = std::max(m, std::fabs(v - oi));
  int q = 38;
  while (q > 0 && std::ldexp(m, q) * (1 + 1e-9) + 1 >= std::ldexp(1.0, 38) * 1.9) q--;
  const int ks = (nx + 63) / 64;
  if (ks > kSgMaxKs) return;
  std::vector<std::array<int8_t, kSgDigits>> dg((size_t)nx * ny);
  for (int v = 0; v < ny; v++)
    for (int u = 0; u < nx; u++) {
      const long double a = (long double)std::ldexp(imp[(size_t)v * nx + u], q);
      const long double b = (long double)std::ldexp(oi, q);
      int64_t x = (int64_t)std::llrintl(a - b);
      auto &d = dg[(size_t)v * nx + u];
      for (int i = 0; i < kSgDigits; i++) {
        const int64_t r = ((x + 128) & 255) - 128;
        d[i] = (int8_t)r;
        out->S[i] += (int32_t)r;
        x = (x - r) / 256;
      }
      if (x != 0) return;  // |Tq| beyond five digits (cannot happen with q above)
    }
  out->q = q;
  out->ks = ks;
  out->nrows = ny + step * (nslot - 1);
  out->frag.assign((size_t)out->nrows * ks * 256, 0);
  for (int r = 0; r < out->nrows; r++)
    for (int t = 0; t < ks; t++) {
      uint8_t *f = reinterpret_cast<uint8_t *>(&out->frag[((size_t)r * ks + t) * 256]);
      for (int l = 0; l < 64; l++) {
        const int n = l & 15, slot = n / kSgDigits, digit = n % kSgDigits;
        if (slot >= nslot) continue;
        const int v = r - step * slot;
        if (v < 0 || v >= ny) continue;
        for (int j = 0; j < 16; j++) {
          const int u = 64 * t + mfma_i8_k(l, j);
          if (u < nx) f[l * 16 + j] = (uint8_t)dg[(size_t)v * nx + u][digit];
        }
      }
    }
  out->ok = true;
}

// ---- ScaleImage contribution lists (resize.c ScaleImage; oracle
// or_im_scale_q16 is the literal loop) ----------------------------------------
void im_scale_rows(int H, int oh, ScaleList *L) {
  *L = ScaleList();
  L->off.push_back(0);
  if (oh == H) {  // rows copied (scanline = x_vector)
    for (int y = 0; y < oh; y++) {
      L->idx.push_back(y);
      L->w.push_back(1.0);
      L->off.push_back((int32_t)L->idx.size());
    }
    return;
  }
  int number_rows = 0, i = 0, cur = -1;
  bool next_row = true;
  double span_y = 1.0, scale_y = (double)oh / (double)H;
  for (int y = 0; y < oh; y++) {
    while (scale_y < span_y) {
      if (next_row && number_rows < H) {
        cur = i++;
        number_rows++;
      }
      L->idx.push_back(cur);
      L->w.push_back(scale_y);
      span_y -= scale_y;
      scale_y = (double)oh / (double)H;
      next_row = true;
    }
    if (next_row && number_rows < H) {
      cur = i++;
      number_rows++;
      next_row = false;
    }
    L->idx.push_back(cur);
    L->w.push_back(span_y);
    L->off.push_back((int32_t)L->idx.size());
    scale_y -= span_y;
    if (scale_y <= 0) {
      scale_y = (double)oh / (double)H;
      next_row = true;
    }
    span_y = 1.0;
  }
}

void im_scale_cols(int W, int ow, ScaleList *L) {
  *L = ScaleList();
  std::vector<std::vector<std::pair<int32_t, double>>> col(ow);
  if (ow == W) {
    for (int x = 0; x < ow; x++) col[x].push_back({x, 1.0});
  } else {
    std::vector<std::pair<int32_t, double>> cur;  // additions to `pixel` since its last reset
    bool next_column = false;
    int t = 0;
    double span_x = 1.0, scale_x = 0;
    for (int x = 0; x < W; x++) {
      scale_x = (double)ow / (double)W;
      while (scale_x >= span_x) {
        if (next_column) {
          cur.clear();
          t++;
        }
        cur.push_back({x, span_x});
        if (t < ow) col[t] = cur;  // scale_scanline[t] = pixel
        scale_x -= span_x;
        span_x = 1.0;
        next_column = true;
      }
      if (scale_x > 0) {
        if (next_column) {
          cur.clear();
          next_column = false;
          t++;
        }
        cur.push_back({x, scale_x});
        span_x -= scale_x;
      }
    }
    if (span_x > 0) cur.push_back({W - 1, span_x});
    if (!next_column && t < ow) col[t] = cur;
  }
  L->off.push_back(0);
  for (int x = 0; x < ow; x++) {
    for (auto &e : col[x]) {
      L->idx.push_back(e.first);
      L->w.push_back(e.second);
    }
    L->off.push_back((int32_t)L->idx.size());
  }
}

int im_percent_size(int size, double percent) { return (int)floor(percent * (double)size / 100.0 + 0.5); }

}  // namespace fi
