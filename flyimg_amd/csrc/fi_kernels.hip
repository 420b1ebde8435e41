// fi_kernels.hip -- gfx950 kernels of the flyimg hot path.
//
// Built with -ffp-contract=off: every float/double operation that mirrors a
// reference computation is one IEEE-rounded op (fast-path accumulations that
// are *allowed* to fuse use explicit fma()).
//
//   resample (ImageMagick -thumbnail/-resize, ImageProcessor.php:66-110):
//     k_rs_v_u8     vertical pass  RGB8 src  -> Q16 mid      (V-first images)
//     k_rs_h_final  horizontal pass Q16 mid  -> RGB8/Gray dst + extent/gray/rotate
//     k_rs_h_u8     horizontal pass RGB8 src -> Q16 mid      (H-first images)
//     k_rs_v_final  vertical pass  Q16 mid   -> dst + epilogue
//     k_rs_copy     no resample (ResizeImage clone) -> dst + epilogue
//     (the fused vertical-first kernel lives in fi_fused.hip)
//   smartcrop (python/smartcrop.py:79-191):
//     k_sc_reduce / k_sc_hpass / k_sc_vpass   Pillow thumbnail (integer, exact)
//     k_sc_maps                               L, edge, skin, saturation
//     k_sc_score                              fast bounded scores + exact re-score
//   k_crop_apply   convert -crop (SmartCropProcessor.php:30-34)
//   k_synth        seeded synthetic RGB8 (flyimg_amd/synth.py)
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "fi_internal.h"

namespace fi {

// ---------------------------------------------------------------------------
// helpers
// ---------------------------------------------------------------------------
// Find the image owning flat tile index t (prefix[i] = first tile of image i,
// prefix[n] = total).  Binary search, wave-uniform.
__device__ __forceinline__ int find_image(const int32_t *__restrict__ prefix, int n, int t) {
  int lo = 0, hi = n;  // invariant prefix[lo] <= t < prefix[hi]
  while (hi - lo > 1) {
    const int mid = (lo + hi) >> 1;
    if (prefix[mid] <= t)
      lo = mid;
    else
      hi = mid;
  }
  return lo;
}

__device__ __forceinline__ uint32_t clamp_q16(float v) {
  // ClampToQuantum (Q16, non-HDRI): <=0 -> 0, >=65535 -> 65535, else (v+0.5) truncated
  if (!(v > 0.0f)) return 0u;
  if (v >= 65535.0f) return 65535u;
  return (uint32_t)(v + 0.5f);
}
__device__ __forceinline__ uint32_t clamp_q16d(double v) {
  if (!(v > 0.0)) return 0u;
  if (v >= 65535.0) return 65535u;
  return (uint32_t)(v + 0.5);
}
__device__ __forceinline__ uint8_t q16_to_u8(uint32_t q) {  // ScaleQuantumToChar
  return (uint8_t)(((q + 128u) - ((q + 128u) >> 8)) >> 8);
}

// Epilogue: Q16 RGB of extent pixel (x, y) -> gray?/8-bit -> rotated store.
__device__ __forceinline__ void store_pixel(const ResizeDesc &D, int x, int y, uint32_t r, uint32_t g,
                                            uint32_t b) {
  int dx = x, dy = y;
  if (D.rot == 90) {
    dx = D.eh - 1 - y;
    dy = x;
  } else if (D.rot == 180) {
    dx = D.ew - 1 - x;
    dy = D.eh - 1 - y;
  } else if (D.rot == 270) {
    dx = y;
    dy = D.ew - 1 - x;
  }
  uint8_t *o = D.dst + (int64_t)dy * D.dst_stride;
  if (D.gray) {
    // -colorspace Gray: Rec709Luma on gamma-encoded Q16, ClampToQuantum
    const double gv = 0.212656 * (double)r + 0.715158 * (double)g + 0.072186 * (double)b;
    o[dx] = q16_to_u8(clamp_q16d(gv));
  } else {
    o[dx * 3 + 0] = q16_to_u8(r);
    o[dx * 3 + 1] = q16_to_u8(g);
    o[dx * 3 + 2] = q16_to_u8(b);
  }
}

// ---------------------------------------------------------------------------
// generic two-pass resample
// ---------------------------------------------------------------------------
// V-first, pass 1: mid[y][e] = Q16(257 * sum_j w[y][j] * src[start_y + j][b_lo + e])
// one workgroup per (image, output row); 8 consecutive bytes per thread.
__global__ __launch_bounds__(256) void k_rs_v_u8(const ResizeDesc *__restrict__ descs,
                                                 const int32_t *__restrict__ prefix, int nimg,
                                                 const int32_t *__restrict__ ai,
                                                 const float *__restrict__ af) {
  const int t = blockIdx.x;
  const int i = find_image(prefix, nimg, t);
  const ResizeDesc &D = descs[i];
  const int y = t - prefix[i];
  const int s = ai[D.v.start + y], n = ai[D.v.count + y];
  const float *w = af + ai[D.v.woff + y];
  const int nel = D.mid_cols;  // bytes of the strip row held in mid
  const int64_t b_lo = D.mid_c0;
  uint16_t *out = D.mid + (int64_t)y * D.mid_stride;
  for (int e = threadIdx.x * 8; e < nel; e += 256 * 8) {
    float acc[8];
#pragma unroll
    for (int k = 0; k < 8; k++) acc[k] = 0.0f;
    const bool full = e + 8 <= nel;
    for (int j = 0; j < n; j++) {
      const uint8_t *p = D.src + (int64_t)(s + j) * D.src_stride + b_lo + e;
      const float wj = w[j];
      if (full && ((((uintptr_t)p) & 7) == 0)) {
        const uint2 v = *reinterpret_cast<const uint2 *>(p);
#pragma unroll
        for (int k = 0; k < 4; k++) acc[k] += wj * (float)((v.x >> (8 * k)) & 255u);
#pragma unroll
        for (int k = 0; k < 4; k++) acc[4 + k] += wj * (float)((v.y >> (8 * k)) & 255u);
      } else {
        for (int k = 0; k < 8 && e + k < nel; k++) acc[k] += wj * (float)p[k];
      }
    }
    for (int k = 0; k < 8 && e + k < nel; k++) out[e + k] = (uint16_t)clamp_q16(acc[k] * 257.0f);
  }
}

// V-first, pass 2: out[y][x] = Q16(sum_j w[x][j] * mid[y][3*(start_x + j) - b_lo + c]) + epilogue
__global__ __launch_bounds__(256) void k_rs_h_final(const ResizeDesc *__restrict__ descs,
                                                    const int32_t *__restrict__ prefix, int nimg,
                                                    const int32_t *__restrict__ ai,
                                                    const float *__restrict__ af) {
  const int t = blockIdx.x;
  const int i = find_image(prefix, nimg, t);
  const ResizeDesc &D = descs[i];
  const int y = t - prefix[i];
  const uint16_t *row = D.mid + (int64_t)y * D.mid_stride;
  for (int x = threadIdx.x; x < D.ew; x += 256) {
    const int s = ai[D.h.start + x], n = ai[D.h.count + x];
    const float *w = af + ai[D.h.woff + x];
    const uint16_t *p = row + (int64_t)3 * s - D.mid_c0;
    float r = 0.f, g = 0.f, b = 0.f;
    for (int j = 0; j < n; j++) {
      const float wj = w[j];
      r += wj * (float)p[3 * j + 0];
      g += wj * (float)p[3 * j + 1];
      b += wj * (float)p[3 * j + 2];
    }
    store_pixel(D, x, y, clamp_q16(r), clamp_q16(g), clamp_q16(b));
  }
}

// H-first, pass 1: mid[r - r0][3x + c] = Q16(257 * sum_j w[x][j] * src[r][3(start_x+j) + c])
__global__ __launch_bounds__(256) void k_rs_h_u8(const ResizeDesc *__restrict__ descs,
                                                 const int32_t *__restrict__ prefix, int nimg,
                                                 const int32_t *__restrict__ ai,
                                                 const float *__restrict__ af) {
  const int t = blockIdx.x;
  const int i = find_image(prefix, nimg, t);
  const ResizeDesc &D = descs[i];
  const int rr = t - prefix[i];
  const uint8_t *row = D.src + (int64_t)(D.mid_r0 + rr) * D.src_stride;
  uint16_t *out = D.mid + (int64_t)rr * D.mid_stride;
  for (int x = threadIdx.x; x < D.ew; x += 256) {
    const int s = ai[D.h.start + x], n = ai[D.h.count + x];
    const float *w = af + ai[D.h.woff + x];
    const uint8_t *p = row + 3 * (int64_t)s;
    float r = 0.f, g = 0.f, b = 0.f;
    for (int j = 0; j < n; j++) {
      const float wj = w[j];
      r += wj * (float)p[3 * j + 0];
      g += wj * (float)p[3 * j + 1];
      b += wj * (float)p[3 * j + 2];
    }
    out[3 * x + 0] = (uint16_t)clamp_q16(r * 257.0f);
    out[3 * x + 1] = (uint16_t)clamp_q16(g * 257.0f);
    out[3 * x + 2] = (uint16_t)clamp_q16(b * 257.0f);
  }
}

// H-first, pass 2: out[y][x] = Q16(sum_j w[y][j] * mid[start_y + j - r0][3x + c]) + epilogue
__global__ __launch_bounds__(256) void k_rs_v_final(const ResizeDesc *__restrict__ descs,
                                                    const int32_t *__restrict__ prefix, int nimg,
                                                    const int32_t *__restrict__ ai,
                                                    const float *__restrict__ af) {
  const int t = blockIdx.x;
  const int i = find_image(prefix, nimg, t);
  const ResizeDesc &D = descs[i];
  const int y = t - prefix[i];
  const int s = ai[D.v.start + y], n = ai[D.v.count + y];
  const float *w = af + ai[D.v.woff + y];
  for (int x = threadIdx.x; x < D.ew; x += 256) {
    float r = 0.f, g = 0.f, b = 0.f;
    for (int j = 0; j < n; j++) {
      const uint16_t *p = D.mid + (int64_t)(s + j - D.mid_r0) * D.mid_stride + 3 * x;
      const float wj = w[j];
      r += wj * (float)p[0];
      g += wj * (float)p[1];
      b += wj * (float)p[2];
    }
    store_pixel(D, x, y, clamp_q16(r), clamp_q16(g), clamp_q16(b));
  }
}

// No resample (ResizeImage clone path): extent crop + gray + rotate.
__global__ __launch_bounds__(256) void k_rs_copy(const ResizeDesc *__restrict__ descs,
                                                 const int32_t *__restrict__ prefix, int nimg) {
  const int t = blockIdx.x;
  const int i = find_image(prefix, nimg, t);
  const ResizeDesc &D = descs[i];
  const int y = t - prefix[i];
  const uint8_t *row = D.src + (int64_t)(D.ey0 + y) * D.src_stride + 3 * (int64_t)D.ex0;
  for (int x = threadIdx.x; x < D.ew; x += 256)
    store_pixel(D, x, y, 257u * row[3 * x], 257u * row[3 * x + 1], 257u * row[3 * x + 2]);
}

// ---------------------------------------------------------------------------
// smartcrop prescale: Pillow reduce + LANCZOS resample (exact integer math)
// ---------------------------------------------------------------------------
__device__ __forceinline__ void load_rgb(const uint8_t *img, int64_t stride, int C, int x, int y,
                                         uint32_t *r, uint32_t *g, uint32_t *b) {
  const uint8_t *p = img + (int64_t)y * stride;
  if (C == 3) {
    *r = p[3 * x];
    *g = p[3 * x + 1];
    *b = p[3 * x + 2];
  } else {  // smartcrop.py:357-365 pastes L into a new RGB image
    *r = *g = *b = p[x];
  }
}

// Reduce.c: out = ((sum + n/2) * (u32)(2^32f / (f32)(256 n))) >> 24
__device__ __forceinline__ uint32_t pil_div_u32(int n) {
  const float max_int = 4294967296.0f;
  return (uint32_t)(max_int / (float)(256u * (uint32_t)n));
}
__global__ __launch_bounds__(256) void k_sc_reduce(const ScDesc *__restrict__ descs,
                                                   const int32_t *__restrict__ prefix, int nimg) {
  const int t = blockIdx.x;
  const int i = find_image(prefix, nimg, t);
  const ScDesc &D = descs[i];
  const int y = t - prefix[i];
  const int y0 = y * D.fy, y1 = min(y0 + D.fy, D.H);
  for (int x = threadIdx.x; x < D.rw; x += 256) {
    const int x0 = x * D.fx, x1 = min(x0 + D.fx, D.W);
    const int n = (x1 - x0) * (y1 - y0);
    const uint32_t mult = pil_div_u32(n), amend = (uint32_t)(n / 2);
    uint32_t s0 = amend, s1 = amend, s2 = amend;
    for (int yy = y0; yy < y1; yy++)
      for (int xx = x0; xx < x1; xx++) {
        uint32_t r, g, b;
        load_rgb(D.img, D.stride, D.C, xx, yy, &r, &g, &b);
        s0 += r;
        s1 += g;
        s2 += b;
      }
    uint8_t *o = D.red + ((int64_t)y * D.rw + x) * 3;
    o[0] = (uint8_t)((s0 * mult) >> 24);
    o[1] = (uint8_t)((s1 * mult) >> 24);
    o[2] = (uint8_t)((s2 * mult) >> 24);
  }
}

__device__ __forceinline__ uint8_t pil_clip8(int32_t v) {
  v >>= 22;
  return (uint8_t)(v < 0 ? 0 : v > 255 ? 255 : v);
}

// Horizontal pass over rows [ybox_first, ybox_first + hrows) of the (reduced) image.
__global__ __launch_bounds__(256) void k_sc_hpass(const ScDesc *__restrict__ descs,
                                                  const int32_t *__restrict__ prefix, int nimg,
                                                  const int32_t *__restrict__ ai) {
  const int t = blockIdx.x;
  const int i = find_image(prefix, nimg, t);
  const ScDesc &D = descs[i];
  const int yy = t - prefix[i];
  const bool reduced = D.fx > 1 || D.fy > 1;
  const uint8_t *src = reduced ? D.red : D.img;
  const int64_t stride = reduced ? (int64_t)D.rw * 3 : D.stride;
  const int C = reduced ? 3 : D.C;
  const int32_t *bounds = ai + D.hb;
  const int32_t *kk = ai + D.hk;
  for (int xx = threadIdx.x; xx < D.aw; xx += 256) {
    const int xmin = bounds[2 * xx], xmax = bounds[2 * xx + 1];
    const int32_t *k = kk + (int64_t)xx * D.ksh;
    int32_t s0 = 1 << 21, s1 = 1 << 21, s2 = 1 << 21;
    for (int x = 0; x < xmax; x++) {
      uint32_t r, g, b;
      load_rgb(src, stride, C, x + xmin, yy + D.ybox_first, &r, &g, &b);
      s0 += (int32_t)r * k[x];
      s1 += (int32_t)g * k[x];
      s2 += (int32_t)b * k[x];
    }
    uint8_t *o = D.hbuf + ((int64_t)yy * D.aw + xx) * 3;
    o[0] = pil_clip8(s0);
    o[1] = pil_clip8(s1);
    o[2] = pil_clip8(s2);
  }
}

// Vertical pass -> prescaled image (aw x ah x 3).
__global__ __launch_bounds__(256) void k_sc_vpass(const ScDesc *__restrict__ descs,
                                                  const int32_t *__restrict__ prefix, int nimg,
                                                  const int32_t *__restrict__ ai) {
  const int t = blockIdx.x;
  const int i = find_image(prefix, nimg, t);
  const ScDesc &D = descs[i];
  const int yy = t - prefix[i];
  const bool reduced = D.fx > 1 || D.fy > 1;
  const uint8_t *src;
  int64_t stride;
  int C;
  if (D.need_h) {
    src = D.hbuf;
    stride = (int64_t)D.aw * 3;
    C = 3;
  } else if (reduced) {
    src = D.red;
    stride = (int64_t)D.rw * 3;
    C = 3;
  } else {
    src = D.img;
    stride = D.stride;
    C = D.C;
  }
  const int vw = D.aw;
  uint8_t *o = D.pre + (int64_t)yy * D.aw * 3;
  if (!D.need_v) {
    for (int xx = threadIdx.x; xx < vw; xx += 256) {
      uint32_t r, g, b;
      load_rgb(src, stride, C, xx, yy, &r, &g, &b);
      o[3 * xx] = (uint8_t)r;
      o[3 * xx + 1] = (uint8_t)g;
      o[3 * xx + 2] = (uint8_t)b;
    }
    return;
  }
  const int ymin = ai[D.vb + 2 * yy], ymax = ai[D.vb + 2 * yy + 1];
  const int32_t *k = ai + D.vk + (int64_t)yy * D.ksv;
  for (int xx = threadIdx.x; xx < vw; xx += 256) {
    int32_t s0 = 1 << 21, s1 = 1 << 21, s2 = 1 << 21;
    for (int y = 0; y < ymax; y++) {
      uint32_t r, g, b;
      load_rgb(src, stride, C, xx, y + ymin, &r, &g, &b);
      s0 += (int32_t)r * k[y];
      s1 += (int32_t)g * k[y];
      s2 += (int32_t)b * k[y];
    }
    o[3 * xx] = pil_clip8(s0);
    o[3 * xx + 1] = pil_clip8(s1);
    o[3 * xx + 2] = pil_clip8(s2);
  }
}

// ---------------------------------------------------------------------------
// smartcrop maps (analyse(), smartcrop.py:94-101)
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint32_t sc_luma(uint32_t r, uint32_t g, uint32_t b) {
  // Pillow ImagingConvertMatrix: float sum in order, +0.5 in double, CLIPF
  float v = 0.2126f * (float)r + 0.7152f * (float)g;
  v = v + 0.0722f * (float)b;
  v = v + 0.0f;
  v = (float)((double)v + 0.5);
  return v <= 0.0f ? 0u : v >= 255.0f ? 255u : (uint32_t)v;
}

__device__ __forceinline__ uint32_t pre_luma(const ScDesc &D, const uint8_t *pre, int64_t stride, int C,
                                             int x, int y) {
  uint32_t r, g, b;
  load_rgb(pre, stride, C, x, y, &r, &g, &b);
  return sc_luma(r, g, b);
}

__global__ __launch_bounds__(256) void k_sc_maps(const ScDesc *__restrict__ descs,
                                                 const int32_t *__restrict__ prefix, int nimg,
                                                 const ScParamsDev P) {
  const int t = blockIdx.x;
  const int i = find_image(prefix, nimg, t);
  const ScDesc &D = descs[i];
  const int y = t - prefix[i];
  const int W = D.aw, H = D.ah;
  // the analysed image is D.pre (3 channels) unless no prescale ran
  const bool own = D.pre != nullptr;
  const uint8_t *img = own ? D.pre : D.img;
  const int64_t stride = own ? (int64_t)W * 3 : D.stride;
  const int C = own ? 3 : D.C;
  for (int x = threadIdx.x; x < W; x += 256) {
    uint32_t r, g, b;
    load_rgb(img, stride, C, x, y, &r, &g, &b);
    const uint32_t L = sc_luma(r, g, b);
    // detect_edge: ImagingFilter3x3; border copies L; < 3x3 images copied
    uint32_t E = L;
    if (W >= 3 && H >= 3 && x > 0 && y > 0 && x < W - 1 && y < H - 1) {
      const int v = 4 * (int)L - (int)pre_luma(D, img, stride, C, x, y - 1) -
                    (int)pre_luma(D, img, stride, C, x, y + 1) - (int)pre_luma(D, img, stride, C, x - 1, y) -
                    (int)pre_luma(D, img, stride, C, x + 1, y) + 1;
      E = (uint32_t)(v <= 0 ? 0 : v >= 255 ? 255 : v);
    }
    const double rd_ = (double)r, gd_ = (double)g, bd_ = (double)b;
    // detect_skin (smartcrop.py:250-274)
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
    // saturation() + detect_saturation (smartcrop.py:16-27, 234-248)
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
    D.maps[(int64_t)y * W + x] = S | (E << 8) | (T << 16);
  }
}

// ---------------------------------------------------------------------------
// smartcrop scoring (score() smartcrop.py:300-338 for every crop + argmax
// analyse() :116-133).
//
// Fast pass: per crop, inside-window sums of importance x term by one wave
// (importance from a per-geometry f64 table); the outside part from the
// image totals (summed-area identity: outside = total - inside) times
// outside_importance.  Each fast total carries a rigorous bound on its
// distance to the reference's left-to-right f64 sum.  Crops whose bound
// interval reaches the best lower bound are re-scored exactly: one lane per
// crop, every pixel in the reference's row-major order, same IEEE operations.
// ---------------------------------------------------------------------------
__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

constexpr int kMaxCrops = 2048;  // per image; LDS holds totals + bounds

__global__ __launch_bounds__(256) void k_sc_score(const ScDesc *__restrict__ descs,
                                                  const DevCrop *__restrict__ crops,
                                                  const double *__restrict__ ad, CropScore *scores,
                                                  ScResult *results, const ScParamsDev P) {
  const ScDesc &D = descs[blockIdx.x];
  __shared__ double lut[256];
  __shared__ double part[4][3];
  __shared__ double T[3];
  __shared__ double s_tot[kMaxCrops];
  __shared__ double s_bnd[kMaxCrops];
  __shared__ int32_t cand[kMaxCrops];
  __shared__ int32_t ncand_s;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  if (D.ncrops > kMaxCrops) {
    if (tid == 0) {
      results[D.result].top = -1;
      results[D.result].n_candidates = D.ncrops;
      results[D.result].total = 0;
    }
    return;
  }
  lut[tid] = (double)tid / 255.0;  // Python int / 255 (correctly rounded)
  __syncthreads();
  const int W = D.aw, H = D.ah, npx = W * H;
  const uint32_t *maps = D.maps;
  const double sb = P.skin_bias, tb = P.saturation_bias, oi = P.outside_importance;

  // image totals of the three per-pixel terms (outside part of every crop)
  {
    double t0 = 0, t1 = 0, t2 = 0;
    for (int p = tid; p < npx; p += 256) {
      const uint32_t m = maps[p];
      const double d = lut[(m >> 8) & 255];
      t0 += d;
      t1 += lut[m & 255] * (d + sb);
      t2 += lut[(m >> 16) & 255] * (d + tb);
    }
    t0 = wave_sum(t0);
    t1 = wave_sum(t1);
    t2 = wave_sum(t2);
    if (lane == 0) {
      part[wave][0] = t0;
      part[wave][1] = t1;
      part[wave][2] = t2;
    }
    __syncthreads();
    if (tid < 3) T[tid] = (part[0][tid] + part[1][tid]) + (part[2][tid] + part[3][tid]);
    __syncthreads();
  }
  const double u = 1.1102230246251565e-16;  // 2^-53
  const double nn = (double)npx + 1.0;
  const double gam = nn * u / (1.0 - nn * u);
  const double aoi = fabs(oi);
  const double wd = P.detail_weight, ws = P.skin_weight, wt = P.saturation_weight;

  for (int c = wave; c < D.ncrops; c += 4) {
    const DevCrop cr = crops[D.crop0 + c];
    const double *tab = ad + cr.table;
    double sd = 0, ss = 0, st = 0, ad_ = 0, as_ = 0, at_ = 0, id = 0, is = 0, it = 0;
    for (int dy = 0; dy < cr.nin_y; dy++) {
      const uint32_t *mrow = maps + (int64_t)(cr.y0 + dy) * W + cr.x0;
      const double *trow = tab + (int64_t)dy * cr.table_w;
      for (int dx = lane; dx < cr.nin_x; dx += 64) {
        const uint32_t m = mrow[dx];
        const double imp = trow[dx];
        const double d = lut[(m >> 8) & 255];
        const double a1 = lut[m & 255] * (d + sb);
        const double a2 = lut[(m >> 16) & 255] * (d + tb);
        const double ai_ = fabs(imp);
        sd = fma(imp, d, sd);
        ss = fma(imp, a1, ss);
        st = fma(imp, a2, st);
        ad_ = fma(ai_, d, ad_);
        as_ = fma(ai_, a1, as_);
        at_ = fma(ai_, a2, at_);
        id += d;
        is += a1;
        it += a2;
      }
    }
    sd = wave_sum(sd);
    ss = wave_sum(ss);
    st = wave_sum(st);
    ad_ = wave_sum(ad_);
    as_ = wave_sum(as_);
    at_ = wave_sum(at_);
    id = wave_sum(id);
    is = wave_sum(is);
    it = wave_sum(it);
    if (lane == 0) {
      const double Fd = sd + oi * (T[0] - id), Fs = ss + oi * (T[1] - is), Ft = st + oi * (T[2] - it);
      // |python_sum - F| <= 5 gamma(n+1) (sum |imp| a)   ("bound-and-verify")
      const double Ed = 5.0 * gam * (ad_ + aoi * T[0]) * 1.0000001;
      const double Es = 5.0 * gam * (as_ + aoi * T[1]) * 1.0000001;
      const double Et = 5.0 * gam * (at_ + aoi * T[2]) * 1.0000001;
      const double area = cr.fw * cr.fh;
      const double tot = (Fd * wd + Fs * ws + Ft * wt) / area;
      const double mag = fabs(wd) * (fabs(Fd) + Ed) + fabs(ws) * (fabs(Fs) + Es) + fabs(wt) * (fabs(Ft) + Et);
      const double B = ((fabs(wd) * Ed + fabs(ws) * Es + fabs(wt) * Et) * (1.0 + 16.0 * u) + 16.0 * u * mag) /
                       area * 1.01;
      s_tot[c] = tot;
      s_bnd[c] = B;
      CropScore &o = scores[D.crop0 + c];
      o.detail = Fd;
      o.saturation = Ft;
      o.skin = Fs;
      o.total = tot;
      o.bound = B;
      o.exact = 0;
    }
  }
  __syncthreads();
  // candidate set: every crop whose interval reaches the best lower bound
  if (tid == 0) {
    double best_lo = -1.0e308;
    for (int c = 0; c < D.ncrops; c++) best_lo = fmax(best_lo, s_tot[c] - s_bnd[c]);
    int k = 0;
    for (int c = 0; c < D.ncrops; c++)
      if (D.exact_all || s_tot[c] + s_bnd[c] >= best_lo) cand[k++] = c;
    ncand_s = k;
  }
  __syncthreads();
  const int ncand = ncand_s;
  const bool need_exact = D.exact_all || ncand > 1;
  if (need_exact) {
    // exact re-score: one lane per candidate, the reference's row-major order
    for (int k = tid; k < ncand; k += 256) {
      const int c = cand[k];
      const DevCrop cr = crops[D.crop0 + c];
      const double *tab = ad + cr.table;
      double skin = 0, detail = 0, sat = 0;
      for (int y = 0; y < H; y++) {
        const bool yin = y >= cr.y0 && y < cr.y0 + cr.nin_y;
        const uint32_t *mrow = maps + (int64_t)y * W;
        const int64_t trow = (int64_t)(y - cr.y0) * cr.table_w - cr.x0;
        for (int x = 0; x < W; x++) {
          const bool in = yin && x >= cr.x0 && x < cr.x0 + cr.nin_x;
          const double tv = tab[in ? trow + x : 0];
          const double imp = in ? tv : oi;
          const uint32_t m = mrow[x];
          const double det = lut[(m >> 8) & 255];
          skin = skin + lut[m & 255] * (det + sb) * imp;
          detail = detail + det * imp;
          sat = sat + lut[(m >> 16) & 255] * (det + tb) * imp;
        }
      }
      const double tot = (detail * wd + skin * ws + sat * wt) / (cr.fw * cr.fh);
      s_tot[c] = tot;
      CropScore &o = scores[D.crop0 + c];
      o.detail = detail;
      o.saturation = sat;
      o.skin = skin;
      o.total = tot;
      o.bound = 0;
      o.exact = 1;
    }
    __syncthreads();
  }
  if (tid == 0) {
    int top = cand[0];
    double best = s_tot[top];
    if (need_exact) {
      best = -9223372036854775807.0;  // -sys.maxsize; strict > keeps the first max
      for (int k = 0; k < ncand; k++) {
        const double v = s_tot[cand[k]];
        if (v > best) {
          best = v;
          top = cand[k];
        }
      }
    }
    results[D.result].top = top;
    results[D.result].n_candidates = ncand;
    results[D.result].total = best;
  }
}

// ---------------------------------------------------------------------------
// convert <out> -crop WxH+X+Y (SmartCropProcessor.php:30-34), W = w + x,
// H = h + y as smartcrop.py prints them (:372-377); CropImage clips to the
// image.  src is the resized image; per-image box from ScResult + crops.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_crop_apply(const ApplyDesc *__restrict__ descs,
                                                    const int32_t *__restrict__ prefix, int nimg,
                                                    const DevCrop *__restrict__ crops,
                                                    const ScResult *__restrict__ results) {
  const int t = blockIdx.x;
  const int i = find_image(prefix, nimg, t);
  const ApplyDesc &A = descs[i];
  const int y = t - prefix[i];
  const ScResult r = results[A.result];
  if (r.top < 0) return;
  const DevCrop c = crops[A.crop0 + r.top];
  const int gw = c.rw + c.rx, gh = c.rh + c.ry;
  const int ow = min(gw, A.W - c.rx), oh = min(gh, A.H - c.ry);
  if (y == 0 && threadIdx.x == 0) {
    A.out_wh[0] = ow;
    A.out_wh[1] = oh;
  }
  if (y >= oh) return;
  const uint8_t *s = A.src + (int64_t)(c.ry + y) * A.src_stride + (int64_t)c.rx * A.C;
  uint8_t *d = A.dst + (int64_t)y * ow * A.C;
  for (int k = threadIdx.x; k < ow * A.C; k += 256) d[k] = s[k];
}

// ---------------------------------------------------------------------------
// synthetic images (flyimg_amd/synth.py, integer-exact)
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint32_t mix32(uint32_t x) {
  x ^= x >> 16;
  x *= 0x7FEB352Du;
  x ^= x >> 15;
  x *= 0x846CA68Bu;
  x ^= x >> 16;
  return x;
}
__device__ __forceinline__ uint32_t hash4(uint32_t seed, uint32_t a, uint32_t b, uint32_t c) {
  const uint32_t s = seed * 0x9E3779B1u;
  const uint32_t tt = mix32(b * 0xC2B2AE3Du ^ c);
  const uint32_t uu = mix32(a * 0x85EBCA77u ^ tt);
  return mix32(s ^ uu);
}
__global__ __launch_bounds__(256) void k_synth(uint8_t *dst, int W, int H, int64_t stride, uint32_t seed) {
  const int64_t idx = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (idx >= (int64_t)W * H) return;
  const uint32_t x = (uint32_t)(idx % W), y = (uint32_t)(idx / W);
  const uint32_t GRID = 64, NOISE = 24, CELL = 96;
  const uint32_t gi = x / GRID, gj = y / GRID;
  const int64_t fx = x % GRID, fy = y % GRID;
  uint8_t px[3];
  for (uint32_t c = 0; c < 3; c++) {
    const int64_t g00 = hash4(seed, gi, gj, c) & 255, g10 = hash4(seed, gi + 1, gj, c) & 255;
    const int64_t g01 = hash4(seed, gi, gj + 1, c) & 255, g11 = hash4(seed, gi + 1, gj + 1, c) & 255;
    const int64_t smooth = (g00 * (GRID - fx) * (GRID - fy) + g10 * fx * (GRID - fy) + g01 * (GRID - fx) * fy +
                            g11 * fx * fy) >> 12;
    const int64_t noise = (int64_t)(hash4(seed ^ 0xA5A5A5A5u, x, y, c) % NOISE) - (int64_t)(NOISE / 2);
    int64_t v = smooth + noise;
    px[c] = (uint8_t)(v < 0 ? 0 : v > 255 ? 255 : v);
  }
  const uint32_t ci = x / CELL, cj = y / CELL;
  const uint32_t h = hash4(seed ^ 0x51D1u, ci, cj, 7);
  if ((h & 3) == 0) {
    const int64_t cx = (int64_t)(ci * CELL + 24 + ((h >> 8) & 47));
    const int64_t cy = (int64_t)(cj * CELL + 24 + ((h >> 16) & 47));
    const int64_t r = 12 + ((h >> 24) & 15);
    const int64_t dx = (int64_t)x - cx, dy = (int64_t)y - cy;
    if (dx * dx + dy * dy <= r * r) {
      const int64_t shade = (h >> 4) & 31;
      px[0] = (uint8_t)min<int64_t>(190 + shade, 255);
      px[1] = (uint8_t)min<int64_t>(135 + shade, 255);
      px[2] = (uint8_t)min<int64_t>(105 + shade, 255);
    }
  }
  uint8_t *o = dst + (int64_t)y * stride + 3 * (int64_t)x;
  o[0] = px[0];
  o[1] = px[1];
  o[2] = px[2];
}

}  // namespace fi
