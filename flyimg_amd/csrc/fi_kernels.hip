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
//   smartcrop (python/smartcrop.py:79-191):
//     k_sc_reduce / k_sc_hpass / k_sc_vpass   Pillow thumbnail (integer, exact)
//     k_sc_maps                               L, edge, skin, saturation
//     k_sc_score                              fast bounded scores + exact re-score
//   k_crop_apply   convert -crop (SmartCropProcessor.php:30-34)
//   k_synth        seeded synthetic RGB8 (flyimg_amd/synth.py)
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "fi_internal.h"
#include "fi_sc_device.h"

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
  if (D.q16out) {
    // the rotated Q16 image of the forwarded convolutions (fi_conv.hip)
    uint16_t *q = reinterpret_cast<uint16_t *>(o);
    if (D.gray) {
      const double gv = 0.212656 * (double)r + 0.715158 * (double)g + 0.072186 * (double)b;
      q[dx] = (uint16_t)clamp_q16d(gv);
    } else {
      q[dx * 3 + 0] = (uint16_t)r;
      q[dx * 3 + 1] = (uint16_t)g;
      q[dx * 3 + 2] = (uint16_t)b;
    }
  } else if (D.gray == 2) {
    // -monochrome input: the Q16 gray value itself (u16 scratch, fi_mono.hip; rot = 0)
    const double gv = 0.212656 * (double)r + 0.715158 * (double)g + 0.072186 * (double)b;
    reinterpret_cast<uint16_t *>(o)[dx] = (uint16_t)clamp_q16d(gv);
  } else if (D.gray) {
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
    const uint8_t *p0 = D.src + (int64_t)s * D.src_stride + b_lo + e;
    if (full && ((((uintptr_t)p0 | (uintptr_t)D.src_stride) & 7) == 0)) {
      for (int j0 = 0; j0 < n; j0 += 8) {
        // 8 rows' loads in flight, then accumulated in tap order (same fp32 ops)
        uint2 v[8];
        float wq[8];
#pragma unroll
        for (int u = 0; u < 8; u++) {
          const int j = min(j0 + u, n - 1);
          v[u] = *reinterpret_cast<const uint2 *>(p0 + (int64_t)j * D.src_stride);
          wq[u] = w[j];
        }
#pragma unroll
        for (int u = 0; u < 8; u++) {
          if (j0 + u < n) {
#pragma unroll
            for (int k = 0; k < 4; k++) acc[k] += wq[u] * (float)((v[u].x >> (8 * k)) & 255u);
#pragma unroll
            for (int k = 0; k < 4; k++) acc[4 + k] += wq[u] * (float)((v[u].y >> (8 * k)) & 255u);
          }
        }
      }
    } else {
      for (int j = 0; j < n; j++) {
        const uint8_t *p = p0 + (int64_t)j * D.src_stride;
        const float wj = w[j];
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
    for (int j0 = 0; j0 < n; j0 += 8) {
      // 8 taps' loads in flight, then accumulated in tap order (same fp32 ops)
      uint16_t q[8][3];
      float wq[8];
#pragma unroll
      for (int u = 0; u < 8; u++) {
        const int j = min(j0 + u, n - 1);
        q[u][0] = p[3 * j + 0];
        q[u][1] = p[3 * j + 1];
        q[u][2] = p[3 * j + 2];
        wq[u] = w[j];
      }
#pragma unroll
      for (int u = 0; u < 8; u++) {
        if (j0 + u < n) {
          r += wq[u] * (float)q[u][0];
          g += wq[u] * (float)q[u][1];
          b += wq[u] * (float)q[u][2];
        }
      }
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

// H-first, pass 1 (tiled): one workgroup = (image, kHTRows mid rows, 256
// output columns).  The source bytes the 256 columns' windows touch are staged
// in LDS for the rows with coalesced dword loads, and the columns' weights
// transposed [tap][column] (zero padded to the axis' longest window, so the
// tap loop is uniform; a zero weight adds +0.0 and changes nothing).  Each
// thread then reads a tap's weight once for all rows and a pixel's three
// bytes with one two-dword LDS read + v_alignbyte.  Same fp32 operation
// order per output as k_rs_h_u8, so the same Q16 values.
constexpr int kHTRows = 16;
__global__ __launch_bounds__(256) void k_rs_h_tile(const ResizeDesc *__restrict__ descs,
                                                   const int32_t *__restrict__ prefix, int nimg,
                                                   const int32_t *__restrict__ ai, const float *__restrict__ af,
                                                   int pitch) {
  extern __shared__ __attribute__((aligned(16))) uint8_t hl[];  // [kHTRows][pitch] bytes, then wT[taps][256]
  const int t = blockIdx.x;
  const int i = find_image(prefix, nimg, t);
  const ResizeDesc &D = descs[i];
  const int ncc = (D.ew + 255) >> 8, lt = t - prefix[i];
  const int rb = lt / ncc, cc = lt - rb * ncc;
  const int r0 = rb * kHTRows, nr = min(kHTRows, D.mid_rows - r0);
  const int x0 = cc * 256, x1 = min(D.ew, x0 + 256);
  const int s_lo = ai[D.h.start + x0];
  const int s_hi = ai[D.h.start + x1 - 1] + ai[D.h.count + x1 - 1];
  const int tid = threadIdx.x;
  const int x = x0 + tid;
  const bool valid = x < x1;
  const int taps = D.h.maxtaps;
  float *wT = reinterpret_cast<float *>(hl + kHTRows * pitch);
  int s = s_lo, n = 0;
  if (valid) {
    s = ai[D.h.start + x];
    n = ai[D.h.count + x];
    const float *w = af + ai[D.h.woff + x];
    for (int j0 = 0; j0 < taps; j0 += 8) {  // 8 weight loads in flight, then the LDS stores
      float t8[8];
#pragma unroll
      for (int u = 0; u < 8; u++) t8[u] = j0 + u < n ? w[j0 + u] : 0.0f;
#pragma unroll
      for (int u = 0; u < 8; u++)
        if (j0 + u < taps) wT[(j0 + u) * 256 + tid] = t8[u];
    }
  }
  int shr[kHTRows];
#pragma unroll
  for (int r = 0; r < kHTRows; r++) {
    const uint8_t *row = D.src + (int64_t)(D.mid_r0 + r0 + min(r, nr - 1)) * D.src_stride;
    shr[r] = (int)(((uintptr_t)row + 3 * (uintptr_t)s_lo) & 3u);
  }
  {
    // dwords wholly inside the window's bytes, then the tail bytes one by one
    // (never a byte past the window: the source may end right after it).
    // Batches of 16 loads per thread are in flight before the first LDS
    // store (a load-store pair per iteration put one HBM round trip per
    // staged dword on the critical path).
    const int ndw = (3 * (s_hi - s_lo) + 3 + 3) >> 2;
    const int total = nr * ndw;
    constexpr int kB = 16;
    for (int base = 0; base < total; base += 256 * kB) {
      uint32_t v[kB];
#pragma unroll
      for (int u = 0; u < kB; u++) {
        const int it = base + u * 256 + tid;
        v[u] = 0;
        if (it < total) {
          const int r = it / ndw, k = it - r * ndw;
          const uint8_t *row = D.src + (int64_t)(D.mid_r0 + r0 + r) * D.src_stride;
          const uintptr_t a0 = ((uintptr_t)row + 3 * (uintptr_t)s_lo) & ~(uintptr_t)3;
          const uintptr_t end = (uintptr_t)row + 3 * (uintptr_t)s_hi;
          if (a0 + 4 * (uintptr_t)k + 4 <= end) {
            v[u] = reinterpret_cast<const uint32_t *>(a0)[k];
          } else {
            for (int b = 0; b < 4; b++) {
              const uintptr_t a = a0 + 4 * (uintptr_t)k + b;
              if (a >= (uintptr_t)row + 3 * (uintptr_t)s_lo && a < end) v[u] |= (uint32_t)(*(const uint8_t *)a) << (8 * b);
            }
          }
        }
      }
#pragma unroll
      for (int u = 0; u < kB; u++) {
        const int it = base + u * 256 + tid;
        if (it < total) {
          const int r = it / ndw, k = it - r * ndw;
          reinterpret_cast<uint32_t *>(hl + r * pitch)[k] = v[u];
        }
      }
    }
  }
  __syncthreads();
  if (!valid) return;
  float acc[kHTRows][3];
#pragma unroll
  for (int r = 0; r < kHTRows; r++) acc[r][0] = acc[r][1] = acc[r][2] = 0.f;
  const int ob = 3 * (s - s_lo);
  for (int j = 0; j < taps; j++) {
    const float wj = wT[j * 256 + tid];
#pragma unroll
    for (int r = 0; r < kHTRows; r++) {
      const int o = r * pitch + shr[r] + ob + 3 * j;
      // bytes o .. o + 2 of the staged row from the two dwords around them
      const uint32_t *dw = reinterpret_cast<const uint32_t *>(hl + (o & ~3));
      const uint32_t v = __builtin_amdgcn_alignbyte(dw[1], dw[0], (uint32_t)(o & 3));
      acc[r][0] += wj * (float)(v & 255u);
      acc[r][1] += wj * (float)((v >> 8) & 255u);
      acc[r][2] += wj * (float)((v >> 16) & 255u);
    }
  }
#pragma unroll
  for (int r = 0; r < kHTRows; r++) {  // unrolled: acc stays in registers (a dynamic index spills it to scratch)
    if (r < nr) {
      uint16_t *out = D.mid + (int64_t)(r0 + r) * D.mid_stride;
      out[3 * x + 0] = (uint16_t)clamp_q16(acc[r][0] * 257.0f);
      out[3 * x + 1] = (uint16_t)clamp_q16(acc[r][1] * 257.0f);
      out[3 * x + 2] = (uint16_t)clamp_q16(acc[r][2] * 257.0f);
    }
  }
}
size_t rs_h_tile_lds(int pitch, int taps) { return (size_t)kHTRows * pitch + (size_t)taps * 256 * 4 + 16; }
int launch_rs_h_tile(hipStream_t s, const ResizeDesc *descs, const int32_t *prefix, int n, int tiles,
                     const int32_t *ai, const float *af, int pitch, int taps) {
  if (tiles <= 0) return 0;
  hipLaunchKernelGGL(k_rs_h_tile, dim3(tiles), dim3(256), rs_h_tile_lds(pitch, taps), s, descs, prefix, n, ai, af,
                     pitch);
  return 0;
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
// RGBA sources: ImageMagick's matte resample (IM 6 resize.c HorizontalFilter /
// VerticalFilter, the image->matte branch), f64 as IM's MagickRealType, f64
// tap weights (DevAxis::wd).  Q16 intermediate RGBA with the alpha channel
// (IM keeps opacity = QuantumRange - alpha: converted at each pass).  Generic
// two-pass structure as above, one workgroup per output / intermediate row.
// ---------------------------------------------------------------------------
struct Px4 {
  uint32_t c[4];
};
// One output of a matte pass: tap j at p + j * step (Q16 RGBA, or 8-bit RGBA
// scaled by 257 when U8).
template <bool U8, class T>
__device__ __forceinline__ Px4 matte_taps(const T *p, int64_t step, const double *w, int n) {
  const double qs = 1.0 / 65535.0;  // QuantumScale
  double r = 0.0, g = 0.0, b = 0.0, op = 0.0, gamma = 0.0;
  for (int j = 0; j < n; j++) {
    const T *q = p + (int64_t)j * step;
    const double k = U8 ? 257.0 : 1.0;
    const double A = k * (double)q[3];
    const double alpha = w[j] * qs * A;
    r += alpha * (k * (double)q[0]);
    g += alpha * (k * (double)q[1]);
    b += alpha * (k * (double)q[2]);
    op += w[j] * (65535.0 - A);
    gamma += alpha;
  }
  // PerceptibleReciprocal
  const double sg = gamma < 0.0 ? -1.0 : 1.0;
  gamma = (sg * gamma) >= 1.0e-12 ? 1.0 / gamma : sg / 1.0e-12;
  Px4 o;
  o.c[0] = clamp_q16d(gamma * r);
  o.c[1] = clamp_q16d(gamma * g);
  o.c[2] = clamp_q16d(gamma * b);
  o.c[3] = 65535u - clamp_q16d(op);
  return o;
}
__device__ __forceinline__ const double *axis_wd(const DevAxis &a, const int32_t *ai, const double *ad, int o) {
  return ad + a.wd + (ai[a.woff + o] - a.wbase);
}
// Epilogue of a matte image: extent pixel (x, y) -> RGBA8 or gray + alpha, rotated.
__device__ __forceinline__ void store_pixel4(const ResizeDesc &D, int x, int y, const Px4 &v) {
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
    const double gv = 0.212656 * (double)v.c[0] + 0.715158 * (double)v.c[1] + 0.072186 * (double)v.c[2];
    o[dx * 2 + 0] = q16_to_u8(clamp_q16d(gv));
    o[dx * 2 + 1] = q16_to_u8(v.c[3]);
  } else {
#pragma unroll
    for (int c = 0; c < 4; c++) o[dx * 4 + c] = q16_to_u8(v.c[c]);
  }
}
// V-first pass 1: mid[y][e] (source column mid_c0 + e) over the rows of output row y
__global__ __launch_bounds__(256) void k_rs4_v_mid(const ResizeDesc *__restrict__ descs,
                                                   const int32_t *__restrict__ prefix, int nimg,
                                                   const int32_t *__restrict__ ai, const double *__restrict__ ad) {
  const int t = blockIdx.x;
  const int i = find_image(prefix, nimg, t);
  const ResizeDesc &D = descs[i];
  const int y = t - prefix[i];
  const int s = ai[D.v.start + y], n = ai[D.v.count + y];
  const double *w = axis_wd(D.v, ai, ad, y);
  uint16_t *out = D.mid + (int64_t)y * D.mid_stride;
  for (int e = threadIdx.x; e < D.mid_cols; e += 256) {
    const Px4 v = matte_taps<true>(D.src + (int64_t)s * D.src_stride + 4 * ((int64_t)D.mid_c0 + e), D.src_stride, w, n);
#pragma unroll
    for (int c = 0; c < 4; c++) out[4 * e + c] = (uint16_t)v.c[c];
  }
}
// V-first pass 2: output row y from mid row y over the columns
__global__ __launch_bounds__(256) void k_rs4_h_final(const ResizeDesc *__restrict__ descs,
                                                     const int32_t *__restrict__ prefix, int nimg,
                                                     const int32_t *__restrict__ ai, const double *__restrict__ ad) {
  const int t = blockIdx.x;
  const int i = find_image(prefix, nimg, t);
  const ResizeDesc &D = descs[i];
  const int y = t - prefix[i];
  const uint16_t *row = D.mid + (int64_t)y * D.mid_stride;
  for (int x = threadIdx.x; x < D.ew; x += 256) {
    const int s = ai[D.h.start + x], n = ai[D.h.count + x];
    store_pixel4(D, x, y, matte_taps<false>(row + 4 * ((int64_t)s - D.mid_c0), 4, axis_wd(D.h, ai, ad, x), n));
  }
}
// H-first pass 1: mid row rr (source row mid_r0 + rr) over the columns
__global__ __launch_bounds__(256) void k_rs4_h_mid(const ResizeDesc *__restrict__ descs,
                                                   const int32_t *__restrict__ prefix, int nimg,
                                                   const int32_t *__restrict__ ai, const double *__restrict__ ad) {
  const int t = blockIdx.x;
  const int i = find_image(prefix, nimg, t);
  const ResizeDesc &D = descs[i];
  const int rr = t - prefix[i];
  const uint8_t *row = D.src + (int64_t)(D.mid_r0 + rr) * D.src_stride;
  uint16_t *out = D.mid + (int64_t)rr * D.mid_stride;
  for (int x = threadIdx.x; x < D.ew; x += 256) {
    const int s = ai[D.h.start + x], n = ai[D.h.count + x];
    const Px4 v = matte_taps<true>(row + 4 * (int64_t)s, 4, axis_wd(D.h, ai, ad, x), n);
#pragma unroll
    for (int c = 0; c < 4; c++) out[4 * x + c] = (uint16_t)v.c[c];
  }
}
// H-first pass 2: output row y over the mid rows
__global__ __launch_bounds__(256) void k_rs4_v_final(const ResizeDesc *__restrict__ descs,
                                                     const int32_t *__restrict__ prefix, int nimg,
                                                     const int32_t *__restrict__ ai, const double *__restrict__ ad) {
  const int t = blockIdx.x;
  const int i = find_image(prefix, nimg, t);
  const ResizeDesc &D = descs[i];
  const int y = t - prefix[i];
  const int s = ai[D.v.start + y], n = ai[D.v.count + y];
  const double *w = axis_wd(D.v, ai, ad, y);
  const uint16_t *col0 = D.mid + (int64_t)(s - D.mid_r0) * D.mid_stride;
  for (int x = threadIdx.x; x < D.ew; x += 256)
    store_pixel4(D, x, y, matte_taps<false>(col0 + 4 * x, D.mid_stride, w, n));
}
// No resample (ResizeImage clone): extent crop + gray + rotate of a matte image
__global__ __launch_bounds__(256) void k_rs4_copy(const ResizeDesc *__restrict__ descs,
                                                  const int32_t *__restrict__ prefix, int nimg) {
  const int t = blockIdx.x;
  const int i = find_image(prefix, nimg, t);
  const ResizeDesc &D = descs[i];
  const int y = t - prefix[i];
  const uint8_t *row = D.src + (int64_t)(D.ey0 + y) * D.src_stride + 4 * (int64_t)D.ex0;
  for (int x = threadIdx.x; x < D.ew; x += 256) {
    Px4 v;
#pragma unroll
    for (int c = 0; c < 4; c++) v.c[c] = 257u * row[4 * x + c];
    store_pixel4(D, x, y, v);
  }
}
int launch_rs4(hipStream_t s, int mode, const ResizeDesc *d1, const int32_t *p1, int n1, int tiles1,
               const ResizeDesc *d2, const int32_t *p2, int n2, int tiles2, const int32_t *ai, const double *ad) {
  if (mode == 0) {
    if (tiles1 > 0) hipLaunchKernelGGL(k_rs4_copy, dim3(tiles1), dim3(256), 0, s, d1, p1, n1);
  } else if (mode == 1) {
    if (tiles1 > 0) hipLaunchKernelGGL(k_rs4_v_mid, dim3(tiles1), dim3(256), 0, s, d1, p1, n1, ai, ad);
    if (tiles2 > 0) hipLaunchKernelGGL(k_rs4_h_final, dim3(tiles2), dim3(256), 0, s, d2, p2, n2, ai, ad);
  } else {
    if (tiles1 > 0) hipLaunchKernelGGL(k_rs4_h_mid, dim3(tiles1), dim3(256), 0, s, d1, p1, n1, ai, ad);
    if (tiles2 > 0) hipLaunchKernelGGL(k_rs4_v_final, dim3(tiles2), dim3(256), 0, s, d2, p2, n2, ai, ad);
  }
  return 0;
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
    D.maps[(int64_t)y * W + x] = sc_skin_sat(r, g, b, L, P) | (E << 8);
  }
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
