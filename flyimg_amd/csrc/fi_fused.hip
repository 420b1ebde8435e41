// fi_fused.hip -- fused vertical-first resample (ImageMagick ResizeImage with
// the ThumbnailImage sample pre-step folded into the tap tables), one launch
// per batch:
//
//   source rows --(16 B/lane global_load_dwordx4, D rows in flight)-->
//   registers: K-slot ring of fp32 accumulators (one slot per output row
//   whose vertical window contains the row; weights are wave-uniform SGPRs)
//   --(row complete: Q16 round, ds_write_b128)--> LDS row buffer
//   --(horizontal taps from LDS, weights transposed in LDS)--> Q16
//   --> extent window / -colorspace Gray / -rotate epilogue --> RGB8/Gray dst.
//
// Every needed source byte crosses HBM once; the Q16 intermediate of
// VerticalFilter never leaves the CU.  Work item = (image, column strip,
// output-row band); see DESIGN.md "Fused resample kernel".
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "fi_internal.h"

namespace fi {

// Pointers fetched from descriptors are generic (flat) pointers to the
// compiler; flat loads are waited with vmcnt(0)+lgkmcnt(0) and defeat the
// row prefetch.  Force the global address space explicitly.
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) const u32x4 g_u32x4;
typedef __attribute__((address_space(1))) uint8_t g_u8;
__device__ __forceinline__ u32x4 gload16(const uint8_t *p) { return *(g_u32x4 *)(p); }

__device__ __forceinline__ uint32_t clamp_q16f(float v) {
  if (!(v > 0.0f)) return 0u;
  if (v >= 65535.0f) return 65535u;
  return (uint32_t)(v + 0.5f);
}
__device__ __forceinline__ uint8_t q16_to_u8f(uint32_t q) {
  return (uint8_t)(((q + 128u) - ((q + 128u) >> 8)) >> 8);
}
__device__ __forceinline__ void store_pixel_f(const ResizeDesc &D, int x, int y, uint32_t r, uint32_t g,
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
  g_u8 *o = (g_u8 *)(D.dst + (int64_t)dy * D.dst_stride);
  if (D.gray) {
    const double gv = 0.212656 * (double)r + 0.715158 * (double)g + 0.072186 * (double)b;
    uint32_t q;
    if (!(gv > 0.0))
      q = 0;
    else if (gv >= 65535.0)
      q = 65535;
    else
      q = (uint32_t)(gv + 0.5);
    o[dx] = q16_to_u8f(q);
  } else {
    o[dx * 3 + 0] = q16_to_u8f(r);
    o[dx * 3 + 1] = q16_to_u8f(g);
    o[dx * 3 + 2] = q16_to_u8f(b);
  }
}

__device__ __forceinline__ void unpack16(const u32x4 v, float *f) {
  const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
  for (int q = 0; q < 4; q++) {
    f[4 * q + 0] = (float)(w[q] & 255u);
    f[4 * q + 1] = (float)((w[q] >> 8) & 255u);
    f[4 * q + 2] = (float)((w[q] >> 16) & 255u);
    f[4 * q + 3] = (float)(w[q] >> 24);
  }
}

constexpr int kDepth = 4;  // source rows in flight per lane

template <int K>
__global__ __launch_bounds__(256, 2) void k_rs_fused(const ResizeDesc *__restrict__ descs,
                                                     const FusedTile *__restrict__ tiles,
                                                     const int32_t *__restrict__ ai,
                                                     const float *__restrict__ af, int lds_hw_pitch) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const FusedTile T = tiles[blockIdx.x];
  const ResizeDesc &D = descs[T.image];
  const int tid = threadIdx.x;
  const int nx = T.x1 - T.x0;
  const int maxT = D.h.maxtaps;
  const int NBp = (T.nbytes + 63) & ~63;
  float *hw = lds;                                   // [maxT][lds_hw_pitch]
  float *vrow = lds + maxT * lds_hw_pitch;           // [2][NBp]
  // ---- horizontal tap table of this strip -> LDS (transposed: conflict-free)
  const int32_t *hstart = ai + D.h.start, *hcount = ai + D.h.count, *hwoff = ai + D.h.woff;
  for (int i = tid; i < nx * maxT; i += 256) {
    const int x = i % nx, j = i / nx;
    const int gx = T.x0 + x;
    hw[j * lds_hw_pitch + x] = j < hcount[gx] ? af[hwoff[gx] + j] : 0.0f;
  }
  // per-thread output columns (at most 2 per thread: strips are <= 512 wide)
  int hb0 = 0, hn0 = 0, hb1 = 0, hn1 = 0;
  if (tid < nx) {
    hb0 = 3 * hstart[T.x0 + tid] - T.b0;
    hn0 = hcount[T.x0 + tid];
  }
  if (tid + 256 < nx) {
    hb1 = 3 * hstart[T.x0 + tid + 256] - T.b0;
    hn1 = hcount[T.x0 + tid + 256];
  }
  __syncthreads();

  // ---- vertical ring
  const bool vlane = tid * 16 < T.nbytes;
  const float *ring_w = af + D.ring_w;       // [n][K]
  const int32_t *rows = ai + D.ring_rows;    // source row per list index
  const int32_t *ringy = ai + D.ring_y;      // [n][K] owning output row or -1
  const int32_t *flush = ai + D.ring_flush;  // [n][2] output rows completing at list row i
  const uint8_t *src = D.src + T.b0 + (int64_t)tid * 16;
  float acc[K][16];
#pragma unroll
  for (int k = 0; k < K; k++)
#pragma unroll
    for (int e = 0; e < 16; e++) acc[k][e] = 0.0f;

  u32x4 pf[kDepth];
#pragma unroll
  for (int d = 0; d < kDepth; d++) {
    const int i = T.i0 + d;
    if (vlane && i < T.i1) pf[d] = gload16(src + (int64_t)rows[i] * D.src_stride);
  }
  for (int ib = T.i0; ib < T.i1; ib += kDepth) {
#pragma unroll
    for (int d = 0; d < kDepth; d++) {
      const int i = ib + d;
      if (i < T.i1) {
        float f[16];
        if (vlane) {
          unpack16(pf[d], f);
          const int inext = i + kDepth;
          if (inext < T.i1) pf[d] = gload16(src + (int64_t)rows[inext] * D.src_stride);
#pragma unroll
          for (int k = 0; k < K; k++) {
            const int yk = ringy[i * K + k];
            const float w = ring_w[i * K + k];
            if (w != 0.0f && yk >= T.y0 && yk < T.y1) {
#pragma unroll
              for (int e = 0; e < 16; e++) acc[k][e] = fmaf(w, f[e], acc[k][e]);
            }
          }
        }
        // rows of the band whose last tap is list row i
        const int ylo = max(flush[2 * i], T.y0), yhi = min(flush[2 * i + 1], T.y1);
        for (int y = ylo; y < yhi; y++) {
          float *buf = vrow + (y & 1) * NBp;
          const int ks = y % K;
#pragma unroll
          for (int k = 0; k < K; k++) {
            if (k == ks) {
              if (vlane) {
                float4 *o = reinterpret_cast<float4 *>(buf + tid * 16);
#pragma unroll
                for (int q = 0; q < 4; q++) {
                  float4 v;
                  v.x = (float)clamp_q16f(acc[k][4 * q + 0] * 257.0f);
                  v.y = (float)clamp_q16f(acc[k][4 * q + 1] * 257.0f);
                  v.z = (float)clamp_q16f(acc[k][4 * q + 2] * 257.0f);
                  v.w = (float)clamp_q16f(acc[k][4 * q + 3] * 257.0f);
                  o[q] = v;
                }
              }
#pragma unroll
              for (int e = 0; e < 16; e++) acc[k][e] = 0.0f;
            }
          }
          __syncthreads();
          // horizontal pass of output row y from the LDS row
          if (tid < nx) {
            float r = 0.f, g = 0.f, b = 0.f;
            const float *p = buf + hb0;
            for (int j = 0; j < hn0; j++) {
              const float w = hw[j * lds_hw_pitch + tid];
              r = fmaf(w, p[3 * j + 0], r);
              g = fmaf(w, p[3 * j + 1], g);
              b = fmaf(w, p[3 * j + 2], b);
            }
            store_pixel_f(D, T.x0 + tid, y, clamp_q16f(r), clamp_q16f(g), clamp_q16f(b));
          }
          if (tid + 256 < nx) {
            float r = 0.f, g = 0.f, b = 0.f;
            const float *p = buf + hb1;
            for (int j = 0; j < hn1; j++) {
              const float w = hw[j * lds_hw_pitch + tid + 256];
              r = fmaf(w, p[3 * j + 0], r);
              g = fmaf(w, p[3 * j + 1], g);
              b = fmaf(w, p[3 * j + 2], b);
            }
            store_pixel_f(D, T.x0 + tid + 256, y, clamp_q16f(r), clamp_q16f(g), clamp_q16f(b));
          }
        }
      }
    }
  }
}

int launch_fused(hipStream_t s, int K, const ResizeDesc *descs, const FusedTile *tiles, int ntiles,
                 const int32_t *ai, const float *af, int hw_pitch, int max_taps, int max_nbytes) {
  const int NBp = (max_nbytes + 63) & ~63;
  const size_t lds = (size_t)max_taps * hw_pitch * 4 + (size_t)2 * NBp * 4;
  if (lds > 160 * 1024) return -1;
  switch (K) {
    case 4:
      hipLaunchKernelGGL(k_rs_fused<4>, dim3(ntiles), dim3(256), lds, s, descs, tiles, ai, af, hw_pitch);
      break;
    case 8:
      hipLaunchKernelGGL(k_rs_fused<8>, dim3(ntiles), dim3(256), lds, s, descs, tiles, ai, af, hw_pitch);
      break;
    default:
      return -2;
  }
  return 0;
}

}  // namespace fi
