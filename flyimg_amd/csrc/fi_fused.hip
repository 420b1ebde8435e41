// fi_fused.hip -- fused vertical-first resample (ImageMagick ResizeImage with
// the ThumbnailImage sample pre-step folded into the tap tables), one launch
// per batch.  Work item = (image, column strip, output-row band), one
// 512-thread workgroup per item, two wave roles:
//
//   streaming waves 0-3: every touched source row of the strip is read once
//     (16 B/lane global_load_dwordx4, kDepth rows in flight per lane) into a
//     K-slot ring of fp32 accumulators (slot = output row % K, weights are
//     wave-uniform SGPRs).  When an output row's last tap has arrived its
//     slot is rounded to Q16 (ClampToQuantum) and written to an LDS row
//     buffer (double buffered), then one s_barrier.
//   epilogue waves 4-7: per output row, the horizontal taps from LDS
//     (weights transposed in LDS), ClampToQuantum, then -extent window /
//     -colorspace Gray / -rotate and the 8-bit store.
//
// The roles are split by wave because stores count on vmcnt: in a streaming
// wave a data-dependent number of stores per row would force vmcnt(0) at
// every loop head and serialise the prefetch.  The Q16 intermediate of
// VerticalFilter never leaves the CU; every needed source byte crosses HBM
// once.  See DESIGN.md "Fused resample kernel".
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "fi_internal.h"

namespace fi {

// Pointers fetched from descriptors are generic (flat) pointers to the
// compiler; flat loads are waited with vmcnt(0)+lgkmcnt(0).  Force global.
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) const u32x4 g_u32x4;
typedef __attribute__((address_space(1))) uint8_t g_u8;
__device__ __forceinline__ u32x4 gload16(const uint8_t *p) { return *(g_u32x4 *)(p); }

// ClampToQuantum (Q16, non-HDRI) without branches: med3 clamp, +0.5,
// truncate.  Equal to "v<=0 ? 0 : v>=65535 ? 65535 : (int)(v+0.5f)" for every
// float (NaN -> 0); result kept as a float.
__device__ __forceinline__ float clamp_q16_bf(float v) {
  return truncf(__builtin_amdgcn_fmed3f(v, 0.0f, 65535.0f) + 0.5f);
}
__device__ __forceinline__ uint8_t q16_to_u8f(uint32_t q) {  // ScaleQuantumToChar
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
  if (D.gray) {  // -colorspace Gray: Rec709Luma on gamma-encoded Q16
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

constexpr int kDepth = 8;  // source rows in flight per streaming lane (host pads 2*kDepth rows)
constexpr int kStreamThreads = 256;
constexpr int kThreads = 512;

template <int K>
__global__ __launch_bounds__(kThreads, 2) void k_rs_fused(const ResizeDesc *__restrict__ descs,
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
  float *hw = lds;                          // [maxT][lds_hw_pitch]
  float *vrow = lds + maxT * lds_hw_pitch;  // [2][NBp]
  const int32_t *hstart = ai + D.h.start, *hcount = ai + D.h.count, *hwoff = ai + D.h.woff;
  // horizontal tap table of this strip -> LDS, transposed (conflict-free reads)
  for (int i = tid; i < nx * maxT; i += kThreads) {
    const int x = i % nx, j = i / nx;
    const int gx = T.x0 + x;
    hw[j * lds_hw_pitch + x] = j < hcount[gx] ? af[hwoff[gx] + j] : 0.0f;
  }
  __syncthreads();

  if (tid < kStreamThreads) {
    // ------------------------------------------------------------ streaming
    const bool vlane = tid * 16 < T.nbytes;
    const float *ring_w = af + D.ring_w;       // [n + pad][K]
    const int32_t *rows = ai + D.ring_rows;    // source row per list index
    const int32_t *flush = ai + D.ring_flush;  // [n + pad][2] output rows completing at list row
    // lanes past the strip load lane 0's bytes: every load is unconditional
    const uint8_t *src = D.src + T.b0 + (vlane ? (int64_t)tid * 16 : 0);
    const int64_t sstride = D.src_stride;
    float acc[K][16];
#pragma unroll
    for (int k = 0; k < K; k++)
#pragma unroll
      for (int e = 0; e < 16; e++) acc[k][e] = 0.0f;
    // The ring list is padded on the host with zero-weight rows so the
    // unrolled body runs unconditionally (a guarded body makes the number of
    // outstanding loads path dependent -> vmcnt(0) at the loop head).  Issue
    // order of the prologue must match the loop's (pf[0] oldest).
    u32x4 pf[kDepth];
#pragma unroll
    for (int d = 0; d < kDepth; d++) {
      pf[d] = gload16(src + (int64_t)rows[T.i0 + d] * sstride);
      __builtin_amdgcn_sched_barrier(0);
    }
    for (int ib = T.i0; ib < T.i1; ib += kDepth) {
#pragma unroll
      for (int d = 0; d < kDepth; d++) {
        const int i = ib + d;
        float f[16];
        unpack16(pf[d], f);
        pf[d] = gload16(src + (int64_t)rows[i + kDepth] * sstride);
        float w[K];
#pragma unroll
        for (int k = 0; k < K; k++) w[k] = ring_w[i * K + k];
        // slots of rows outside the band accumulate too; never written out
#pragma unroll
        for (int k = 0; k < K; k++) {
          if (w[k] != 0.0f) {
#pragma unroll
            for (int e = 0; e < 16; e++) acc[k][e] = fmaf(w[k], f[e], acc[k][e]);
          }
        }
        const int ylo = flush[2 * i], yhi = flush[2 * i + 1];
        for (int y = ylo; y < yhi; y++) {
          const int ks = y % K;
          const bool inband = y >= T.y0 && y < T.y1;
          float *buf = vrow + (y & 1) * NBp;
#pragma unroll
          for (int k = 0; k < K; k++) {
            if (k == ks) {
              if (inband && vlane) {
                float4 *o = reinterpret_cast<float4 *>(buf + tid * 16);
#pragma unroll
                for (int q = 0; q < 4; q++) {
                  float4 v;
                  v.x = clamp_q16_bf(acc[k][4 * q + 0] * 257.0f);
                  v.y = clamp_q16_bf(acc[k][4 * q + 1] * 257.0f);
                  v.z = clamp_q16_bf(acc[k][4 * q + 2] * 257.0f);
                  v.w = clamp_q16_bf(acc[k][4 * q + 3] * 257.0f);
                  o[q] = v;
                }
              }
#pragma unroll
              for (int e = 0; e < 16; e++) acc[k][e] = 0.0f;
            }
          }
          if (inband) __syncthreads();  // row y ready in buf[y & 1]
        }
      }
    }
  } else {
    // ------------------------------------------------------------- epilogue
    const int h = tid - kStreamThreads;
    int hb0 = 0, hn0 = 0, hb1 = 0, hn1 = 0;
    if (h < nx) {
      hb0 = 3 * hstart[T.x0 + h] - T.b0;
      hn0 = hcount[T.x0 + h];
    }
    if (h + 256 < nx) {
      hb1 = 3 * hstart[T.x0 + h + 256] - T.b0;
      hn1 = hcount[T.x0 + h + 256];
    }
    for (int y = T.y0; y < T.y1; y++) {
      __syncthreads();
      const float *buf = vrow + (y & 1) * NBp;
      if (h < nx) {
        float r = 0.f, g = 0.f, b = 0.f;
        const float *p = buf + hb0;
        for (int j = 0; j < hn0; j++) {
          const float w = hw[j * lds_hw_pitch + h];
          r = fmaf(w, p[3 * j + 0], r);
          g = fmaf(w, p[3 * j + 1], g);
          b = fmaf(w, p[3 * j + 2], b);
        }
        store_pixel_f(D, T.x0 + h, y, (uint32_t)clamp_q16_bf(r), (uint32_t)clamp_q16_bf(g),
                      (uint32_t)clamp_q16_bf(b));
      }
      if (h + 256 < nx) {
        float r = 0.f, g = 0.f, b = 0.f;
        const float *p = buf + hb1;
        for (int j = 0; j < hn1; j++) {
          const float w = hw[j * lds_hw_pitch + h + 256];
          r = fmaf(w, p[3 * j + 0], r);
          g = fmaf(w, p[3 * j + 1], g);
          b = fmaf(w, p[3 * j + 2], b);
        }
        store_pixel_f(D, T.x0 + h + 256, y, (uint32_t)clamp_q16_bf(r), (uint32_t)clamp_q16_bf(g),
                      (uint32_t)clamp_q16_bf(b));
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
      hipLaunchKernelGGL(k_rs_fused<4>, dim3(ntiles), dim3(kThreads), lds, s, descs, tiles, ai, af, hw_pitch);
      break;
    case 8:
      hipLaunchKernelGGL(k_rs_fused<8>, dim3(ntiles), dim3(kThreads), lds, s, descs, tiles, ai, af, hw_pitch);
      break;
    default:
      return -2;
  }
  return 0;
}

}  // namespace fi
