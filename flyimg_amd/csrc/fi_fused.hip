// fi_fused.hip -- fused vertical-first resample (ImageMagick ResizeImage with
// the ThumbnailImage sample pre-step folded into the tap tables), one launch
// per batch.  Work item = (image, column strip, output-row band), one
// 512-thread workgroup per item, two wave roles:
//
//   streaming waves 0-3: every touched source row of the strip is read once
//     (8 B/lane global_load_dwordx2, kDepth rows in flight per lane) into a
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
#include <stdlib.h>
#include <string.h>

#include "fi_internal.h"

namespace fi {

// Pointers fetched from descriptors are generic (flat) pointers to the
// compiler; flat loads are waited with vmcnt(0)+lgkmcnt(0).  Force global.
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) const u32x4 g_u32x4;
typedef __attribute__((address_space(1))) uint8_t g_u8;
__device__ __forceinline__ u32x4 gload16(const uint8_t *p) { return *(g_u32x4 *)(p); }
typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
typedef __attribute__((address_space(1))) const u32x2 g_u32x2;
__device__ __forceinline__ u32x2 gload8(const uint8_t *p) { return *(g_u32x2 *)(p); }

// ClampToQuantum (Q16, non-HDRI) without branches: med3 clamp, +0.5,
// truncate.  Equal to "v<=0 ? 0 : v>=65535 ? 65535 : (int)(v+0.5f)" for every
// float (NaN -> 0); result kept as a float.
__device__ __forceinline__ float clamp_q16_bf(float v) {
  return truncf(__builtin_amdgcn_fmed3f(v, 0.0f, 65535.0f) + 0.5f);
}
__device__ __forceinline__ uint8_t q16_to_u8f(uint32_t q) {  // ScaleQuantumToChar
  return (uint8_t)(((q + 128u) - ((q + 128u) >> 8)) >> 8);
}
// Epilogue constants of one image, held in registers (a reference into the
// descriptor array would be re-read after every store: the stores may alias).
struct Epi {
  uint8_t *dst;
  int64_t stride;
  int ew, eh, rot, gray;
};
__device__ __forceinline__ void store_pixel_f(const Epi &D, int x, int y, uint32_t r, uint32_t g, uint32_t b) {
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
  g_u8 *o = (g_u8 *)(D.dst + (int64_t)dy * D.stride);
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

__device__ __forceinline__ void unpack8(const u32x2 v, float *f) {
#pragma unroll
  for (int q = 0; q < 2; q++) {
    const uint32_t w = q ? v.y : v.x;
    f[4 * q + 0] = (float)(w & 255u);
    f[4 * q + 1] = (float)((w >> 8) & 255u);
    f[4 * q + 2] = (float)((w >> 16) & 255u);
    f[4 * q + 3] = (float)(w >> 24);
  }
}

// source rows in flight per streaming lane is the template parameter DEPTH
// (host pads every ring list with 32 zero-weight rows >= 2 * DEPTH)
constexpr int kLaneBytes = 8;       // source bytes per streaming lane (dwordx2)
constexpr int kStreamThreads = 256; // streaming waves 0-3 -> strips of <= 2048 bytes
constexpr int kThreads = 512;       // + epilogue waves 4-7

// MODE: 0 = production; 1 = ablation without epilogue work (barriers only);
// 2 = ablation without the vertical FMAs (loads + flushes only).  The
// ablations produce wrong pixels and exist for profiling (FI_FUSED_VARIANT).
template <int K, int DEPTH, int MODE>
__global__ __launch_bounds__(kThreads, 4) void k_rs_fused(const ResizeDesc *__restrict__ descs,
                                                          const FusedTile *__restrict__ tiles,
                                                          const int32_t *__restrict__ ai,
                                                          const float *__restrict__ af, int lds_hw_pitch) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const FusedTile T = tiles[blockIdx.x];
  const ResizeDesc &D = descs[T.image];
  const int tid = threadIdx.x;
  const int nx = T.x1 - T.x0;
  const int HT = T.htaps;
  const int NBp = (T.nbytes + 63) & ~63;
  float *hw = lds;                         // [HT][lds_hw_pitch]
  int *hs = (int *)(lds + HT * lds_hw_pitch);  // [lds_hw_pitch] window start (LDS row offset)
  float *vrow = lds + (HT + 1) * lds_hw_pitch;  // [2][NBp]
  // strip's horizontal table -> LDS (already transposed and padded by the host)
  for (int i = tid; i < nx * HT; i += kThreads) {
    const int j = i / nx, x = i - j * nx;
    hw[j * lds_hw_pitch + x] = af[T.hw + i];
  }
  for (int x = tid; x < nx; x += kThreads) hs[x] = 3 * ai[T.hstart + x] - T.b0;
  __syncthreads();

  if (tid < kStreamThreads) {
    // ------------------------------------------------------------ streaming
    const bool vlane = tid * kLaneBytes < T.nbytes;
    const float *ring_w = af + D.ring_w;       // [n + pad][K]
    const int32_t *rows = ai + D.ring_rows;    // source row per list index
    const int32_t *flush = ai + D.ring_flush;  // [n + pad][2] output rows completing at list row
    // lanes past the strip load lane 0's bytes: every load is unconditional
    const uint8_t *src = D.src + T.b0 + (vlane ? (int64_t)tid * kLaneBytes : 0);
    const int64_t sstride = D.src_stride;
    float acc[K][kLaneBytes];
#pragma unroll
    for (int k = 0; k < K; k++)
#pragma unroll
      for (int e = 0; e < kLaneBytes; e++) acc[k][e] = 0.0f;
    // The ring list is padded on the host with zero-weight rows so the
    // unrolled body runs unconditionally (a guarded body makes the number of
    // outstanding loads path dependent -> vmcnt(0) at the loop head).  Issue
    // order of the prologue must match the loop's (pf[0] oldest).
    u32x2 pf[DEPTH];
#pragma unroll
    for (int d = 0; d < DEPTH; d++) {
      pf[d] = gload8(src + (int64_t)rows[T.i0 + d] * sstride);
      __builtin_amdgcn_sched_barrier(0);
    }
    // Per-row metadata (the row to prefetch next, the K slot weights, the
    // output rows completing) is loaded ONE ROW AHEAD: scalar loads can only
    // be waited with lgkmcnt(0), so a value loaded and used in the same row
    // exposes the scalar-cache/L2 latency on every row.
    float wc[K];
#pragma unroll
    for (int k = 0; k < K; k++) wc[k] = ring_w[T.i0 * K + k];
    int rnext = rows[T.i0 + DEPTH];
    int f0 = flush[2 * T.i0], f1 = flush[2 * T.i0 + 1];
    for (int ib = T.i0; ib < T.i1; ib += DEPTH) {
#pragma unroll
      for (int d = 0; d < DEPTH; d++) {
        const int i = ib + d;
        // metadata of row i + 1
        float wn[K];
#pragma unroll
        for (int k = 0; k < K; k++) wn[k] = ring_w[(i + 1) * K + k];
        const int rn = rows[i + 1 + DEPTH];
        const int g0 = flush[2 * (i + 1)], g1 = flush[2 * (i + 1) + 1];
        float f[kLaneBytes];
        unpack8(pf[d], f);
        pf[d] = gload8(src + (int64_t)rnext * sstride);
        if (MODE != 2) {
#pragma unroll
          for (int k = 0; k < K; k++)
#pragma unroll
            for (int e = 0; e < kLaneBytes; e++) acc[k][e] = fmaf(wc[k], f[e], acc[k][e]);
        } else {
#pragma unroll
          for (int e = 0; e < kLaneBytes; e++) acc[0][e] += f[e];
        }
        for (int y = f0; y < f1; y++) {
          const int ks = y % K;
          const bool inband = y >= T.y0 && y < T.y1;
          float *buf = vrow + (y & 1) * NBp;
#pragma unroll
          for (int k = 0; k < K; k++) {
            if (k == ks) {
              if (inband && vlane) {
                float4 *o = reinterpret_cast<float4 *>(buf + tid * kLaneBytes);
#pragma unroll
                for (int q = 0; q < kLaneBytes / 4; q++) {
                  float4 v;
                  v.x = clamp_q16_bf(acc[k][4 * q + 0] * 257.0f);
                  v.y = clamp_q16_bf(acc[k][4 * q + 1] * 257.0f);
                  v.z = clamp_q16_bf(acc[k][4 * q + 2] * 257.0f);
                  v.w = clamp_q16_bf(acc[k][4 * q + 3] * 257.0f);
                  o[q] = v;
                }
              }
#pragma unroll
              for (int e = 0; e < kLaneBytes; e++) acc[k][e] = 0.0f;
            }
          }
          if (inband) __syncthreads();  // row y ready in buf[y & 1]
        }
#pragma unroll
        for (int k = 0; k < K; k++) wc[k] = wn[k];
        rnext = rn;
        f0 = g0;
        f1 = g1;
      }
    }
  } else {
    // ------------------------------------------------------------- epilogue
    const int h = tid - kStreamThreads;
    Epi E;
    E.dst = D.dst;
    E.stride = D.dst_stride;
    E.ew = D.ew;
    E.eh = D.eh;
    E.rot = D.rot;
    E.gray = D.gray;
    for (int y = T.y0; y < T.y1; y++) {
      __syncthreads();
      if (MODE == 1) continue;
      const float *buf = vrow + (y & 1) * NBp;
      for (int x = h; x < nx; x += kThreads - kStreamThreads) {
        const float *p = buf + hs[x];
        float r = 0.f, g = 0.f, b = 0.f;
#pragma unroll 4
        for (int j = 0; j < HT; j++) {
          const float w = hw[j * lds_hw_pitch + x];
          r = fmaf(w, p[3 * j + 0], r);
          g = fmaf(w, p[3 * j + 1], g);
          b = fmaf(w, p[3 * j + 2], b);
        }
        store_pixel_f(E, T.x0 + x, y, (uint32_t)clamp_q16_bf(r), (uint32_t)clamp_q16_bf(g),
                      (uint32_t)clamp_q16_bf(b));
      }
    }
  }
}

int launch_fused(hipStream_t s, int K, const ResizeDesc *descs, const FusedTile *tiles, int ntiles,
                 const int32_t *ai, const float *af, int hw_pitch, int max_taps, int max_nbytes) {
  const int NBp = (max_nbytes + 63) & ~63;
  const size_t lds = (size_t)(max_taps + 1) * hw_pitch * 4 + (size_t)2 * NBp * 4;
  if (lds > 160 * 1024) return -1;
  static const char *variant = getenv("FI_FUSED_VARIANT");  // profiling ablations only
  const int v = !variant ? 0 : !strcmp(variant, "d16") ? 1 : !strcmp(variant, "noepi") ? 2
              : !strcmp(variant, "noflops") ? 3 : 0;
#define FI_LAUNCH(KK, DD, MM) \
  hipLaunchKernelGGL((k_rs_fused<KK, DD, MM>), dim3(ntiles), dim3(kThreads), lds, s, descs, tiles, ai, af, hw_pitch)
  if (K == 4) {
    FI_LAUNCH(4, 8, 0);
  } else if (K == 8) {
    switch (v) {
      case 1: FI_LAUNCH(8, 16, 0); break;
      case 2: FI_LAUNCH(8, 8, 1); break;
      case 3: FI_LAUNCH(8, 8, 2); break;
      default: FI_LAUNCH(8, 8, 0); break;
    }
  } else {
    return -2;
  }
#undef FI_LAUNCH
  return 0;
}

}  // namespace fi
