// fi_mfma.hip -- ImageMagick ResizeImage (vertical pass first, the
// ThumbnailImage sample pre-step folded into the tap tables) as exact
// integer matrix-core work: v_mfma_i32_16x16x64_i8.
//
// Weights are quantized to W = rint(w * 2^22) and split into three signed
// byte limbs W = L0 + 256 L1 + 65536 L2; pixels enter as p - 128.  Every
// product is exact in int32, so the only rounding is the weight quantization
// (|dw| <= 2^-23) and one float conversion per output: results are within
// the +-1 LSB contract of the fp32/f64 paths and bit-reproducible.
//
// One workgroup (4 waves) = (image, column strip <= 512 B of source bytes,
// band of 16-row output blocks, looped over; the next block's first loads
// are in flight during the current block's horizontal pass).  Per block:
//   vertical   waves take 64-byte column chunks; 64 list rows x 64 bytes are
//              loaded (global_load_dwordx4, rows from the touched-row list),
//              written to the wave's LDS tile and read back transposed with
//              ds_read_b64_tr_b8 -> B fragments (16 rows x 16 columns);
//              A = weight fragments (host tables, L2 resident).  The Q16
//              result (ClampToQuantum of 257 * sum) is written as two signed
//              byte planes per channel, compacted to the touched columns.
//   horizontal waves take (16-px output block, channel) items: A = the Q16
//              planes (16 rows x 64 columns), B = weight fragments; six MFMAs
//              per k-step (2 data bytes x 3 limbs) -> Q16 out tile in LDS.
//   epilogue   ScaleQuantumToChar, -extent window, -colorspace Gray,
//              -rotate, byte stores (store_pixel_f semantics of fi_fused.hip).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

#include "fi_internal.h"

namespace fi {

typedef int32_t i32x4 __attribute__((ext_vector_type(4)));
typedef int32_t i32x2 __attribute__((ext_vector_type(2)));
typedef uint32_t u32x4m __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) const u32x4m g_u32x4m;
typedef __attribute__((address_space(1))) uint8_t g_u8m;
typedef __attribute__((address_space(3))) i32x2 l_i32x2;

__device__ __forceinline__ float clamp_q16m(float v) {  // ClampToQuantum (Q16), branch free
  return truncf(__builtin_amdgcn_fmed3f(v, 0.0f, 65535.0f) + 0.5f);
}
__device__ __forceinline__ uint8_t q16_to_u8m(uint32_t q) {  // ScaleQuantumToChar
  return (uint8_t)(((q + 128u) - ((q + 128u) >> 8)) >> 8);
}
__device__ __forceinline__ i32x2 tr8(const uint8_t *p) {
  return __builtin_amdgcn_ds_read_tr8_b64_v2i32((l_i32x2 *)(p));
}
__device__ __forceinline__ i32x4 mfma8(i32x4 a, i32x4 b, i32x4 c) {
  return __builtin_amdgcn_mfma_i32_16x16x64_i8(a, b, c, 0, 0, 0);
}
// sum = D0 + 256 D1 + 65536 D2 in modular int32 (limb partial sums may wrap,
// the total fits)
__device__ __forceinline__ int32_t fold3(int32_t d0, int32_t d1, int32_t d2) {
  return (int32_t)((uint32_t)d0 + ((uint32_t)d1 << 8) + ((uint32_t)d2 << 16));
}

// LDS pitch of a wave's transposition tile: 72 B rows make the
// ds_read_b64_tr_b8 reads of both 16-lane groups of a half-wave hit disjoint
// banks (rows 16 apart land 32 banks apart); rows are written as two b64.
constexpr int kTilePitch = 72;

// second bound = waves per SIMD: 4 (two 8-wave workgroups per CU, <= 128 VGPRs)
// MODE (profiling ablations, FI_MFMA_VARIANT; wrong pixels): 0 production,
// 1 vertical only, 2 no vertical MFMA/fold, 3 loads only.
// Second launch bound = waves per SIMD: 3 (three 4-wave workgroups per CU,
// <= 168 VGPRs; ~41 KB of LDS each).
#ifndef FI_MFMA_WAVES_PER_SIMD
#define FI_MFMA_WAVES_PER_SIMD 3
#endif
template <int MODE>
__global__ __launch_bounds__(kMfmaThreads, FI_MFMA_WAVES_PER_SIMD) void k_rs_mfma(const MDesc *__restrict__ descs,
                                                            const MStrip *__restrict__ strips,
                                                            const MTile *__restrict__ tiles,
                                                            const int32_t *__restrict__ ai) {
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  const MTile T = tiles[blockIdx.x];
  const MDesc D = descs[T.img];
  const MStrip S = strips[T.strip];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  constexpr int kWaves = kMfmaThreads / 64;
  constexpr int P = kMfmaPitch;
  uint8_t *wtile = lds + wave * (64 * kTilePitch);              // [64 rows][72 B] per wave
  uint16_t *otile = reinterpret_cast<uint16_t *>(lds);          // [16][nx][3] Q16 (aliases the wave tiles)
  uint8_t *vpl = lds + kWaves * 64 * kTilePitch;                // [2 bytes][3 ch][16 rows][P]
  int32_t *win = reinterpret_cast<int32_t *>(vpl + 96 * P);     // [blocks][2] window start / rows
  const int nblk = T.yb1 - T.yb0;
  for (int i = tid; i < nblk; i += kMfmaThreads) {
    win[2 * i] = ai[D.ya + T.yb0 + i];
    win[2 * i + 1] = ai[D.yn + T.yb0 + i];
  }
  const int nx = S.x1 - S.x0;
  const int nchunk = (S.nbytes + 63) >> 6;  // 64-byte column chunks, <= 2 per wave (512 B strips)
  const int KS = D.ks;
  const int32_t *rows = ai + D.rows;
  const uint8_t *srcb = D.src + S.b0;
  // LDS offset of this lane's V-plane column for its (at most 2) chunks x 4 column
  // blocks: channel plane + compacted column (0xFFFF: byte not needed), packed
  // as 16-bit pairs.  Loads are unconditional: a guarded load in divergent
  // code is waited for on the spot.
  const int32_t *lut = ai + S.lut;
  int32_t ciw[2][4];
#pragma unroll
  for (int u = 0; u < 2; u++)
#pragma unroll
    for (int cb = 0; cb < 4; cb++) {
      const int col = (wave + kWaves * u) * 64 + 16 * cb + (lane & 15);
      const int abs = S.b0 + min(col, S.nbytes - 1);
      ciw[u][cb] = lut[abs / 3 - S.lut_px0];
    }
  uint32_t vcolp[4];
#pragma unroll
  for (int u = 0; u < 2; u++)
#pragma unroll
    for (int cb = 0; cb < 4; cb++) {
      const int col = (wave + kWaves * u) * 64 + 16 * cb + (lane & 15);
      const int abs = S.b0 + col, px = abs / 3, chn = abs - 3 * px;
      const int ci = ciw[u][cb];
      const int o = (col < S.nbytes && ci >= 0) ? (chn * 16 + 4 * (lane >> 4)) * P + ci : 0xFFFF;
      const int e = 4 * u + cb;
      if (e & 1)
        vcolp[e >> 1] |= (uint32_t)o << 16;
      else
        vcolp[e >> 1] = (uint32_t)o;
    }
  __syncthreads();  // win

  // Load one 64-byte chunk of block b's window (both k-steps): every lane loads
  // unconditionally (rows past the window read its first row, bytes past the
  // strip its first byte); validity bits say which values count.
  u32x4m v[2][4];
  uint32_t rvalid = 0;
  auto issue = [&](int bi, int u) {
    const int ya = win[2 * bi], yn = win[2 * bi + 1];
    const int seg = (wave + kWaves * u) * 64 + 16 * (lane & 3);
    const bool sv_ok = seg < S.nbytes;
    const uint8_t *sp = srcb + (sv_ok ? seg : 0);
    // all row indices first (one uniform branch), then the loads back to back:
    // a branch between loads would wait for every load issued before it
    int32_t rr[2][4];
    rvalid = 0;
#pragma unroll
    for (int t = 0; t < 2; t++)
#pragma unroll
      for (int i = 0; i < 4; i++) {
        const int k = 64 * t + 16 * i + (lane >> 2);
        const bool ok = sv_ok && k < yn && t < KS;
        rr[t][i] = ya + (ok ? k : 0);
        rvalid |= (ok ? 1u : 0u) << (4 * t + i);
      }
    if (D.rstep > 0) {
#pragma unroll
      for (int t = 0; t < 2; t++)
#pragma unroll
        for (int i = 0; i < 4; i++) rr[t][i] = D.row0 + D.rstep * rr[t][i];
    } else {
#pragma unroll
      for (int t = 0; t < 2; t++)
#pragma unroll
        for (int i = 0; i < 4; i++) rr[t][i] = rows[rr[t][i]];
    }
#pragma unroll
    for (int i = 0; i < 4; i++) v[0][i] = *(g_u32x4m *)(sp + (int64_t)rr[0][i] * D.src_stride);
    if (KS > 1) {
#pragma unroll
      for (int i = 0; i < 4; i++) v[1][i] = *(g_u32x4m *)(sp + (int64_t)rr[1][i] * D.src_stride);
    }
  };
  if (wave < nchunk) issue(0, 0);
  for (int bi = 0; bi < nblk; bi++) {
    const int b = T.yb0 + bi;
    int32_t w128[4];  // 128 * sum of the quantized weights of this lane's 4 output rows
#pragma unroll
    for (int i = 0; i < 4; i++) w128[i] = 128 * ai[D.vwsum + 16 * b + 4 * (lane >> 4) + i];
    const i32x4 *vf = reinterpret_cast<const i32x4 *>(ai + D.vfrag) + (size_t)b * KS * 3 * 64;
    // ------------------------------------------------------------ vertical
#pragma unroll
    for (int u = 0; u < 2; u++) {
      const int ch = wave + kWaves * u;
      if (ch >= nchunk) break;
      if (u == 1) issue(bi, 1);
      const bool last = u == 1 || ch + kWaves >= nchunk;
      if (MODE != 3) {
        i32x4 acc[4][3];
#pragma unroll
        for (int cb = 0; cb < 4; cb++)
#pragma unroll
          for (int q = 0; q < 3; q++) acc[cb][q] = i32x4{0, 0, 0, 0};
        const uint8_t *pb = wtile + (16 * (lane >> 4) + ((lane & 15) >> 1)) * kTilePitch + 8 * (lane & 1);
#pragma unroll
        for (int t = 0; t < 2; t++) {
          if (t >= KS) break;
          const i32x4 A0 = vf[(3 * t + 0) * 64 + lane], A1 = vf[(3 * t + 1) * 64 + lane],
                      A2 = vf[(3 * t + 2) * 64 + lane];
#pragma unroll
          for (int i = 0; i < 4; i++) {
            // p - 128 as signed bytes; rows/bytes outside the window contribute 0
            const u32x4m x = ((rvalid >> (4 * t + i)) & 1u)
                                 ? (v[t][i] ^ u32x4m{0x80808080u, 0x80808080u, 0x80808080u, 0x80808080u})
                                 : u32x4m{0u, 0u, 0u, 0u};
            uint8_t *w = wtile + (16 * i + (lane >> 2)) * kTilePitch + 16 * (lane & 3);
            *reinterpret_cast<i32x2 *>(w) = i32x2{(int32_t)x.x, (int32_t)x.y};
            *reinterpret_cast<i32x2 *>(w + 8) = i32x2{(int32_t)x.z, (int32_t)x.w};
          }
          if (MODE == 2) continue;
          // the wave's own LDS writes -> its transposed reads (in order per wave)
#pragma unroll
          for (int cb = 0; cb < 4; cb++) {
            const i32x2 lo = tr8(pb + 16 * cb), hi = tr8(pb + 16 * cb + 8 * kTilePitch);
            const i32x4 B = {lo.x, lo.y, hi.x, hi.y};
            acc[cb][0] = mfma8(A0, B, acc[cb][0]);
            acc[cb][1] = mfma8(A1, B, acc[cb][1]);
            acc[cb][2] = mfma8(A2, B, acc[cb][2]);
          }
        }
        if (MODE != 2) {
          // fold: rows 4 (lane >> 4) + i of the block, column from vcolp
#pragma unroll
          for (int cb = 0; cb < 4; cb++) {
            const int e = 4 * u + cb;
            const uint32_t o = (vcolp[e >> 1] >> (16 * (e & 1))) & 0xFFFFu;
            if (o == 0xFFFFu) continue;
            uint8_t *ph = vpl + o;
#pragma unroll
            for (int i = 0; i < 4; i++) {
              const int32_t sv = fold3(acc[cb][0][i], acc[cb][1][i], acc[cb][2][i]) + w128[i];
              // ClampToQuantum: the conversion saturates below 0; v + 0.5 truncated
              const uint32_t q =
                  min(__float2uint_rz(fmaf((float)sv, 257.0f / 4194304.0f, 0.5f)), 65535u) ^ 0x8080u;
              ph[i * P] = (uint8_t)(q >> 8);
              ph[i * P + 48 * P] = (uint8_t)q;
            }
          }
        }
        // the next block's first chunk is in flight during this block's
        // horizontal pass and epilogue (issued once the accumulators are dead)
        if (last && bi + 1 < nblk) issue(bi + 1, 0);
      } else {
        uint32_t z = 0;
#pragma unroll
        for (int t = 0; t < 2; t++)
#pragma unroll
          for (int i = 0; i < 4; i++) z ^= v[t][i].x ^ v[t][i].w;
        if (z == 0x12345678u) wtile[0] = 1;
        if (last && bi + 1 < nblk) issue(bi + 1, 0);
      }
    }
    __syncthreads();
    if (MODE == 1 || MODE == 3) continue;
    // ---------------------------------------------------------- horizontal
    const int32_t *hwsum = ai + D.hwsum;
    const i32x4 *hfrag = reinterpret_cast<const i32x4 *>(ai + S.frag);
    const int k0 = mfma_i8_k(lane, 0), k8 = mfma_i8_k(lane, 8);
    for (int it = wave; it < S.nocb * 3; it += kWaves) {
      const int ob = it / 3, chn = it - 3 * ob;
      const int w0 = ai[S.s0 + 2 * ob], ksob = ai[S.s0 + 2 * ob + 1];
      i32x4 hh[3], hl[3];
#pragma unroll
      for (int q = 0; q < 3; q++) hh[q] = hl[q] = i32x4{0, 0, 0, 0};
#pragma unroll
      for (int t = 0; t < 2; t++) {
        if (t >= ksob) break;
        const uint8_t *ph = vpl + (chn * 16 + (lane & 15)) * P + w0 + 64 * t;
        const uint8_t *pl = ph + 48 * P;
        const i32x2 h0 = *reinterpret_cast<const i32x2 *>(ph + k0), h1 = *reinterpret_cast<const i32x2 *>(ph + k8);
        const i32x2 l0 = *reinterpret_cast<const i32x2 *>(pl + k0), l1 = *reinterpret_cast<const i32x2 *>(pl + k8);
        const i32x4 Ah = {h0.x, h0.y, h1.x, h1.y}, Al = {l0.x, l0.y, l1.x, l1.y};
        const i32x4 *hf = hfrag + (size_t)(ob * S.ks + t) * 3 * 64;
        const i32x4 B0 = hf[lane], B1 = hf[64 + lane], B2 = hf[128 + lane];
        hh[0] = mfma8(Ah, B0, hh[0]);
        hh[1] = mfma8(Ah, B1, hh[1]);
        hh[2] = mfma8(Ah, B2, hh[2]);
        hl[0] = mfma8(Al, B0, hl[0]);
        hl[1] = mfma8(Al, B1, hl[1]);
        hl[2] = mfma8(Al, B2, hl[2]);
      }
      const int x = 16 * ob + (lane & 15);
      if (x < nx) {
        const float ws = 32896.0f * (float)hwsum[S.x0 + x];  // V = 256 (h - 128) + (l - 128) + 32896
        uint16_t *o = otile + (4 * (lane >> 4) * nx + x) * 3 + chn;
#pragma unroll
        for (int i = 0; i < 4; i++) {
          const float tot = 256.0f * (float)fold3(hh[0][i], hh[1][i], hh[2][i]) +
                            (float)fold3(hl[0][i], hl[1][i], hl[2][i]) + ws;
          o[i * nx * 3] = (uint16_t)min(__float2uint_rz(fmaf(tot, 1.0f / 4194304.0f, 0.5f)), 65535u);
        }
      }
    }
    __syncthreads();
    // ------------------------------------------------------------ epilogue
    const int rows_here = min(16, D.eh - 16 * b);
    const float inv_nx = 1.0f / (float)nx;
    for (int it = tid; it < rows_here * nx; it += kMfmaThreads) {
      const int yl = (int)(((float)it + 0.5f) * inv_nx), x = it - yl * nx, y = 16 * b + yl;
      const uint16_t *o = otile + it * 3;
      const uint32_t r = o[0], g = o[1], bl = o[2];
      const int ox = S.x0 + x;
      int dx = ox, dy = y;
      if (D.rot == 90) {
        dx = D.eh - 1 - y;
        dy = ox;
      } else if (D.rot == 180) {
        dx = D.ew - 1 - ox;
        dy = D.eh - 1 - y;
      } else if (D.rot == 270) {
        dx = y;
        dy = D.ew - 1 - ox;
      }
      g_u8m *out = (g_u8m *)(D.dst + (int64_t)dy * D.dst_stride);
      if (D.gray) {  // -colorspace Gray: Rec709Luma on gamma-encoded Q16
        const double gv = 0.212656 * (double)r + 0.715158 * (double)g + 0.072186 * (double)bl;
        uint32_t q;
        if (!(gv > 0.0))
          q = 0;
        else if (gv >= 65535.0)
          q = 65535;
        else
          q = (uint32_t)(gv + 0.5);
        out[dx] = q16_to_u8m(q);
      } else {
        out[dx * 3 + 0] = q16_to_u8m(r);
        out[dx * 3 + 1] = q16_to_u8m(g);
        out[dx * 3 + 2] = q16_to_u8m(bl);
      }
    }
    __syncthreads();
  }
}

size_t mfma_lds_bytes(int nblocks) {
  return (size_t)(kMfmaThreads / 64) * 64 * kTilePitch + (size_t)96 * kMfmaPitch + (size_t)8 * nblocks;
}

int launch_mfma(hipStream_t s, const MDesc *descs, const MStrip *strips, const MTile *tiles, int ntiles,
                const int32_t *ai, size_t lds) {
  if (ntiles <= 0) return 0;
  if (lds > 160 * 1024) return -1;
  static const char *variant = getenv("FI_MFMA_VARIANT");  // profiling ablations only
  const int v = variant ? atoi(variant) : 0;
  if (v == 1)
    hipLaunchKernelGGL((k_rs_mfma<1>), dim3(ntiles), dim3(kMfmaThreads), lds, s, descs, strips, tiles, ai);
  else if (v == 2)
    hipLaunchKernelGGL((k_rs_mfma<2>), dim3(ntiles), dim3(kMfmaThreads), lds, s, descs, strips, tiles, ai);
  else if (v == 3)
    hipLaunchKernelGGL((k_rs_mfma<3>), dim3(ntiles), dim3(kMfmaThreads), lds, s, descs, strips, tiles, ai);
  else
    hipLaunchKernelGGL((k_rs_mfma<0>), dim3(ntiles), dim3(kMfmaThreads), lds, s, descs, strips, tiles, ai);
  return 0;
}

}  // namespace fi
