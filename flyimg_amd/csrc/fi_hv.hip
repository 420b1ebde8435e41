// fi_hv.hip -- ImageMagick ResizeImage for horizontal-first geometries
// (resize.c: HorizontalFilter before VerticalFilter when x_factor > y_factor)
// as a streaming, exact-integer matrix-core kernel: k_rs_vm's arithmetic with
// the two passes' roles exchanged, IM's pass order and intermediate rounding
// kept (the Q16 HorizontalFilter rows are ClampToQuantum'd before the
// vertical pass reads them).
//
// One workgroup (8 waves) = (image, column strip of <= 48 output px, band of
// 16-row output blocks).  The strip's source rows stream through ONCE, top to
// bottom, in blocks of 16 (fi_plan.h HvH / HvV):
//
//   stage       16 source rows x the strip's window [px0, px0 + pp) ->
//               per-channel planes of (p - 128), row-major (items of 16 px:
//               three 16-byte loads, deinterleaved with v_perm);
//   horizontal  items (16-px output block, channel) over the waves: 3 weight
//               limbs x <= 2 k-steps of v_mfma_i32_16x16x64_i8, exact int32;
//               ClampToQuantum(257 acc / 2^22) -> the Q16 row's hi / lo bytes
//               (as value - 128) into an LDS ring of kHvRing intermediate rows;
//   vertical    as soon as the ring holds output block b's window (K0, <= 2
//               k-steps of 64 rows): 16-column tiles over the waves, B from
//               transposing ds_read_b64_tr_b8 reads of the ring, 2 data limbs
//               x 3 weight limbs, V = 256 (h - 128) + (l - 128) + 32896;
//               ClampToQuantum -> Q16 output tile;
//   epilogue    ScaleQuantumToChar / -colorspace Gray / -monochrome Q16,
//               -extent window, -rotate (k_rs_vm's store paths).
//
// Every product is exact in int32; the only roundings are the weight
// quantization (|dw| <= 2^-23) and one float conversion per pass: within
// +-1 LSB of the f64 reference and bit-reproducible.
//
// Measured (rocprofv3, cfg4 8192-image run, 1197 horizontal-first images):
// 18.7 ms vs 33.0 ms for the two-pass k_rs_h_tile + k_rs_v_final.  Tried and
// dropped: 9 waves (one per item; 96 VGPRs at 5 waves/SIMD, spills) 36 ms;
// 32-px strips 21.7 ms; next-step loads in flight across output blocks, and
// a stream of its own beside k_rs_vm: no change.  Bands of output blocks
// (host, ~8192 workgroups) took it from 24.6 to 18.7 ms.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "fi_internal.h"

namespace fi {

typedef int32_t i32x4h __attribute__((ext_vector_type(4)));
typedef int32_t i32x2h __attribute__((ext_vector_type(2)));
typedef uint32_t u32x4h __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) const i32x4h g_i32x4h;
typedef __attribute__((address_space(1))) const u32x4h g_u32x4h;
typedef __attribute__((address_space(1))) uint8_t g_u8h;
typedef __attribute__((address_space(1))) uint16_t g_u16h;
typedef __attribute__((address_space(1))) uint32_t g_u32h;
typedef __attribute__((address_space(3))) i32x2h l_i32x2h;

constexpr int kHvWaves = kHvThreads / 64;

__device__ __forceinline__ i32x4h hv_mfma(i32x4h a, i32x4h b, i32x4h c) {
  return __builtin_amdgcn_mfma_i32_16x16x64_i8(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ int32_t hv_fold3(int32_t d0, int32_t d1, int32_t d2) {  // modular limb fold
  return (int32_t)((uint32_t)d0 + ((uint32_t)d1 << 8) + ((uint32_t)d2 << 16));
}
__device__ __forceinline__ uint32_t hv_q16_to_u8(uint32_t q) {  // ScaleQuantumToChar
  return ((q + 128u) - ((q + 128u) >> 8)) >> 8;
}
__device__ __forceinline__ uint32_t hv_gray_q16(uint32_t r, uint32_t g, uint32_t b) {
  // -colorspace Gray: Rec709Luma on gamma-encoded Q16, ClampToQuantum
  const double gv = 0.212656 * (double)r + 0.715158 * (double)g + 0.072186 * (double)b;
  return !(gv > 0.0) ? 0u : (gv >= 65535.0 ? 65535u : (uint32_t)(gv + 0.5));
}

// LDS: [ring hi][ring lo] kHvRing x kHvOpitch each | planes [3][16][pp] |
//      output tile [16][kHvOtPitch] u16 | horizontal fragments [nocb][2][3][64] x 16 B
size_t hv_lds_bytes(int pp, int nocb) {
  return (size_t)2 * kHvRing * kHvOpitch + (size_t)3 * 16 * pp + (size_t)16 * kHvOtPitch * 2 +
         (size_t)nocb * 2 * 3 * 1024;
}

__global__ __launch_bounds__(kHvThreads, 4) void k_rs_hv(const HvDesc *__restrict__ descs,
                                                         const HvStripD *__restrict__ strips,
                                                         const HvTile *__restrict__ tiles,
                                                         const int32_t *__restrict__ ai) {
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  const HvTile T = tiles[blockIdx.x];
  const HvDesc D = descs[T.img];
  const HvStripD S = strips[T.strip];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int nx = S.x1 - S.x0, nb = 3 * nx, PP = S.pp;
  const int oc = D.gray ? 1 : 3;
  uint8_t *ringH = lds, *ringL = lds + kHvRing * kHvOpitch;
  uint8_t *planes = ringL + kHvRing * kHvOpitch;  // [c][16][PP]
  uint16_t *otile = reinterpret_cast<uint16_t *>(planes + 3 * 16 * PP);
  i32x4h *hbl = reinterpret_cast<i32x4h *>(planes + 3 * 16 * PP + 16 * kHvOtPitch * 2);
  {
    const g_i32x4h *hf = (const g_i32x4h *)(ai + S.frag);
    const int nf = S.nocb * 2 * 3 * 64;
    for (int i = tid; i < nf; i += kHvThreads) hbl[i] = hf[i];
  }
  const int64_t sstride = D.src_stride;

  // ---- stage 16 source rows (list k0 .. k0 + 15) as planes of p - 128: the
  // next block's three 16-byte loads per item are issued (stage_load) before
  // the current block's horizontal pass, deinterleaved and stored after it
  const int ng = PP >> 4, nitem = 16 * ng;
  const int srr = tid / ng, sg = tid - srr * ng, spx = S.px0 + 16 * sg;
  u32x4h q0, q1, q2;
  auto stage_load = [&](int k0) {
    const int k = k0 + srr;
    if (tid < nitem && k < D.nrows && spx + 16 <= D.W) {
      const uint8_t *s = D.src + (int64_t)(D.row0 + k) * sstride + 3 * spx;
      q0 = *(g_u32x4h *)(s);
      q1 = *(g_u32x4h *)(s + 16);
      q2 = *(g_u32x4h *)(s + 32);
    }
  };
  auto stage_store = [&](int k0) {
    if (tid >= nitem) return;
    const int rr = srr, g = sg;
    const int k = k0 + rr, px = spx;
    const bool rowok = k < D.nrows;
    const uint8_t *s = D.src + (int64_t)(D.row0 + min(k, D.nrows - 1)) * sstride;
    u32x4h w0, w1, w2;
    if (rowok && px + 16 <= D.W) {
      const uint32_t d[12] = {q0.x, q0.y, q0.z, q0.w, q1.x, q1.y, q1.z, q1.w, q2.x, q2.y, q2.z, q2.w};
#pragma unroll
      for (int j = 0; j < 4; j++) {
        const uint32_t a0 = d[3 * j], a1 = d[3 * j + 1], a2 = d[3 * j + 2];
        w0[j] = __builtin_amdgcn_perm(a2, __builtin_amdgcn_perm(a1, a0, 0x00060300u), 0x05020100u) ^ 0x80808080u;
        w1[j] = __builtin_amdgcn_perm(a2, __builtin_amdgcn_perm(a1, a0, 0x00070401u), 0x06020100u) ^ 0x80808080u;
        w2[j] = __builtin_amdgcn_perm(a2, __builtin_amdgcn_perm(a1, a0, 0x00000502u), 0x07040100u) ^ 0x80808080u;
      }
    } else {
#pragma unroll 1
      for (int j = 0; j < 4; j++) {
        uint32_t a = 0, b = 0, c = 0;
#pragma unroll 1
        for (int e = 0; e < 4; e++) {
          const int x = px + 4 * j + e;
          const bool ok = rowok && x < D.W;
          a |= (ok ? (uint32_t)s[3 * x] : 128u) << (8 * e);
          b |= (ok ? (uint32_t)s[3 * x + 1] : 128u) << (8 * e);
          c |= (ok ? (uint32_t)s[3 * x + 2] : 128u) << (8 * e);
        }
        w0[j] = a ^ 0x80808080u;
        w1[j] = b ^ 0x80808080u;
        w2[j] = c ^ 0x80808080u;
      }
    }
    *reinterpret_cast<u32x4h *>(planes + (0 * 16 + rr) * PP + 16 * g) = w0;
    *reinterpret_cast<u32x4h *>(planes + (1 * 16 + rr) * PP + 16 * g) = w1;
    *reinterpret_cast<u32x4h *>(planes + (2 * 16 + rr) * PP + 16 * g) = w2;
  };

  // ---- horizontal pass of the staged block -> ring rows k0 .. k0 + 15
  const int k0l = mfma_i8_k(lane, 0), k8l = mfma_i8_k(lane, 8);
  const int32_t *s0t = ai + S.s0;
  const int32_t *hw128 = ai + D.hw128 + S.x0;
  auto hpass = [&](int k0) {
#pragma unroll 1
    for (int it = wave; it < 3 * S.nocb; it += kHvWaves) {
      const int ob = it / 3, c = it - 3 * ob;
      const int w0 = s0t[2 * ob], ks = s0t[2 * ob + 1];
      i32x4h a0 = {0, 0, 0, 0}, a1 = a0, a2 = a0;
#pragma unroll
      for (int t = 0; t < 2; t++) {
        if (t >= ks) break;
        const uint8_t *base = planes + (c * 16 + (lane & 15)) * PP + w0 + 64 * t;
        const i32x2h lo = *reinterpret_cast<const i32x2h *>(base + k0l);
        const i32x2h hi = *reinterpret_cast<const i32x2h *>(base + k8l);
        const i32x4h A = {lo.x, lo.y, hi.x, hi.y};
        const i32x4h *B = hbl + (size_t)(ob * 2 + t) * 3 * 64 + lane;
        a0 = hv_mfma(A, B[0], a0);
        a1 = hv_mfma(A, B[64], a1);
        a2 = hv_mfma(A, B[128], a2);
      }
      const int x = 16 * ob + (lane & 15);
      if (x < nx) {
        const int32_t w128 = hw128[x];
#pragma unroll
        for (int i = 0; i < 4; i++) {
          // sum W p = sum W (p - 128) + 128 sum W (exact); ClampToQuantum(257 / 2^22 x)
          const int32_t tot = hv_fold3(a0[i], a1[i], a2[i]) + w128;
          const uint32_t q = __float2uint_rz(fmaf((float)tot, 257.0f / 4194304.0f, 0.5f));
          const uint32_t qc = min(q, 65535u);
          const int row = (k0 + 4 * (lane >> 4) + i) % kHvRing;
          ringH[row * kHvOpitch + 3 * x + c] = (uint8_t)((qc >> 8) ^ 0x80u);
          ringL[row * kHvOpitch + 3 * x + c] = (uint8_t)((qc & 255u) ^ 0x80u);
        }
      }
    }
  };

  // ---- epilogue: the block's Q16 tile -> destination
  auto out_byte = [&](int yl, int k) -> uint32_t {  // byte k of block row yl's segment
    const uint16_t *o = otile + yl * kHvOtPitch;
    if (!D.gray) return hv_q16_to_u8(o[k]);
    return hv_q16_to_u8(hv_gray_q16(o[3 * k], o[3 * k + 1], o[3 * k + 2]));
  };
  auto store_block = [&](int b) {
    const int rows_here = min(16, D.eh - 16 * b);
    const int nbo = nx * oc;
    if (D.gray == 2) {  // -monochrome input: Q16 gray (u16 scratch, rot = 0) for fi_mono.hip
      for (int it = tid; it < rows_here * nx; it += kHvThreads) {
        const int yl = it / nx, x = it - yl * nx;
        const uint16_t *o = otile + yl * kHvOtPitch + 3 * x;
        ((g_u16h *)(D.dst + (int64_t)(16 * b + yl) * D.dst_stride))[S.x0 + x] =
            (uint16_t)hv_gray_q16(o[0], o[1], o[2]);
      }
      return;
    }
    if (D.rot == 0) {
      // items = (row, destination dword): interior dwords as one dword store,
      // the partial first / last dword of a row byte by byte
      const int ndw = (nbo + 3) / 4 + 1;
      for (int it = tid; it < rows_here * ndw; it += kHvThreads) {
        const int yl = it / ndw, d = it - yl * ndw;
        uint8_t *a0 = D.dst + (int64_t)(16 * b + yl) * D.dst_stride + (int64_t)S.x0 * oc;
        const int kb = 4 * d - (int)((uintptr_t)a0 & 3u);  // segment byte of the dword's first byte
        if (kb >= nbo) continue;
        if (kb >= 0 && kb + 4 <= nbo) {
          const uint32_t w = out_byte(yl, kb) | (out_byte(yl, kb + 1) << 8) | (out_byte(yl, kb + 2) << 16) |
                             (out_byte(yl, kb + 3) << 24);
          *(g_u32h *)(a0 + kb) = w;
        } else {
          for (int k = max(kb, 0); k < min(kb + 4, nbo); k++) *(g_u8h *)(a0 + k) = (uint8_t)out_byte(yl, k);
        }
      }
      return;
    }
    for (int it = tid; it < rows_here * nx; it += kHvThreads) {
      const int yl = it / nx, x = it - yl * nx, y = 16 * b + yl;
      const int ox = S.x0 + x;
      int dx, dy;
      if (D.rot == 90) {
        dx = D.eh - 1 - y;
        dy = ox;
      } else if (D.rot == 180) {
        dx = D.ew - 1 - ox;
        dy = D.eh - 1 - y;
      } else {  // 270
        dx = y;
        dy = D.ew - 1 - ox;
      }
      g_u8h *out = (g_u8h *)(D.dst + (int64_t)dy * D.dst_stride) + dx * oc;
      for (int c = 0; c < oc; c++) out[c] = (uint8_t)out_byte(yl, x * oc + c);
    }
  };

  // ---- stream: produce ring rows until block b's window is in, then its vertical pass
  const int32_t *vk = ai + D.vk;
  const g_i32x4h *vfrag = (const g_i32x4h *)(ai + D.vfrag);
  const g_i32x4h *vws = (const g_i32x4h *)(ai + D.vws);
  const int rA = 16 * (lane >> 4) + ((lane & 15) >> 1);
  const int ntile = (nb + 15) >> 4;
  int produced = vk[2 * T.b0];
#pragma unroll 1
  for (int b = T.b0; b < T.b1; b++) {
    const int K0 = vk[2 * b], ks = vk[2 * b + 1];
    const int need = min(K0 + 64 * ks, D.nrows);
    // the next production step's loads are in flight during this one's
    // horizontal pass, within one output block (none live across the
    // vertical pass and epilogue)
    // the block's A fragments and row weight sums (L2 hits), in flight during production
    i32x4h A[2][3];
#pragma unroll
    for (int t = 0; t < 2; t++)
#pragma unroll
      for (int q = 0; q < 3; q++) A[t][q] = vfrag[((size_t)(b * 2 + t) * 3 + q) * 64 + lane];
    const i32x4h ws = vws[4 * b + (lane >> 4)];
    bool have = false;
#pragma unroll 1
    while (produced < need) {
      if (!have) stage_load(produced);
      __syncthreads();  // the planes' previous readers are done
      stage_store(produced);
      have = produced + 16 < need;
      if (have) stage_load(produced + 16);
      __syncthreads();
      hpass(produced);
      produced += 16;
    }
    __syncthreads();  // ring rows of the window written; the previous block's tile stored
#pragma unroll 1
    for (int j = wave; j < ntile; j += kHvWaves) {
      // one data limb at a time (hi, then lo): 12 accumulator registers live, not 24
      float fh[4];
#pragma unroll
      for (int limb = 0; limb < 2; limb++) {
        const uint8_t *ring = limb == 0 ? ringH : ringL;
        i32x4h acc[3];
#pragma unroll
        for (int q = 0; q < 3; q++) acc[q] = i32x4h{0, 0, 0, 0};
#pragma unroll
        for (int t = 0; t < 2; t++) {
          if (t >= ks) break;
          const int ra = ((K0 + 64 * t + rA) % kHvRing) * kHvOpitch + 16 * j + 8 * (lane & 1);
          const int rb = ((K0 + 64 * t + rA + 8) % kHvRing) * kHvOpitch + 16 * j + 8 * (lane & 1);
          const i32x2h v0 = __builtin_amdgcn_ds_read_tr8_b64_v2i32((l_i32x2h *)(ring + ra));
          const i32x2h v1 = __builtin_amdgcn_ds_read_tr8_b64_v2i32((l_i32x2h *)(ring + rb));
          const i32x4h B = {v0.x, v0.y, v1.x, v1.y};
#pragma unroll
          for (int q = 0; q < 3; q++) acc[q] = hv_mfma(A[t][q], B, acc[q]);
        }
        const int col = 16 * j + (lane & 15);
#pragma unroll
        for (int i = 0; i < 4; i++) {
          const float f = (float)hv_fold3(acc[0][i], acc[1][i], acc[2][i]);
          if (limb == 0) {
            fh[i] = 256.0f * f;
          } else if (col < nb) {
            // V = 256 (h - 128) + (l - 128) + 32896; ClampToQuantum
            const float tot = fh[i] + f + 32896.0f * (float)ws[i];
            const uint32_t q = min(__float2uint_rz(fmaf(tot, 1.0f / 4194304.0f, 0.5f)), 65535u);
            otile[(4 * (lane >> 4) + i) * kHvOtPitch + col] = (uint16_t)q;
          }
        }
      }
    }
    __syncthreads();
    store_block(b);
  }
}

int launch_hv(hipStream_t s, const HvDesc *descs, const HvStripD *strips, const HvTile *tiles, int ntiles,
              const int32_t *ai, size_t lds) {
  if (ntiles <= 0) return 0;
  if (lds > (size_t)kVmMaxLds) return -1;  // two workgroups per CU
  hipLaunchKernelGGL(k_rs_hv, dim3(ntiles), dim3(kHvThreads), lds, s, descs, strips, tiles, ai);
  return 0;
}

}  // namespace fi
