// fi_vm.hip -- ImageMagick ResizeImage (vertical pass first, the
// ThumbnailImage sample pre-step folded into the tap tables) as a streaming,
// exact-integer matrix-core kernel: v_mfma_i32_16x16x64_i8.
//
// One workgroup (4 waves) = (image, column strip of <= 512 source bytes,
// range of row pieces).  The touched source rows are streamed ONCE, top to
// bottom, in pieces of <= 64 rows (fi_plan.h VmV): every lane owns 8 16-byte
// loads of a piece (two full 512-byte row segments per wave-instruction);
// piece p+1 is in flight in registers while piece p is computed.
//
//   piece buffer  64 rows x 512 B in LDS (pixels as p - 128), byte c of row
//                 r at r * 528 + (c ^ 128 ((r >> 4) & 1)): the
//                 ds_read_b64_tr_b8 transposing reads of both 8-row groups
//                 of a half-wave hit disjoint banks.
//   vertical      wave w owns byte columns [128 w, 128 w + 128) = 8 tiles of
//                 16.  Per tile: B = 2 tr8 reads (64 rows x 16 columns);
//                 two accumulator slots -- the block the piece belongs to and
//                 the next one (whose window starts inside the piece) -- each
//                 3 MFMAs (weight limbs L0 + 256 L1 + 65536 L2, A fragments
//                 from the host table) folded into one int32 accumulator:
//                 acc += A0 B + ((A1 B + ((A2 B) << 8)) << 8), exact.
//   block done    ClampToQuantum(257 * acc / 2^22) -> Q16 hi/lo byte planes
//                 per channel, compacted to the touched columns, stored
//                 column-major ([column][16 rows], one dword per 4 rows) so a
//                 lane writes its 4 rows at once and the horizontal pass
//                 reads its A operand with the same transposing reads;
//   horizontal    wave = 16-px output block: 2 data limbs x 3 weight limbs x
//                 <= 2 k-steps MFMAs per channel, then ScaleQuantumToChar /
//                 -colorspace Gray -> 8-bit tile in LDS;
//   epilogue      one piece later: -extent window / -rotate byte stores.
//
// Every product is exact in int32; the only roundings are the weight
// quantization (|dw| <= 2^-23) and one float conversion per pass: results
// are within +-1 LSB of the f64 reference and bit-reproducible.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

#include "fi_internal.h"

namespace fi {

typedef int32_t i32x4 __attribute__((ext_vector_type(4)));
typedef int32_t i32x2 __attribute__((ext_vector_type(2)));
typedef uint32_t u32x4v __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) const u32x4v g_u32x4v;
typedef __attribute__((address_space(1))) const i32x4 g_i32x4;
typedef __attribute__((address_space(1))) uint8_t g_u8v;
typedef __attribute__((address_space(3))) i32x2 l_i32x2v;

__device__ __forceinline__ i32x2 vm_tr8(const uint8_t *p) {
  return __builtin_amdgcn_ds_read_tr8_b64_v2i32((l_i32x2v *)(p));
}
__device__ __forceinline__ i32x4 vm_mfma(i32x4 a, i32x4 b, i32x4 c) {
  return __builtin_amdgcn_mfma_i32_16x16x64_i8(a, b, c, 0, 0, 0);
}
// Q16 plane column ci (16 rows = 16 bytes): bit 7 of the offset flipped in odd
// 16-column groups, so the two 8-column groups of a transposing half-wave read
// (columns 16 apart) land 32 banks apart
__device__ __forceinline__ int vm_col_off(int ci) { return (ci * 16) ^ (((ci >> 4) & 1) << 7); }
__device__ __forceinline__ uint8_t vm_q16_to_u8(uint32_t q) {  // ScaleQuantumToChar
  return (uint8_t)(((q + 128u) - ((q + 128u) >> 8)) >> 8);
}
// modular int32 limb fold: the partial sums may wrap, the total fits
__device__ __forceinline__ int32_t vm_fold3(int32_t d0, int32_t d1, int32_t d2) {
  return (int32_t)((uint32_t)d0 + ((uint32_t)d1 << 8) + ((uint32_t)d2 << 16));
}

// per-workgroup phase sums of MODE 9 (read by fi_debug_vm_stamps)
constexpr int kVmStampSlots = 4096;
__device__ uint64_t g_vm_stamps[kVmStampSlots * 9];

// MODE (profiling ablations, FI_VM_VARIANT; wrong pixels): 0 production,
// 1 loads + LDS writes only, 2 no horizontal pass / epilogue, 3 no stores,
// 4 no horizontal MFMA (planes + stores kept), 9 production + per-phase
// s_memtime sums written over the first bytes of the output (tools/vm_timing.py).
template <int MODE>
__global__ __launch_bounds__(kVmThreads, 2) void k_rs_vm(const VDesc *__restrict__ descs,
                                                         const MStrip *__restrict__ strips,
                                                         const VTile *__restrict__ tiles,
                                                         const int32_t *__restrict__ ai) {
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  const VTile T = tiles[blockIdx.x];
  const VDesc D = descs[T.img];
  const MStrip S = strips[T.strip];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  // LDS: [piece buffer][Q16 planes [limb][ch][column][16 rows]][8-bit tile][horizontal fragments]
  uint8_t *vpl = lds + kVmChunkBytes;
  uint8_t *otile = vpl + kVmPlaneBytes;                                  // [16][nx * oc]
  i32x4 *hbl = reinterpret_cast<i32x4 *>(otile + kVmOtileBytes);         // [nocb][ks][3][64]
  const int oc = D.gray ? 1 : 3;
  const int nx = S.x1 - S.x0;
  const int64_t sstride = D.src_stride;

  // ---- per-lane constants -------------------------------------------------
  // Q16-plane offset (hi limb; lo = + 3 planes) of this lane's 4 rows of each of its
  // 8 tile columns (0xFFFF: column not needed)
  const int32_t *lut = ai + S.lut;
  uint32_t vcolp[4];
#pragma unroll
  for (int j = 0; j < 8; j++) {
    const int col = 128 * wave + 16 * j + (lane & 15);
    const int abs = S.b0 + min(col, S.nbytes - 1), px = abs / 3, chn = abs - 3 * px;
    const int ci = lut[px - S.lut_px0];
    const int o = (col < S.nbytes && ci >= 0) ? chn * kVmPlane + vm_col_off(ci) + 4 * (lane >> 4) : 0xFFFF;
    if (j & 1)
      vcolp[j >> 1] |= (uint32_t)o << 16;
    else
      vcolp[j >> 1] = (uint32_t)o;
  }
  // horizontal: this wave's 16-px output block (ob = wave); the strip's B
  // fragments are staged in LDS once (read back per block)
  const bool hwave = wave < S.nocb;
  const int ob = hwave ? wave : 0;
  const int hw0 = ai[S.s0 + 2 * ob], hks = ai[S.s0 + 2 * ob + 1];
  {
    const g_i32x4 *hf = (const g_i32x4 *)(ai + S.frag);
    const int nf = S.nocb * S.ks * 3 * 64;
    for (int i = tid; i < nf; i += kVmThreads) hbl[i] = hf[i];
  }
  const int hx = 16 * ob + (lane & 15);
  const float hws = 32896.0f * (float)((hwave && hx < nx) ? ai[D.hwsum + S.x0 + hx] : 0);
  // transposing reads of the A operand: column k0 + 16 (l >> 4) + (l & 15) / 2 (+8), rows 8 (l & 1)
  int hoff[2][2];
#pragma unroll
  for (int t = 0; t < 2; t++)
#pragma unroll
    for (int h = 0; h < 2; h++)
      hoff[t][h] = vm_col_off(hw0 + 64 * t + 16 * (lane >> 4) + ((lane & 15) >> 1) + 8 * h) + 8 * (lane & 1);

  // ---- piece loads: lane = (16-byte column c16, row phase rs) ---------------
  // Rows 8 i + 2 w and 8 i + 2 w + 1 of a piece are wave-uniform: their list
  // entries come in through scalar loads, so the only vector-memory traffic in
  // the loop is (A fragments, w128, source rows) in a fixed order and the
  // vmcnt waits stay exact (a data-dependent VMEM load here would make the
  // compiler wait for the whole prefetch before the first MFMA).
  const int wv = __builtin_amdgcn_readfirstlane(wave);
  const int c16 = tid & 31, rs = tid >> 5;
  const bool hi_row = (lane & 32) != 0;
  const uint8_t *sb = D.src + S.b0 + (16 * c16 < S.nbytes ? 16 * c16 : 0);
  const int32_t *rows = ai + D.rows;
  u32x4v v[8];
  // piece metadata {list start, rows, block, block completes}, one piece ahead
  typedef int32_t i32x4m __attribute__((ext_vector_type(4)));
  const i32x4m *pmeta = reinterpret_cast<const i32x4m *>(ai + D.pmeta);
  auto issue = [&](const i32x4m m) {
    const int lo = m.x, n = m.y;
#pragma unroll
    for (int i = 0; i < 8; i++) {
      const int ra = 8 * i + 2 * wv;
      const int k0 = min(lo + (ra < n ? ra : 0), D.nrows - 1), k1 = min(lo + (ra + 1 < n ? ra + 1 : 0), D.nrows - 1);
      // regular lists (rows[k] = row0 + rstep k) need no table lookups (uniform branch)
      const int r0 = D.rstep > 0 ? D.row0 + D.rstep * k0 : rows[k0];
      const int r1 = D.rstep > 0 ? D.row0 + D.rstep * k1 : rows[k1];
      const int64_t o0 = (int64_t)r0 * sstride, o1 = (int64_t)r1 * sstride;
      v[i] = *(g_u32x4v *)(sb + (hi_row ? o1 : o0));
    }
  };
  // A fragments of piece p: [slot][limb], and the w128 rows of block pblk(p) + 2
  // (w128 is padded with two zero blocks: the load is unconditional)
  const g_i32x4 *vfrag = (const g_i32x4 *)(ai + D.frag);
  const g_i32x4 *w128 = (const g_i32x4 *)(ai + D.w128) + (lane >> 4);
  auto load_a = [&](int p, int blk, i32x4 (&A)[2][3], i32x4 &w2) {
#pragma unroll
    for (int s2 = 0; s2 < 2; s2++)
#pragma unroll
      for (int q = 0; q < 3; q++) A[s2][q] = vfrag[((size_t)(2 * p + s2) * 3 + q) * 64 + lane];
    w2 = w128[4 * (blk + 2)];
  };

  // accumulators: slot 0 = block pblk(p0), slot 1 = the next block
  i32x4 acc0[8], acc1[8];
  {
    const int b0 = pmeta[T.p0].z;
    const i32x4 w0 = w128[4 * b0], w1 = w128[4 * (b0 + 1)];
#pragma unroll
    for (int j = 0; j < 8; j++) {
      acc0[j] = w0;
      acc1[j] = w1;
    }
  }
  i32x4 A[2][3], W2;
  i32x4m mc = pmeta[T.p0];
  issue(mc);

  // transposing-read offsets: lane reads rows 16 (l >> 4) + (l & 15) / 2 (+8), bytes 8 (l & 1)
  // (rows rA and rA + 8 share the 16-row group (lane >> 4): same column swizzle)
  const int rA = 16 * (lane >> 4) + ((lane & 15) >> 1);
  const int csw = 128 * (wave ^ ((lane >> 4) & 1)) + 8 * (lane & 1);
  const int offA = rA * kVmPitch + csw, offB = (rA + 8) * kVmPitch + csw;
  const int woff_st = rs * kVmPitch;  // + row 8 i and the swizzled column below

  // ---- epilogue of a completed block (run one piece later, before that
  // piece's loads are issued, so the stores never sit behind a prefetch in
  // the vmcnt queue): -extent window, -rotate, byte stores of the 8-bit tile
  // 8-bit tile rows are placed so that tile byte k of row yl sits at the same
  // offset mod 4 as its destination byte (rot 0): whole dwords go out as dword stores.
  auto row_shift = [&](int y) -> int {
    return (int)(((uintptr_t)D.dst + (uint64_t)y * (uint64_t)D.dst_stride + (uint64_t)S.x0 * oc) & 3u);
  };
  auto store_block = [&](int b) {
    const int rows_here = min(16, D.eh - 16 * b);
    const int nb = nx * oc;
    if (D.rot == 0) {
      // items = (row, destination dword): interior dwords as one dword store,
      // the partial first/last dword of a row byte by byte
      const int ndw = (nb + 3) / 4 + 1;
      const float inv = 1.0f / (float)ndw;
      const int nit = rows_here * ndw;
      for (int it0 = tid; it0 < nit; it0 += 2 * kVmThreads) {
        // two items per lane per round: both tile reads before either store
        uint32_t w[2];
        uint8_t *a[2];
        int k0[2], yl[2];
#pragma unroll
        for (int u = 0; u < 2; u++) {
          const int it = min(it0 + u * kVmThreads, nit - 1);
          yl[u] = (int)(((float)it + 0.5f) * inv);
          const int d = it - yl[u] * ndw;
          a[u] = D.dst + (int64_t)(16 * b + yl[u]) * D.dst_stride + (int64_t)S.x0 * oc;
          const int sh = (int)((uintptr_t)a[u] & 3u);
          k0[u] = 4 * d - sh;  // tile byte of the dword's first byte (tile row starts at byte sh)
          w[u] = *reinterpret_cast<const uint32_t *>(otile + yl[u] * kVmOtilePitch + min(4 * d, kVmOtilePitch - 4));
        }
#pragma unroll
        for (int u = 0; u < 2; u++) {
          if (it0 + u * kVmThreads >= nit || k0[u] >= nb) continue;
          if (k0[u] >= 0 && k0[u] + 4 <= nb) {
            *(__attribute__((address_space(1))) uint32_t *)(a[u] + k0[u]) = w[u];
          } else {
            const uint8_t *o = otile + yl[u] * kVmOtilePitch + ((uintptr_t)a[u] & 3u);
            for (int k = max(k0[u], 0); k < min(k0[u] + 4, nb); k++) *(g_u8v *)(a[u] + k) = o[k];
          }
        }
      }
      return;
    }
    for (int it = tid; it < rows_here * nx; it += kVmThreads) {
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
      g_u8v *out = (g_u8v *)(D.dst + (int64_t)dy * D.dst_stride) + dx * oc;
      const uint8_t *o = otile + yl * kVmOtilePitch + x * oc;
      for (int c = 0; c < oc; c++) out[c] = o[c];
    }
  };

  int pend = -1;  // block whose Q16 tile waits in otile for its stores
  constexpr bool kStamp = MODE == 9;
  uint64_t tsum[8] = {0, 0, 0, 0, 0, 0, 0, 0}, tprev = 0;
  auto stamp = [&](int k) {
    if (kStamp) {
      const uint64_t t = __builtin_amdgcn_s_memtime();
      tsum[k] += t - tprev;
      tprev = t;
    }
  };
  if (kStamp) tprev = __builtin_amdgcn_s_memtime();
  for (int p = T.p0; p < T.p1; p++) {
    stamp(0);  // end of the previous iteration's tail
    const i32x4m mn = pmeta[min(p + 1, T.p1 - 1)];  // scalar load, used after the piece write
    __syncthreads();  // previous piece's readers of the (aliased) buffer are done
    stamp(1);
    // piece p: registers -> LDS as signed bytes p - 128
#pragma unroll
    for (int i = 0; i < 8; i++) {
      const u32x4v x = v[i] ^ u32x4v{0x80808080u, 0x80808080u, 0x80808080u, 0x80808080u};
      // row 8 i + rs (rs < 8): its 16-row group is i >> 1, a compile-time swizzle
      *reinterpret_cast<u32x4v *>(lds + woff_st + 8 * i * kVmPitch + ((16 * c16) ^ (128 * ((i >> 1) & 1)))) = x;
    }
    stamp(2);
    if ((MODE == 0 || MODE == 4 || MODE == 9) && pend >= 0) {
      store_block(pend);
      pend = -1;
    }
    // this piece's weight fragments, then the next piece's source rows (in
    // flight during compute; the fragments are waited for with vmcnt(8))
    // (unconditional: the last piece re-issues itself, an L2 hit, so the
    // count of younger loads -- and so every vmcnt -- is the same on all paths)
    stamp(7);
    load_a(p, mc.z, A, W2);
    issue(mn);
    stamp(3);
    __syncthreads();
    stamp(4);
    const bool last = mc.w != 0;
    if (MODE != 1) {
#pragma unroll
      for (int j = 0; j < 8; j++) {
        const i32x2 lo = vm_tr8(lds + offA + 16 * j), hi = vm_tr8(lds + offB + 16 * j);
        const i32x4 B = {lo.x, lo.y, hi.x, hi.y};
        {
          const i32x4 d2 = vm_mfma(A[0][2], B, i32x4{0, 0, 0, 0});
          const i32x4 d1 = vm_mfma(A[0][1], B, d2 << 8);
          const i32x4 d0 = vm_mfma(A[0][0], B, acc0[j]);
          acc0[j] = d0 + (d1 << 8);
        }
        {
          const i32x4 d2 = vm_mfma(A[1][2], B, i32x4{0, 0, 0, 0});
          const i32x4 d1 = vm_mfma(A[1][1], B, d2 << 8);
          const i32x4 d0 = vm_mfma(A[1][0], B, acc1[j]);
          acc1[j] = d0 + (d1 << 8);
        }
      }
    }
    stamp(5);
    if (last) {
      const int b = mc.z;
      if ((MODE == 0 || MODE >= 3) && b >= T.emit0) {  // (9: production + stamps)
        // ---- block b: Q16 planes, one dword (4 rows) per limb and column
#pragma unroll
        for (int j = 0; j < 8; j++) {
          const uint32_t o = (vcolp[j >> 1] >> (16 * (j & 1))) & 0xFFFFu;
          if (o == 0xFFFFu) continue;
          uint32_t q[4];
#pragma unroll
          for (int i = 0; i < 4; i++)  // ClampToQuantum: +0.5 truncated; the conversions saturate
            q[i] = __float2uint_rz(fmaf((float)acc0[j][i], 257.0f / 4194304.0f, 0.5f));
          const auto p01 = __builtin_amdgcn_cvt_pk_u16(q[0], q[1]);
          const auto p23 = __builtin_amdgcn_cvt_pk_u16(q[2], q[3]);
          // signed limbs: (hi - 128, lo - 128)
          const uint32_t x01 = __builtin_bit_cast(uint32_t, p01) ^ 0x80808080u;
          const uint32_t x23 = __builtin_bit_cast(uint32_t, p23) ^ 0x80808080u;
          *reinterpret_cast<uint32_t *>(vpl + o) = __builtin_amdgcn_perm(x23, x01, 0x07050301u);
          *reinterpret_cast<uint32_t *>(vpl + o + 3 * kVmPlane) = __builtin_amdgcn_perm(x23, x01, 0x06040200u);
        }
        __syncthreads();
        // ---- horizontal: wave = output block ob, the three channels interleaved
        if (hwave && MODE != 4) {
          i32x4 HB[2][3];
#pragma unroll
          for (int t = 0; t < 2; t++)
#pragma unroll
            for (int q = 0; q < 3; q++)
              HB[t][q] = t < hks ? hbl[((ob * S.ks + t) * 3 + q) * 64 + lane] : i32x4{0, 0, 0, 0};
          i32x4 hh[3][3], hl[3][3];  // [channel][limb]
#pragma unroll
          for (int c = 0; c < 3; c++)
#pragma unroll
            for (int q = 0; q < 3; q++) hh[c][q] = hl[c][q] = i32x4{0, 0, 0, 0};
#pragma unroll
          for (int t = 0; t < 2; t++) {
            if (t >= hks) break;
#pragma unroll
            for (int c = 0; c < 3; c++) {
              const uint8_t *ph = vpl + c * kVmPlane, *pl = ph + 3 * kVmPlane;
              const i32x2 h0 = vm_tr8(ph + hoff[t][0]), h1 = vm_tr8(ph + hoff[t][1]);
              const i32x2 l0 = vm_tr8(pl + hoff[t][0]), l1 = vm_tr8(pl + hoff[t][1]);
              const i32x4 Ah = {h0.x, h0.y, h1.x, h1.y}, Al = {l0.x, l0.y, l1.x, l1.y};
#pragma unroll
              for (int q = 0; q < 3; q++) {
                hh[c][q] = vm_mfma(Ah, HB[t][q], hh[c][q]);
                hl[c][q] = vm_mfma(Al, HB[t][q], hl[c][q]);
              }
            }
          }
          if (hx < nx) {
#pragma unroll
            for (int i = 0; i < 4; i++) {
              uint32_t q[3];
#pragma unroll
              for (int c = 0; c < 3; c++) {
                // V = 256 (h - 128) + (l - 128) + 32896; ClampToQuantum
                const float tot = 256.0f * (float)vm_fold3(hh[c][0][i], hh[c][1][i], hh[c][2][i]) +
                                  (float)vm_fold3(hl[c][0][i], hl[c][1][i], hl[c][2][i]) + hws;
                q[c] = min(__float2uint_rz(fmaf(tot, 1.0f / 4194304.0f, 0.5f)), 65535u);
              }
              const int yl = 4 * (lane >> 4) + i;
              uint8_t *o = otile + yl * kVmOtilePitch + (D.rot == 0 ? row_shift(16 * b + yl) : 0) + hx * oc;
              if (D.gray) {  // -colorspace Gray: Rec709Luma on gamma-encoded Q16
                const double gv = 0.212656 * (double)q[0] + 0.715158 * (double)q[1] + 0.072186 * (double)q[2];
                uint32_t g;
                if (!(gv > 0.0))
                  g = 0;
                else if (gv >= 65535.0)
                  g = 65535;
                else
                  g = (uint32_t)(gv + 0.5);
                o[0] = vm_q16_to_u8(g);
              } else {
                o[0] = vm_q16_to_u8(q[0]);
                o[1] = vm_q16_to_u8(q[1]);
                o[2] = vm_q16_to_u8(q[2]);
              }
            }
          }
        }
        pend = b;  // stored at the top of the next piece (after its barrier)
        stamp(6);
      }
      if (MODE != 0 && MODE != 9) {  // ablations: keep the work alive
        uint32_t z = 0;
#pragma unroll
        for (int j = 0; j < 8; j++) z ^= (uint32_t)acc0[j][0] ^ (uint32_t)acc1[j][1];
#pragma unroll
        for (int i = 0; i < 8; i++) z ^= v[i].x ^ v[i].w;
        if (z == 0x9E3779B9u) D.dst[tid] = (uint8_t)z;
      }
      // slot 1 becomes slot 0; the new slot 1 (block b + 2) starts at its weight correction
#pragma unroll
      for (int j = 0; j < 8; j++) {
        acc0[j] = acc1[j];
        acc1[j] = W2;
      }
    }
    mc = mn;
  }
  if ((MODE == 0 || MODE == 4 || MODE == 9) && pend >= 0) {
    __syncthreads();
    store_block(pend);
  }
  if (kStamp && tid == 0 && blockIdx.x < kVmStampSlots) {
    for (int k = 0; k < 8; k++) g_vm_stamps[blockIdx.x * 9 + k] = tsum[k];
    g_vm_stamps[blockIdx.x * 9 + 8] = (uint64_t)(T.p1 - T.p0);
  }
}

int vm_read_stamps(uint64_t *out, int slots) {
  if (slots > kVmStampSlots) slots = kVmStampSlots;
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_vm_stamps), (size_t)slots * 9 * sizeof(uint64_t)) == hipSuccess ? 0 : -1;
}

// piece buffer + Q16 planes + 8-bit output tile + the strip's horizontal fragments
size_t vm_lds_bytes(int nocb, int ks) {
  return (size_t)kVmChunkBytes + kVmPlaneBytes + kVmOtileBytes + (size_t)nocb * ks * 3 * 1024;
}

int launch_vm(hipStream_t s, const VDesc *descs, const MStrip *strips, const VTile *tiles, int ntiles,
              const int32_t *ai, size_t lds) {
  if (ntiles <= 0) return 0;
  if (lds > (size_t)kVmMaxLds) return -1;  // two workgroups per CU
  static const char *variant = getenv("FI_VM_VARIANT");  // profiling ablations only
  const int v = variant ? atoi(variant) : 0;
  if (v == 1)
    hipLaunchKernelGGL((k_rs_vm<1>), dim3(ntiles), dim3(kVmThreads), lds, s, descs, strips, tiles, ai);
  else if (v == 2)
    hipLaunchKernelGGL((k_rs_vm<2>), dim3(ntiles), dim3(kVmThreads), lds, s, descs, strips, tiles, ai);
  else if (v == 3)
    hipLaunchKernelGGL((k_rs_vm<3>), dim3(ntiles), dim3(kVmThreads), lds, s, descs, strips, tiles, ai);
  else if (v == 4)
    hipLaunchKernelGGL((k_rs_vm<4>), dim3(ntiles), dim3(kVmThreads), lds, s, descs, strips, tiles, ai);
  else if (v == 9)
    hipLaunchKernelGGL((k_rs_vm<9>), dim3(ntiles), dim3(kVmThreads), lds, s, descs, strips, tiles, ai);
  else
    hipLaunchKernelGGL((k_rs_vm<0>), dim3(ntiles), dim3(kVmThreads), lds, s, descs, strips, tiles, ai);
  return 0;
}

}  // namespace fi
