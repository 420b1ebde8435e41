// fi_smartcrop.hip -- smartcrop.py's saliency stage, one workgroup per image.
//
//   k_sc_fz       (default) Pillow thumbnail (22-bit fixed-point Lanczos,
//                 Resample.c) horizontal pass as exact-integer MFMA into an LDS
//                 ring, vertical MFMA pass, then the analyse() maps (luma,
//                 Laplacian edge, skin and saturation from the 2^24-colour
//                 table of k_sc_skinsat; smartcrop.py:94-101, 231-274) -> packed
//                 maps (skin | edge << 8 | sat << 16).
//   k_sc_hmfma + k_sc_vq  the same two passes as two kernels (H-stage rows
//                 through HBM) where k_sc_fz's LDS does not fit (reduced
//                 sources, wide analysed images).
//   k_sc_vmaps    the vertical pass + maps on the VALU, where a 16-row
//                 MFMA block's window exceeds 64 H-stage rows (prescale
//                 factors > ~3: cfg5's 400 -> 111).
//   k_sc_score2   every crop's score (smartcrop.py:300-338) + the argmax
//                 (:116-133), maps resident in LDS: fast f64 pass with a
//                 rigorous error bound, exact sequential re-score of the
//                 crops whose interval reaches the best lower bound.
//   k_crop_apply3 convert -crop of the winning box (SmartCropProcessor.php:30-34).
//
// The generic per-row kernels in fi_kernels.hip remain for geometries the
// per-image kernels do not take (no prescale, staging that does not fit LDS).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "fi_internal.h"
#include "fi_sc_device.h"

namespace fi {

constexpr int kPrepThreads = 256;


// ---- k_sc_hmfma: the same horizontal pass as exact integer MFMA.  One
// workgroup per (image, chunk of hm_rows H-stage rows).  Source rows are
// staged as three planar channels of (p - 128) in signed bytes; each wave
// takes 16-column output blocks: D = A(16 rows x 64 cols of one channel)
// x B(64 cols x 16 outputs) with v_mfma_i32_16x16x64_i8 per coefficient limb,
// then sum = D0 + 256 D1 + 65536 D2 + 2^21 + 128 sum(k) is Pillow's int32
// accumulator bit for bit (Resample.c ImagingResampleHorizontal_8bpc).
typedef int32_t i32x4 __attribute__((ext_vector_type(4)));
typedef int32_t i32x2 __attribute__((ext_vector_type(2)));

__global__ __launch_bounds__(kPrepThreads) void k_sc_hmfma(const ScDesc *__restrict__ descs,
                                                           const int32_t *__restrict__ ai) {
  extern __shared__ __attribute__((aligned(16))) uint8_t lds8[];
  const ScDesc &D = descs[blockIdx.x];
  const int R = D.hm_rows, P = D.hm_pitch, KS = D.hm_ks, nb = D.hm_nb;
  const int r0 = blockIdx.y * R;
  if (r0 >= D.hrows) return;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const bool reduced = D.fx > 1 || D.fy > 1;
  const uint8_t *src = reduced ? D.red : D.img;
  const int64_t sstride = reduced ? (int64_t)D.rw * 3 : D.stride;
  const int sC = reduced ? 3 : D.C;
  const int sW = reduced ? D.rw : D.W;
  const int aw = D.aw, hrows = D.hrows, yoff = D.ybox_first;
  const int apitch = (aw * 3 + 15) & ~15;
  const int nch = sC == 3 ? 3 : 1;
  // ---- stage rows [r0, r0 + R) as planes [c][row][P] of (p - 128); zero pad.
  // One item = 16 pixels of a row: three 16-byte loads (dword-aligned rows),
  // deinterleaved into one 16-byte LDS store per plane; row tails pad with 128.
  typedef uint32_t u32x4a __attribute__((ext_vector_type(4), aligned(4)));
  typedef uint32_t u32x4s __attribute__((ext_vector_type(4)));
  const int ng = P >> 4;  // 16-pixel groups per plane row
  const bool a4 = (((uintptr_t)src | (uintptr_t)sstride) & 3) == 0;
  // batches of 4 items per thread: all 12 loads of a batch are issued before
  // the first is consumed (one HBM round trip per batch, not per item)
  for (int base = 0; base < R * ng; base += 4 * kPrepThreads) {
    u32x4a q[4][3];
    bool fast[4];
#pragma unroll
    for (int u = 0; u < 4; u++) {
      const int it = base + u * kPrepThreads + tid;
      const int rr = it / ng, g = it - rr * ng;
      const uint8_t *s = src + (int64_t)(r0 + rr + yoff) * sstride;
      fast[u] = it < R * ng && r0 + rr < hrows && sC == 3 && a4 && 16 * g + 16 <= sW;
      if (fast[u]) {
#pragma unroll
        for (int k = 0; k < 3; k++) q[u][k] = *reinterpret_cast<const u32x4a *>(s + 48 * g + 16 * k);
      }
    }
#pragma unroll
    for (int u = 0; u < 4; u++) {
      const int it = base + u * kPrepThreads + tid;
      if (it >= R * ng) break;
      const int rr = it / ng, g = it - rr * ng;
      const bool rowok = r0 + rr < hrows;
      const uint8_t *s = src + (int64_t)(r0 + rr + yoff) * sstride;
      u32x4s w0, w1, w2;
      if (fast[u]) {
        // deinterleave 16 RGB pixels: plane dword k takes bytes 12k + {0,3,6,9}
        // (+1 / +2 for G / B) of the three source dwords 3k .. 3k + 2
        const uint32_t d[12] = {q[u][0].x, q[u][0].y, q[u][0].z, q[u][0].w, q[u][1].x, q[u][1].y,
                                q[u][1].z, q[u][1].w, q[u][2].x, q[u][2].y, q[u][2].z, q[u][2].w};
#pragma unroll
        for (int k = 0; k < 4; k++) {
          const uint32_t a0 = d[3 * k], a1 = d[3 * k + 1], a2 = d[3 * k + 2];
          w0[k] = __builtin_amdgcn_perm(a2, __builtin_amdgcn_perm(a1, a0, 0x00060300u), 0x05020100u) ^ 0x80808080u;
          w1[k] = __builtin_amdgcn_perm(a2, __builtin_amdgcn_perm(a1, a0, 0x00070401u), 0x06020100u) ^ 0x80808080u;
          w2[k] = __builtin_amdgcn_perm(a2, __builtin_amdgcn_perm(a1, a0, 0x00000502u), 0x07040100u) ^ 0x80808080u;
        }
      } else {
        for (int k = 0; k < 4; k++) {
          uint32_t a = 0, b = 0, c = 0;
          for (int j = 0; j < 4; j++) {
            const int x = 16 * g + 4 * k + j;
            const bool ok = rowok && x < sW;
            uint32_t vr, vg, vb;
            if (sC == 3) {
              vr = ok ? s[3 * x] : 128u;
              vg = ok ? s[3 * x + 1] : 128u;
              vb = ok ? s[3 * x + 2] : 128u;
            } else {
              vr = vg = vb = ok ? s[x] : 128u;
            }
            a |= vr << (8 * j);
            b |= vg << (8 * j);
            c |= vb << (8 * j);
          }
          w0[k] = a ^ 0x80808080u;
          w1[k] = b ^ 0x80808080u;
          w2[k] = c ^ 0x80808080u;
        }
      }
      *reinterpret_cast<u32x4s *>(lds8 + (0 * R + rr) * P + 16 * g) = w0;
      if (nch == 3) {
        *reinterpret_cast<u32x4s *>(lds8 + (1 * R + rr) * P + 16 * g) = w1;
        *reinterpret_cast<u32x4s *>(lds8 + (2 * R + rr) * P + 16 * g) = w2;
      }
    }
  }
  __syncthreads();
  const int32_t *hmS0 = ai + D.hmS0, *hmC = ai + D.hmC;
  const i32x4 *hmB = reinterpret_cast<const i32x4 *>(ai + D.hmB);
  const int k0 = mfma_i8_k(lane, 0), k8 = mfma_i8_k(lane, 8);
  for (int b = wave; b < nb; b += kPrepThreads / 64) {
    const int s0 = hmS0[b];
    i32x4 Bf[2][3];
#pragma unroll
    for (int t = 0; t < 2; t++)
#pragma unroll
      for (int q = 0; q < 3; q++) Bf[t][q] = t < KS ? hmB[((b * KS + t) * 3 + q) * 64 + lane] : i32x4{0, 0, 0, 0};
    const int x = 16 * b + (lane & 15);
    const int32_t cx = x < aw ? hmC[x] : 0;
    for (int c = 0; c < nch; c++) {
      for (int rb = 0; rb < R; rb += 16) {
        i32x4 acc0 = {0, 0, 0, 0}, acc1 = {0, 0, 0, 0}, acc2 = {0, 0, 0, 0};
#pragma unroll
        for (int t = 0; t < 2; t++) {
          if (t < KS) {
            const uint8_t *base = lds8 + (c * R + rb + (lane & 15)) * P + s0 + 64 * t;
            const i32x2 lo = *reinterpret_cast<const i32x2 *>(base + k0);
            const i32x2 hi = *reinterpret_cast<const i32x2 *>(base + k8);
            const i32x4 a = {lo.x, lo.y, hi.x, hi.y};
            acc0 = __builtin_amdgcn_mfma_i32_16x16x64_i8(a, Bf[t][0], acc0, 0, 0, 0);
            acc1 = __builtin_amdgcn_mfma_i32_16x16x64_i8(a, Bf[t][1], acc1, 0, 0, 0);
            acc2 = __builtin_amdgcn_mfma_i32_16x16x64_i8(a, Bf[t][2], acc2, 0, 0, 0);
          }
        }
#pragma unroll
        for (int i = 0; i < 4; i++) {
          const int row = r0 + rb + 4 * (lane >> 4) + i;
          if (x < aw && row < hrows) {
            // modular int32: the limbs' partial products may wrap, the sum fits
            const uint32_t v = (uint32_t)acc0[i] + ((uint32_t)acc1[i] << 8) + ((uint32_t)acc2[i] << 16) + (uint32_t)cx;
            const uint8_t o = pil_clip8((int32_t)v);
            uint8_t *dst = D.hbuf + (int64_t)row * apitch + 3 * x;
            if (nch == 3) {
              dst[c] = o;
            } else {
              dst[0] = dst[1] = dst[2] = o;
            }
          }
        }
      }
    }
  }
}


// ---- k_sc_vmaps: Pillow's vertical pass + analyse() maps, one workgroup per
// (image, chunk of kPrepRows output rows).  The H-stage rows the chunk and its
// one-row halo need are staged in LDS (from hbuf, or from the source when no
// horizontal pass runs), the prescaled rows [y0-1, y1+1) are computed into
// LDS, then the maps of [y0, y1) are written.
__global__ __launch_bounds__(kPrepThreads) void k_sc_vmaps(const ScDesc *__restrict__ descs,
                                                           const int32_t *__restrict__ ai, const ScParamsDev P) {
  extern __shared__ __attribute__((aligned(16))) uint8_t lds8[];
  const ScDesc &D = descs[blockIdx.x];
  const int aw = D.aw, ah = D.ah;
  const int y0 = blockIdx.y * kPrepRows;
  if (y0 >= ah) return;
  const int y1 = min(y0 + kPrepRows, ah);
  const int pa = max(0, y0 - 1), pb = min(ah, y1 + 1);
  const int tid = threadIdx.x;
  const int apitch = (aw * 3 + 15) & ~15;
  const int32_t *vb = ai + D.vb, *vk = ai + D.vk;
  const bool need_v = D.need_v;
  int lo = pa, hi = pb;
  if (need_v) {
    lo = vb[2 * pa];
    hi = 0;
    for (int y = pa; y < pb; y++) hi = max(hi, vb[2 * y] + vb[2 * y + 1]);
  }
  uint8_t *rows = lds8;                        // [hi - lo][apitch] H-stage rows
  uint8_t *prer = lds8 + (hi - lo) * apitch;   // [pb - pa][apitch] prescaled rows
  if (D.need_h) {
    const int nq = apitch >> 4;
    for (int it = tid; it < (hi - lo) * nq; it += kPrepThreads) {
      const int rr = it / nq, k = it - rr * nq;
      reinterpret_cast<uint4 *>(rows + rr * apitch)[k] =
          reinterpret_cast<const uint4 *>(D.hbuf + (int64_t)(lo + rr) * apitch)[k];
    }
  } else {
    const bool reduced = D.fx > 1 || D.fy > 1;
    const uint8_t *src = reduced ? D.red : D.img;
    const int64_t sstride = reduced ? (int64_t)D.rw * 3 : D.stride;
    const int sC = reduced ? 3 : D.C;
    for (int it = tid; it < (hi - lo) * aw; it += kPrepThreads) {
      const int rr = it / aw, x = it - rr * aw;
      const uint8_t *s = src + (int64_t)(lo + rr) * sstride + x * sC;
      uint8_t *o = rows + rr * apitch + 3 * x;
      o[0] = s[0];
      o[1] = s[sC == 3 ? 1 : 0];
      o[2] = s[sC == 3 ? 2 : 0];
    }
  }
  __syncthreads();
  for (int it = tid; it < (pb - pa) * aw; it += kPrepThreads) {
    const int yr = it / aw, x = it - yr * aw, y = pa + yr;
    uint8_t *q = prer + yr * apitch + 3 * x;
    if (need_v) {
      const int ymin = vb[2 * y], cnt = vb[2 * y + 1];
      const int32_t *k = vk + y * D.ksv;
      const uint8_t *p = rows + (ymin - lo) * apitch + 3 * x;
      int32_t s0 = 1 << 21, s1 = 1 << 21, s2 = 1 << 21;
      for (int j = 0; j < cnt; j++) {
        const int32_t kj = k[j];
        s0 += (int32_t)p[j * apitch] * kj;
        s1 += (int32_t)p[j * apitch + 1] * kj;
        s2 += (int32_t)p[j * apitch + 2] * kj;
      }
      q[0] = pil_clip8(s0);
      q[1] = pil_clip8(s1);
      q[2] = pil_clip8(s2);
    } else {
      const uint8_t *p = rows + (y - lo) * apitch + 3 * x;
      q[0] = p[0];
      q[1] = p[1];
      q[2] = p[2];
    }
  }
  __syncthreads();
  for (int it = tid; it < (y1 - y0) * aw; it += kPrepThreads) {
    const int yr = it / aw, x = it - yr * aw, y = y0 + yr;
    const uint8_t *row = prer + (y - pa) * apitch;
    const uint32_t r = row[3 * x], g = row[3 * x + 1], b = row[3 * x + 2];
    if (D.pre) {
      uint8_t *o = D.pre + ((int64_t)y * aw + x) * 3;
      o[0] = (uint8_t)r;
      o[1] = (uint8_t)g;
      o[2] = (uint8_t)b;
    }
    const uint32_t L = sc_luma(r, g, b);
    // detect_edge: ImagingFilter3x3 interior, border copies L
    uint32_t E = L;
    if (aw >= 3 && ah >= 3 && x > 0 && y > 0 && x < aw - 1 && y < ah - 1) {
      const uint8_t *up = row - apitch, *dn = row + apitch;
      const int v = 4 * (int)L - (int)sc_luma(up[3 * x], up[3 * x + 1], up[3 * x + 2]) -
                    (int)sc_luma(dn[3 * x], dn[3 * x + 1], dn[3 * x + 2]) -
                    (int)sc_luma(row[3 * x - 3], row[3 * x - 2], row[3 * x - 1]) -
                    (int)sc_luma(row[3 * x + 3], row[3 * x + 4], row[3 * x + 5]) + 1;
      E = (uint32_t)(v <= 0 ? 0 : v >= 255 ? 255 : v);
    }
    D.maps[(int64_t)y * aw + x] = sc_skin_sat(r, g, b, L, P) | (E << 8);
  }
}

// ---- k_sc_vq: Pillow's vertical pass (Resample.c ImagingResampleVertical_8bpc)
// as exact integer MFMA, fused with analyse()'s maps.  One workgroup per
// (image, chunk of kVqRows analysed rows): the chunk's 16 prescaled rows
// (with the one-row edge halo) are ONE 16-row MFMA block over a window of <= 64
// H-stage rows; N = 16 interleaved channel bytes per tile (the vertical pass
// never mixes columns).  sum = D0 + 256 D1 + 65536 D2 + C[y] is Pillow's int32
// accumulator bit for bit (pixels enter as p - 128, C = 2^21 + 128 sum k).
// Luma is computed once per prescaled pixel into LDS for the 3x3 edge filter.
typedef __attribute__((address_space(3))) i32x2 l_i32x2q;
__global__ __launch_bounds__(kPrepThreads) void k_sc_vq(const ScDesc *__restrict__ descs,
                                                        const int32_t *__restrict__ ai, const ScParamsDev P) {
  extern __shared__ __attribute__((aligned(16))) uint8_t lds8[];
  const ScDesc &D = descs[blockIdx.x];
  const int c = blockIdx.y;
  const int aw = D.aw, ah = D.ah;
  const int y0 = kVqRows * c;
  if (y0 >= ah) return;
  const int y1 = min(y0 + kVqRows, ah), pa = max(0, y0 - 1), pe = min(ah, pa + 16);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int apitch = (aw * 3 + 15) & ~15, lpitch = (aw + 3) & ~3;
  uint8_t *stg = lds8;                    // [64][apitch] H-stage rows as p - 128
  uint8_t *prer = lds8 + 64 * apitch;     // [16][apitch] prescaled rows pa..pe-1
  uint8_t *lum = prer + 16 * apitch;      // [16][lpitch] their luma
  const int k0 = ai[D.vqK0 + c], hrows = D.hrows;
  // ---- stage the window (rows past the H stage are zero-weight: any bytes)
  const int nq = apitch >> 4;
  for (int it = tid; it < 64 * nq; it += kPrepThreads) {
    const int r = it / nq, q = it - r * nq;
    const int hr = min(k0 + r, hrows - 1);
    uint4 v = reinterpret_cast<const uint4 *>(D.hbuf + (int64_t)hr * apitch)[q];
    v.x ^= 0x80808080u;
    v.y ^= 0x80808080u;
    v.z ^= 0x80808080u;
    v.w ^= 0x80808080u;
    reinterpret_cast<uint4 *>(stg + r * apitch)[q] = v;
  }
  const i32x4 *af = reinterpret_cast<const i32x4 *>(ai + D.vqA) + (size_t)c * 3 * 64;
  const i32x4 A0 = af[lane], A1 = af[64 + lane], A2 = af[128 + lane];
  int32_t cy[4];
#pragma unroll
  for (int i = 0; i < 4; i++) cy[i] = ai[D.vqC + min(pa + 4 * (lane >> 4) + i, ah - 1)];
  __syncthreads();
  // ---- vertical pass: tiles of 16 byte columns over the waves
  const int rA = 16 * (lane >> 4) + ((lane & 15) >> 1);
  const uint8_t *pA = stg + rA * apitch + 8 * (lane & 1), *pB = pA + 8 * apitch;
  const int nbytes = 3 * aw;
  for (int t = wave; t < nq; t += kPrepThreads / 64) {
    const i32x2 lo = __builtin_amdgcn_ds_read_tr8_b64_v2i32((l_i32x2q *)(pA + 16 * t));
    const i32x2 hi = __builtin_amdgcn_ds_read_tr8_b64_v2i32((l_i32x2q *)(pB + 16 * t));
    const i32x4 B = {lo.x, lo.y, hi.x, hi.y};
    const i32x4 d2 = __builtin_amdgcn_mfma_i32_16x16x64_i8(A2, B, i32x4{0, 0, 0, 0}, 0, 0, 0);
    const i32x4 d1 = __builtin_amdgcn_mfma_i32_16x16x64_i8(A1, B, d2 << 8, 0, 0, 0);
    const i32x4 d0 = __builtin_amdgcn_mfma_i32_16x16x64_i8(A0, B, i32x4{0, 0, 0, 0}, 0, 0, 0);
    const int col = 16 * t + (lane & 15);
#pragma unroll
    for (int i = 0; i < 4; i++) {
      const int m = 4 * (lane >> 4) + i;
      // modular int32: the limbs' partial products may wrap, the sum fits
      const int32_t sv = (int32_t)((uint32_t)d0[i] + ((uint32_t)d1[i] << 8) + (uint32_t)cy[i]);
      if (col < nbytes && pa + m < pe) prer[m * apitch + col] = pil_clip8(sv);
    }
  }
  __syncthreads();
  // ---- luma of every prescaled pixel (and the prescaled image when kept)
  const int nr = pe - pa;
  for (int it = tid; it < nr * aw; it += kPrepThreads) {
    const int m = it / aw, x = it - m * aw;
    const uint8_t *q = prer + m * apitch + 3 * x;
    lum[m * lpitch + x] = (uint8_t)sc_luma(q[0], q[1], q[2]);
    const int y = pa + m;
    if (D.pre && y >= y0 && y < y1) {
      uint8_t *o = D.pre + ((int64_t)y * aw + x) * 3;
      o[0] = q[0];
      o[1] = q[1];
      o[2] = q[2];
    }
  }
  __syncthreads();
  // ---- maps of the chunk's rows: detect_edge (ImagingFilter3x3 interior,
  // border copies L), skin and saturation
  for (int it = tid; it < (y1 - y0) * aw; it += kPrepThreads) {
    const int yr = it / aw, x = it - yr * aw, y = y0 + yr, m = y - pa;
    const uint8_t *lrow = lum + m * lpitch;
    const uint32_t L = lrow[x];
    uint32_t E = L;
    if (aw >= 3 && ah >= 3 && x > 0 && y > 0 && x < aw - 1 && y < ah - 1) {
      const int v = 4 * (int)L - (int)lrow[x - lpitch] - (int)lrow[x + lpitch] - (int)lrow[x - 1] - (int)lrow[x + 1] + 1;
      E = (uint32_t)(v <= 0 ? 0 : v >= 255 ? 255 : v);
    }
    const uint8_t *q = prer + m * apitch + 3 * x;
    D.maps[(int64_t)y * aw + x] = sc_skin_sat(q[0], q[1], q[2], L, P) | (E << 8);
  }
}

// ---- k_sc_fz: the whole prescale + maps of ONE image per workgroup (k_sc_hmfma
// and k_sc_vq fused; no H-stage round trip through HBM).  The image's source
// rows stream through in blocks of 16 (one MFMA row block of the horizontal
// pass); their H-stage rows (p - 128 bytes) go to an LDS ring of kFzRing rows;
// each chunk of kVqRows analysed rows runs as soon as the ring holds its
// 64-row window (k_sc_vq's vertical MFMA, luma, edge / skin / saturation).
// Two workgroups per CU overlap one's loads with the other's MFMAs.  LDS: ring kFzRing x apitch, then one region shared by the
// source planes (horizontal phase) and the prescaled rows + luma (vertical).
// Arithmetic is k_sc_hmfma's and k_sc_vq's: Pillow's int32 accumulators bit
// for bit.
constexpr int kFzRing = 80;  // a 64-row window at any 16-row block alignment
#ifndef FI_FZ_THREADS
#define FI_FZ_THREADS 512
#endif
constexpr int kFzThreads = FI_FZ_THREADS;  // 8 waves; two workgroups per CU (LDS)
#ifndef FI_FZ_ABL
#define FI_FZ_ABL 0
#endif
// profiling ablations (wrong maps): 1 no source loads, 2 no horizontal pass,
// 4 no vertical pass, 8 no luma loop, 16 no maps loop
constexpr int kFzAbl = FI_FZ_ABL;
#ifndef FI_FZ_REV
#define FI_FZ_REV 0
#endif
constexpr bool kFzRev = FI_FZ_REV;
constexpr int kFzGather = 4;                // skin/saturation table reads in flight per thread
// skin | saturation << 8 of every 24-bit colour (sc_skin_sat of the colour and
// its luma) at sc_colour_key(r, g, b): built once per parameter set, a gather replaces ~200 f64 VALU
// instructions per analysed pixel in k_sc_fz<true>; bit-identical by construction.
__global__ __launch_bounds__(256) void k_sc_skinsat(uint16_t *__restrict__ t, const ScParamsDev P) {
  const uint32_t c = blockIdx.x * 256u + threadIdx.x;  // (r << 16) | (g << 8) | b
  const uint32_t r = c >> 16, g = (c >> 8) & 255u, b = c & 255u;
  const uint32_t L = sc_luma(r, g, b);
  uint32_t v;
  if (!sc_skin_sat_est(sc_fast_params(P), r, g, b, L, v)) v = sc_skin_sat(r, g, b, L, P);
  t[sc_colour_key(r, g, b)] = (uint16_t)((v & 255u) | ((v >> 16) << 8));
}

// n / d for 0 <= n < 2^22, 0 < d < 2^12 from a float reciprocal and one
// correction each way (exact: the float quotient is within 1 of n / d)
__device__ __forceinline__ int fz_div(int n, int d, float rcp) {
  int q = (int)((float)n * rcp);
  const int r = n - q * d;
  q += r >= d ? 1 : 0;
  q -= r < 0 ? 1 : 0;
  return q;
}

template <bool LUT>
__global__ __launch_bounds__(kFzThreads, 4) void k_sc_fz(const ScDesc *__restrict__ descs,
                                                        const int32_t *__restrict__ ai, const ScParamsDev P,
                                                        const uint16_t *__restrict__ skinsat) {
  extern __shared__ __attribute__((aligned(16))) uint8_t lds8[];
  const ScDesc &D = descs[kFzRev ? gridDim.x - 1 - blockIdx.x : blockIdx.x];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int aw = D.aw, ah = D.ah, hrows = D.hrows, yoff = D.ybox_first;
  const int apitch = (aw * 3 + 15) & ~15, lpitch = (aw + 3) & ~3;
  const int PP = D.hm_pitch, KS = D.hm_ks, nb = D.hm_nb;
  const uint8_t *src = D.img;
  const int64_t sstride = D.stride;
  const int sC = D.C, sW = D.W, nch = sC == 3 ? 3 : 1;
  uint8_t *ring = lds8;                                   // [kFzRing][apitch] H-stage rows, p - 128
  uint8_t *shared = lds8 + kFzRing * apitch;              // source planes [c][16][PP] | prer + lum
  uint8_t *prer = shared, *lum = shared + 16 * apitch;    // [16][apitch] prescaled rows, [16][lpitch] luma
  typedef uint32_t u32x4a __attribute__((ext_vector_type(4), aligned(4)));
  typedef uint32_t u32x4s __attribute__((ext_vector_type(4)));
  const int ng = PP >> 4;                                 // 16-pixel groups per plane row
  const float rcp_ng = 1.0f / (float)ng;
  const int nitem = 16 * ng;                              // items of one 16-row block
  const bool a4 = (((uintptr_t)src | (uintptr_t)sstride) & 3) == 0;
  // one block of 16 source rows -> planes of (p - 128): items of 16 pixels of a
  // row, two per thread at a time (six 16-byte loads in flight, then the
  // deinterleave); RGB row tails as dword + byte loads issued together (a
  // byte-by-byte tail loop serialised ~16 load round trips per block); gray
  // or unaligned sources byte by byte
  auto stage_block = [&](int r0) {
#pragma unroll 1
    for (int base = 0; base < nitem; base += 2 * kFzThreads) {
      u32x4a q[2][3];
      bool fast[2];
      int rrs[2], gs[2];
#pragma unroll
      for (int u = 0; u < 2; u++) {
        const int it = base + u * kFzThreads + tid;
        const int rr = fz_div(it, ng, rcp_ng), g = it - rr * ng;
        rrs[u] = rr;
        gs[u] = g;
        fast[u] = it < nitem && sC == 3 && a4;
        if (fast[u]) {
          const uint8_t *s = src + (int64_t)(r0 + rr + yoff) * sstride + 48 * g;
          const int remb = r0 + rr < hrows ? 3 * (sW - 16 * g) : 0;  // the group's bytes inside the row
          if (kFzAbl & 1) {  // profiling ablation: no source loads
#pragma unroll
            for (int k = 0; k < 3; k++) q[u][k] = u32x4a{(uint32_t)it, (uint32_t)r0, (uint32_t)k, (uint32_t)g};
          } else if (remb >= 48) {
#pragma unroll
            for (int k = 0; k < 3; k++) q[u][k] = *reinterpret_cast<const u32x4a *>(s + 16 * k);
          } else {
            // row tail (or a row / group past the source): whole dwords, then
            // the last bytes, all loads in flight together; pixels past the
            // row read as 128 like the plane padding
            uint32_t d[12];
#pragma unroll
            for (int k = 0; k < 12; k++) {
              if (4 * k + 4 <= remb) {
                d[k] = *reinterpret_cast<const uint32_t *>(s + 4 * k);
              } else {
                uint32_t v = 0x80808080u;
#pragma unroll
                for (int j = 0; j < 3; j++)
                  if (4 * k + j < remb) v = (v & ~(0xFFu << (8 * j))) | ((uint32_t)s[4 * k + j] << (8 * j));
                d[k] = v;
              }
            }
#pragma unroll
            for (int k = 0; k < 3; k++) q[u][k] = u32x4a{d[4 * k], d[4 * k + 1], d[4 * k + 2], d[4 * k + 3]};
          }
        }
      }
#pragma unroll
      for (int u = 0; u < 2; u++) {
        const int it = base + u * kFzThreads + tid;
        if (it >= nitem) break;
        const int rr = rrs[u], g = gs[u];
        const bool rowok = r0 + rr < hrows;
        const uint8_t *s = src + (int64_t)(r0 + rr + yoff) * sstride;
        u32x4s w0, w1, w2;
        if (fast[u]) {
          const uint32_t d[12] = {q[u][0].x, q[u][0].y, q[u][0].z, q[u][0].w, q[u][1].x, q[u][1].y,
                                  q[u][1].z, q[u][1].w, q[u][2].x, q[u][2].y, q[u][2].z, q[u][2].w};
#pragma unroll
          for (int k = 0; k < 4; k++) {
            const uint32_t a0 = d[3 * k], a1 = d[3 * k + 1], a2 = d[3 * k + 2];
            w0[k] = __builtin_amdgcn_perm(a2, __builtin_amdgcn_perm(a1, a0, 0x00060300u), 0x05020100u) ^ 0x80808080u;
            w1[k] = __builtin_amdgcn_perm(a2, __builtin_amdgcn_perm(a1, a0, 0x00070401u), 0x06020100u) ^ 0x80808080u;
            w2[k] = __builtin_amdgcn_perm(a2, __builtin_amdgcn_perm(a1, a0, 0x00000502u), 0x07040100u) ^ 0x80808080u;
          }
        } else {
#pragma unroll 1
          for (int k = 0; k < 4; k++) {
            uint32_t a = 0, b = 0, c = 0;
#pragma unroll 1
            for (int j = 0; j < 4; j++) {
              const int x = 16 * g + 4 * k + j;
              const bool ok = rowok && x < sW;
              uint32_t vr, vg, vb;
              if (sC == 3) {
                vr = ok ? s[3 * x] : 128u;
                vg = ok ? s[3 * x + 1] : 128u;
                vb = ok ? s[3 * x + 2] : 128u;
              } else {
                vr = vg = vb = ok ? s[x] : 128u;
              }
              a |= vr << (8 * j);
              b |= vg << (8 * j);
              c |= vb << (8 * j);
            }
            w0[k] = a ^ 0x80808080u;
            w1[k] = b ^ 0x80808080u;
            w2[k] = c ^ 0x80808080u;
          }
        }
        *reinterpret_cast<u32x4s *>(shared + (0 * 16 + rr) * PP + 16 * g) = w0;
        if (nch == 3) {
          *reinterpret_cast<u32x4s *>(shared + (1 * 16 + rr) * PP + 16 * g) = w1;
          *reinterpret_cast<u32x4s *>(shared + (2 * 16 + rr) * PP + 16 * g) = w2;
        }
      }
    }
  };
  const int32_t *hmS0 = ai + D.hmS0, *hmC = ai + D.hmC;
  const i32x4 *hmB = reinterpret_cast<const i32x4 *>(ai + D.hmB);
  const int k0l = mfma_i8_k(lane, 0), k8l = mfma_i8_k(lane, 8);
  auto hpass = [&](int r0) {  // the staged block -> H-stage rows r0 .. r0 + 15 into the ring
    // a wave's two column blocks (b, b + 8) per pass: both blocks' weight
    // fragments are loaded before the first block's MFMAs, so the second
    // block's load latency hides behind the first block's work
    constexpr int kW = kFzThreads / 64;
    if (kFzAbl & 2) return;
#pragma unroll 1
    for (int bp = wave; bp < nb; bp += 2 * kW) {
      i32x4 Bfs[2][2][3];
      int s0s[2];
      int32_t cxs[2];
#pragma unroll
      for (int h = 0; h < 2; h++) {
        const int b = bp + h * kW;
        if (b < nb) {
          s0s[h] = hmS0[b];
#pragma unroll
          for (int t = 0; t < 2; t++)
#pragma unroll
            for (int qq = 0; qq < 3; qq++)
              Bfs[h][t][qq] = t < KS ? hmB[((b * KS + t) * 3 + qq) * 64 + lane] : i32x4{0, 0, 0, 0};
          const int x = 16 * b + (lane & 15);
          cxs[h] = x < aw ? hmC[x] : 0;
        }
      }
#pragma unroll
      for (int h = 0; h < 2; h++) {
      const int b = bp + h * kW;
      if (b >= nb) break;
      const int s0 = s0s[h];
      const int x = 16 * b + (lane & 15);
      const int32_t cx = cxs[h];
      i32x4 (&Bf)[2][3] = Bfs[h];
#pragma unroll 1
      for (int c = 0; c < nch; c++) {
        i32x4 acc0 = {0, 0, 0, 0}, acc1 = {0, 0, 0, 0}, acc2 = {0, 0, 0, 0};
#pragma unroll
        for (int t = 0; t < 2; t++) {
          if (t < KS) {
            const uint8_t *base = shared + (c * 16 + (lane & 15)) * PP + s0 + 64 * t;
            const i32x2 lo = *reinterpret_cast<const i32x2 *>(base + k0l);
            const i32x2 hi = *reinterpret_cast<const i32x2 *>(base + k8l);
            const i32x4 a = {lo.x, lo.y, hi.x, hi.y};
            acc0 = __builtin_amdgcn_mfma_i32_16x16x64_i8(a, Bf[t][0], acc0, 0, 0, 0);
            acc1 = __builtin_amdgcn_mfma_i32_16x16x64_i8(a, Bf[t][1], acc1, 0, 0, 0);
            acc2 = __builtin_amdgcn_mfma_i32_16x16x64_i8(a, Bf[t][2], acc2, 0, 0, 0);
          }
        }
#pragma unroll
        for (int i = 0; i < 4; i++) {
          const int row = r0 + 4 * (lane >> 4) + i;
          if (x < aw && row < hrows) {
            const uint32_t v = (uint32_t)acc0[i] + ((uint32_t)acc1[i] << 8) + ((uint32_t)acc2[i] << 16) + (uint32_t)cx;
            const uint8_t o = (uint8_t)(pil_clip8((int32_t)v) ^ 0x80u);
            uint8_t *dst = ring + (row % kFzRing) * apitch + 3 * x;
            if (nch == 3) {
              dst[c] = o;
            } else {
              dst[0] = dst[1] = dst[2] = o;
            }
          }
        }
      }
      }
    }
  };
  // ---- stream the H stage, run each analysed-row chunk once its window is in
  const int chunks = (ah + kVqRows - 1) / kVqRows;
  int produced = 0;  // H-stage rows in the ring: [produced - ring span, produced)
  const int rA = 16 * (lane >> 4) + ((lane & 15) >> 1);
  const int nq = apitch >> 4, nbytes = 3 * aw;
  // per-thread (row, column) walks over [rows][aw] items in steps of
  // kFzThreads: start and step once, no integer division per item
  const int stepy = kFzThreads / aw, stepx = kFzThreads - stepy * aw;
  const int lm0 = tid / aw, lx0 = tid - lm0 * aw;
#pragma unroll 1
  for (int c = 0; c < chunks; c++) {
    const int k0 = ai[D.vqK0 + c];
    const int need = min(k0 + 64, hrows);
    while (produced < need) {
      __syncthreads();  // the shared region's previous readers (vertical phase) are done
      stage_block(produced);
      __syncthreads();
      hpass(produced);
      produced += 16;
    }
    __syncthreads();  // ring rows of the window complete; the shared region is free
    const int y0 = kVqRows * c, y1 = min(y0 + kVqRows, ah), pa = max(0, y0 - 1), pe = min(ah, pa + 16);
    const i32x4 *af = reinterpret_cast<const i32x4 *>(ai + D.vqA) + (size_t)c * 3 * 64;
    const i32x4 A0 = af[lane], A1 = af[64 + lane], A2 = af[128 + lane];
    int32_t cy[4];
#pragma unroll
    for (int i = 0; i < 4; i++) cy[i] = ai[D.vqC + min(pa + 4 * (lane >> 4) + i, ah - 1)];
    // window row r lives in ring row (k0 + r) % kFzRing
    const uint8_t *pA = ring + ((k0 + rA) % kFzRing) * apitch + 8 * (lane & 1);
    const uint8_t *pB = ring + ((k0 + rA + 8) % kFzRing) * apitch + 8 * (lane & 1);
#pragma unroll 1
    for (int t = wave; t < ((kFzAbl & 4) ? 0 : nq); t += kFzThreads / 64) {
      const i32x2 lo = __builtin_amdgcn_ds_read_tr8_b64_v2i32((l_i32x2q *)(pA + 16 * t));
      const i32x2 hi = __builtin_amdgcn_ds_read_tr8_b64_v2i32((l_i32x2q *)(pB + 16 * t));
      const i32x4 B = {lo.x, lo.y, hi.x, hi.y};
      const i32x4 d2 = __builtin_amdgcn_mfma_i32_16x16x64_i8(A2, B, i32x4{0, 0, 0, 0}, 0, 0, 0);
      const i32x4 d1 = __builtin_amdgcn_mfma_i32_16x16x64_i8(A1, B, d2 << 8, 0, 0, 0);
      const i32x4 d0 = __builtin_amdgcn_mfma_i32_16x16x64_i8(A0, B, i32x4{0, 0, 0, 0}, 0, 0, 0);
      const int col = 16 * t + (lane & 15);
#pragma unroll
      for (int i = 0; i < 4; i++) {
        const int m = 4 * (lane >> 4) + i;
        const int32_t sv = (int32_t)((uint32_t)d0[i] + ((uint32_t)d1[i] << 8) + (uint32_t)cy[i]);
        if (col < nbytes && pa + m < pe) prer[m * apitch + col] = pil_clip8(sv);
      }
    }
    __syncthreads();
    const int nr = pe - pa;
    int m = lm0, x = lx0;  // (m, x) of it, stepped by (stepy, stepx) without a division
#pragma unroll 1
    for (int it = tid; it < ((kFzAbl & 8) ? 0 : nr * aw); it += kFzThreads, m += stepy, x += stepx) {
      if (x >= aw) {
        x -= aw;
        m++;
      }
      const uint8_t *qq = prer + m * apitch + 3 * x;
      lum[m * lpitch + x] = (uint8_t)sc_luma(qq[0], qq[1], qq[2]);
      const int y = pa + m;
      if (D.pre && y >= y0 && y < y1) {
        uint8_t *o = D.pre + ((int64_t)y * aw + x) * 3;
        o[0] = qq[0];
        o[1] = qq[1];
        o[2] = qq[2];
      }
    }
    __syncthreads();
    // maps of the chunk's rows: detect_edge (ImagingFilter3x3 interior,
    // border copies L), skin and saturation (LUT: kFzGather table reads in
    // flight per thread before they are used)
    const int nit = (y1 - y0) * aw;
    constexpr int kG = LUT ? kFzGather : 1;
    int yr_n = lm0, x_n = lx0;  // (row, column) of the next item
#pragma unroll 1
    for (int base = tid; base < ((kFzAbl & 16) ? 0 : nit); base += kG * kFzThreads) {
      uint32_t sv[kG];
      int yrs[kG], xs[kG];
#pragma unroll
      for (int u = 0; u < kG; u++) {
        if (x_n >= aw) {
          x_n -= aw;
          yr_n++;
        }
        yrs[u] = yr_n;
        xs[u] = x_n;
        yr_n += stepy;
        x_n += stepx;
      }
      if (LUT) {
#pragma unroll
        for (int u = 0; u < kG; u++) {
          const int it = base + u * kFzThreads;
          sv[u] = 0;
          if (it < nit) {
            const uint8_t *qq = prer + (y0 + yrs[u] - pa) * apitch + 3 * xs[u];
            sv[u] = skinsat[sc_colour_key(qq[0], qq[1], qq[2])];
          }
        }
      }
#pragma unroll
      for (int u = 0; u < kG; u++) {
        const int it = base + u * kFzThreads;
        if (it >= nit) break;
        const int yr = yrs[u], x = xs[u], y = y0 + yr, m = y - pa;
        const uint8_t *lrow = lum + m * lpitch;
        const uint32_t L = lrow[x];
        uint32_t E = L;
        if (aw >= 3 && ah >= 3 && x > 0 && y > 0 && x < aw - 1 && y < ah - 1) {
          const int v = 4 * (int)L - (int)lrow[x - lpitch] - (int)lrow[x + lpitch] - (int)lrow[x - 1] - (int)lrow[x + 1] + 1;
          E = (uint32_t)(v <= 0 ? 0 : v >= 255 ? 255 : v);
        }
        uint32_t st;
        if (LUT) {
          st = (sv[u] & 255u) | ((sv[u] >> 8) << 16);
        } else {
          const uint8_t *qq = prer + m * apitch + 3 * x;
          st = sc_skin_sat(qq[0], qq[1], qq[2], L, P);
        }
        D.maps[(int64_t)y * aw + x] = st | (E << 8);
      }
    }
  }
}

// ---- k_sc_fd: k_sc_fz's passes (same tables, same arithmetic, bit-identical
// maps) with the source stream decoupled from the compute.  One 16-wave
// workgroup per CU: waves 0-13 run the horizontal pass, the vertical pass,
// luma and maps; waves 14-15 copy 16-row source blocks by LDS-DMA
// (global_load_lds_dwordx4, no VGPRs, no VALU) into kFdSlots raw slots, two
// blocks ahead of the horizontal pass, and wait for each with an exact vmcnt.
// k_sc_fz has one block of loads in flight per workgroup only while it stages
// (ablation: 0.24 of its 0.55 ms per cfg2 step are that load latency); here
// they stay in flight through the MFMA and maps phases.  The horizontal pass
// reads its A fragments straight from the raw interleaved rows (three 8-byte
// LDS reads per 8 pixels, v_perm into the three channels), so there is no
// staging pass and no plane buffer.  One barrier per source block, plus three
// per analysed-row chunk.  Needs 3-channel sources with 16-B aligned rows
// readable to fd_rp(W) bytes (the host's ScDesc.fd).
constexpr int kFdThreads = 1024;
constexpr int kFdC = kFdCWaves * 64;
#ifndef FI_FD_ABL
#define FI_FD_ABL 0
#endif
// profiling ablations (wrong maps): 1 no source DMA, 2 no horizontal pass,
// 4 no vertical pass, 8 no luma loop, 16 no maps loop, 32 no table reads,
// 64 no map stores
constexpr int kFdAbl = FI_FD_ABL;
// skin / saturation: 1 = every pixel from k_sc_skinsat's table (k_sc_fz's
// way), 0 = sc_skin_sat_est per pixel and the table only for what it leaves
// open: one workgroup per CU has no second workgroup to cover the gathers'
// latency, and the L2 serves divergent gathers one line per request
#ifndef FI_FD_LUT
#define FI_FD_LUT 0
#endif
constexpr bool kFdLut = FI_FD_LUT;
__device__ __forceinline__ void fd_dma16(uint32_t m0, const uint8_t *sbase, uint32_t voff) {
  // lane i's 16 bytes at sbase + voff land at LDS m0 + 16 i (m0, sbase uniform)
  unsigned keep;
  const uint64_t sb = (uint64_t)(uintptr_t)sbase;
  sbase = reinterpret_cast<const uint8_t *>((uintptr_t)(
      ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(sb >> 32)) << 32) |
      (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)sb)));
  m0 = (uint32_t)__builtin_amdgcn_readfirstlane((int)m0);
  asm volatile(
      "s_mov_b32 %0, m0\n\t"
      "s_mov_b32 m0, %3\n\t"
      "s_nop 0\n\t"
      "global_load_lds_dwordx4 %1, %2\n\t"
      "s_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(voff), "s"(sbase), "s"(m0)
      : "memory");
}
// s_waitcnt vmcnt(n) for n <= 15 (larger n wait for 15: conservative)
__device__ __forceinline__ void fd_wait_vm(int n) {
  switch (n) {
    case 0: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
    case 1: asm volatile("s_waitcnt vmcnt(1)" ::: "memory"); break;
    case 2: asm volatile("s_waitcnt vmcnt(2)" ::: "memory"); break;
    case 3: asm volatile("s_waitcnt vmcnt(3)" ::: "memory"); break;
    case 4: asm volatile("s_waitcnt vmcnt(4)" ::: "memory"); break;
    case 5: asm volatile("s_waitcnt vmcnt(5)" ::: "memory"); break;
    case 6: asm volatile("s_waitcnt vmcnt(6)" ::: "memory"); break;
    case 7: asm volatile("s_waitcnt vmcnt(7)" ::: "memory"); break;
    case 8: asm volatile("s_waitcnt vmcnt(8)" ::: "memory"); break;
    case 9: asm volatile("s_waitcnt vmcnt(9)" ::: "memory"); break;
    case 10: asm volatile("s_waitcnt vmcnt(10)" ::: "memory"); break;
    case 11: asm volatile("s_waitcnt vmcnt(11)" ::: "memory"); break;
    case 12: asm volatile("s_waitcnt vmcnt(12)" ::: "memory"); break;
    case 13: asm volatile("s_waitcnt vmcnt(13)" ::: "memory"); break;
    case 14: asm volatile("s_waitcnt vmcnt(14)" ::: "memory"); break;
    default: asm volatile("s_waitcnt vmcnt(15)" ::: "memory"); break;
  }
}
__device__ __forceinline__ uint32_t fd_ch(int c, uint32_t a0, uint32_t a1, uint32_t a2) {
  // channel c of 4 interleaved RGB pixels (12 bytes a0 a1 a2), as p - 128
  const uint32_t s1 = c == 0 ? 0x00060300u : c == 1 ? 0x00070401u : 0x00000502u;
  const uint32_t s2 = c == 0 ? 0x05020100u : c == 1 ? 0x06020100u : 0x07040100u;
  return __builtin_amdgcn_perm(a2, __builtin_amdgcn_perm(a1, a0, s1), s2) ^ 0x80808080u;
}

// workgroup barrier without the vmcnt(0) that __syncthreads' fence adds: the
// loader waves' DMAs for the next blocks stay in flight across it (LDS
// accesses are complete at lgkmcnt(0); nothing here reads a global store of
// this kernel)
__device__ __forceinline__ void fd_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

__global__ __launch_bounds__(kFdThreads) void k_sc_fd(const ScDesc *__restrict__ descs,
                                                      const int32_t *__restrict__ ai, const ScParamsDev P,
                                                      const uint16_t *__restrict__ skinsat) {
  extern __shared__ __attribute__((aligned(16))) uint8_t lds8[];
  const ScDesc &D = descs[blockIdx.x];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const bool loader = wave >= kFdCWaves;
  const int aw = D.aw, ah = D.ah, hrows = D.hrows, yoff = D.ybox_first;
  const int apitch = (aw * 3 + 15) & ~15, lpitch = (aw + 3) & ~3;
  const int PP = D.hm_pitch, KS = D.hm_ks, nb = D.hm_nb;
  const int RP = fd_rp(D.W), slotB = fd_slot_bytes(D.W);
  const int64_t sstride = D.stride;
  uint8_t *raw = lds8;                                         // [kFdSlots][16][RP] source rows
  uint8_t *ring = lds8 + fd_ring_off(D.W, PP);                 // [kFzRing][apitch] H-stage rows, p - 128
  uint8_t *prer = ring + kFzRing * apitch, *lum = prer + 16 * apitch;  // [16][apitch], [16][lpitch]
  uint8_t *abuf = lds8 + fd_tab_off(D.W, PP, aw);             // [chunks][3][64] i32x4 vertical A fragments
  const int chunks = (ah + kVqRows - 1) / kVqRows;
  int32_t *cbuf = reinterpret_cast<int32_t *>(abuf + chunks * 3072);  // [ah] vertical bias
  const int nblk = (min(ai[D.vqK0 + chunks - 1] + 64, hrows) + 15) >> 4;  // blocks the last chunk needs
  // ---- loader side: block blk -> slot blk % kFdSlots, DMA steps i = lw, lw + 2, ...
  const int ninstr = slotB >> 10, lw = wave - kFdCWaves;
  const int cnt = (ninstr - lw + 1) >> 1;  // this loader wave's DMAs per block
  const int rpc = RP >> 4;                 // 16-byte chunks per row
  const float rcp_rpc = 1.0f / (float)rpc;
  const uint32_t raw_m0 = (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) uint8_t *)raw;
  const uint32_t ab_m0 = (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) uint8_t *)abuf;
  auto issue = [&](int blk) {
    if (blk >= nblk || (kFdAbl & 1)) return;
    const int r0 = blk << 4;
    const uint8_t *sb = D.img + (int64_t)(r0 + yoff) * sstride;
    const int last = hrows - 1 - r0;  // rows past the analysed rows repeat the last one (never used)
#pragma unroll 1
    for (int i = lw; i < ninstr; i += 2) {
      const int j = 64 * i + lane;
      int row = fz_div(j, rpc, rcp_rpc);
      const int col = j - row * rpc;
      row = min(row, min(15, last));  // lanes past the block's 16 rows land in the slot's padding
      fd_dma16(raw_m0 + (uint32_t)((blk % kFdSlots) * slotB + 1024 * i), sb,
               (uint32_t)(row * sstride + 16 * col));
    }
  };
  // ---- compute side: wave w owns column block w (the host admits images of
  // <= kFdCWaves blocks: aw <= 224; cfg2: 13); its B fragments stay in
  // registers for the whole image
  const int32_t *hmS0 = ai + D.hmS0, *hmC = ai + D.hmC;
  const i32x4 *hmB = reinterpret_cast<const i32x4 *>(ai + D.hmB);
  const int k0l = mfma_i8_k(lane, 0), k8l = mfma_i8_k(lane, 8);
  auto load_b = [&](int b, i32x4 (&Bf)[2][3], int &s0, int32_t &cx) {
    s0 = hmS0[b];
#pragma unroll
    for (int t = 0; t < 2; t++)
#pragma unroll
      for (int q = 0; q < 3; q++) Bf[t][q] = t < KS ? hmB[((b * KS + t) * 3 + q) * 64 + lane] : i32x4{0, 0, 0, 0};
    const int x = 16 * b + (lane & 15);
    cx = x < aw ? hmC[x] : 0;
  };
  i32x4 Bh[2][3];
  int s0h = 0;
  int32_t cxh = 0;
  if (!loader && wave < nb) load_b(wave, Bh, s0h, cxh);
  // the slot's 16 rows x column block b -> H-stage rows r0 .. r0 + 15
  auto hpass_block = [&](int r0, const uint8_t *slot, int b, const i32x4 (&Bf)[2][3], int s0, int32_t cx) {
    const int x = 16 * b + (lane & 15);
    i32x4 acc[3][3];
#pragma unroll
    for (int c = 0; c < 3; c++)
#pragma unroll
      for (int q = 0; q < 3; q++) acc[c][q] = i32x4{0, 0, 0, 0};
#pragma unroll
    for (int t = 0; t < 2; t++) {
      if (t < KS) {
        const uint8_t *rp = slot + (lane & 15) * RP + 3 * (s0 + 64 * t);
        const i32x2 *p0 = reinterpret_cast<const i32x2 *>(rp + 3 * k0l);
        const i32x2 *p1 = reinterpret_cast<const i32x2 *>(rp + 3 * k8l);
        const i32x2 u0 = p0[0], u1 = p0[1], u2 = p0[2], v0 = p1[0], v1 = p1[1], v2 = p1[2];
#pragma unroll
        for (int c = 0; c < 3; c++) {
          const i32x4 a = {(int32_t)fd_ch(c, u0.x, u0.y, u1.x), (int32_t)fd_ch(c, u1.y, u2.x, u2.y),
                           (int32_t)fd_ch(c, v0.x, v0.y, v1.x), (int32_t)fd_ch(c, v1.y, v2.x, v2.y)};
#pragma unroll
          for (int q = 0; q < 3; q++) acc[c][q] = __builtin_amdgcn_mfma_i32_16x16x64_i8(a, Bf[t][q], acc[c][q], 0, 0, 0);
        }
      }
    }
#pragma unroll
    for (int i = 0; i < 4; i++) {
      const int row = r0 + 4 * (lane >> 4) + i;
      if (x < aw && row < hrows) {
        uint8_t *dst = ring + (row % kFzRing) * apitch + 3 * x;
#pragma unroll
        for (int c = 0; c < 3; c++) {
          const uint32_t v = (uint32_t)acc[c][0][i] + ((uint32_t)acc[c][1][i] << 8) + ((uint32_t)acc[c][2][i] << 16) +
                             (uint32_t)cx;
          dst[c] = (uint8_t)(pil_clip8((int32_t)v) ^ 0x80u);
        }
      }
    }
  };
  auto hpass = [&](int r0, const uint8_t *slot) {
    if (wave < nb) hpass_block(r0, slot, wave, Bh, s0h, cxh);
  };
  const int rA = 16 * (lane >> 4) + ((lane & 15) >> 1);
  const int nq = apitch >> 4, nbytes = 3 * aw;
  const int stepy = kFdC / aw, stepx = kFdC - stepy * aw;
  const int lm0 = tid / aw, lx0 = tid - lm0 * aw;
  const ScFast F = sc_fast_params(P);
  const int ng4 = (aw + 3) >> 2;  // luma: 4-pixel groups per row
  const float rcp_ng4 = 1.0f / (float)ng4;
  // ---- prologue: every chunk's vertical A fragments, source blocks 0 and 1
  // in flight; the vertical bias into LDS; block 0 and the fragments landed
  if (loader) {
    const uint8_t *afrag = reinterpret_cast<const uint8_t *>(ai + D.vqA);
#pragma unroll 1
    for (int k = lw; k < 3 * chunks; k += 2) fd_dma16(ab_m0 + 1024 * k, afrag, (uint32_t)(1024 * k + 16 * lane));
    issue(0);
    issue(1);
    fd_wait_vm(1 < nblk ? cnt : 0);
  } else {
#pragma unroll 1
    for (int i = tid; i < ah; i += kFdC) cbuf[i] = ai[D.vqC + i];
  }
  fd_barrier();
  int blk = 0;  // next block for the horizontal pass (in slot blk % kFdSlots)
#pragma unroll 1
  for (int c = 0; c < chunks; c++) {
    const int k0 = ai[D.vqK0 + c];
    const int need = min(k0 + 64, hrows);
    bool phased = false;
#pragma unroll 1
    while (16 * blk < need) {
      if (loader) {
        issue(blk + 2);                        // into the slot block blk - 1 left
        fd_wait_vm(blk + 2 < nblk ? cnt : 0);  // block blk + 1 landed
      } else if (!(kFdAbl & 2)) {
        hpass(16 * blk, raw + (blk % kFdSlots) * slotB);
      }
      fd_barrier();
      blk++;
      phased = true;
    }
    // the chunk's window is in the ring; the last chunk's maps are done with
    // prer / lum (a barrier of their own when no block ran in between)
    if (!phased) fd_barrier();
    const int y0 = kVqRows * c, y1 = min(y0 + kVqRows, ah), pa = max(0, y0 - 1), pe = min(ah, pa + 16);
    if (!loader) {
      const i32x4 *af = reinterpret_cast<const i32x4 *>(abuf + c * 3072);
      const i32x4 A0 = af[lane], A1 = af[64 + lane], A2 = af[128 + lane];
      int32_t cy[4];
#pragma unroll
      for (int i = 0; i < 4; i++) cy[i] = cbuf[min(pa + 4 * (lane >> 4) + i, ah - 1)];
      const uint8_t *pA = ring + ((k0 + rA) % kFzRing) * apitch + 8 * (lane & 1);
      const uint8_t *pB = ring + ((k0 + rA + 8) % kFzRing) * apitch + 8 * (lane & 1);
#pragma unroll 1
      for (int t = wave; t < ((kFdAbl & 4) ? 0 : nq); t += kFdCWaves) {
        const i32x2 lo = __builtin_amdgcn_ds_read_tr8_b64_v2i32((l_i32x2q *)(pA + 16 * t));
        const i32x2 hi = __builtin_amdgcn_ds_read_tr8_b64_v2i32((l_i32x2q *)(pB + 16 * t));
        const i32x4 B = {lo.x, lo.y, hi.x, hi.y};
        const i32x4 d2 = __builtin_amdgcn_mfma_i32_16x16x64_i8(A2, B, i32x4{0, 0, 0, 0}, 0, 0, 0);
        const i32x4 d1 = __builtin_amdgcn_mfma_i32_16x16x64_i8(A1, B, d2 << 8, 0, 0, 0);
        const i32x4 d0 = __builtin_amdgcn_mfma_i32_16x16x64_i8(A0, B, i32x4{0, 0, 0, 0}, 0, 0, 0);
        const int col = 16 * t + (lane & 15);
#pragma unroll
        for (int i = 0; i < 4; i++) {
          const int m = 4 * (lane >> 4) + i;
          const int32_t sv = (int32_t)((uint32_t)d0[i] + ((uint32_t)d1[i] << 8) + (uint32_t)cy[i]);
          if (col < nbytes && pa + m < pe) prer[m * apitch + col] = pil_clip8(sv);
        }
      }
    }
    fd_barrier();
    // maps items (analysed rows y0 .. y1 - 1): the first kFzGather skin /
    // saturation table reads per thread go out before the luma pass, so their
    // latency overlaps it and its barrier
    const int nit = (y1 - y0) * aw;
    int yr_n = lm0, x_n = lx0;  // (row, column) of the thread's next item
    uint32_t sv[kFzGather];
    // the kFzGather items of a step: (row, column) from the walk; walk() is
    // run twice per step (for the table reads, then for the maps) so only the
    // reads' results stay live across the luma pass
    auto walk = [&](int (&yrs)[kFzGather], int (&xs)[kFzGather]) {
#pragma unroll
      for (int u = 0; u < kFzGather; u++) {
        if (x_n >= aw) {
          x_n -= aw;
          yr_n++;
        }
        yrs[u] = yr_n;
        xs[u] = x_n;
        yr_n += stepy;
        x_n += stepx;
      }
    };
    auto gather = [&](int base) {
      int yrs[kFzGather], xs[kFzGather];
      walk(yrs, xs);
#pragma unroll
      for (int u = 0; u < kFzGather; u++) {
        const int it = base + u * kFdC;
        sv[u] = 0;
        if (it < nit) {
          const uint8_t *qq = prer + (y0 + yrs[u] - pa) * apitch + 3 * xs[u];
          sv[u] = (kFdAbl & 32) ? qq[0] * 0x101u : skinsat[sc_colour_key(qq[0], qq[1], qq[2])];
        }
      }
    };
    const int nr = pe - pa;
    if (!loader) {
      if (kFdLut && !(kFdAbl & 16)) gather(tid);
      // luma of the prescaled rows pa .. pe - 1, four pixels per item
#pragma unroll 1
      for (int it = tid; it < ((kFdAbl & 8) ? 0 : nr * ng4); it += kFdC) {
        const int m = fz_div(it, ng4, rcp_ng4), g = it - m * ng4;
        const uint32_t *q = reinterpret_cast<const uint32_t *>(prer + m * apitch + 12 * g);
        const uint32_t a0 = q[0], a1 = q[1], a2 = q[2];
        const uint32_t R = fd_ch(0, a0, a1, a2) ^ 0x80808080u, G = fd_ch(1, a0, a1, a2) ^ 0x80808080u,
                       B = fd_ch(2, a0, a1, a2) ^ 0x80808080u;
        uint32_t l4 = 0;
#pragma unroll
        for (int j = 0; j < 4; j++)
          l4 |= sc_luma((R >> (8 * j)) & 255u, (G >> (8 * j)) & 255u, (B >> (8 * j)) & 255u) << (8 * j);
        *reinterpret_cast<uint32_t *>(lum + m * lpitch + 4 * g) = l4;
        const int y = pa + m;
        if (D.pre && y >= y0 && y < y1) {
#pragma unroll
          for (int j = 0; j < 4; j++) {
            const int x = 4 * g + j;
            if (x < aw) {
              uint8_t *o = D.pre + ((int64_t)y * aw + x) * 3;
              o[0] = (uint8_t)(R >> (8 * j));
              o[1] = (uint8_t)(G >> (8 * j));
              o[2] = (uint8_t)(B >> (8 * j));
            }
          }
        }
      }
    }
    fd_barrier();
    if (!loader && !kFdLut) {
      // kFzGather items per step: skin / saturation by sc_skin_sat_est, the
      // table read only for the items it leaves open (skin candidates,
      // saturation bytes at an integer boundary), all in flight together
      int yr_w = lm0, x_w = lx0;
#pragma unroll 1
      for (int base = tid; base < ((kFdAbl & 16) ? 0 : nit); base += kFzGather * kFdC) {
        uint32_t stv[kFzGather];
        int yrs[kFzGather], xs[kFzGather];
#pragma unroll
        for (int u = 0; u < kFzGather; u++) {
          if (x_w >= aw) {
            x_w -= aw;
            yr_w++;
          }
          yrs[u] = yr_w;
          xs[u] = x_w;
          yr_w += stepy;
          x_w += stepx;
          stv[u] = 0;
          if (base + u * kFdC < nit) {
            const int m = y0 + yrs[u] - pa;
            const uint8_t *qq = prer + m * apitch + 3 * xs[u];
            const uint32_t r = qq[0], g = qq[1], b = qq[2];
            if (!sc_skin_sat_est(F, r, g, b, lum[m * lpitch + xs[u]], stv[u])) {
              const uint32_t t = skinsat[sc_colour_key(r, g, b)];
              stv[u] = (t & 255u) | ((t >> 8) << 16);
            }
          }
        }
#pragma unroll
        for (int u = 0; u < kFzGather; u++) {
          const int it = base + u * kFdC;
          if (it >= nit) break;
          const int yr = yrs[u], x = xs[u], y = y0 + yr, m = y - pa;
          const uint8_t *lrow = lum + m * lpitch;
          const uint32_t L = lrow[x];
          uint32_t E = L;
          if (aw >= 3 && ah >= 3 && x > 0 && y > 0 && x < aw - 1 && y < ah - 1) {
            const int v = 4 * (int)L - (int)lrow[x - lpitch] - (int)lrow[x + lpitch] - (int)lrow[x - 1] - (int)lrow[x + 1] + 1;
            E = (uint32_t)(v <= 0 ? 0 : v >= 255 ? 255 : v);
          }
          if (!(kFdAbl & 64)) D.maps[(int64_t)y * aw + x] = stv[u] | (E << 8);
        }
      }
    }
    if (!loader && kFdLut) {
      yr_n = lm0;
      x_n = lx0;
#pragma unroll 1
      for (int base = tid; base < ((kFdAbl & 16) ? 0 : nit); base += kFzGather * kFdC) {
        if (base != tid) {
          const int ys = yr_n, xs0 = x_n;
          gather(base);
          yr_n = ys;
          x_n = xs0;
        }
        int yrs[kFzGather], xs[kFzGather];
        walk(yrs, xs);
#pragma unroll
        for (int u = 0; u < kFzGather; u++) {
          const int it = base + u * kFdC;
          if (it >= nit) break;
          const int yr = yrs[u], x = xs[u], y = y0 + yr, m = y - pa;
          const uint8_t *lrow = lum + m * lpitch;
          const uint32_t L = lrow[x];
          uint32_t E = L;
          if (aw >= 3 && ah >= 3 && x > 0 && y > 0 && x < aw - 1 && y < ah - 1) {
            const int v = 4 * (int)L - (int)lrow[x - lpitch] - (int)lrow[x + lpitch] - (int)lrow[x - 1] - (int)lrow[x + 1] + 1;
            E = (uint32_t)(v <= 0 ? 0 : v >= 255 ? 255 : v);
          }
          if (!(kFdAbl & 64)) D.maps[(int64_t)y * aw + x] = ((sv[u] & 255u) | ((sv[u] >> 8) << 16)) | (E << 8);
        }
      }
    }
  }
  if (loader) fd_wait_vm(0);  // every DMA landed before the workgroup retires
}

// ---- k_sc_hx + k_sc_vx: the same prescale + maps (same integer arithmetic,
// bit-identical maps) shaped to run BESIDE the next batch's k_rs_vr: no LDS,
// <= 64 VGPRs (launch_bounds(256, 8)), so their waves take the one wave slot
// per SIMD that k_rs_vr's workgroup leaves free (as k_crop_apply3p does),
// instead of a serial stage between two resamples.
//  * k_sc_hx: one wave per (image, 16-column block b), looping over 16-row
//    blocks of the H stage (k_sc_hmfma's B fragments stay in registers).  A
//    lane's A operand is 16 consecutive source pixels (48 contiguous bytes);
//    limbs fold through the accumulator (t = A B2; t = A B1 + (t << 8);
//    t = A B0 + (t << 8) + C', C' = Pillow's bias - 2^29, so the H-stage byte
//    as p - 128 is med3(t >> 22, -128, 127)).  The MFMA result lane
//    (g, n) holds rows 4g .. 4g + 3 of column n: one dword store per channel
//    into the TRANSPOSED H stage tbuf[b][ch][n][row] (p - 128 bytes).
//  * k_sc_vx: one wave per (image, chunk of kVqRows analysed rows): per
//    column block, the chunk's 16 prescaled rows = one MFMA block whose B
//    operand is 16 contiguous bytes of a tbuf column (rows K0 + 16 g ..); the
//    lane then holds R, G, B of 4 vertically adjacent pixels.  Luma is packed
//    4 bytes a dword; the Laplacian's row neighbours come from lanes -+16
//    (ds_bpermute), its column neighbours by DPP within the 16-lane row, the
//    previous / next block's edge column through the rotate's `old` operand, so
//    a block's maps are written one block late.  Skin / saturation: k_sc_fd's
//    estimator, k_sc_skinsat's table for what it leaves open.
// The host runs both on the apply stream behind the batch's resample, so they
// overlap the next batch's k_rs_vr (fi_api.cpp launch_batch).
// (the RGB two-k-step forms at 128 VGPRs: at 64 they spill, and they never
// run beside k_rs_vr -- FI_SC_CX=3 is for uniform cfg2-like batches)
template <int KS, int NCH>
__global__ __launch_bounds__(256, KS == 2 && NCH == 3 ? 4 : 8) void k_sc_hx(const ScDesc *__restrict__ descs,
                                                                          const int32_t *__restrict__ tiles,
                                                                          const int32_t *__restrict__ ai) {
  typedef uint32_t u32x4a __attribute__((ext_vector_type(4), aligned(4)));
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int di = tiles[3 * blockIdx.x];
  if (di < 0) return;
  const ScDesc &D = descs[di];
  const int b = tiles[3 * blockIdx.x + 1] + wave, rb0 = tiles[3 * blockIdx.x + 2];
  if (b >= D.hm_nb) return;
  const int g = lane >> 4, r = lane & 15;
  const int aw = D.aw, hrows = D.hrows, yoff = D.ybox_first, tp = D.cx_tp;
  const int rp = NCH == 3 ? fd_rp(D.W) : (D.W + 15) & ~15;  // readable bytes of a row
  const int s0 = ai[D.hmS0 + b];
  const i32x4 *hmB = reinterpret_cast<const i32x4 *>(ai + D.hmB) + (size_t)b * KS * 3 * 64 + lane;
  // B fragments in registers, except at two k-steps of RGB (64 VGPRs: from L1 per item)
  constexpr bool kKeepB = !(KS == 2 && NCH == 3);
  i32x4 Bf[kKeepB ? KS : 1][3];
  if (kKeepB)
#pragma unroll
    for (int t = 0; t < KS; t++)
#pragma unroll
      for (int q = 0; q < 3; q++) Bf[kKeepB ? t : 0][q] = hmB[(t * 3 + q) * 64];
  auto bfrag = [&](int t, int q) {
    const i32x4 *hb = hmB;
    if (!kKeepB) asm volatile("" : "+v"(hb));  // re-read per use: not hoisted out of the row loop
    return kKeepB ? Bf[kKeepB ? t : 0][q] : hb[(t * 3 + q) * 64];
  };
  const int x = 16 * b + r;
  const int32_t cxp = x < aw ? ai[D.hmC + x] - (1 << 29) : 0;
  constexpr int NQ = NCH == 3 ? 3 : 1;  // 16-B loads per k-step
  const int64_t sstride = D.stride;
  // tbuf tiles [b][ch][row block][16 columns][16 rows]: a store instruction
  // writes one whole 256-B tile (lane (g, n): column n, rows 4g .. 4g + 3)
  const int nrbt = tp >> 4;
  uint8_t *tcol = D.tbuf + (int64_t)b * NCH * nrbt * 256 + 16 * r + 4 * g;
  auto load = [&](int rb, u32x4a (&q)[KS][NQ]) {
    const int hr = min(16 * rb + r, hrows - 1);
    const uint8_t *row = D.img + (int64_t)(hr + yoff) * sstride;
#pragma unroll
    for (int t = 0; t < KS; t++)
#pragma unroll
      for (int i = 0; i < NQ; i++) {
        const int off = (NCH == 3 ? 3 : 1) * (s0 + 64 * t + 16 * g) + 16 * i;  // 8-B aligned
        u32x4a v = *reinterpret_cast<const u32x4a *>(row + min(off, rp - 16));
        if (off > rp - 16) v = off == rp - 8 ? u32x4a{v.z, v.w, 0u, 0u} : u32x4a{0u, 0u, 0u, 0u};
        q[t][i] = v;
      }
  };
  // row blocks [rb0, rb0 + kHxRb) of the H stage (the last tile row block is
  // the V pass's straddle margin, never read as data)
  const int nrb = min(nrbt - 1, rb0 + kHxRb);
  constexpr bool kPre = KS * NQ <= 3;  // the next row block's loads in flight (within 64 VGPRs)
  u32x4a cur[KS][NQ], nxt[KS][NQ];
  load(rb0, cur);
#pragma unroll 1
  for (int rb = rb0; rb < nrb; rb++) {
    if (!kPre && rb > rb0) load(rb, cur);
    if (kPre && rb + 1 < nrb) load(rb + 1, nxt);
#pragma unroll
    for (int ch = 0; ch < NCH; ch++) {
      i32x4 A[KS];
#pragma unroll
      for (int t = 0; t < KS; t++) {
        if (NCH == 3) {
          const uint32_t d[12] = {cur[t][0].x, cur[t][0].y, cur[t][0].z, cur[t][0].w, cur[t][1].x, cur[t][1].y,
                                  cur[t][1].z, cur[t][1].w, cur[t][2].x, cur[t][2].y, cur[t][2].z, cur[t][2].w};
          A[t] = i32x4{(int32_t)fd_ch(ch, d[0], d[1], d[2]), (int32_t)fd_ch(ch, d[3], d[4], d[5]),
                       (int32_t)fd_ch(ch, d[6], d[7], d[8]), (int32_t)fd_ch(ch, d[9], d[10], d[11])};
        } else {
          A[t] = i32x4{(int32_t)(cur[t][0].x ^ 0x80808080u), (int32_t)(cur[t][0].y ^ 0x80808080u),
                       (int32_t)(cur[t][0].z ^ 0x80808080u), (int32_t)(cur[t][0].w ^ 0x80808080u)};
        }
      }
      // limbs folded through the accumulator (modular int32)
      i32x4 acc = {0, 0, 0, 0};
#pragma unroll
      for (int t = 0; t < KS; t++) acc = __builtin_amdgcn_mfma_i32_16x16x64_i8(A[t], bfrag(t, 2), acc, 0, 0, 0);
      acc = acc << 8;
#pragma unroll
      for (int t = 0; t < KS; t++) acc = __builtin_amdgcn_mfma_i32_16x16x64_i8(A[t], bfrag(t, 1), acc, 0, 0, 0);
      acc = (acc << 8) + i32x4{cxp, cxp, cxp, cxp};
#pragma unroll
      for (int t = 0; t < KS; t++) acc = __builtin_amdgcn_mfma_i32_16x16x64_i8(A[t], bfrag(t, 0), acc, 0, 0, 0);
      uint32_t w = 0;
#pragma unroll
      for (int i = 0; i < 4; i++) w |= ((uint32_t)min(max(acc[i] >> 22, -128), 127) & 255u) << (8 * i);
      *reinterpret_cast<uint32_t *>(tcol + ((int64_t)ch * nrbt + rb) * 256) = w;
    }
    if (kPre)
#pragma unroll
      for (int t = 0; t < KS; t++)
#pragma unroll
        for (int i = 0; i < NQ; i++) cur[t][i] = nxt[t][i];
  }
}

__device__ __forceinline__ uint32_t vx_byte(uint32_t v, int i) { return (v >> (8 * i)) & 255u; }

template <int KV, int NCH>
__global__ __launch_bounds__(256, KV == 2 && NCH == 3 ? 4 : 8) void k_sc_vx(const ScDesc *__restrict__ descs,
                                                                          const int32_t *__restrict__ tiles,
                                                                          const int32_t *__restrict__ ai, const ScFast F,
                                                                          const uint16_t *__restrict__ skinsat) {
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int tix = 4 * blockIdx.x + wave;
  const int di = tiles[2 * tix], c = tiles[2 * tix + 1];
  if (di < 0) return;
  const ScDesc &D = descs[di];
  const int g = lane >> 4, n = lane & 15;
  const int aw = D.aw, ah = D.ah, tp = D.cx_tp, nb = D.hm_nb;
  const int y0 = kVqRows * c, y1 = min(y0 + kVqRows, ah), pa = max(0, y0 - 1);
  // the chunk's A fragments, read per block (L1 hits): registers are the budget
  const i32x4 *af = reinterpret_cast<const i32x4 *>(ai + D.cxA) + (size_t)c * KV * 3 * 64 + lane;
  int32_t cy[4];
#pragma unroll
  for (int i = 0; i < 4; i++) cy[i] = ai[D.vqC + min(pa + 4 * g + i, ah - 1)];
  // the window's rows K0 + 64 t + 16 g .. + 15 of column n straddle row blocks
  // rb0 + 4 t + g and the next at dword offset m = (K0 & 15) / 4 (uniform)
  const int K0 = ai[D.cxK0 + c], nrbt = tp >> 4, m4 = (K0 & 15) >> 2;
  const uint8_t *tb = D.tbuf + ((int64_t)(K0 >> 4) + g) * 256 + 16 * n;
  const bool edges = aw >= 3 && ah >= 3;
  // block b's prescaled bytes of the lane's 4 rows, one dword per channel
  auto vpass = [&](int b, uint32_t (&rgb)[3]) {
    const i32x4 *afb = af;
    asm volatile("" : "+v"(afb));  // re-read per block: not hoisted into 12-24 live VGPRs
#pragma unroll
    for (int ch = 0; ch < NCH; ch++) {
      const uint8_t *col = tb + (int64_t)(b * NCH + ch) * nrbt * 256;
      i32x4 B[KV];
#pragma unroll
      for (int t = 0; t < KV; t++) {
        const i32x4 lo = *reinterpret_cast<const i32x4 *>(col + 1024 * t);
        if (m4 == 0) {
          B[t] = lo;
        } else {
          const i32x4 hi = *reinterpret_cast<const i32x4 *>(col + 1024 * t + 256);
          B[t] = m4 == 1 ? i32x4{lo.y, lo.z, lo.w, hi.x} : m4 == 2 ? i32x4{lo.z, lo.w, hi.x, hi.y}
                                                             : i32x4{lo.w, hi.x, hi.y, hi.z};
        }
      }
      i32x4 acc = {0, 0, 0, 0};
#pragma unroll
      for (int t = 0; t < KV; t++) acc = __builtin_amdgcn_mfma_i32_16x16x64_i8(afb[(t * 3 + 2) * 64], B[t], acc, 0, 0, 0);
      acc = acc << 8;
#pragma unroll
      for (int t = 0; t < KV; t++) acc = __builtin_amdgcn_mfma_i32_16x16x64_i8(afb[(t * 3 + 1) * 64], B[t], acc, 0, 0, 0);
      acc = (acc << 8) + i32x4{cy[0], cy[1], cy[2], cy[3]};
#pragma unroll
      for (int t = 0; t < KV; t++) acc = __builtin_amdgcn_mfma_i32_16x16x64_i8(afb[(t * 3 + 0) * 64], B[t], acc, 0, 0, 0);
      uint32_t w = 0;
#pragma unroll
      for (int i = 0; i < 4; i++) w |= (uint32_t)pil_clip8(acc[i]) << (8 * i);
      rgb[ch] = w;
      asm volatile("" ::: "memory");  // one channel's fragments live at a time (64 VGPRs)
    }
    if (NCH == 1) rgb[1] = rgb[2] = rgb[0];
  };
  auto luma4 = [&](const uint32_t (&rgb)[3]) {
    uint32_t l4 = 0;
#pragma unroll
    for (int i = 0; i < 4; i++) l4 |= sc_luma(vx_byte(rgb[0], i), vx_byte(rgb[1], i), vx_byte(rgb[2], i)) << (8 * i);
    return l4;
  };
  uint32_t cur[3] = {0, 0, 0}, prv[3] = {0, 0, 0};
  uint32_t Lc = 0, Lp = 0, Lpp = 0;  // luma of blocks b, b - 1, b - 2
#pragma unroll 1
  for (int b = 0; b <= nb; b++) {
    if (b < nb) {
      vpass(b, cur);
      Lc = luma4(cur);
    }
    if (b > 0) {  // maps of block b - 1
      const int x = 16 * (b - 1) + n;
      const uint32_t up = (uint32_t)__shfl((int)Lp, lane - 16, 64), dn = (uint32_t)__shfl((int)Lp, lane + 16, 64);
      const uint32_t lt = (uint32_t)__builtin_amdgcn_update_dpp(
          __builtin_amdgcn_update_dpp(0, (int)Lpp, 0x121, 0xF, 0xF, false), (int)Lp, 0x111, 0xF, 0xF, false);
      const uint32_t rt = (uint32_t)__builtin_amdgcn_update_dpp(
          __builtin_amdgcn_update_dpp(0, (int)Lc, 0x12F, 0xF, 0xF, false), (int)Lp, 0x101, 0xF, 0xF, false);
      uint32_t stv[4];
#pragma unroll
      for (int i = 0; i < 4; i++) {
        const uint32_t rr = vx_byte(prv[0], i), gg = vx_byte(prv[1], i), bb = vx_byte(prv[2], i);
        if (!sc_skin_sat_est(F, rr, gg, bb, vx_byte(Lp, i), stv[i])) {
          const uint32_t t = skinsat[sc_colour_key(rr, gg, bb)];
          stv[i] = (t & 255u) | ((t >> 8) << 16);
        }
      }
#pragma unroll
      for (int i = 0; i < 4; i++) {
        const int y = pa + 4 * g + i;
        if (x >= aw || y < y0 || y >= y1) continue;
        const uint32_t L = vx_byte(Lp, i);
        uint32_t E = L;
        if (edges && x > 0 && y > 0 && x < aw - 1 && y < ah - 1) {
          const uint32_t u = i > 0 ? vx_byte(Lp, i - 1) : vx_byte(up, 3);
          const uint32_t d = i < 3 ? vx_byte(Lp, i + 1) : vx_byte(dn, 0);
          const int v = 4 * (int)L - (int)u - (int)d - (int)vx_byte(lt, i) - (int)vx_byte(rt, i) + 1;
          E = (uint32_t)(v <= 0 ? 0 : v >= 255 ? 255 : v);
        }
        D.maps[(int64_t)y * aw + x] = stv[i] | (E << 8);
        if (D.pre) {  // the prescaled image, when the caller keeps it
          uint8_t *o = D.pre + ((int64_t)y * aw + x) * 3;
          o[0] = (uint8_t)vx_byte(prv[0], i);
          o[1] = (uint8_t)vx_byte(prv[1], i);
          o[2] = (uint8_t)vx_byte(prv[2], i);
        }
      }
    }
    Lpp = Lp;
    Lp = Lc;
#pragma unroll
    for (int k = 0; k < 3; k++) prv[k] = cur[k];
  }
}

int launch_sc_hx(hipStream_t s, int ks, int nch, const ScDesc *descs, const int32_t *tiles, int ntiles,
                 const int32_t *ai) {
  if (ntiles <= 0) return 0;
  const dim3 grid(ntiles), blk(256);
  if (ks == 1 && nch == 3) hipLaunchKernelGGL((k_sc_hx<1, 3>), grid, blk, 0, s, descs, tiles, ai);
  else if (ks == 2 && nch == 3) hipLaunchKernelGGL((k_sc_hx<2, 3>), grid, blk, 0, s, descs, tiles, ai);
  else if (ks == 1 && nch == 1) hipLaunchKernelGGL((k_sc_hx<1, 1>), grid, blk, 0, s, descs, tiles, ai);
  else if (ks == 2 && nch == 1) hipLaunchKernelGGL((k_sc_hx<2, 1>), grid, blk, 0, s, descs, tiles, ai);
  else return -1;
  return 0;
}
int launch_sc_vx(hipStream_t s, int kv, int nch, const ScDesc *descs, const int32_t *tiles, int ntiles,
                 const int32_t *ai, const ScParamsDev &P, const uint16_t *skinsat) {
  if (ntiles <= 0) return 0;
  if (ntiles % 4) return -1;  // four waves (tiles) a workgroup; the host pads
  const dim3 grid(ntiles / 4), blk(256);
  const ScFast F = sc_fast_params(P);  // host-side: kernel arguments stay in SGPRs
  if (kv == 1 && nch == 3) hipLaunchKernelGGL((k_sc_vx<1, 3>), grid, blk, 0, s, descs, tiles, ai, F, skinsat);
  else if (kv == 2 && nch == 3) hipLaunchKernelGGL((k_sc_vx<2, 3>), grid, blk, 0, s, descs, tiles, ai, F, skinsat);
  else if (kv == 1 && nch == 1) hipLaunchKernelGGL((k_sc_vx<1, 1>), grid, blk, 0, s, descs, tiles, ai, F, skinsat);
  else if (kv == 2 && nch == 1) hipLaunchKernelGGL((k_sc_vx<2, 1>), grid, blk, 0, s, descs, tiles, ai, F, skinsat);
  else return -1;
  return 0;
}

// ---------------------------------------------------------------------------
constexpr int kScoreThreads = 1024;
constexpr int kScoreWaves = kScoreThreads / 64;
#ifndef FI_SC_BANDS
#define FI_SC_BANDS 0
#endif
constexpr bool kScoreBands = FI_SC_BANDS;

// MODE 0: maps read from global memory; 1: maps in LDS.
template <int MODE>
__global__ __launch_bounds__(kScoreThreads) void k_sc_score2(const ScDesc *__restrict__ descs,
                                                             const DevCrop *__restrict__ crops,
                                                             const double *__restrict__ ad,
                                                             CropScore *__restrict__ scores,
                                                             ScResult *__restrict__ results, const ScParamsDev P,
                                                             const int32_t *__restrict__ ai) {
  constexpr bool LDS_MAPS = MODE >= 1;
  extern __shared__ __attribute__((aligned(16))) uint32_t smaps[];
  __shared__ double lut[256];
  __shared__ double part[kScoreWaves][3];
  __shared__ double T[3];
  __shared__ double s_tot[kScoreMaxCrops];
  __shared__ double s_bnd[kScoreMaxCrops];
  __shared__ int32_t cand[kScoreMaxCrops];
  __shared__ double s_part[kScoreMaxCrops][3];  // band partial sums (crop-major)
  __shared__ int32_t ncand_s, first_cand_s;
  const ScDesc &D = descs[blockIdx.x];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int ncrops = D.ncrops;
  // more crops than the LDS arrays hold (analysed images beyond ~14:1, or a
  // small step): totals, bounds and the candidate marks live in the image's
  // CropScore slots instead (exact = 2 marks a candidate until re-scored)
  const bool big = ncrops > kScoreMaxCrops;
  CropScore *const sco = scores + D.score0;
  const int W = D.aw, H = D.ah, npx = W * H;
  const uint32_t *maps = D.maps;
  if (LDS_MAPS) {
    const uint4 *g = reinterpret_cast<const uint4 *>(D.maps);
    for (int k = tid; k < (npx >> 2); k += kScoreThreads) reinterpret_cast<uint4 *>(smaps)[k] = g[k];
    for (int k = (npx & ~3) + tid; k < npx; k += kScoreThreads) smaps[k] = D.maps[k];
    maps = smaps;
  }
  if (tid < 256) lut[tid] = (double)tid / 255.0;  // Python int / 255 (correctly rounded)
  __syncthreads();
  const double sb = P.skin_bias, tb = P.saturation_bias, oi = P.outside_importance;
  // image totals of the three per-pixel terms (the outside part of every crop)
  {
    double t0 = 0, t1 = 0, t2 = 0;
    for (int p = tid; p < npx; p += kScoreThreads) {
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
    if (tid < 3) {
      double s = 0;
      for (int w = 0; w < kScoreWaves; w++) s += part[w][tid];
      T[tid] = s;
    }
    __syncthreads();
  }
  const double u = 1.1102230246251565e-16;  // 2^-53
  const double nn = (double)npx + 1.0;
  const double aoi = fabs(oi);
  const double wd = P.detail_weight, ws = P.skin_weight, wt = P.saturation_weight;

  // ---- fast pass: one wave per (crop, band of the window's rows), lanes
  // across the window's columns.  Bands (FI_SC_BANDS=1) balance the waves
  // when the crops are few (cfg2: 37 crops -> 74 items on 16 waves, not 3
  // rounds of 16 / 16 / 5) but measured slower (0.40 vs 0.37 ms per cfg2
  // step: per-item reductions), so the default is one band per crop.
  // F = sum_in (imp - oi) a + oi * total(a): the outside pixels need no pass,
  // the inside ones weigh by the table of fl(importance - oi) -- 7 f64
  // operations per (crop, pixel) instead of 10
  auto finalize = [&](int c, double sd, double ss, double st) {
    const DevCrop &cr = crops[D.crop0 + c];
    const double Fd = sd + oi * T[0], Fs = ss + oi * T[1], Ft = st + oi * T[2];
    // |python_sum - F| <= 6 gamma(n+4) (imax + imax2 + |oi|) total(a), a >= 0 (biases
    // >= 0, host-checked): python's sequential sum (5 gamma(n+1) sum |imp a|) plus
    // this pass (fl(imp - oi), one FMA per term, <= nin_y + 16 additions deep
    // with the band and wave reductions)
    const double g4 = (nn + 3.0) * u / (1.0 - (nn + 3.0) * u);
    const double kb = 6.0 * g4 * (cr.imax + cr.imax2 + aoi) * 1.0000001;
    const double Ed = kb * T[0], Es = kb * T[1], Et = kb * T[2];
    const double area = cr.fw * cr.fh;
    const double tot = (Fd * wd + Fs * ws + Ft * wt) / area;
    const double mag = fabs(wd) * (fabs(Fd) + Ed) + fabs(ws) * (fabs(Fs) + Es) + fabs(wt) * (fabs(Ft) + Et);
    const double B = ((fabs(wd) * Ed + fabs(ws) * Es + fabs(wt) * Et) * (1.0 + 16.0 * u) + 16.0 * u * mag) /
                     area * 1.01;
    if (!big) {
      s_tot[c] = tot;
      s_bnd[c] = B;
    }
    CropScore &o = sco[c];
    o.detail = Fd;
    o.saturation = Ft;
    o.skin = Fs;
    o.total = tot;
    o.bound = B;
    o.exact = 0;
  };
  const int nbands = big || !kScoreBands ? 1 : max(1, min(min(8, kScoreMaxCrops / ncrops), (4 * kScoreWaves + ncrops - 1) / ncrops));
  const int nitems = ncrops * nbands;
  for (int item = __builtin_amdgcn_readfirstlane(wave); item < nitems; item += kScoreWaves) {
    const int c = item / nbands, band = item - c * nbands;
    const DevCrop cr = crops[D.crop0 + c];
    const int bh = (cr.nin_y + nbands - 1) / nbands;
    const int ya = min(cr.nin_y, band * bh), yb = min(cr.nin_y, ya + bh);
    const int t2w = cr.table2_w;
    const __amdgpu_buffer_rsrc_t trs =
        __builtin_amdgcn_make_buffer_rsrc((void *)(ad + cr.table2), (short)0, cr.nin_y * t2w * 8, 0x00020000);
    double sd = 0, ss = 0, st = 0;
    auto row_terms = [&](uint32_t m, double imp) {
      const double d = lut[(m >> 8) & 255];
      const double a1 = lut[m & 255] * (d + sb);
      const double a2 = lut[(m >> 16) & 255] * (d + tb);
      sd = fma(imp, d, sd);
      ss = fma(imp, a1, ss);
      st = fma(imp, a2, st);
    };
    for (int dx0 = 0; dx0 < cr.nin_x; dx0 += 64) {
      const int dx = dx0 + lane;
      // LDS maps: lanes past the window read whatever lies there (finite
      // terms) and weigh it by the table's zero padding, so no lane test and
      // the table rows load by scalar base + lane offset; global maps keep
      // the column clamp (the read must stay inside the buffer)
      const bool act = LDS_MAPS || dx < cr.nin_x;
      const int dxc = act ? dx : 0;
      const uint32_t *mcol = maps + (int64_t)cr.y0 * W + cr.x0 + dxc;
      // table row r, column dxc: buffer load, row offset in an SGPR
      auto tload = [&](int r) {
        return __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(trs, 8u * (uint32_t)dxc,
                                                                               (uint32_t)(r * t2w * 8), 0));
      };
      // rows in groups of 4: the four map words, then the four table values,
      // go out together (a conditional read put an exec-masked block and a
      // full LDS wait between consecutive rows)
      int dy = ya;
#pragma unroll 1
      for (; dy + 4 <= yb; dy += 4) {
        uint32_t m[4];
        double imp[4];
#pragma unroll
        for (int u = 0; u < 4; u++) m[u] = mcol[(dy + u) * W];
#pragma unroll
        for (int u = 0; u < 4; u++) imp[u] = tload(dy + u);
#pragma unroll
        for (int u = 0; u < 4; u++) row_terms(act ? m[u] : 0u, imp[u]);  // m = 0: every term is 0
      }
#pragma unroll 1
      for (; dy < yb; dy++) {
        const uint32_t m = mcol[dy * W];
        row_terms(act ? m : 0u, tload(dy));
      }
    }
    sd = wave_sum(sd);
    ss = wave_sum(ss);
    st = wave_sum(st);
    if (lane == 0) {
      if (nbands == 1) {
        finalize(c, sd, ss, st);
      } else {
        s_part[item][0] = sd;
        s_part[item][1] = ss;
        s_part[item][2] = st;
      }
    }
  }
  if (nbands > 1) {
    __syncthreads();
    for (int c = tid; c < ncrops; c += kScoreThreads) {
      double sd = 0, ss = 0, st = 0;  // bands in order: deterministic
      for (int k = 0; k < nbands; k++) {
        sd += s_part[c * nbands + k][0];
        ss += s_part[c * nbands + k][1];
        st += s_part[c * nbands + k][2];
      }
      finalize(c, sd, ss, st);
    }
  }
  __syncthreads();
  // candidates: every crop whose interval reaches the best lower bound
  auto tot_of = [&](int c) { return big ? sco[c].total : s_tot[c]; };
  auto bnd_of = [&](int c) { return big ? sco[c].bound : s_bnd[c]; };
  if (tid == 0) {
    double best_lo = -1.0e308;
    for (int c = 0; c < ncrops; c++) best_lo = fmax(best_lo, tot_of(c) - bnd_of(c));
    int k = 0, first = -1;
    for (int c = 0; c < ncrops; c++)
      if (D.exact_all || tot_of(c) + bnd_of(c) >= best_lo) {
        if (first < 0) first = c;
        if (big)
          sco[c].exact = 2;
        else
          cand[k] = c;
        k++;
      }
    ncand_s = k;
    first_cand_s = first;
  }
  __syncthreads();
  const int ncand = ncand_s;
  const bool need_exact = D.exact_all || ncand > 1;
  if (need_exact) {
    // exact re-score: one lane per candidate, the reference's row-major order
    for (int k = tid; k < (big ? ncrops : ncand); k += kScoreThreads) {
      if (big && sco[k].exact != 2) continue;
      const int c = big ? k : cand[k];
      const DevCrop cr = crops[D.crop0 + c];
      const double *tab = ad + cr.table;
      double skin = 0, detail = 0, sat = 0;
      for (int y = 0; y < H; y++) {
        const bool yin = y >= cr.y0 && y < cr.y0 + cr.nin_y;
        const uint32_t *mrow = maps + (int64_t)y * W;
        const int64_t trow = (int64_t)(y - cr.y0) * cr.table_w - cr.x0;
#pragma unroll 4
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
      if (!big) s_tot[c] = tot;
      CropScore &o = sco[c];
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
    int top = first_cand_s;
    double best = tot_of(top);
    if (need_exact) {
      best = -9223372036854775807.0;  // -sys.maxsize; strict > keeps the first max
      // candidates in crop order (the re-scored ones carry exact = 1)
      for (int k = 0; k < (big ? ncrops : ncand); k++) {
        const int c = big ? k : cand[k];
        if (big && sco[c].exact != 1) continue;
        const double v = tot_of(c);
        if (v > best) {
          best = v;
          top = c;
        }
      }
    }
    if (big && !need_exact) sco[top].exact = 0;  // the one candidate's mark (fast score kept)
    results[D.result].top = top;
    results[D.result].n_candidates = ncand;
    results[D.result].total = best;
  }
}

// ---------------------------------------------------------------------------
// k_sc_score3: k_sc_score2's fast pass as exact-integer MFMA (fi_internal.h
// ScGroup).  One 16-wave workgroup per image:
//   1. the maps -> seven signed-byte planes in LDS (edge, skin, sat and the
//      low / high bytes of skin * edge, sat * edge, each as value - 128) and
//      the f64 image totals of the three terms (the outside part);
//   2. the waves take the groups' rows r = wave, wave + 16, ...: per 64-px
//      k-step, the B fragment (digits of Tq over that row segment, one per
//      y slot) from the host table, and per plane one MFMA whose A rows are
//      the 16 x origins' 64 pixels -- D[plane][x origin][digit, slot] sums
//      sum_window Tq_digit (value - 128) exactly in int32;
//   3. cross-wave sums in LDS (the planes are dead), then per crop
//        sum_in Tq x = sum_digit 256^digit D + 128 sum_window Tq
//      for x = edge, skin, sat, skin * edge, sat * edge, and the three terms
//        detail     = 2^-q sum Tq e / 255
//        skin       = 2^-q (sum Tq s e / 65025 + skin_bias sum Tq s / 255)
//        saturation = 2^-q (sum Tq t e / 65025 + sat_bias sum Tq t / 255)
//      are the exact-real sums of (importance - oi) a over the window, up to
//      the quantisation of Tq; F = that + oi total(a) as in k_sc_score2;
//   4. the rigorous bound, candidates, the exact sequential re-score and the
//      argmax exactly as k_sc_score2 (maps reloaded into LDS when needed).
// Bound per term (a >= 0: biases >= 0, host-checked):
//   |python - F| <= [2 gamma(n+5) (imax + |oi|) + 2^-(q+1) + |oi| gamma(n+16)]
//                   total(a) (1 + gamma(n+16)) + gamma(24) |F|_abs
// python's per-term roundings and sequential sum, the rint of Tq, the f64
// image totals (from exact integer sums), and the f64 combination of the integer sums (its absolute
// value carried alongside).
constexpr int kS3Threads = 1024;
constexpr int kS3Waves = kS3Threads / 64;
constexpr int kS3Pre = 8;  // plane items per thread with their map loads in flight together
#ifndef FI_S3_ABL
#define FI_S3_ABL 0
#endif
constexpr int kS3Abl = FI_S3_ABL;  // profiling ablations (wrong scores): 1 no MFMA pass, 2 no plane build, 4 no finalize

__global__ __launch_bounds__(kS3Threads) void k_sc_score3(const ScDesc *__restrict__ descs,
                                                          const DevCrop *__restrict__ crops,
                                                          const ScGroup *__restrict__ groups,
                                                          const double *__restrict__ ad,
                                                          CropScore *__restrict__ scores,
                                                          ScResult *__restrict__ results, const ScParamsDev P,
                                                          const int32_t *__restrict__ ai) {
  typedef __attribute__((address_space(3))) const i32x2 l_ci32x2;
  extern __shared__ __attribute__((aligned(16))) uint8_t lds3[];
  __shared__ double lut[256];
  __shared__ uint32_t ipart[kS3Waves][5];
  __shared__ double T[3];
  __shared__ double s_tot[kSgMaxCrops];
  __shared__ double s_bnd[kSgMaxCrops];
  __shared__ int32_t cand[kSgMaxCrops];
  __shared__ int32_t ncand_s, first_cand_s;
  const ScDesc &D = descs[blockIdx.x];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int ncrops = D.ncrops;
  CropScore *const sco = scores + D.score0;
  const int W = D.aw, H = D.ah, npx = W * H;
  const int pitch = sg_pitch(W), psz = H * pitch;
  const int ng = D.ngrp;
  const ScGroup *G = groups + D.sg0;
  const double sb = P.skin_bias, tb = P.saturation_bias, oi = P.outside_importance;
  if (tid < 256) lut[tid] = (double)tid / 255.0;  // Python int / 255 (correctly rounded)
  __syncthreads();
  // ---- 1. planes + image totals ----
  // items (row, 4-pixel quad), kS3Pre per thread with every map load in flight
  // before the first is used; the totals as exact integer sums (sum e, s, t,
  // s e, t e) turned into the three f64 terms at the end (|error| <= 3 u T)
  {
    const int nq = (W + 3) >> 2, nit = H * nq;
    uint32_t se_s = 0, te_s = 0, e_s = 0, s_s = 0, t_s = 0;
#pragma unroll 1
    for (int base = 0; base < ((kS3Abl & 2) ? 0 : nit); base += kS3Pre * kS3Threads) {
      uint32_t mm[kS3Pre][4];
#pragma unroll
      for (int j = 0; j < kS3Pre; j++) {
        const int it = base + tid + j * kS3Threads;
        const int y = it / nq, x = 4 * (it - y * nq);
#pragma unroll
        for (int k = 0; k < 4; k++) mm[j][k] = (it < nit && x + k < W) ? D.maps[(int64_t)y * W + x + k] : 0u;
      }
#pragma unroll
      for (int j = 0; j < kS3Pre; j++) {
        const int it = base + tid + j * kS3Threads;
        if (it >= nit) break;
        const int y = it / nq, x = 4 * (it - y * nq);
        uint32_t pl[kSgPlanes] = {0, 0, 0, 0, 0, 0, 0};
#pragma unroll
        for (int k = 0; k < 4; k++) {
          const uint32_t m = mm[j][k];  // 0 past the row end: adds nothing
          const uint32_t sk = m & 255u, e = (m >> 8) & 255u, t = (m >> 16) & 255u;
          const uint32_t se = sk * e, te = t * e;
          pl[0] |= e << (8 * k);
          pl[1] |= sk << (8 * k);
          pl[2] |= t << (8 * k);
          pl[3] |= (se & 255u) << (8 * k);
          pl[4] |= (se >> 8) << (8 * k);
          pl[5] |= (te & 255u) << (8 * k);
          pl[6] |= (te >> 8) << (8 * k);
          e_s += e;
          s_s += sk;
          t_s += t;
          se_s += se;
          te_s += te;
        }
#pragma unroll
        for (int p = 0; p < kSgPlanes; p++)
          *reinterpret_cast<uint32_t *>(lds3 + p * psz + y * pitch + x) = pl[p] ^ 0x80808080u;  // value - 128
      }
    }
    // wave sums (each < 2^32: <= 22.7 K pixels per image fit k_sc_score3's LDS)
    uint32_t v5[5] = {e_s, s_s, t_s, se_s, te_s};
#pragma unroll
    for (int i = 0; i < 5; i++)
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) v5[i] += __shfl_xor(v5[i], o, 64);
    if (lane == 0)
#pragma unroll
      for (int i = 0; i < 5; i++) ipart[wave][i] = v5[i];
    __syncthreads();
    if (tid == 0) {
      uint64_t S5[5] = {0, 0, 0, 0, 0};
      for (int w = 0; w < kS3Waves; w++)
        for (int i = 0; i < 5; i++) S5[i] += ipart[w][i];
      T[0] = (double)S5[0] / 255.0;
      T[1] = (double)S5[3] / 65025.0 + sb * ((double)S5[1] / 255.0);
      T[2] = (double)S5[4] / 65025.0 + tb * ((double)S5[2] / 255.0);
    }
  }
  // ---- 2. MFMA pass: the waves split between the groups in proportion to
  // their rows (one group's accumulators per wave); a wave takes rows
  // r, r + nw, ... of its group, each row's B fragments (L2) loaded three of
  // its rows ahead ----
  int gw = 0, w0 = 0, nw = kS3Waves;
  if (ng == 2) {
    const int r0 = G[0].nrows, r1 = G[1].nrows;
    const int n0 = min(kS3Waves - 1, max(1, (kS3Waves * r0 + (r0 + r1) / 2) / (r0 + r1)));
    if (wave >= n0) {
      gw = 1;
      w0 = n0;
      nw = kS3Waves - n0;
    } else {
      nw = n0;
    }
  }
  i32x4 acc[kSgPlanes];
#pragma unroll
  for (int p = 0; p < kSgPlanes; p++) acc[p] = i32x4{0, 0, 0, 0};
  if (!(kS3Abl & 1)) {
    const ScGroup *Gg = G + gw;
    const int nrows = __builtin_amdgcn_readfirstlane(Gg->nrows);
    const int ks = __builtin_amdgcn_readfirstlane(Gg->ks);
    const int ybase = __builtin_amdgcn_readfirstlane(Gg->ybase);
    const int nB = kSgDigits * __builtin_amdgcn_readfirstlane(Gg->nslot);
    const bool bl = (lane & 15) < nB;
    const i32x4 *bf = reinterpret_cast<const i32x4 *>(ai + Gg->bfrag);
    const int aoff = Gg->x0[lane & 15] + 16 * (lane >> 4);
    auto loadb = [&](int r, i32x4 (&b)[kSgMaxKs]) {
#pragma unroll
      for (int t = 0; t < kSgMaxKs; t++)
        b[t] = (r < nrows && t < ks && bl) ? bf[((int64_t)r * ks + t) * 64 + lane] : i32x4{0, 0, 0, 0};
    };
    auto row = [&](int r, const i32x4 (&b)[kSgMaxKs]) {
      const uint8_t *rowp = lds3 + (ybase + r) * pitch + aoff;
#pragma unroll
      for (int t = 0; t < kSgMaxKs; t++) {
        if (t < ks) {
#pragma unroll
          for (int p = 0; p < kSgPlanes; p++) {
            const uint8_t *a = rowp + p * psz + 64 * t;
            const i32x2 lo = *(l_ci32x2 *)(const __attribute__((address_space(3))) uint8_t *)a;
            const i32x2 hi = *(l_ci32x2 *)(const __attribute__((address_space(3))) uint8_t *)(a + 8);
            acc[p] = __builtin_amdgcn_mfma_i32_16x16x64_i8(i32x4{lo.x, lo.y, hi.x, hi.y}, b[t], acc[p], 0, 0, 0);
          }
        }
      }
    };
    const int rs = wave - w0;
    i32x4 b0[kSgMaxKs], b1[kSgMaxKs], b2[kSgMaxKs];
    loadb(rs, b0);
    loadb(rs + nw, b1);
    loadb(rs + 2 * nw, b2);
#pragma unroll 1
    for (int r = rs; r < nrows; r += 3 * nw) {
      row(r, b0);
      loadb(r + 3 * nw, b0);
      if (r + nw < nrows) row(r + nw, b1);
      loadb(r + 4 * nw, b1);
      if (r + 2 * nw < nrows) row(r + 2 * nw, b2);
      loadb(r + 5 * nw, b2);
    }
  }
  // ---- 3. cross-wave sums (the planes are dead), then per crop ----
  __syncthreads();
  int32_t *red = reinterpret_cast<int32_t *>(lds3);  // [g][plane][16 x origins][16 (digit, slot)]
  auto red_at = [&](int g, int p, int i) { return ((g * kSgPlanes + p) * 16 + 4 * (lane >> 4) + i) * 16 + (lane & 15); };
  // the first wave of each group stores, the others add
  if (wave == w0) {
#pragma unroll
    for (int p = 0; p < kSgPlanes; p++)
#pragma unroll
      for (int i = 0; i < 4; i++) red[red_at(gw, p, i)] = acc[p][i];
  }
  __syncthreads();
  if (wave != w0) {
#pragma unroll
    for (int p = 0; p < kSgPlanes; p++)
#pragma unroll
      for (int i = 0; i < 4; i++) atomicAdd(&red[red_at(gw, p, i)], acc[p][i]);
  }
  __syncthreads();
  const double u = 1.1102230246251565e-16;  // 2^-53
  auto gam = [&](double n) { return n * u / (1.0 - n * u); };
  const double aoi = fabs(oi);
  const double wd = P.detail_weight, ws = P.skin_weight, wt = P.saturation_weight;
  if (kS3Abl & 4)
    for (int c = tid; c < ncrops; c += kS3Threads) {
      s_tot[c] = c;  // one candidate, no re-score
      s_bnd[c] = 0;
    }
  for (int c = tid; c < ((kS3Abl & 4) ? 0 : ncrops); c += kS3Threads) {
    const DevCrop cr = crops[D.crop0 + c];
    const ScGroup &Gr = G[cr.sg];
    double V[kSgPlanes], A[kSgPlanes];
#pragma unroll
    for (int p = 0; p < kSgPlanes; p++) {
      V[p] = 0;
      A[p] = 0;
#pragma unroll
      for (int k = 0; k < kSgDigits; k++) {
        const double v = ldexp((double)red[((cr.sg * kSgPlanes + p) * 16 + cr.sm) * 16 + kSgDigits * cr.sj + k], 8 * k);
        V[p] += v;
        A[p] += fabs(v);
      }
    }
    double S = 0, AS = 0;
#pragma unroll
    for (int k = 0; k < kSgDigits; k++) {
      const double v = ldexp(128.0 * (double)Gr.S[k], 8 * k);
      S += v;
      AS += fabs(v);
    }
    // sum_window Tq x (x = e, s, t, s e, t e) and their absolute counterparts
    const double xe = V[0] + S, xs = V[1] + S, xt = V[2] + S;
    const double xse = 256.0 * (V[4] + S) + (V[3] + S), xte = 256.0 * (V[6] + S) + (V[5] + S);
    const double ae = A[0] + AS, as = A[1] + AS, at = A[2] + AS;
    const double ase = 256.0 * (A[4] + AS) + (A[3] + AS), ate = 256.0 * (A[6] + AS) + (A[5] + AS);
    const double sc = ldexp(1.0, -Gr.q);
    const double Fd = xe * sc / 255.0 + oi * T[0];
    const double Fs = (xse / 65025.0 + sb * xs / 255.0) * sc + oi * T[1];
    const double Ft = (xte / 65025.0 + tb * xt / 255.0) * sc + oi * T[2];
    const double Ad = ae * sc / 255.0 + aoi * T[0];
    const double As = (ase / 65025.0 + sb * as / 255.0) * sc + aoi * T[1];
    const double At = (ate / 65025.0 + tb * at / 255.0) * sc + aoi * T[2];
    const double nn = (double)npx;
    const double kb = (2.0 * gam(nn + 5.0) * (cr.imax + aoi) + ldexp(1.0, -Gr.q - 1) + aoi * gam(nn + 16.0)) *
                      (1.0 + gam(nn + 16.0));
    const double Ed = kb * T[0] + gam(24.0) * Ad, Es = kb * T[1] + gam(24.0) * As, Et = kb * T[2] + gam(24.0) * At;
    const double area = cr.fw * cr.fh;
    const double tot = (Fd * wd + Fs * ws + Ft * wt) / area;
    const double mag = fabs(wd) * (fabs(Fd) + Ed) + fabs(ws) * (fabs(Fs) + Es) + fabs(wt) * (fabs(Ft) + Et);
    const double B = ((fabs(wd) * Ed + fabs(ws) * Es + fabs(wt) * Et) * (1.0 + 16.0 * u) + 16.0 * u * mag) /
                     area * 1.01;
    s_tot[c] = tot;
    s_bnd[c] = B;
    CropScore &o = sco[c];
    o.detail = Fd;
    o.saturation = Ft;
    o.skin = Fs;
    o.total = tot;
    o.bound = B;
    o.exact = 0;
  }
  __syncthreads();
  // ---- 4. candidates, exact re-score, argmax (k_sc_score2's non-"big" path) ----
  if (tid == 0) {
    double best_lo = -1.0e308;
    for (int c = 0; c < ncrops; c++) best_lo = fmax(best_lo, s_tot[c] - s_bnd[c]);
    int k = 0, first = -1;
    for (int c = 0; c < ncrops; c++)
      if (D.exact_all || s_tot[c] + s_bnd[c] >= best_lo) {
        if (first < 0) first = c;
        cand[k++] = c;
      }
    ncand_s = k;
    first_cand_s = first;
  }
  __syncthreads();
  const int ncand = ncand_s;
  const bool need_exact = D.exact_all || ncand > 1;
  if (need_exact) {
    uint32_t *smaps = reinterpret_cast<uint32_t *>(lds3);
    for (int k = tid; k < npx; k += kS3Threads) smaps[k] = D.maps[k];
    __syncthreads();
    for (int k = tid; k < ncand; k += kS3Threads) {
      const int c = cand[k];
      const DevCrop cr = crops[D.crop0 + c];
      const double *tab = ad + cr.table;
      double skin = 0, detail = 0, sat = 0;
      for (int y = 0; y < H; y++) {
        const bool yin = y >= cr.y0 && y < cr.y0 + cr.nin_y;
        const uint32_t *mrow = smaps + (int64_t)y * W;
        const int64_t trow = (int64_t)(y - cr.y0) * cr.table_w - cr.x0;
#pragma unroll 4
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
      CropScore &o = sco[c];
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
    int top = first_cand_s;
    double best = s_tot[top];
    if (need_exact) {
      best = -9223372036854775807.0;  // -sys.maxsize; strict > keeps the first max
      for (int k = 0; k < ncand; k++) {
        const int c = cand[k];
        if (s_tot[c] > best) {
          best = s_tot[c];
          top = c;
        }
      }
    }
    results[D.result].top = top;
    results[D.result].n_candidates = ncand;
    results[D.result].total = best;
  }
}

// ---------------------------------------------------------------------------
// convert <out> -crop WxH+X+Y with W = w + x, H = h + y as smartcrop.py prints
// them (:372-377); CropImage clips to the image.  kApplyBands workgroups per
// image, rows interleaved.
#ifndef FI_APPLY_WG
#define FI_APPLY_WG 8
#endif
constexpr int kApplyChunks = FI_APPLY_WG;  // workgroups per image
// The output is one contiguous byte array (oh rows of ow * C bytes): 16-byte
// destination chunks, each assembled from 5 aligned source dwords with
// v_alignbyte (the crop origin has any byte alignment); chunks that straddle a
// row end, and the unaligned head/tail of the array, go byte by byte.
__device__ __forceinline__ uint32_t ap_align(uint32_t hi, uint32_t lo, uint32_t sh) {
  return __builtin_amdgcn_alignbyte(hi, lo, sh);
}
#ifndef FI_APPLY_U
#define FI_APPLY_U 2
#endif
constexpr int kApplyU = FI_APPLY_U;  // chunks per thread whose loads go out together
// one (image, part) of the crop copy: part of nparts workgroup-sized slices
__device__ __forceinline__ void crop_apply_item(const ApplyDesc *__restrict__ descs, const DevCrop *__restrict__ crops,
                                                const ScResult *__restrict__ results, int img, int part, int nparts) {
  const ApplyDesc &A = descs[img];
  const ScResult r = results[A.result];
  if (r.top < 0) return;
  const DevCrop c = crops[A.crop0 + r.top];
  const int gw = c.rw + c.rx, gh = c.rh + c.ry;
  const int ow = min(gw, A.W - c.rx), oh = min(gh, A.H - c.ry);
  if (part == 0 && threadIdx.x == 0) {
    A.out_wh[0] = ow;
    A.out_wh[1] = oh;
  }
  const int rowb = ow * A.C;
  const int64_t total = (int64_t)rowb * oh;
  if (total <= 0) return;
  const uint8_t *src0 = A.src + (int64_t)c.ry * A.src_stride + (int64_t)c.rx * A.C;
  // (row, byte) of output offset o: float reciprocal + exact correction (no
  // 64-bit division; total = rowb * oh < 2^31 for any thumbnail)
  const float inv_rowb = 1.0f / (float)rowb;
  auto rowcol = [&](int64_t o, int *y_, int *x_) {
    const int oo = (int)o;
    int y = (int)((float)oo * inv_rowb);
    int x = oo - y * rowb;
    while (x < 0) {
      y--;
      x += rowb;
    }
    while (x >= rowb) {
      y++;
      x -= rowb;
    }
    *y_ = y;
    *x_ = x;
  };
  auto src_of = [&](int64_t o) {
    int y, x;
    rowcol(o, &y, &x);
    return src0 + (int64_t)y * A.src_stride + x;
  };
  const int head = (int)((16 - ((uintptr_t)A.dst & 15)) & 15);
  const int64_t nchunk = head < total ? (total - head) / 16 : 0;
  const int64_t tail0 = head + 16 * nchunk;
  const int tid = threadIdx.x;
  if (part == 0) {
    for (int64_t o = tid; o < min<int64_t>(head, total); o += 256) A.dst[o] = *src_of(o);
    for (int64_t o = tail0 + tid; o < total; o += 256) A.dst[o] = *src_of(o);
  }
  const int64_t cs = (int64_t)nparts * 256;
  for (int64_t k0 = (int64_t)part * 256 + tid; k0 < nchunk; k0 += kApplyU * cs) {
    uint4 out[kApplyU];
#pragma unroll
    for (int u = 0; u < kApplyU; u++) {
      const int64_t k = k0 + u * cs;
      if (k >= nchunk) break;
      const int64_t o = head + 16 * k;
      int y, x;
      rowcol(o, &y, &x);
      if (x + 16 <= rowb) {
        const uint8_t *s = src0 + (int64_t)y * A.src_stride + x;
        const uint32_t *sa = reinterpret_cast<const uint32_t *>((uintptr_t)s & ~(uintptr_t)3);
        const uint32_t sh = (uint32_t)((uintptr_t)s & 3);
        const uint32_t w0 = sa[0], w1 = sa[1], w2 = sa[2], w3 = sa[3], w4 = sh ? sa[4] : 0u;
        out[u].x = ap_align(w1, w0, sh);
        out[u].y = ap_align(w2, w1, sh);
        out[u].z = ap_align(w3, w2, sh);
        out[u].w = ap_align(w4, w3, sh);
      } else {
        uint8_t b[16];
        int yy = y, xx = x;
#pragma unroll
        for (int j = 0; j < 16; j++) {  // straddles a row end
          b[j] = src0[(int64_t)yy * A.src_stride + xx];
          if (++xx == rowb) {
            xx = 0;
            yy++;
          }
        }
        out[u].x = b[0] | (b[1] << 8) | (b[2] << 16) | ((uint32_t)b[3] << 24);
        out[u].y = b[4] | (b[5] << 8) | (b[6] << 16) | ((uint32_t)b[7] << 24);
        out[u].z = b[8] | (b[9] << 8) | (b[10] << 16) | ((uint32_t)b[11] << 24);
        out[u].w = b[12] | (b[13] << 8) | (b[14] << 16) | ((uint32_t)b[15] << 24);
      }
    }
#pragma unroll
    for (int u = 0; u < kApplyU; u++) {
      const int64_t k = k0 + u * cs;
      if (k >= nchunk) break;
      *reinterpret_cast<uint4 *>(A.dst + head + 16 * k) = out[u];
    }
  }
}
__global__ __launch_bounds__(256) void k_crop_apply3(const ApplyDesc *__restrict__ descs,
                                                     const DevCrop *__restrict__ crops,
                                                     const ScResult *__restrict__ results) {
  crop_apply_item(descs, crops, results, blockIdx.y, blockIdx.x, gridDim.x);
}
// the same work from one workgroup per CU walking the (image, part) items: runs
// beside the next batch's persistent resample (no LDS, few VGPRs: it fits next
// to a 16-wave k_rs_vr workgroup, so neither kernel waits for the other's CUs)
__global__ __launch_bounds__(256, 8) void k_crop_apply3p(const ApplyDesc *__restrict__ descs,
                                                      const DevCrop *__restrict__ crops,
                                                      const ScResult *__restrict__ results, int n) {
  for (int item = blockIdx.x; item < n * kApplyChunks; item += gridDim.x)
    crop_apply_item(descs, crops, results, item / kApplyChunks, item % kApplyChunks, kApplyChunks);
}

int launch_sc_h(hipStream_t s, const ScDesc *descs, int n, int chunks, int lds, const int32_t *ai) {
  if (n <= 0 || chunks <= 0) return 0;
  if (lds > kHmMaxLds) return -1;
  hipLaunchKernelGGL(k_sc_hmfma, dim3(n, chunks), dim3(kPrepThreads), lds, s, descs, ai);
  return 0;
}
int launch_sc_skinsat(hipStream_t s, uint16_t *table, const ScParamsDev &P) {
  hipLaunchKernelGGL(k_sc_skinsat, dim3(1u << 16), dim3(256), 0, s, table, P);
  return 0;
}
int launch_sc_fz(hipStream_t s, const ScDesc *descs, int n, int lds, const int32_t *ai, const ScParamsDev &P,
                 const uint16_t *skinsat) {
  if (n <= 0) return 0;
  if (lds > kFzMaxLds || !skinsat) return -1;
  hipLaunchKernelGGL((k_sc_fz<true>), dim3(n), dim3(kFzThreads), lds, s, descs, ai, P, skinsat);
  return 0;
}
int launch_sc_fd(hipStream_t s, const ScDesc *descs, int n, int lds, const int32_t *ai, const ScParamsDev &P,
                 const uint16_t *skinsat) {
  if (n <= 0) return 0;
  if (lds > kFdMaxLds || !skinsat) return -1;
  hipLaunchKernelGGL(k_sc_fd, dim3(n), dim3(kFdThreads), lds, s, descs, ai, P, skinsat);
  return 0;
}
int launch_sc_vq(hipStream_t s, const ScDesc *descs, int n, int chunks, int lds, const int32_t *ai,
                 const ScParamsDev &P) {
  if (n <= 0) return 0;
  if (lds > kPrepMaxLds) return -1;
  hipLaunchKernelGGL(k_sc_vq, dim3(n, chunks), dim3(kPrepThreads), lds, s, descs, ai, P);
  return 0;
}
int launch_sc_v(hipStream_t s, const ScDesc *descs, int n, int chunks, int lds, const int32_t *ai,
                const ScParamsDev &P) {
  if (n <= 0) return 0;
  if (lds > kPrepMaxLds) return -1;
  hipLaunchKernelGGL(k_sc_vmaps, dim3(n, chunks), dim3(kPrepThreads), lds, s, descs, ai, P);
  return 0;
}
int launch_sc_score(hipStream_t s, int mode, const ScDesc *descs, int n, size_t lds, const DevCrop *crops,
                    const double *ad, CropScore *scores, ScResult *results, const ScParamsDev &P, const int32_t *ai) {
  if (n <= 0) return 0;
  if (mode == 1) {
    if (lds > (size_t)kScoreLdsMaps) return -1;
    hipLaunchKernelGGL((k_sc_score2<1>), dim3(n), dim3(kScoreThreads), lds, s, descs, crops, ad, scores, results, P,
                       ai);
  } else {
    hipLaunchKernelGGL((k_sc_score2<0>), dim3(n), dim3(kScoreThreads), 0, s, descs, crops, ad, scores, results, P,
                       ai);
  }
  return 0;
}
int launch_sc_score3(hipStream_t s, const ScDesc *descs, int n, size_t lds, const DevCrop *crops, const ScGroup *groups,
                     const double *ad, CropScore *scores, ScResult *results, const ScParamsDev &P, const int32_t *ai) {
  if (n <= 0) return 0;
  if (lds > (size_t)kScore3Lds) return -1;
  hipLaunchKernelGGL(k_sc_score3, dim3(n), dim3(kS3Threads), lds, s, descs, crops, groups, ad, scores, results, P,
                     ai);
  return 0;
}
int launch_crop_apply(hipStream_t s, const ApplyDesc *descs, int n, const DevCrop *crops, const ScResult *results,
                      int persistent_wgs) {
  if (n <= 0) return 0;
  if (persistent_wgs > 0)
    hipLaunchKernelGGL(k_crop_apply3p, dim3(min(persistent_wgs, n * kApplyChunks)), dim3(256), 0, s, descs, crops,
                       results, n);
  else
    hipLaunchKernelGGL(k_crop_apply3, dim3(kApplyChunks, n), dim3(256), 0, s, descs, crops, results);
  return 0;
}

}  // namespace fi
