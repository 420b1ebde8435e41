// fi_jpeg.hip -- baseline JPEG decode on the GPU, bit-exact with the
// libjpeg-turbo decoder the host codec path uses (Pillow 12.2.0 bundles
// libjpeg-turbo 3.x; SURVEY.md 8(f) 1: "nvJPEG-style batched decode").
//
//   host     marker parse (SOF0/SOF1 8-bit, DQT, DHT, DRI, one SOS), canonical
//            Huffman tables deduplicated over the batch, restart intervals
//            located by their RSTn markers;
//   k_jpeg_huff   one 64-lane workgroup per restart interval (the whole scan
//            when there is none), the lanes in lockstep on wave-uniform state,
//            the segment window spread over the lanes: jdhuff.c's sequential decode -- DC prediction, AC run /
//            size symbols, HUFF_EXTEND -- into int16 coefficient blocks in
//            zigzag order (the IDCT reads them back in natural order); byte stuffing and markers as jdhuff.c (a marker
//            feeds zero bits);
//   k_jpeg_idct   one thread per 8x8 block: jidctint.c jpeg_idct_islow
//            (dequantise, 13-bit constants, PASS1_BITS 2, range limit);
//   k_jpeg_color  one thread per output pixel: jdsample.c fancy upsampling
//            (h2v1 / h2v2 triangle filters, edge replication) and jdcolor.c
//            ycc_rgb_convert with its 16-bit fixed-point tables.
//
// Unsupported streams (progressive, arithmetic, 12-bit, CMYK / Adobe
// transforms, other samplings, several scans) return FI_EUNSUPPORTED from
// jpeg_parse so the caller decodes them on the host.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string.h>

#include <atomic>
#include <functional>
#include <map>
#include <string>
#include <thread>
#include <vector>

#include "fi_internal.h"
#include "fi_jpeg.h"

namespace fi {

// ---------------------------------------------------------------------------
// device: Huffman decode
// ---------------------------------------------------------------------------
constexpr int kJpegLdsTabs = 8;  // distinct Huffman tables staged in LDS (more: read from global)

typedef __attribute__((address_space(1))) const uint32_t g_u32;
// All 64 lanes of the workgroup decode the same interval in lockstep (the
// values are wave-uniform, so no lane diverges): the 256-byte window of the
// segment is spread over the lanes, lane i holding bytes [wbase + 4 i, + 4),
// read with v_readlane; the next 256 bytes are in flight in `nxt` (their
// latency hides behind the decode of the current window).  The segment is
// zero padded by >= 512 bytes.
struct BitReader {
  const uint8_t *p;
  uint32_t win, nxt;
  int wbase, pos, end;
  uint64_t buf;
  int nbits;
  bool marker;
  __device__ __forceinline__ void advance_window() {
    if (pos - wbase >= 256) {  // bytes [pos, pos + 4) stay inside win + the first dword of nxt
      win = nxt;
      wbase += 256;
      nxt = *(g_u32 *)(p + wbase + 256 + 4 * (threadIdx.x & 63));
    }
  }
  // the 4 bytes at pos, little-endian
  __device__ __forceinline__ uint32_t word_at_pos() const {
    const int o = __builtin_amdgcn_readfirstlane(pos - wbase), k = o >> 2;
    const uint32_t lo = __builtin_amdgcn_readlane(win, k);
    const uint32_t hi = k < 63 ? __builtin_amdgcn_readlane(win, k + 1) : __builtin_amdgcn_readfirstlane(nxt);
    return __builtin_amdgcn_alignbyte(hi, lo, (uint32_t)(o & 3));
  }
  __device__ void init(const uint8_t *ecs, int byte0, int len) {
    p = ecs;
    wbase = byte0 & ~255;
    win = *(g_u32 *)(p + wbase + 4 * (threadIdx.x & 63));
    nxt = *(g_u32 *)(p + wbase + 256 + 4 * (threadIdx.x & 63));
    pos = byte0;
    end = len;
    buf = 0;
    nbits = 0;
    marker = false;
  }
  // jdhuff.c jpeg_fill_bit_buffer: stuffed 0xFF00 -> 0xFF; at a marker (or the
  // end of the data) zero bits are supplied.  Called once per symbol: leaves
  // >= 32 bits, enough for a code (<= 16) and its value bits (<= 16); four
  // bytes at a time while they hold no 0xFF, else byte by byte.
  __device__ __forceinline__ void fill() {
    if (nbits >= 32) return;
    const uint32_t w = word_at_pos();
    const uint32_t t = ~w;
    const bool ff = ((t - 0x01010101u) & ~t & 0x80808080u) != 0u;  // some byte of w is 0xFF
    if (!ff && !marker && pos + 4 <= end) {
      buf = (buf << 32) | __builtin_bswap32(w);
      nbits += 32;
      pos += 4;
      advance_window();
      return;
    }
    while (nbits < 32) {
      uint32_t b = 0;
      if (!marker && pos < end) {
        const uint32_t x = word_at_pos();
        b = x & 255u;
        if (b == 0xFFu) {
          if (((x >> 8) & 255u) == 0u) {
            pos += 2;
          } else {
            marker = true;
            b = 0;
          }
        } else {
          pos++;
        }
        advance_window();
      }
      buf = (buf << 8) | b;
      nbits += 8;
    }
  }
  __device__ __forceinline__ uint32_t peek(int n) const { return (uint32_t)(buf >> (nbits - n)) & ((1u << n) - 1u); }
  __device__ __forceinline__ void skip(int n) { nbits -= n; }
};

template <typename TAB>
__device__ __forceinline__ int jpeg_decode_sym(BitReader &br, const TAB *t) {
  br.fill();
  const uint32_t lk = t->look[br.peek(9)];
  if (lk) {
    br.skip(lk >> 8);
    return lk & 255;
  }
  int l = 10;
  int32_t code = (int32_t)br.peek(10);
  while (l <= 16 && code > t->maxcode[l]) {
    l++;
    code = (int32_t)br.peek(l);
  }
  if (l > 16) {  // corrupt data: jdhuff.c warns and returns 0
    br.skip(0);
    return 0;
  }
  br.skip(l);
  return t->huffval[(code + t->valoff[l]) & 255];
}
__device__ __forceinline__ int jpeg_extend(uint32_t r, int s) {  // HUFF_EXTEND
  return r < (1u << (s - 1)) ? (int)r - (1 << s) + 1 : (int)r;
}

template <bool LDS>
__global__ __launch_bounds__(64) void k_jpeg_huff(const JpegDesc *__restrict__ descs,
                                                  const JpegInterval *__restrict__ ivs, int niv,
                                                  const JpegHuff *__restrict__ huff, int nhuff,
                                                  uint8_t *__restrict__ work) {
  __shared__ JpegHuff sh[kJpegLdsTabs];
  __shared__ __attribute__((aligned(16))) int16_t blk[64];
  const int tid = threadIdx.x;
  if (LDS) {
    const uint32_t *src = reinterpret_cast<const uint32_t *>(huff);
    uint32_t *dstw = reinterpret_cast<uint32_t *>(sh);
    const int nw = nhuff * (int)sizeof(JpegHuff) / 4;
    for (int i = tid; i < nw; i += 64) dstw[i] = src[i];
  }
  if (tid < 32) reinterpret_cast<uint32_t *>(blk)[tid] = 0;
  __syncthreads();
  const int iv = blockIdx.x;
  if (iv >= niv) return;
  const JpegInterval I = ivs[iv];
  const JpegDesc *Dp = descs + I.img;
  // the descriptor in registers (the block stores below may alias it for the
  // compiler: fields read through the pointer would be reloaded per block)
  const int ncomp = Dp->ncomp, mcux = Dp->mcux;
  int tdc[3], tac[3], hs[3], vs[3], bw[3];
  int64_t co[3];
#pragma unroll
  for (int c = 0; c < 3; c++) {
    const bool on = c < ncomp;
    tdc[c] = on ? Dp->ht[Dp->td[c]] : 0;
    tac[c] = on ? Dp->ht[2 + Dp->ta[c]] : 0;
    hs[c] = on ? Dp->h[c] : 0;
    vs[c] = on ? Dp->v[c] : 0;
    bw[c] = on ? Dp->bw[c] : 0;
    co[c] = on ? Dp->coef[c] : 0;
  }
  // the address space of the table reads is static: LDS reads (ds_read, ~100
  // cycles) or global ones, never flat pointers into either
  typedef __attribute__((address_space(3))) const JpegHuff l_huff;
  typedef __attribute__((address_space(1))) const JpegHuff g_huff;
  BitReader br;
  br.init(Dp->ecs, I.byte0, Dp->ecs_len);
  int pred[3] = {0, 0, 0};  // DC predictions (static indices only: registers)
  int16_t *b = blk;
  for (int mcu = I.mcu0; mcu < I.mcu1; mcu++) {
    const int my = mcu / mcux, mx = mcu - my * mcux;
#pragma unroll
    for (int c = 0; c < 3; c++) {
      if (c >= ncomp) break;
      for (int by = 0; by < vs[c]; by++)
        for (int bx = 0; bx < hs[c]; bx++) {
          // DC: difference from the component's previous block
          int s = LDS ? jpeg_decode_sym(br, (l_huff *)(sh + tdc[c])) : jpeg_decode_sym(br, (g_huff *)(huff + tdc[c]));
          if (s) {  // (the symbol's fill left enough bits for its value)
            const uint32_t r = br.peek(s);
            br.skip(s);
            s = jpeg_extend(r, s);
          }
          pred[c] += s;
          b[0] = (int16_t)pred[c];
          // AC: run / size symbols
          for (int k = 1; k < 64; k++) {
            br.fill();
            const int fa = LDS ? ((l_huff *)(sh + tac[c]))->fast_ac[br.peek(9)]
                               : ((g_huff *)(huff + tac[c]))->fast_ac[br.peek(9)];
            if (fa) {  // code + value in one lookahead
              k += (fa >> 4) & 15;
              br.skip(fa & 15);
              b[k < 63 ? k : 63] = (int16_t)(fa >> 8);
              continue;
            }
            const int rs = LDS ? jpeg_decode_sym(br, (l_huff *)(sh + tac[c]))
                               : jpeg_decode_sym(br, (g_huff *)(huff + tac[c]));
            const int r = rs >> 4, sz = rs & 15;
            if (sz) {
              k += r;
              const uint32_t v = br.peek(sz);
              br.skip(sz);
              b[k < 63 ? k : 63] = (int16_t)jpeg_extend(v, sz);  // zigzag order (k > 63: jpeg_natural_order's guard -> 63)
            } else {
              if (r != 15) break;
              k += 15;
            }
          }
          // block -> work (lanes 0-7: 16 bytes each), and clear the staging block
          const int row = my * vs[c] + by, col = mx * hs[c] + bx;
          if (tid < 8) {
            uint4 *o = reinterpret_cast<uint4 *>(work + co[c] + ((int64_t)row * bw[c] + col) * 128);
            uint4 *bb = reinterpret_cast<uint4 *>(b);
            o[tid] = bb[tid];
            bb[tid] = uint4{0, 0, 0, 0};
          }
        }
    }
  }
}

// ---------------------------------------------------------------------------
// device: islow IDCT (jidctint.c), one thread per block
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint8_t jpeg_range_limit(int x) {  // IDCT_range_limit[x & RANGE_MASK]
  const int m = x & 1023;
  const int v = (m >= 512 ? m - 1024 : m) + 128;
  return (uint8_t)(v < 0 ? 0 : v > 255 ? 255 : v);
}

// one thread per 8x8 block of the batch; blk0[j] = first block of the j-th
// (image, component) pair (3 pairs per image, empty ones for gray), blk0[3 n] = total
__device__ __forceinline__ void jpeg_idct_block(const JpegDesc *__restrict__ descs, const int64_t *__restrict__ blk0,
                                                int nimg, const uint16_t *__restrict__ qts, uint8_t *__restrict__ work,
                                                int64_t i);
// (grid-stride, as k_jpeg_color)
__global__ __launch_bounds__(256) void k_jpeg_idct(const JpegDesc *__restrict__ descs,
                                                   const int64_t *__restrict__ blk0, int nimg,
                                                   const uint16_t *__restrict__ qts, uint8_t *__restrict__ work) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < blk0[3 * nimg]; i += (int64_t)gridDim.x * 256)
    jpeg_idct_block(descs, blk0, nimg, qts, work, i);
}
__device__ __forceinline__ void jpeg_idct_block(const JpegDesc *__restrict__ descs, const int64_t *__restrict__ blk0,
                                                int nimg, const uint16_t *__restrict__ qts, uint8_t *__restrict__ work,
                                                int64_t i) {
  int lo = 0, hi = 3 * nimg;
  while (hi - lo > 1) {
    const int mid = (lo + hi) >> 1;
    if (blk0[mid] <= i)
      lo = mid;
    else
      hi = mid;
  }
  struct {
    int img, comp, blk;
  } R = {lo / 3, lo % 3, (int)(i - blk0[lo])};
  const JpegDesc &D = descs[R.img];
  const int c = R.comp;
  const int by = R.blk / D.bw[c], bx = R.blk - by * D.bw[c];
  const int16_t *in = reinterpret_cast<const int16_t *>(work + D.coef[c] + (int64_t)R.blk * 128);
  const uint16_t *q = qts + (int64_t)(D.qt + D.tq[c]) * 64;
  constexpr int CB = 13, P1 = 2;
  constexpr int F0298 = 2446, F0390 = 3196, F0541 = 4433, F0765 = 6270, F0899 = 7373, F1175 = 9633, F1501 = 12299,
                F1847 = 15137, F1961 = 16069, F2053 = 16819, F2562 = 20995, F3072 = 25172;
  int ws[64];
  int cf[64];
  // coefficient blocks are stored in zigzag order: natural k = jpeg_natural_order[z]
  constexpr uint8_t zz[64] = {0,  1,  8,  16, 9,  2,  3,  10, 17, 24, 32, 25, 18, 11, 4,  5,
                              12, 19, 26, 33, 40, 48, 41, 34, 27, 20, 13, 6,  7,  14, 21, 28,
                              35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23, 30, 37, 44, 51,
                              58, 59, 52, 45, 38, 31, 39, 46, 53, 60, 61, 54, 47, 55, 62, 63};
#pragma unroll
  for (int z = 0; z < 64; z++) cf[zz[z]] = (int)in[z] * (int)q[zz[z]];
  // pass 1: columns
#pragma unroll
  for (int x = 0; x < 8; x++) {
    int z2 = cf[16 + x], z3 = cf[48 + x];
    int z1 = (z2 + z3) * F0541;
    int tmp2 = z1 + z3 * (-F1847);
    int tmp3 = z1 + z2 * F0765;
    z2 = cf[x];
    z3 = cf[32 + x];
    int tmp0 = (z2 + z3) * (1 << CB);
    int tmp1 = (z2 - z3) * (1 << CB);
    const int tmp10 = tmp0 + tmp3, tmp13 = tmp0 - tmp3, tmp11 = tmp1 + tmp2, tmp12 = tmp1 - tmp2;
    tmp0 = cf[56 + x];
    tmp1 = cf[40 + x];
    tmp2 = cf[24 + x];
    tmp3 = cf[8 + x];
    z1 = tmp0 + tmp3;
    z2 = tmp1 + tmp2;
    z3 = tmp0 + tmp2;
    int z4 = tmp1 + tmp3;
    const int z5 = (z3 + z4) * F1175;
    tmp0 *= F0298;
    tmp1 *= F2053;
    tmp2 *= F3072;
    tmp3 *= F1501;
    z1 *= -F0899;
    z2 *= -F2562;
    z3 *= -F1961;
    z4 *= -F0390;
    z3 += z5;
    z4 += z5;
    tmp0 += z1 + z3;
    tmp1 += z2 + z4;
    tmp2 += z2 + z3;
    tmp3 += z1 + z4;
    constexpr int S = CB - P1, R1 = 1 << (S - 1);
    ws[x] = (tmp10 + tmp3 + R1) >> S;
    ws[56 + x] = (tmp10 - tmp3 + R1) >> S;
    ws[8 + x] = (tmp11 + tmp2 + R1) >> S;
    ws[48 + x] = (tmp11 - tmp2 + R1) >> S;
    ws[16 + x] = (tmp12 + tmp1 + R1) >> S;
    ws[40 + x] = (tmp12 - tmp1 + R1) >> S;
    ws[24 + x] = (tmp13 + tmp0 + R1) >> S;
    ws[32 + x] = (tmp13 - tmp0 + R1) >> S;
  }
  // pass 2: rows -> samples
  uint8_t *out = work + D.plane[c] + (int64_t)(by * 8) * (D.bw[c] * 8) + bx * 8;
  const int pitch = D.bw[c] * 8;
#pragma unroll
  for (int y = 0; y < 8; y++) {
    const int *w = ws + 8 * y;
    int z2 = w[2], z3 = w[6];
    int z1 = (z2 + z3) * F0541;
    int tmp2 = z1 + z3 * (-F1847);
    int tmp3 = z1 + z2 * F0765;
    int tmp0 = (w[0] + w[4]) * (1 << CB);
    int tmp1 = (w[0] - w[4]) * (1 << CB);
    const int tmp10 = tmp0 + tmp3, tmp13 = tmp0 - tmp3, tmp11 = tmp1 + tmp2, tmp12 = tmp1 - tmp2;
    tmp0 = w[7];
    tmp1 = w[5];
    tmp2 = w[3];
    tmp3 = w[1];
    z1 = tmp0 + tmp3;
    z2 = tmp1 + tmp2;
    z3 = tmp0 + tmp2;
    int z4 = tmp1 + tmp3;
    const int z5 = (z3 + z4) * F1175;
    tmp0 *= F0298;
    tmp1 *= F2053;
    tmp2 *= F3072;
    tmp3 *= F1501;
    z1 *= -F0899;
    z2 *= -F2562;
    z3 *= -F1961;
    z4 *= -F0390;
    z3 += z5;
    z4 += z5;
    tmp0 += z1 + z3;
    tmp1 += z2 + z4;
    tmp2 += z2 + z3;
    tmp3 += z1 + z4;
    constexpr int S = CB + P1 + 3, R2 = 1 << (S - 1);
    uint32_t lo = 0, hi = 0;
    lo |= (uint32_t)jpeg_range_limit((tmp10 + tmp3 + R2) >> S);
    lo |= (uint32_t)jpeg_range_limit((tmp11 + tmp2 + R2) >> S) << 8;
    lo |= (uint32_t)jpeg_range_limit((tmp12 + tmp1 + R2) >> S) << 16;
    lo |= (uint32_t)jpeg_range_limit((tmp13 + tmp0 + R2) >> S) << 24;
    hi |= (uint32_t)jpeg_range_limit((tmp13 - tmp0 + R2) >> S);
    hi |= (uint32_t)jpeg_range_limit((tmp12 - tmp1 + R2) >> S) << 8;
    hi |= (uint32_t)jpeg_range_limit((tmp11 - tmp2 + R2) >> S) << 16;
    hi |= (uint32_t)jpeg_range_limit((tmp10 - tmp3 + R2) >> S) << 24;
    *reinterpret_cast<uint2 *>(out + (int64_t)y * pitch) = uint2{lo, hi};
  }
}

// ---------------------------------------------------------------------------
// device: fancy upsampling + YCbCr -> RGB (jdsample.c, jdcolor.c)
// ---------------------------------------------------------------------------
// chroma sample of output pixel (x, y) for luma sampling (hs, vs) over 1x1 chroma
__device__ __forceinline__ int jpeg_up(const uint8_t *pl, int pitch, int dw, int dh, int hs, int vs, int x, int y) {
  if (hs == 1 && vs == 1) return pl[(int64_t)y * pitch + x];
  const int cx = x >> 1;
  const int cl = cx > 0 ? cx - 1 : 0, cr = cx < dw - 1 ? cx + 1 : dw - 1;
  const bool odd = x & 1;
  if (vs == 1) {  // h2v1_fancy_upsample
    const uint8_t *r = pl + (int64_t)y * pitch;
    return odd ? (3 * r[cx] + r[cr] + 2) >> 2 : (3 * r[cx] + r[cl] + 1) >> 2;
  }
  // h2v2_fancy_upsample: column sums 3 * nearer row + further row (edge rows replicated)
  const int cy = y >> 1;
  const int fy = (y & 1) ? (cy < dh - 1 ? cy + 1 : dh - 1) : (cy > 0 ? cy - 1 : 0);
  const uint8_t *r0 = pl + (int64_t)cy * pitch, *r1 = pl + (int64_t)fy * pitch;
  const int t = 3 * r0[cx] + r1[cx];
  if (odd) return (3 * t + 3 * r0[cr] + r1[cr] + 7) >> 4;
  return (3 * t + 3 * r0[cl] + r1[cl] + 8) >> 4;
}
__device__ __forceinline__ uint8_t jpeg_clamp(int v) { return (uint8_t)(v < 0 ? 0 : v > 255 ? 255 : v); }

__device__ __forceinline__ void jpeg_color_px(const JpegDesc *__restrict__ descs, const int64_t *__restrict__ px0,
                                              int nimg, const uint8_t *__restrict__ work, int64_t i) {
  // image of pixel i: binary search over the per-image pixel prefix
  int lo = 0, hi = nimg;
  while (hi - lo > 1) {
    const int mid = (lo + hi) >> 1;
    if (px0[mid] <= i)
      lo = mid;
    else
      hi = mid;
  }
  if (i >= px0[nimg]) return;
  const JpegDesc &D = descs[lo];
  const int64_t k = i - px0[lo];
  const int y = (int)(k / D.W), x = (int)(k - (int64_t)y * D.W);
  const int yp = D.bw[0] * 8;
  const uint8_t Y = work[D.plane[0] + (int64_t)y * yp + x];
  if (D.ncomp == 1) {
    uint8_t *o = D.dst + (int64_t)y * D.dst_stride + x * D.dst_c;
    for (int k = 0; k < D.dst_c; k++) o[k] = Y;
    return;
  }
  const int hs = D.h[0], vs = D.v[0];
  const int cb = jpeg_up(work + D.plane[1], D.bw[1] * 8, D.dw[1], D.dh[1], hs, vs, x, y);
  const int cr = jpeg_up(work + D.plane[2], D.bw[2] * 8, D.dw[2], D.dh[2], hs, vs, x, y);
  // build_ycc_rgb_table: FIX(x) = (int)(x * 65536 + 0.5), ONE_HALF = 1 << 15
  const int xr = cr - 128, xb = cb - 128;
  const int r = Y + ((91881 * xr + 32768) >> 16);
  const int g = Y + ((-22554 * xb + 32768 + -46802 * xr) >> 16);
  const int b = Y + ((116130 * xb + 32768) >> 16);
  uint8_t *o = D.dst + (int64_t)y * D.dst_stride + 3 * x;
  o[0] = jpeg_clamp(r);
  o[1] = jpeg_clamp(g);
  o[2] = jpeg_clamp(b);
}

// (grid-stride: a dispatch's work-item count is 32-bit, a batch may hold more pixels)
__global__ __launch_bounds__(256) void k_jpeg_color(const JpegDesc *__restrict__ descs, const int64_t *__restrict__ px0,
                                                    int nimg, const uint8_t *__restrict__ work) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < px0[nimg]; i += (int64_t)gridDim.x * 256)
    jpeg_color_px(descs, px0, nimg, work, i);
}

// ---------------------------------------------------------------------------
// host: batch plan + launches
// ---------------------------------------------------------------------------
// Plans and runs one decode batch.  `alloc(which, bytes)` returns memory that
// stays valid until the stream has run: 0 device upload (compressed data +
// tables), 2 device work (coefficients + planes), 3 pinned host staging.
int jpeg_decode_batch(hipStream_t st, const uint8_t *const *data, const size_t *len, int n, uint8_t *const *dst,
                      const int64_t *dst_stride, int out_channels, int32_t *status,
                      void *(*alloc)(void *, int, size_t), void *actx, std::string *err) {
  std::vector<JpegHdr> hd(n);
  std::vector<int> ok(n, 0);
  std::map<std::string, int> huff_ix;
  std::vector<JpegHuff> huffs;
  std::vector<uint16_t> qts;
  std::vector<JpegDesc> descs;
  std::vector<int> desc_img;
  std::vector<JpegInterval> ivs;
  std::vector<int64_t> blk0;  // first block of each (image, component)
  int64_t nblocks = 0;
  std::vector<int64_t> px0(1, 0);
  size_t ecs_total = 0, work_total = 0;
  // header parse (incl. the scan for the end of each entropy-coded segment)
  // and, below, the staging copies run on a few host threads
  const int nthr = (int)std::min<size_t>(8, std::max<size_t>(1, (size_t)n / 16));
  auto parallel = [&](int count, const std::function<void(int)> &fn) {
    if (nthr <= 1 || count < 2) {
      for (int i = 0; i < count; i++) fn(i);
      return;
    }
    std::atomic<int> next(0);
    std::vector<std::thread> th;
    for (int t = 0; t < nthr; t++)
      th.emplace_back([&]() {
        for (int i = next++; i < count; i = next++) fn(i);
      });
    for (auto &t : th) t.join();
  };
  parallel(n, [&](int i) { status[i] = jpeg_parse(data[i], len[i], &hd[i]); });
  for (int i = 0; i < n; i++) {
    if (status[i]) continue;
    JpegHdr &H = hd[i];
    JpegDesc D{};
    D.W = H.W;
    D.H = H.H;
    D.ncomp = H.ncomp;
    D.hmax = D.vmax = 1;
    for (int c = 0; c < H.ncomp; c++) {
      D.hmax = std::max(D.hmax, H.h[c]);
      D.vmax = std::max(D.vmax, H.v[c]);
    }
    D.mcux = (H.W + 8 * D.hmax - 1) / (8 * D.hmax);
    D.mcuy = (H.H + 8 * D.vmax - 1) / (8 * D.vmax);
    D.qt = (int)(qts.size() / 64);
    for (int t = 0; t < 4; t++) qts.insert(qts.end(), H.qt[t], H.qt[t] + 64);
    // the image's four table slots, deduplicated over the batch (an encoder's
    // tables are shared by all its images: a few distinct tables, LDS resident)
    for (int t = 0; t < 4; t++) {
      D.ht[t] = -1;
      if (H.dht[t].empty()) continue;
      const std::string key = std::string(1, t < 2 ? 'D' : 'A') + H.dht[t];  // class + table bytes
      auto it = huff_ix.find(key);
      if (it == huff_ix.end()) {
        JpegHuff hf;
        if (!jpeg_build_huff(H.dht[t], t < 2, &hf)) {
          status[i] = FI_EINVAL;
          break;
        }
        it = huff_ix.emplace(key, (int)huffs.size()).first;
        huffs.push_back(hf);
      }
      D.ht[t] = it->second;
    }
    if (status[i]) continue;
    for (int c = 0; c < H.ncomp; c++) {
      D.h[c] = H.h[c];
      D.v[c] = H.v[c];
      D.tq[c] = H.tq[c];
      D.td[c] = H.td[c];
      D.ta[c] = H.ta[c];
      D.bw[c] = D.mcux * H.h[c];
      D.bh[c] = D.mcuy * H.v[c];
      D.dw[c] = (H.W * H.h[c] + D.hmax - 1) / D.hmax;  // jdmaster.c downsampled_width
      D.dh[c] = (H.H * H.v[c] + D.vmax - 1) / D.vmax;
      D.coef[c] = (int64_t)work_total;
      work_total += (size_t)D.bw[c] * D.bh[c] * 128;
      D.plane[c] = (int64_t)work_total;
      work_total += ((size_t)D.bw[c] * 8 * D.bh[c] * 8 + 255) & ~(size_t)255;
    }
    D.ecs_len = (int32_t)(H.ecs1 - H.ecs0);
    D.ecs = reinterpret_cast<const uint8_t *>(ecs_total);  // offset until placed
    D.dst = dst[i];
    D.dst_stride = dst_stride[i];
    D.dst_c = out_channels == 3 || H.ncomp == 3 ? 3 : 1;
    const int img = (int)descs.size();
    // restart intervals: RSTn markers split the segment
    const int nmcu = D.mcux * D.mcuy;
    if (H.restart > 0) {
      const uint8_t *e = data[i] + H.ecs0;
      int byte0 = 0, mcu0 = 0;
      for (size_t q = 0; q + 1 < (size_t)D.ecs_len && mcu0 < nmcu; q++) {
        if (e[q] == 0xFF && e[q + 1] >= 0xD0 && e[q + 1] <= 0xD7) {
          ivs.push_back({img, mcu0, std::min(mcu0 + H.restart, nmcu), byte0});
          mcu0 += H.restart;
          byte0 = (int)q + 2;
          q++;
        }
      }
      if (mcu0 < nmcu) ivs.push_back({img, mcu0, nmcu, byte0});
    } else {
      ivs.push_back({img, 0, nmcu, 0});
    }
    for (int c = 0; c < 3; c++) {
      blk0.push_back(nblocks);
      if (c < H.ncomp) nblocks += (int64_t)D.bw[c] * D.bh[c];
    }
    px0.push_back(px0.back() + (int64_t)H.W * H.H);
    ecs_total += ((size_t)D.ecs_len + 512 + 255) & ~(size_t)255;  // zero pad: the reader's window
    descs.push_back(D);
    desc_img.push_back(i);
  }
  if (descs.empty()) return 0;
  // one upload: compressed data (each segment zero padded for the reader's
  // window) then tables + descriptors, staged in pinned host memory
  const size_t o_desc = 0, o_iv = o_desc + ((descs.size() * sizeof(JpegDesc) + 255) & ~(size_t)255);
  const size_t o_ref = o_iv + ((ivs.size() * sizeof(JpegInterval) + 255) & ~(size_t)255);
  blk0.push_back(nblocks);
  const size_t o_huff = o_ref + ((blk0.size() * 8 + 255) & ~(size_t)255);
  const size_t o_qt = o_huff + ((huffs.size() * sizeof(JpegHuff) + 255) & ~(size_t)255);
  const size_t o_px = o_qt + ((qts.size() * 2 + 255) & ~(size_t)255);
  const size_t tab0 = (ecs_total + 255) & ~(size_t)255, up_total = tab0 + o_px + px0.size() * 8;
  uint8_t *din = (uint8_t *)alloc(actx, 0, up_total);
  uint8_t *hst = (uint8_t *)alloc(actx, 3, up_total);
  uint8_t *dwork = (uint8_t *)alloc(actx, 2, std::max(work_total, (size_t)256));
  if (!din || !hst || !dwork) {
    *err = "memory for the JPEG batch";
    return FI_ENOMEM;
  }
  uint8_t *dtab = din + tab0, *htab = hst + tab0;
  parallel((int)descs.size(), [&](int k) {
    const JpegDesc &D = descs[k];
    const size_t off = (size_t)reinterpret_cast<uintptr_t>(D.ecs);
    memcpy(hst + off, data[desc_img[k]] + hd[desc_img[k]].ecs0, D.ecs_len);
    const size_t pad_end =
        k + 1 < (int)descs.size() ? (size_t)reinterpret_cast<uintptr_t>(descs[k + 1].ecs) : tab0;
    memset(hst + off + D.ecs_len, 0, pad_end - off - D.ecs_len);
  });
  for (JpegDesc &D : descs) D.ecs = din + (size_t)reinterpret_cast<uintptr_t>(D.ecs);
  memcpy(htab + o_desc, descs.data(), descs.size() * sizeof(JpegDesc));
  memcpy(htab + o_iv, ivs.data(), ivs.size() * sizeof(JpegInterval));
  memcpy(htab + o_ref, blk0.data(), blk0.size() * 8);
  memcpy(htab + o_huff, huffs.data(), huffs.size() * sizeof(JpegHuff));
  memcpy(htab + o_qt, qts.data(), qts.size() * 2);
  memcpy(htab + o_px, px0.data(), px0.size() * 8);
  if (hipMemcpyAsync(din, hst, up_total, hipMemcpyHostToDevice, st) != hipSuccess) {
    *err = "JPEG batch upload";
    return FI_EDEVICE;
  }
  const JpegDesc *dd = (const JpegDesc *)(dtab + o_desc);
  // the distinct Huffman tables go to LDS when they are few (kJpegLdsTabs)
  const int nhuff = (int)huffs.size();
  const dim3 g((unsigned)ivs.size());  // one restart interval per 64-lane workgroup
  if (nhuff <= kJpegLdsTabs)
    hipLaunchKernelGGL(k_jpeg_huff<true>, g, dim3(64), 0, st, dd, (const JpegInterval *)(dtab + o_iv), (int)ivs.size(),
                       (const JpegHuff *)(dtab + o_huff), nhuff, dwork);
  else
    hipLaunchKernelGGL(k_jpeg_huff<false>, g, dim3(64), 0, st, dd, (const JpegInterval *)(dtab + o_iv),
                       (int)ivs.size(), (const JpegHuff *)(dtab + o_huff), nhuff, dwork);
  hipLaunchKernelGGL(k_jpeg_idct, dim3((unsigned)std::min<int64_t>((nblocks + 255) / 256, 1 << 20)), dim3(256), 0, st, dd,
                     (const int64_t *)(dtab + o_ref), (int)descs.size(), (const uint16_t *)(dtab + o_qt), dwork);
  hipLaunchKernelGGL(k_jpeg_color, dim3((unsigned)std::min<int64_t>((px0.back() + 255) / 256, 1 << 20)), dim3(256), 0, st, dd,
                     (const int64_t *)(dtab + o_px), (int)descs.size(), dwork);
  if (hipGetLastError() != hipSuccess || hipStreamSynchronize(st) != hipSuccess) {
    *err = "JPEG decode kernels";
    return FI_EDEVICE;
  }
  return 0;
}

}  // namespace fi
