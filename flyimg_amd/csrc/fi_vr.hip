// fi_vr.hip -- ImageMagick ResizeImage, vertical pass first (the
// ThumbnailImage sample pre-step folded into the tap tables), as a persistent,
// warp-specialised, exact-integer matrix-core pipeline with a BLOCK-MAJOR
// vertical pass: v_mfma_i32_16x16x64_i8.
//
// Weights rint(w 2^s) in two signed-byte limbs, every output row summing to
// 2^s (fi_plan.cpp vr_quant; bounded against IM's f64 weights by
// tests/native/vr_quant_bound.cpp).  k_rs_vm carries the same weights scaled
// to 2^22 in three limbs (axis_q22), so the two kernels give the same pixels;
// what differs is how the vertical pass walks the source rows (DESIGN.md 3.0,
// fi_plan.h VrV):
//
//  * k_rs_vm cuts the touched rows into pieces of <= 64 rows aligned to
//    the 16-row output blocks, and every piece feeds two accumulator slots (its
//    own block and the next) -- so a block whose rows do not fit one piece
//    (every ThumbnailImage geometry: 80 sampled rows per block, 67-80 touched
//    rows) costs two full phases of 64-row MFMAs, and each MFMA triple folds
//    its limbs with VALU shifts;
//  * here the touched rows stream through a RING of R rows in LDS (LDS-DMA,
//    loader waves, as far ahead as the ring allows), and phase p computes ONE
//    output block b from its own window [K0(b), K0(b) + 64 ks) of the ring:
//    ks <= 2 k-steps x 2 weight limbs into two separate accumulators per
//    column tile (folded once per block, the MFMA bias the constant
//    128 * 2^s), then the Q16 planes.
//
//  Roles per phase (one workgroup barrier per phase; NL = 2 or 4 loader waves,
//  7 - NL H waves, chosen per launch by the host, VrLayout::nl):
//    V waves 0-7   block p: vertical MFMAs from the ring (both k-steps' reads
//                  issued first), fold, Q16 planes: into plane buffer p & 1
//                  when there are two (VrLayout::pbuf, the host's choice when
//                  the ring keeps enough rows), else into the single buffer
//                  once the H waves have counted their reads of block p - 1 off
//                  an LDS counter;
//    H waves 8-    block p - 1: both items' plane reads (the counter), then the
//                  horizontal MFMAs -> output tile slot (p - 1) & 1;
//    S wave        the stores of block p - 2;
//    L waves (last NL) the stream cursor: source row pairs by LDS-DMA (ring
//                  slot G mod R, G < K0(p) + R), A fragments of block p + 1, the
//                  record of phase p + 2 (+ the strip's LUT); the end-of-phase
//                  vmcnt waits exactly for the rows of block p + 1.
//  Each workgroup walks its own tile range [t0, t1) (host: LPT over the
//  XCD's workgroups).  Touched rows evenly spaced (rstep > 0) stream from a
//  base and a step; unevenly spaced ones (ThumbnailImage sampling at a
//  non-integral step) from the tile's row list, in per-wave pair classes.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

#include "fi_internal.h"

namespace fi {

namespace {
typedef int32_t i32x4 __attribute__((ext_vector_type(4)));
typedef int32_t i32x2 __attribute__((ext_vector_type(2)));
typedef __attribute__((address_space(1))) const i32x4 g_i32x4;
typedef __attribute__((address_space(1))) uint8_t g_u8;
typedef __attribute__((address_space(1))) uint32_t g_u32;
typedef __attribute__((address_space(1))) uint16_t g_u16;
typedef __attribute__((address_space(3))) i32x2 l_i32x2;
typedef __attribute__((address_space(3))) uint8_t l_u8;

constexpr int kVW = 8;                   // V waves: 64 source bytes (4 column tiles) each
constexpr int kSW = 1;                   // S wave: the stores of the output tile of phase p - 2
// the other 7 waves: NL loader waves (the last ones) and 7 - NL H waves, whose
// items are hw and hw + (7 - NL); the host picks NL per launch (VrLayout::nl,
// fi_api.cpp build_vr_tiles): 4 when every strip of the launch has one 16-px
// output block (3 items; FI_VR_NL=4 forces it where every strip has <= 2),
// else 2 -- evenly or unevenly spaced touched rows alike (the row list's
// 8-row pair classes serve 4 loaders, vr_pair_off)
constexpr int kABytes = 4096;            // [t][limb][64 lanes][16 B]: two limbs, <= 2 k-steps
constexpr int kRecBytes = 32;
constexpr int kLutSlots = 4;
constexpr int kPlanePad = 176;           // 44 (mod 64) dwords: see fi_vm.hip kVmPlanePad
constexpr int kOt8Pitch = 200;           // 8-bit output tile row (<= 64 px x 3 + the row shift)

// record flags (one record per phase, written by L wave 0 two phases ahead)
constexpr int kFirst = 1;                // first block of a tile
constexpr int kSlot = 2;                 // output-tile slot of the block (phase parity)
constexpr int kTslotShift = 4;           // bits 4-5: LUT slot (tile sequence number mod 4)
constexpr int kVshShift = 8;             // bits 8-12: the vertical weight shift (fi_plan.h VrV::shift)

__device__ __forceinline__ i32x2 tr8(const uint8_t *p) { return __builtin_amdgcn_ds_read_tr8_b64_v2i32((l_i32x2 *)(p)); }
__device__ __forceinline__ i32x4 mfma(i32x4 a, i32x4 b, i32x4 c) {
  return __builtin_amdgcn_mfma_i32_16x16x64_i8(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ int col_off(int ci) { return (ci * 16) ^ (((ci >> 4) & 1) << 7); }
__device__ __forceinline__ uint32_t q16_to_u8(uint32_t q) {
  // ScaleQuantumToChar: (q + 128) / 257 = ((q + 128) * 65281) >> 24 on [0, 65535]
  return (uint32_t)(((uint64_t)((q & 0xFFFFu) + 128u) * (65281ull << 8)) >> 32);
}
__device__ __forceinline__ uint32_t gray_q16(uint32_t r, uint32_t g, uint32_t b) {
  // -colorspace Gray: Rec709Luma on gamma-encoded Q16, ClampToQuantum
  const double gv = 0.212656 * (double)r + 0.715158 * (double)g + 0.072186 * (double)b;
  return !(gv > 0.0) ? 0u : (gv >= 65535.0 ? 65535u : (uint32_t)(gv + 0.5));
}
__device__ __forceinline__ int32_t fold2(int32_t d0, int32_t d1) { return (int32_t)((uint32_t)d0 + ((uint32_t)d1 << 8)); }
__device__ __forceinline__ uint32_t lds_addr(const uint8_t *p) { return (uint32_t)(uintptr_t)(const l_u8 *)p; }
// read-only tables through the constant address space (scalar loads)
template <class T>
__device__ __forceinline__ T ldc(const T *p) {
  static_assert(sizeof(T) % 4 == 0, "dword records");
  T r;
  const __attribute__((address_space(4))) int32_t *q = (const __attribute__((address_space(4))) int32_t *)p;
  int32_t *o = reinterpret_cast<int32_t *>(&r);
#pragma unroll
  for (int i = 0; i < (int)(sizeof(T) / 4); i++) o[i] = q[i];
  return r;
}
__device__ __forceinline__ int32_t ldc1(const int32_t *p) { return *(const __attribute__((address_space(4))) int32_t *)p; }
__device__ __forceinline__ int ufl(int x) { return __builtin_amdgcn_readfirstlane(x); }

// LDS-DMA, saddr form: lane i's 16 bytes at sbase + voff land at LDS m0 + 16 i.
// Invisible to hipcc's waitcnt pass: the L loop waits for it explicitly.
__device__ __forceinline__ void dma16(uint32_t m0, const uint8_t *sbase, uint32_t voff) {
  unsigned keep;
  const uint64_t sb = (uint64_t)(uintptr_t)sbase;
  sbase = reinterpret_cast<const uint8_t *>(
      (uintptr_t)(((uint64_t)(uint32_t)ufl((int)(uint32_t)(sb >> 32)) << 32) | (uint32_t)ufl((int)(uint32_t)sb)));
  m0 = (uint32_t)ufl((int)m0);
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
// the row stream's DMA, one asm text per lane pattern: keeps hipcc from
// tail-merging the four sites (a merged site selects its operand with VALU)
// or merging them into the table-lookup path (whose scalar-load wait would
// then run before every DMA)
#define FI_VR_DMA_TAG(name, tag)                                                    \
  __device__ __forceinline__ void name(uint32_t m0, const uint8_t *sbase, uint32_t voff) { \
    unsigned keep;                                                                  \
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\t"                \
                 "global_load_lds_dwordx4 %1, %2 ; " tag "\n\ts_mov_b32 m0, %0"       \
                 : "=&s"(keep)                                                      \
                 : "v"(voff), "s"(sbase), "s"(m0)                                   \
                 : "memory");                                                       \
  }
FI_VR_DMA_TAG(dma16_p0, "p0")
FI_VR_DMA_TAG(dma16_p1, "p1")
FI_VR_DMA_TAG(dma16_p2, "p2")
FI_VR_DMA_TAG(dma16_p3, "p3")
FI_VR_DMA_TAG(dma16_p4, "p4")
FI_VR_DMA_TAG(dma16_p5, "p5")
FI_VR_DMA_TAG(dma16_p6, "p6")
FI_VR_DMA_TAG(dma16_p7, "p7")
#undef FI_VR_DMA_TAG
__device__ __forceinline__ void phase_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }
__device__ __forceinline__ void wait_vm0() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }
// s_waitcnt vmcnt(n): the wave's n youngest vector-memory operations may stay
// in flight (n < 48 exactly; above, 47)
__device__ __forceinline__ void wait_vm_le(int n) {
  switch (n < 48 ? n : 47) {
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
    case 15: asm volatile("s_waitcnt vmcnt(15)" ::: "memory"); break;
    case 16: asm volatile("s_waitcnt vmcnt(16)" ::: "memory"); break;
    case 17: asm volatile("s_waitcnt vmcnt(17)" ::: "memory"); break;
    case 18: asm volatile("s_waitcnt vmcnt(18)" ::: "memory"); break;
    case 19: asm volatile("s_waitcnt vmcnt(19)" ::: "memory"); break;
    case 20: asm volatile("s_waitcnt vmcnt(20)" ::: "memory"); break;
    case 21: asm volatile("s_waitcnt vmcnt(21)" ::: "memory"); break;
    case 22: asm volatile("s_waitcnt vmcnt(22)" ::: "memory"); break;
    case 23: asm volatile("s_waitcnt vmcnt(23)" ::: "memory"); break;
    case 24: asm volatile("s_waitcnt vmcnt(24)" ::: "memory"); break;
    case 25: asm volatile("s_waitcnt vmcnt(25)" ::: "memory"); break;
    case 26: asm volatile("s_waitcnt vmcnt(26)" ::: "memory"); break;
    case 27: asm volatile("s_waitcnt vmcnt(27)" ::: "memory"); break;
    case 28: asm volatile("s_waitcnt vmcnt(28)" ::: "memory"); break;
    case 29: asm volatile("s_waitcnt vmcnt(29)" ::: "memory"); break;
    case 30: asm volatile("s_waitcnt vmcnt(30)" ::: "memory"); break;
    case 31: asm volatile("s_waitcnt vmcnt(31)" ::: "memory"); break;
    case 32: asm volatile("s_waitcnt vmcnt(32)" ::: "memory"); break;
    case 33: asm volatile("s_waitcnt vmcnt(33)" ::: "memory"); break;
    case 34: asm volatile("s_waitcnt vmcnt(34)" ::: "memory"); break;
    case 35: asm volatile("s_waitcnt vmcnt(35)" ::: "memory"); break;
    case 36: asm volatile("s_waitcnt vmcnt(36)" ::: "memory"); break;
    case 37: asm volatile("s_waitcnt vmcnt(37)" ::: "memory"); break;
    case 38: asm volatile("s_waitcnt vmcnt(38)" ::: "memory"); break;
    case 39: asm volatile("s_waitcnt vmcnt(39)" ::: "memory"); break;
    case 40: asm volatile("s_waitcnt vmcnt(40)" ::: "memory"); break;
    case 41: asm volatile("s_waitcnt vmcnt(41)" ::: "memory"); break;
    case 42: asm volatile("s_waitcnt vmcnt(42)" ::: "memory"); break;
    case 43: asm volatile("s_waitcnt vmcnt(43)" ::: "memory"); break;
    case 44: asm volatile("s_waitcnt vmcnt(44)" ::: "memory"); break;
    case 45: asm volatile("s_waitcnt vmcnt(45)" ::: "memory"); break;
    case 46: asm volatile("s_waitcnt vmcnt(46)" ::: "memory"); break;
    case 47: asm volatile("s_waitcnt vmcnt(47)" ::: "memory"); break;
    default: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
  }
}

struct Rec {  // 32 B in LDS (kRecBytes)
  int32_t t, blk, flags, slot0, ks, grend, frag, w128;  // frag / w128: int32 offsets into ai
};
#ifndef FI_VR_PL
#define FI_VR_PL 5
#endif
constexpr int PL = FI_VR_PL;  // k_rs_vr uneven row list: own pairs per scalar load
struct WL {
  int32_t v[2 * PL];
};
struct Lds {  // offsets of the launch's LDS regions
  int ring, a, rec, cnt, lut, planes, otile;
};
__device__ __forceinline__ Lds lds_of(const VrLayout &L) {
  Lds o;
  o.ring = 0;
  o.a = L.R * 512;
  o.rec = o.a + 2 * kABytes;
  o.cnt = o.rec + 8 * kRecBytes;
  o.lut = o.cnt + 16;
  o.planes = o.lut + kLutSlots * 1024;
  o.otile = L.otile_off;
  return o;
}
}  // namespace

// per-wave phase sums of MODE 9 (fi_debug_vr_stamps, tools/vr_timing.py VR=1)
constexpr int kVrStampSlots = 256;
constexpr int kVrStampN = 16 * 6;
__device__ uint64_t g_vr_stamps[kVrStampSlots * kVrStampN];

// MODE (profiling ablations, FI_VR_VARIANT; wrong pixels): 0 production,
// 1 DMA stream only, 2 no H role and no stores, 3 no stores, 4 no A-fragment
// DMAs after the first two blocks, 7 no V fold / float conversion, 8 no H
// conversion, 5 / 6 loader
// priority 1 / 0 (production pixels), 9 production + per-phase s_memtime sums;
// 10 + k: ablation k with the stamps.
template <int MODE, int NL>
__global__ __launch_bounds__(1024, 1) void k_rs_vr(const VDesc *__restrict__ descs, const MStrip *__restrict__ strips,
                                                   const VrTile *__restrict__ tiles, int ntiles,
                                                   const int32_t *__restrict__ wginfo, const int32_t *__restrict__ ai,
                                                   VrLayout Lo) {
  constexpr int M = MODE >= 10 ? MODE - 10 : MODE;
  constexpr int kLW = NL, kHW = 16 - kVW - kSW - NL;
  static_assert(NL == 2 || NL == 4, "loader waves");
  constexpr int kPS = 2 * NL;  // stream rows between a loader wave's own pairs
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wv = ufl(tid >> 6);
  const int g = (int)blockIdx.x;
  // this workgroup's stream: tiles [t0, t1) (host LPT over the XCD's workgroups)
  const int N = ldc1(wginfo + 4 * g);         // phases (blocks)
  const int gend = ldc1(wginfo + 4 * g + 1);  // stream rows
  const int t0 = ldc1(wginfo + 4 * g + 2), t1 = ldc1(wginfo + 4 * g + 3);
  const int R = Lo.R;
  const Lds O = lds_of(Lo);
  Rec *recs = reinterpret_cast<Rec *>(lds + O.rec);
  volatile uint32_t *hcnt = reinterpret_cast<volatile uint32_t *>(lds + O.cnt);
  const int32_t *lut = reinterpret_cast<const int32_t *>(lds + O.lut);  // [kLutSlots][256]
  uint8_t *planes = lds + O.planes;                                      // [6][plane]
  uint8_t *otiles = lds + O.otile;                                       // [2][otile_bytes]
  const int plane = Lo.plane;
  constexpr bool kStamp = MODE == 9 || MODE >= 10;
  uint64_t tsum[5] = {}, tprev = 0;
  auto stamp = [&](int k) {
    if (kStamp) {
      const uint64_t t = __builtin_amdgcn_s_memtime();
      tsum[k] += t - tprev;
      tprev = t;
    }
  };
  auto stamp_out = [&](int n) {
    if (kStamp && lane == 0 && g < kVrStampSlots) {
      uint64_t *o = g_vr_stamps + g * kVrStampN + 6 * wv;
      for (int k = 0; k < 5; k++) o[k] = k < n ? tsum[k] : 0;
      o[5] = (uint64_t)N;
    }
  };
  auto read_rec = [&](int s) -> Rec {
    const Rec x = recs[s & 7];
    return Rec{ufl(x.t), ufl(x.blk), ufl(x.flags), ufl(x.slot0), ufl(x.ks), ufl(x.grend), ufl(x.frag), ufl(x.w128)};
  };

  if (wv >= kVW + kHW + kSW) {
    // ============ L role: phase records, row stream, A fragments ============
    const int li = wv - (kVW + kHW + kSW);
    const int h = lane >> 5;  // half-wave: the two rows of one 1-KB DMA
    // ---- phase cursor (records, A fragments) ----
    struct PI {
      int t, blk, gk0, grend, ks, frag, w128, flags;
    };
    int ct = t0, ck = 0, cb = 0, c_bmeta = 0, c_frag = 0, c_w128 = 0, c_lut = 0, c_lut_n = 0, c_vsh = 0;
    VrTile CT{};
    auto ptile_load = [&]() {
      CT = ldc(tiles + ct);
      const VDesc D = ldc(descs + CT.img);
      const MStrip S = ldc(strips + CT.strip);
      c_bmeta = D.pmeta;
      c_frag = D.frag;
      c_w128 = D.w128;
      c_vsh = D.vsh;
      c_lut = S.lut;
      c_lut_n = S.lut_n;
      cb = CT.b0;
    };
    if (ct < t1) ptile_load();
    // the phase at the cursor; writes its record (slot s) and stages its tile's
    // LUT (first block of a tile) -- L wave 0 only; advances the cursor
    auto next_phase = [&](int s) -> PI {
      const int4 m = ldc(reinterpret_cast<const int4 *>(ai + c_bmeta + 4 * cb));  // {K0, ks, Rend, 0}
      PI r;
      r.t = ct;
      r.blk = cb;
      r.gk0 = CT.g0 + (m.x - CT.kbase);
      r.grend = CT.g0 + (m.z - CT.kbase);
      r.ks = m.y;
      r.frag = c_frag + cb * 4 * 256;
      r.w128 = c_w128 + 16 * cb;
      r.flags = (cb == CT.b0 ? kFirst : 0) | ((s & 1) ? kSlot : 0) | ((ck & (kLutSlots - 1)) << kTslotShift) |
                (c_vsh << kVshShift);
      if (li == 0) {
        if (lane == 0) recs[s & 7] = Rec{r.t, r.blk, r.flags, r.gk0 % R, r.ks, r.grend, r.frag, r.w128};
        if ((r.flags & kFirst) && lane < (c_lut_n + 3) / 4)
          dma16(lds_addr(lds) + (uint32_t)(O.lut + (ck & (kLutSlots - 1)) * 1024),
                reinterpret_cast<const uint8_t *>(ai + c_lut), 16u * lane);
      }
      cb++;
      if (cb >= CT.b1) {
        ck++;
        ct++;
        if (ct < t1) ptile_load();
      }
      return r;
    };
    // A fragments (ks k-steps x 2 limbs x 1 KB) into A slot `slot`
    auto issue_a = [&](const PI &r, int slot) {
      const uint32_t m0 = lds_addr(lds) + (uint32_t)(O.a + slot * kABytes);
      const int nf = 2 * r.ks;
      for (int i = li; i < nf; i += kLW)
        dma16(m0 + 1024 * i, reinterpret_cast<const uint8_t *>(ai + r.frag) + 1024 * i, 16u * lane);
    };
    // ---- row cursor: this wave's row pairs G = kPS m + 2 li of the stream ----
    int rt = t0, rG = 2 * li, rslot = 2 * li, n_issued = 0;
    VrTile RT{};
    const uint8_t *r_src = nullptr;
    int64_t r_stride = 0;
    int r_b0 = 0, r_nbytes = 0, r_row0 = 0, r_rstep = 0, r_nrows = 0, r_rows = 0;
    auto rtile_load = [&]() {
      RT = ldc(tiles + rt);
      const VDesc D = ldc(descs + RT.img);
      const MStrip S = ldc(strips + RT.strip);
      r_src = D.src;
      r_stride = D.src_stride;
      r_b0 = S.b0;
      r_nbytes = S.nbytes;
      r_row0 = D.row0;
      r_rstep = D.rstep;
      r_nrows = D.nrows;
      r_rows = D.rows;
    };
    if (rt < t1) rtile_load();
    const uint32_t lane_c = (uint32_t)((lane & 31) ^ h);  // chunk of this lane before the row swizzle
    uint32_t pat[4] = {0, 0, 0, 0};                          // fast-path lane offsets of tile pat_tile
    int pat_tile = -1;
    // issue this wave's pairs up to stream row `limit`; returns the DMAs issued.
    // Evenly spaced touched rows (rstep > 0): a loop with no loads, bases linear
    // in the pair index, the chunk swizzle from the ring slot.  Uneven ones
    // (ThumbnailImage sampling at a non-integral step, cfg1's 2000 -> 1250): the
    // rows come from the pair-class copy of the touched-row list (vr_pair_off),
    // PL own pairs (2 PL ints) per scalar load, each load waited for before its
    // DMAs are issued.
    auto issue_rows = [&](int limit) -> int {
      int n = 0;
      while (rG < limit) {
        if (rG >= RT.g0 + RT.glen) {
          rt++;
          rtile_load();  // the host makes the stream cover [0, gend): rt < t1 here
          continue;
        }
        const int seg = min(limit, RT.g0 + RT.glen);
        int k0 = RT.kbase + (rG - RT.g0);
        if (r_rstep == 0 && k0 + 1 < r_nrows) {
          const int cnt = min((seg - rG + kPS - 1) / kPS, (r_nrows - 1 - k0 + kPS - 1) / kPS);
          // the host's pair list for kPS-row cycles (after the row list and its
          // 32-entry pad): class k0 mod kPS, own pair m at entry k0 / kPS + m,
          // PL pairs per wait (scalar loads complete out of order: each wait is
          // lgkmcnt(0))
          const WL *lst = reinterpret_cast<const WL *>(ai + r_rows + vr_pair_off(r_nrows, k0, kPS));
          for (int j0 = 0; j0 < cnt; j0 += PL) {
            const WL c0 = ldc(lst + j0 / PL);
            const int jn = cnt - j0;
#pragma unroll
            for (int j = 0; j < PL; j++) {
              if (j >= jn) continue;
              const int r0 = c0.v[2 * j], r1 = c0.v[2 * j + 1];
              const uint32_t f = (uint32_t)((rslot & 7) | (((rslot >> 4) & 1) << 3));
              uint32_t lc = lane_c ^ f;
              if (16 * (int)lc >= r_nbytes) lc = 0;
              const uint32_t voff = (h ? (uint32_t)((int64_t)(r1 - r0) * r_stride) : 0u) + 16u * lc;
              dma16(lds_addr(lds) + (uint32_t)(O.ring + rslot * 512), r_src + (int64_t)r0 * r_stride + r_b0, voff);
              rslot += kPS;
              if (rslot >= R) rslot -= R;
            }
          }
          n += cnt;
          rG += kPS * cnt;
          continue;
        }
        if (k0 + 1 < r_nrows) {
          // pairs with k0 + 1 < nrows and rG < seg
          const int cnt = min((seg - rG + kPS - 1) / kPS, (r_nrows - 1 - k0 + kPS - 1) / kPS);
          const int64_t rs = (int64_t)r_rstep * r_stride;
          const uint8_t *base = r_src + (int64_t)(r_row0 + r_rstep * k0) * r_stride + r_b0;
          if (pat_tile != rt) {
            // this wave's own pair starts 2 li + kPS m have the chunk swizzle
            // f = (s & 7) | 8 ((s >> 4) & 1) of slot s = 2 li + kPS m (R is a
            // multiple of 32): NL 2: 2 li + 4 (m & 1) + 8 ((m >> 2) & 1), four
            // lane patterns; NL 4: 2 li + 8 ((m >> 1) & 1), two
            pat_tile = rt;
            const uint32_t hoff = h ? (uint32_t)rs : 0u;
#pragma unroll
            for (int q = 0; q < 4; q++) {
              uint32_t lc = lane_c ^ (uint32_t)(NL == 2 ? 2 * li + 4 * (q & 1) + 8 * (q >> 1) : 2 * li + 8 * (q & 1));
              if (16 * (int)lc >= r_nbytes) lc = 0;
              pat[q] = hoff + 16u * lc;
            }
          }
          // straight-line DMAs over the 32-row cycle of own pairs (32 / kPS of
          // them: NL 2 pattern (m & 1) | ((m >> 2) & 1) << 1, NL 4 (m >> 1) & 1);
          // a cycle never crosses the ring end (R is a multiple of 32 rows), so
          // the wrap is checked per cycle
          {
            const int rslot0 = rslot;
            uint32_t m0 = lds_addr(lds) + (uint32_t)(O.ring + rslot * 512);
            int left = cnt, ph = (rslot / kPS) & (32 / kPS - 1);
            constexpr uint32_t kStep = 512u * kPS;
            const int64_t bs = (int64_t)kPS * rs;
            for (;;) {
              if constexpr (NL == 2) {
                switch (ph) {
                case 0:
                  dma16_p0(m0, base, pat[0]);
                  base += bs;
                  m0 += kStep;
                  if (--left == 0) goto stream_done;
                case 1:
                  dma16_p1(m0, base, pat[1]);
                  base += bs;
                  m0 += kStep;
                  if (--left == 0) goto stream_done;
                case 2:
                  dma16_p2(m0, base, pat[0]);
                  base += bs;
                  m0 += kStep;
                  if (--left == 0) goto stream_done;
                case 3:
                  dma16_p3(m0, base, pat[1]);
                  base += bs;
                  m0 += kStep;
                  if (--left == 0) goto stream_done;
                case 4:
                  dma16_p4(m0, base, pat[2]);
                  base += bs;
                  m0 += kStep;
                  if (--left == 0) goto stream_done;
                case 5:
                  dma16_p5(m0, base, pat[3]);
                  base += bs;
                  m0 += kStep;
                  if (--left == 0) goto stream_done;
                case 6:
                  dma16_p6(m0, base, pat[2]);
                  base += bs;
                  m0 += kStep;
                  if (--left == 0) goto stream_done;
                case 7:
                  dma16_p7(m0, base, pat[3]);
                  base += bs;
                  m0 += kStep;
                  if (--left == 0) goto stream_done;
                }
              } else {
                switch (ph) {
                case 0:
                  dma16_p0(m0, base, pat[0]);
                  base += bs;
                  m0 += kStep;
                  if (--left == 0) goto stream_done;
                case 1:
                  dma16_p1(m0, base, pat[0]);
                  base += bs;
                  m0 += kStep;
                  if (--left == 0) goto stream_done;
                case 2:
                  dma16_p2(m0, base, pat[1]);
                  base += bs;
                  m0 += kStep;
                  if (--left == 0) goto stream_done;
                case 3:
                  dma16_p3(m0, base, pat[1]);
                  base += bs;
                  m0 += kStep;
                  if (--left == 0) goto stream_done;
                }
              }
              ph = 0;
              int r2 = rslot0 + kPS * (cnt - left);  // the next cycle's first pair
              while (r2 >= R) r2 -= R;
              m0 = lds_addr(lds) + (uint32_t)(O.ring + r2 * 512);
            }
          stream_done:
            rslot = rslot0 + kPS * cnt;
            while (rslot >= R) rslot -= R;
          }
          n += cnt;
          rG += kPS * cnt;
          continue;
        }
        // one pair clamped at the list end
        k0 = min(k0, r_nrows - 1);
        const int k1 = min(k0 + 1, r_nrows - 1);
        const int r0 = r_rstep ? r_row0 + r_rstep * k0 : ldc1(ai + r_rows + k0);
        const int r1 = r_rstep ? r_row0 + r_rstep * k1 : ldc1(ai + r_rows + k1);
        const uint8_t *base = r_src + (int64_t)r0 * r_stride + r_b0;
        const uint32_t f = (uint32_t)((rslot & 7) | (((rslot >> 4) & 1) << 3));  // chunk swizzle of row rslot (rslot + 1: f ^ 1)
        uint32_t lc = lane_c ^ f;
        if (16 * (int)lc >= r_nbytes) lc = 0;
        const uint32_t voff = (h ? (uint32_t)((int64_t)(r1 - r0) * r_stride) : 0u) + 16u * lc;
        dma16(lds_addr(lds) + (uint32_t)(O.ring + rslot * 512), base, voff);
        n++;
        rG += kPS;
        rslot += kPS;
        if (rslot >= R) rslot -= R;
      }
      return n;
    };
    // own pairs (starts kPS m + 2 li) below stream row x
    auto own_below = [&](int x) -> int { return x > 2 * li ? (x - 2 * li + kPS - 1) / kPS : 0; };

    // the loader's few instructions go first on its SIMD (MODE 5 / 6: priority 1 / 0)
    if (M == 5)
      __builtin_amdgcn_s_setprio(1);
    else if (M != 6)
      __builtin_amdgcn_s_setprio(2);
    if (li == 0 && lane == 0) hcnt[0] = 0;
    PI P0{}, P1{};
    if (N > 0) {
      P0 = next_phase(0);
      if (M != 1) issue_a(P0, 0);
    }
    if (N > 1) P1 = next_phase(1);
    if (N > 0) n_issued += issue_rows(min(P0.gk0 + R, gend));
    wait_vm0();
    phase_barrier();  // records 0 / 1, A(0), the rows of block 0 and the first LUT visible
    phase_barrier();
    if (kStamp) tprev = __builtin_amdgcn_s_memtime();
    for (int p = 0; p < N + 2; p++) {
      // A fragments of block p + 1 (its record was written last phase)
      if (M != 1 && M != 4 && p + 1 < N) issue_a(P1, (p + 1) & 1);
      stamp(0);
      PI P2{};
      if (p + 2 < N) P2 = next_phase(p + 2);
      // source rows as far ahead as the ring allows: slots of rows < K0(p) are free
      int nr = 0;
      if (p < N) {
        nr = issue_rows(min(P0.gk0 + R, gend));
        n_issued += nr;
      }
      stamp(1);
      const int ns = 0;
      // block p + 1's rows (every own pair starting below its Rend), A(p + 1) and
      // the LUTs landed; younger row pairs may stay in flight
      if (p + 1 < N) {
        const int after = max(0, n_issued - own_below(P1.grend));
        wait_vm_le(min(after, nr) + ns);
      } else {
        wait_vm0();
      }
      stamp(2);
      phase_barrier();
      stamp(3);
      P0 = P1;
      P1 = P2;
    }
    stamp_out(4);
    return;
  }

  if (wv < kVW) {
    // =================== V role: block-major vertical MFMA + Q16 planes ===================
    // wave w owns source bytes [64 w, 64 w + 64) of the strip = column tiles j < 4
    const int w = wv;
    constexpr int kT = 4;
    // transposing reads: lane reads rows rA (and rA + 8) of a k-step, bytes 8 (lane & 1)
    // of its tile's 16-byte chunk; the chunk swizzle of ring slot s is
    // f(s) = (s & 7) | 8 ((s >> 4) & 1), and with the k-step start a multiple of 16
    // f = fL ^ 8 bit4(start) for both rows
    const int rA = 16 * (lane >> 4) + ((lane & 15) >> 1);
    const int fL = (rA & 7) | (((rA >> 4) & 1) << 3);
    uint32_t offj[kT];
#pragma unroll
    for (int j = 0; j < kT; j++) offj[j] = (uint32_t)(16 * ((4 * w + j) ^ fL) + 8 * (lane & 1));
    uint32_t vcolp[kT / 2] = {0xFFFFFFFFu, 0xFFFFFFFFu};
    phase_barrier();
    phase_barrier();
    Rec rC = N > 0 ? read_rec(0) : Rec{};
    if (kStamp) tprev = __builtin_amdgcn_s_memtime();
    for (int p = 0; p < N + 2; p++) {
      if (p < N && M != 1) {
        const Rec C = rC;
        if (C.flags & kFirst) {
          // new tile: Q16-plane offsets of this lane's columns from the staged LUT
          const VrTile T = ldc(tiles + C.t);
          const MStrip S = ldc(strips + T.strip);
          const int32_t *lt = lut + 256 * ((C.flags >> kTslotShift) & (kLutSlots - 1));
#pragma unroll
          for (int j = 0; j < kT; j++) {
            const int col = 64 * w + 16 * j + (lane & 15);
            const int abs = S.b0 + min(col, S.nbytes - 1), px = abs / 3, chn = abs - 3 * px;
            const int ci = lt[px - S.lut_px0];
            const uint32_t o = (col < S.nbytes && ci >= 0) ? (uint32_t)(chn * plane + col_off(ci) + 4 * (lane >> 4))
                                                            : 0xFFFFu;
            if (j & 1)
              vcolp[j >> 1] = (vcolp[j >> 1] & 0xFFFFu) | (o << 16);
            else
              vcolp[j >> 1] = (vcolp[j >> 1] & 0xFFFF0000u) | o;
          }
        }
        stamp(0);
        const i32x4 *al = reinterpret_cast<const i32x4 *>(lds + O.a + (p & 1) * kABytes);
        // the MFMA bias, 128 * the weight sum of every output row (pixels enter as
        // p - 128): the quantised rows sum to exactly 2^shift (fi_plan.h VrV)
        const int32_t cb = 128 << ((C.flags >> kVshShift) & 31);
        const i32x4 corr = {cb, cb, cb, cb};
        i32x4 acc[2][kT];
        const uint32_t RB = (uint32_t)R * 512u;
        // both k-steps' ring and A reads in flight before the first MFMA
        i32x4 Bt[2][kT], At[2][2];
#pragma unroll
        for (int t = 0; t < 2; t++) {
          if (t >= C.ks) break;
          int sb = C.slot0 + 64 * t;
          if (sb >= R) sb -= R;
          const uint32_t y0 = (uint32_t)(sb + rA) * 512u, y1 = y0 + 8u * 512u;
          const uint32_t Y0 = min(y0, y0 - RB), Y1 = min(y1, y1 - RB);
          const uint32_t sx = (uint32_t)((sb >> 4) & 1) << 7;
#pragma unroll
          for (int j = 0; j < kT; j++) {
            const uint32_t o = offj[j] ^ sx;
            const i32x2 lo = tr8(lds + O.ring + Y0 + o), hi = tr8(lds + O.ring + Y1 + o);
            Bt[t][j] = i32x4{lo.x, lo.y, hi.x, hi.y} ^ i32x4{(int)0x80808080, (int)0x80808080, (int)0x80808080, (int)0x80808080};
          }
#pragma unroll
          for (int q = 0; q < 2; q++) At[t][q] = al[(t * 2 + q) * 64 + lane];
        }
#pragma unroll
        for (int j = 0; j < kT; j++) acc[0][j] = mfma(At[0][0], Bt[0][j], corr);
#pragma unroll
        for (int j = 0; j < kT; j++) acc[1][j] = mfma(At[0][1], Bt[0][j], i32x4{0, 0, 0, 0});
        if (C.ks > 1) {
#pragma unroll
          for (int j = 0; j < kT; j++) acc[0][j] = mfma(At[1][0], Bt[1][j], acc[0][j]);
#pragma unroll
          for (int j = 0; j < kT; j++) acc[1][j] = mfma(At[1][1], Bt[1][j], acc[1][j]);
        }
        stamp(1);
        // the H waves' reads of block p - 1's planes are done (single plane
        // buffer; with two, block p's buffer was read in phase p - 1)
        if (M != 2 && Lo.pbuf == 1) {
          const uint32_t want = (uint32_t)kHW * (uint32_t)(p + 1);
          while (hcnt[0] < want) __builtin_amdgcn_s_sleep(1);
        }
        stamp(4);
        // block done: ClampToQuantum(257 acc / 2^shift) -> Q16 hi / lo signed-byte planes
        const float vscale = __builtin_amdgcn_ldexpf(257.0f, -((C.flags >> kVshShift) & 31));
#pragma unroll
        for (int j = 0; j < kT; j++) {
          const uint32_t o = (vcolp[j >> 1] >> (16 * (j & 1))) & 0xFFFFu;
          uint32_t q[4];
          if (M == 7) {  // ablation: no fold / float conversion (wrong pixels, same LDS traffic)
#pragma unroll
            for (int i = 0; i < 4; i++) q[i] = (uint32_t)acc[0][j][i];
          } else {
            // two rows per packed fma (v_pk_fma_f32: the same IEEE fma per element)
            typedef float f32x2 __attribute__((ext_vector_type(2)));
#pragma unroll
            for (int i = 0; i < 4; i += 2) {
              const f32x2 t = {(float)fold2(acc[0][j][i], acc[1][j][i]), (float)fold2(acc[0][j][i + 1], acc[1][j][i + 1])};
              const f32x2 r = __builtin_elementwise_fma(t, f32x2{vscale, vscale}, f32x2{0.5f, 0.5f});
              q[i] = __float2uint_rz(r.x);
              q[i + 1] = __float2uint_rz(r.y);
            }
          }
          const auto p01 = __builtin_amdgcn_cvt_pk_u16(q[0], q[1]);
          const auto p23 = __builtin_amdgcn_cvt_pk_u16(q[2], q[3]);
          const uint32_t x01 = __builtin_bit_cast(uint32_t, p01) ^ 0x80808080u;
          const uint32_t x23 = __builtin_bit_cast(uint32_t, p23) ^ 0x80808080u;
          if (o != 0xFFFFu) {
            uint8_t *pb = planes + ((Lo.pbuf == 2 && (p & 1)) ? 6 * plane : 0);
            *reinterpret_cast<uint32_t *>(pb + o) = __builtin_amdgcn_perm(x23, x01, 0x07050301u);
            *reinterpret_cast<uint32_t *>(pb + o + 3 * plane) = __builtin_amdgcn_perm(x23, x01, 0x06040200u);
          }
        }
        stamp(2);
      }
      if (p + 1 < N) rC = read_rec(p + 1);
      phase_barrier();
      stamp(3);
    }
    stamp_out(5);
    return;
  }

  if (wv == kVW + kHW) {
    // =================== S role: the output stores ===================
    const int sw = 0;
    int stile = -1;  // tile of the cached store descriptors
    struct StoreD {
      uint8_t *dst;
      int64_t dst_stride;
      int32_t ew, eh, rot, gray, x0, x1;
    } sD{};
    phase_barrier();
    phase_barrier();
    for (int p = 0; p < N + 2; p++) {
      // stores of the block of phase p - 2 (output tile slot (p - 2) & 1): on
      // the loader waves their issue held back the row stream
      bool st_fast = false;
      uint8_t *st_row0 = nullptr;
      int64_t st_stride = 0;
      int st_nb = 0, st_nrow = 0;
      const uint8_t *st_ot = nullptr;
      if (p >= 2 && p - 2 < N && M != 3 && M != 1 && M != 2) {
        const Rec rs = read_rec(p - 2);
        if (stile != rs.t) {
          stile = rs.t;
          const VrTile T = ldc(tiles + rs.t);
          const VDesc D0 = ldc(descs + T.img);
          const MStrip S0 = ldc(strips + T.strip);
          sD = StoreD{D0.dst, D0.dst_stride, D0.ew, D0.eh, D0.rot, D0.gray, S0.x0, S0.x1};
        }
        const StoreD &D = sD;
        const int b = rs.blk;
        const int nx = D.x1 - D.x0;
        const int oc = D.gray ? 1 : 3;
        const int rows_here = min(16, D.eh - 16 * b);
        const int nb = nx * oc;
        uint8_t *ot = otiles + ((rs.flags & kSlot) ? Lo.otile_bytes : 0);
        const uint16_t *otile = reinterpret_cast<const uint16_t *>(ot);
        const bool fastA = !D.gray && D.rot == 0 && (((uintptr_t)D.dst + (uint64_t)D.x0 * 3) & 3u) == 0 &&
                           (D.dst_stride & 3) == 0 && (nb & 3) == 0;
        auto out_byte = [&](int yl, int k) -> uint32_t {
          const uint16_t *o = otile + yl * kVmOtilePitch;
          if (!D.gray) return q16_to_u8(o[k]);
          return q16_to_u8(gray_q16(o[3 * k], o[3 * k + 1], o[3 * k + 2]));
        };
        if (fastA) {
          st_fast = true;
          st_row0 = D.dst + (int64_t)(16 * b + sw) * D.dst_stride + (int64_t)D.x0 * 3;
          st_stride = (int64_t)kSW * D.dst_stride;
          st_nb = nb;
          st_nrow = (rows_here - sw + kSW - 1) / kSW;
          st_ot = ot + sw * kOt8Pitch;
        } else if (D.gray == 2) {
          for (int it = tid - 64 * (kVW + kHW); it < rows_here * nx; it += 64 * kSW) {
            const int yl = it / nx, x = it - yl * nx;
            const uint16_t *o = otile + yl * kVmOtilePitch + 3 * x;
            ((g_u16 *)(D.dst + (int64_t)(16 * b + yl) * D.dst_stride))[D.x0 + x] = (uint16_t)gray_q16(o[0], o[1], o[2]);
          }
        } else if (!D.gray && D.rot == 0) {
          // 8-bit tile, rows shifted to the destination's address mod 4: store wave
          // sw copies rows sw, sw + kSW, ..., one destination dword per lane
          const uint32_t sh0 = (uint32_t)(((uintptr_t)D.dst + (uint64_t)D.x0 * 3) & 3u);
          const uint32_t shs = (uint32_t)(D.dst_stride & 3);
          constexpr int kRows = (16 + kSW - 1) / kSW;
          uint32_t wd[kRows];
  #pragma unroll
          for (int r = 0; r < kRows; r++) wd[r] = sw + kSW * r < 16 ? *reinterpret_cast<const uint32_t *>(ot + (sw + kSW * r) * kOt8Pitch + 4 * lane) : 0u;
  #pragma unroll
          for (int r = 0; r < kRows; r++) {
            const int yl = sw + kSW * r;
            if (yl >= rows_here) break;
            const int sh = (int)((sh0 + (uint32_t)(16 * b + yl) * shs) & 3u);
            const int k0 = 4 * lane - sh;
            uint8_t *a0 = D.dst + (int64_t)(16 * b + yl) * D.dst_stride + (int64_t)D.x0 * 3;
            if (k0 >= 0 && k0 + 4 <= nb) {
              *(g_u32 *)(a0 + k0) = wd[r];
            } else if (k0 < nb && k0 + 4 > 0) {
  #pragma unroll
              for (int j = 0; j < 4; j++)
                if (k0 + j >= 0 && k0 + j < nb) *(g_u8 *)(a0 + k0 + j) = (uint8_t)(wd[r] >> (8 * j));
            }
          }
        } else if (D.rot == 0) {
          const int ndw = (nb + 3) / 4 + 1;
          const float inv = 1.0f / (float)ndw;
          for (int it = tid - 64 * (kVW + kHW); it < rows_here * ndw; it += 64 * kSW) {
            const int yl = (int)(((float)it + 0.5f) * inv), d = it - yl * ndw;
            uint8_t *a0 = D.dst + (int64_t)(16 * b + yl) * D.dst_stride + (int64_t)D.x0 * oc;
            const int k0 = 4 * d - (int)((uintptr_t)a0 & 3u);
            if (k0 >= nb) continue;
            if (k0 >= 0 && k0 + 4 <= nb) {
              const uint32_t wd = out_byte(yl, k0) | (out_byte(yl, k0 + 1) << 8) | (out_byte(yl, k0 + 2) << 16) |
                                  (out_byte(yl, k0 + 3) << 24);
              *(g_u32 *)(a0 + k0) = wd;
            } else {
              for (int k = max(k0, 0); k < min(k0 + 4, nb); k++) *(g_u8 *)(a0 + k) = (uint8_t)out_byte(yl, k);
            }
          }
        } else {
          for (int it = tid - 64 * (kVW + kHW); it < rows_here * nx; it += 64 * kSW) {
            const int yl = it / nx, x = it - yl * nx, y = 16 * b + yl;
            const int ox = D.x0 + x;
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
            g_u8 *out = (g_u8 *)(D.dst + (int64_t)dy * D.dst_stride) + dx * oc;
            for (int c = 0; c < oc; c++) out[c] = (uint8_t)out_byte(yl, x * oc + c);
          }
        }
      }
      // dword-aligned fast8 stores of block p - 2: rows sw, sw + kSW, ... as dwords
      if (st_fast && (st_nb >> 2) <= 64) {
        // one destination dword per lane, row by row: the row base is scalar and
        // the tile row an immediate, so the copy needs no per-element VALU
        if (lane < (st_nb >> 2)) {
#pragma unroll
          for (int r = 0; r < 16; r++) {
            if (r >= st_nrow) break;
            *(g_u32 *)(st_row0 + r * st_stride + 4 * lane) =
                *reinterpret_cast<const uint32_t *>(st_ot + r * kSW * kOt8Pitch + 4 * lane);
          }
        }
      } else if (st_fast) {
        const int U = st_nb >> 2;
        const float invU = 1.0f / (float)U;
        for (int it0 = 0; it0 < st_nrow * U; it0 += 64) {
          const int it = it0 + lane;
          if (it < st_nrow * U) {
            const int r = (int)(((float)it + 0.5f) * invU), u = it - r * U;
            *(g_u32 *)(st_row0 + r * st_stride + 4 * u) =
                *reinterpret_cast<const uint32_t *>(st_ot + r * kSW * kOt8Pitch + 4 * u);
          }
        }
      }

      phase_barrier();
    }
    return;
  }

  // ============ H role: horizontal MFMA of the previous block ============
  const int hw = wv - kVW;  // 0 .. kHW - 1
  int ftile = -1, h_nx = 0, h_items = 0;
  bool h_fast8 = false;
  uint32_t h_sh0 = 0, h_shs = 0;
  i32x4 hb[2][2][2];
  int hw0k[2] = {0, 0}, hksk[2] = {0, 0};
  uint32_t hoff[2][2][2] = {};  // per item and k-step: this lane's two plane-column offsets (tile-constant)
  float hwsk[2] = {0.f, 0.f}, hscale = 0.f;
  __builtin_amdgcn_s_setprio(1);
  phase_barrier();
  phase_barrier();
  Rec rH{};  // record of the block this phase's horizontal pass takes (phase p - 1)
  if (kStamp) tprev = __builtin_amdgcn_s_memtime();
  for (int p = 0; p < N + 2; p++) {
    stamp(0);
    if (M != 1 && M != 2 && p >= 1 && p - 1 < N) {
      const Rec rh = rH;
      const int b = rh.blk;
      if (ftile != rh.t) {
        // a new tile: its strip's horizontal fragments and epilogue constants
        ftile = rh.t;
        const VrTile T = ldc(tiles + rh.t);
        const VDesc D = ldc(descs + T.img);
        const MStrip S = ldc(strips + T.strip);
        h_nx = S.x1 - S.x0;
        h_items = 3 * S.nocb;
        h_fast8 = !D.gray && D.rot == 0;
        h_sh0 = (uint32_t)(((uintptr_t)D.dst + (uint64_t)S.x0 * 3) & 3u);
        h_shs = (uint32_t)(D.dst_stride & 3);
        hscale = __builtin_amdgcn_ldexpf(1.0f, -D.hsh);
        const int nx = h_nx;
        const g_i32x4 *hf = (const g_i32x4 *)(ai + S.frag2);
#pragma unroll
        for (int k = 0; k < 2; k++) {
          const int it = hw + kHW * k, ob = it / 3;
          const bool ok = it < 3 * S.nocb;
          hw0k[k] = ok ? ldc1(ai + S.s0 + 2 * ob) : 0;
          hksk[k] = ok ? ldc1(ai + S.s0 + 2 * ob + 1) : 0;
#pragma unroll
          for (int t = 0; t < 2; t++) {
            const int cA = hw0k[k] + 64 * t + 16 * (lane >> 4) + ((lane & 15) >> 1);
            hoff[k][t][0] = (uint32_t)(col_off(cA) + 8 * (lane & 1));
            hoff[k][t][1] = (uint32_t)(col_off(cA + 8) + 8 * (lane & 1));
          }
          const int hx = 16 * ob + (lane & 15);
          hwsk[k] = (ok && hx < nx) ? 32896.0f * (float)ai[D.hwsum + S.x0 + hx] : 0.0f;
#pragma unroll
          for (int t = 0; t < 2; t++)
#pragma unroll
            for (int q = 0; q < 2; q++)
              hb[k][t][q] = (ok && t < S.ks) ? hf[((ob * S.ks + t) * 2 + q) * 64 + lane] : i32x4{0, 0, 0, 0};
        }
      }
      stamp(1);
      uint8_t *ot = otiles + ((rh.flags & kSlot) ? Lo.otile_bytes : 0);
      uint16_t *otile = reinterpret_cast<uint16_t *>(ot);
      const int nx = h_nx;
      const bool fast8 = h_fast8;
      const uint32_t sh0 = h_sh0, shs = h_shs;
      // both items' plane reads first, then the LDS counter frees the planes for
      // the V waves' next block; MFMAs and epilogues run on registers after that
      const int nk = (hw < h_items ? 1 : 0) + (hw + kHW < h_items ? 1 : 0);
      i32x4 Ahk[2][2], Alk[2][2];
#pragma unroll
      for (int k = 0; k < 2; k++) {
        const int it = hw + kHW * k;
        const int chn = it - 3 * (it / 3);
        const int hks = k < nk ? hksk[k] : 0;
        const uint8_t *ph = planes + ((Lo.pbuf == 2 && ((p - 1) & 1)) ? 6 * plane : 0) + chn * plane,
                      *pl = ph + 3 * plane;
#pragma unroll
        for (int t = 0; t < 2; t++) {
          if (t >= hks) break;
          const uint32_t o0 = hoff[k][t][0], o1 = hoff[k][t][1];
          const i32x2 h0 = tr8(ph + o0), h1 = tr8(ph + o1);
          const i32x2 l0 = tr8(pl + o0), l1 = tr8(pl + o1);
          Ahk[k][t] = i32x4{h0.x, h0.y, h1.x, h1.y};
          Alk[k][t] = i32x4{l0.x, l0.y, l1.x, l1.y};
        }
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      if (lane == 0 && Lo.pbuf == 1) atomicAdd(static_cast<unsigned *>(__builtin_assume_aligned(lds + O.cnt, 16)), 1u);
#pragma unroll
      for (int k = 0; k < 2; k++) {
        if (k >= nk) break;
        const int it = hw + kHW * k;
        const int ob = it / 3, chn = it - 3 * ob;
        const int hks = hksk[k];
        i32x4 hh[2], hl[2];
#pragma unroll
        for (int q = 0; q < 2; q++) hh[q] = hl[q] = i32x4{0, 0, 0, 0};
#pragma unroll
        for (int t = 0; t < 2; t++) {
          if (t >= hks) break;
#pragma unroll
          for (int q = 0; q < 2; q++) {
            hh[q] = mfma(Ahk[k][t], hb[k][t][q], hh[q]);
            hl[q] = mfma(Alk[k][t], hb[k][t][q], hl[q]);
          }
        }
        const int hx = 16 * ob + (lane & 15);
        if (hx < nx) {
          const float hws = hwsk[k];
          // the four rows' conversions first (independent chains, no branch
          // between them), then the stores in the tile's format
          uint32_t q[4];
          // two rows per packed op (v_pk_fma_f32 / v_pk_add_f32: the same IEEE
          // operations per element); 256 a + b as one fma: 256 a is exact in
          // f32, so the one rounding is the add's (bit-identical to the product
          // then the sum)
          typedef float f32x2 __attribute__((ext_vector_type(2)));
#pragma unroll
          for (int i = 0; i < 4; i += 2) {
            const f32x2 a = {(float)fold2(hh[0][i], hh[1][i]), (float)fold2(hh[0][i + 1], hh[1][i + 1])};
            const f32x2 c = {(float)fold2(hl[0][i], hl[1][i]), (float)fold2(hl[0][i + 1], hl[1][i + 1])};
            const f32x2 tot = __builtin_elementwise_fma(f32x2{256.0f, 256.0f}, a, c) + f32x2{hws, hws};
            const f32x2 r = __builtin_elementwise_fma(tot, f32x2{hscale, hscale}, f32x2{0.5f, 0.5f});
            q[i] = M == 8 ? ((uint32_t)hh[0][i] & 0xFFFFu)  // ablation: no H conversion
                          : min(__float2uint_rz(r.x), 65535u);
            q[i + 1] = M == 8 ? ((uint32_t)hh[0][i + 1] & 0xFFFFu) : min(__float2uint_rz(r.y), 65535u);
          }
          if (fast8) {
#pragma unroll
            for (int i = 0; i < 4; i++) {
              const int yl = 4 * (lane >> 4) + i;
              const int sh = (int)((sh0 + (uint32_t)(16 * b + yl) * shs) & 3u);
              ot[yl * kOt8Pitch + sh + 3 * hx + chn] = (uint8_t)q16_to_u8(q[i]);
            }
          } else {
#pragma unroll
            for (int i = 0; i < 4; i++) otile[(4 * (lane >> 4) + i) * kVmOtilePitch + 3 * hx + chn] = (uint16_t)q[i];
          }
        }
      }
      stamp(2);
    } else if (M != 1 && M != 2 && p < N + 1) {
      // no block this phase (p == 0): count the (empty) plane reads
      if (lane == 0 && Lo.pbuf == 1) atomicAdd(static_cast<unsigned *>(__builtin_assume_aligned(lds + O.cnt, 16)), 1u);
    }
    stamp(3);
    if (p < N) rH = read_rec(p);
    phase_barrier();
    stamp(4);
  }
  stamp_out(5);
}

int vr_read_stamps(uint64_t *out, int slots) {
  if (slots > kVrStampSlots) slots = kVrStampSlots;
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_vr_stamps), (size_t)slots * kVrStampN * sizeof(uint64_t)) == hipSuccess
             ? 0
             : -1;
}

// LDS of a launch: the ring takes what the other regions leave (R a multiple
// of 32, at most 256 rows); R = 0 when even the smallest ring does not fit
VrLayout vr_lds_layout(int vpitch, bool q16, int pbuf) {
  VrLayout L{};
  L.plane = 16 * vpitch + kPlanePad;
  L.otile_bytes = ((q16 ? kVmOtileBytes : 16 * kOt8Pitch) + 15) & ~15;
  L.pbuf = pbuf == 2 ? 2 : 1;
  const int rest = 2 * kABytes + 8 * kRecBytes + 16 + kLutSlots * 1024 + 6 * L.pbuf * L.plane;
  const int fixed = ((rest + 15) & ~15) + 2 * L.otile_bytes;
  int R = (kVrMaxLds - fixed) / 512 / 32 * 32;
  if (R > 256) R = 256;
  if (R < 160) R = 0;
  L.R = R;
  L.otile_off = (R * 512 + rest + 15) & ~15;
  L.total = L.otile_off + 2 * L.otile_bytes;
  return L;
}

int launch_vr(hipStream_t s, const VDesc *descs, const MStrip *strips, const VrTile *tiles, int ntiles,
              const int32_t *wginfo, int G, const int32_t *ai, VrLayout L) {
  if (ntiles <= 0 || G <= 0) return 0;
  if (L.R <= 0 || L.total > kVrMaxLds || (L.nl != 2 && L.nl != 4)) return -1;
  // FI_VR_VARIANT: profiling ablations (1-3, 11-13: wrong pixels, reported by
  // the return value 1, which the caller counts as stat "vr_ablation") and the
  // per-phase stamps (9: production pixels)
  static const char *variant = getenv("FI_VR_VARIANT");
  const int v = variant ? atoi(variant) : 0;
#define FI_VR_LAUNCH(m)                                                                                    \
  do {                                                                                                     \
    if (L.nl == 4)                                                                                         \
      hipLaunchKernelGGL((k_rs_vr<m, 4>), dim3(G), dim3(1024), L.total, s, descs, strips, tiles, ntiles, wginfo, \
                         ai, L);                                                                           \
    else                                                                                                   \
      hipLaunchKernelGGL((k_rs_vr<m, 2>), dim3(G), dim3(1024), L.total, s, descs, strips, tiles, ntiles, wginfo, \
                         ai, L);                                                                           \
  } while (0)
  switch (v) {
    case 1: FI_VR_LAUNCH(1); break;
    case 2: FI_VR_LAUNCH(2); break;
    case 3: FI_VR_LAUNCH(3); break;
    case 5: FI_VR_LAUNCH(5); break;
    case 4: FI_VR_LAUNCH(4); break;
    case 6: FI_VR_LAUNCH(6); break;
    case 7: FI_VR_LAUNCH(7); break;
    case 8: FI_VR_LAUNCH(8); break;
    case 9: FI_VR_LAUNCH(9); break;
    case 14: FI_VR_LAUNCH(14); break;
    case 11: FI_VR_LAUNCH(11); break;
    case 12: FI_VR_LAUNCH(12); break;
    case 13: FI_VR_LAUNCH(13); break;
    default: FI_VR_LAUNCH(0); break;
  }
#undef FI_VR_LAUNCH
  return (v == 1 || v == 2 || v == 3 || v == 4 || v == 7 || v == 8 || v == 11 || v == 12 || v == 13 || v == 14) ? 1
                                                                                                             : 0;
}

}  // namespace fi
