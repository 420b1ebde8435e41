// fi_vp.hip -- ImageMagick ResizeImage, vertical pass first (the
// ThumbnailImage sample pre-step folded into the tap tables), as a persistent,
// warp-specialised, exact-integer matrix-core pipeline: v_mfma_i32_16x16x64_i8.
//
// Same arithmetic and host tables as k_rs_vm (fi_vm.hip, fi_plan.h VmV /
// MfmaH): weights W = rint(w 2^22) in three signed-byte limbs, pixels as
// p - 128, every product exact in int32, one float conversion per pass, so the
// two kernels are bit-identical.  What differs is the dataflow:
//
//  * one 1024-thread workgroup per CU, persistent: workgroup g takes the tiles
//    (image, 512-byte column strip, row pieces) g, g + G, g + 2G, ... and walks
//    their pieces as ONE stream, so the memory pipeline never drains between
//    tiles (the host orders tiles so that g % 8 keeps an image on one XCD);
//  * phase p of the stream has ONE workgroup barrier, and two roles run in it
//    side by side:
//      V waves 0-7   LDS-DMA the source rows of piece p + 2 (64 rows x 512 B,
//                    global_load_lds_dwordx4, 3-slot ring) and the weight
//                    fragments of piece p + 1 (2-slot ring), then run piece
//                    p's vertical MFMAs; when p completes block b they write
//                    b's Q16 planes into plane slot s (two slots);
//      H waves 8-15  run the horizontal MFMAs of the block completed in phase
//                    p - 1 (plane slot s^1 -> output tile slot s^1), store the
//                    block completed in p - 2 from the other output tile, and
//                    stage the compact-column LUT of the next tile;
//    so source bytes are in flight two phases ahead, the vertical MFMAs of one
//    block overlap the horizontal MFMAs and stores of the previous one, and no
//    wave waits for another role inside a phase;
//  * the DMAs are inline asm (hipcc would otherwise wait vmcnt(0) before every
//    LDS read); every vmcnt wait of the V loop is explicit and exact, and the
//    V loop holds no compiler-visible vector-memory instruction.  The piece
//    bytes land raw; the XOR to p - 128 is applied to the B operand.
//
// LDS (vp_lds_layout): ring 3 x 32 KB | A ring 2 x 6336 B | records 8 x 16 B |
// LUT 4 x 1 KB | Q16 planes 2 x 6 x plane | output tile 2 x (8-bit or Q16).
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
typedef __attribute__((address_space(1))) uint64_t g_u64;
typedef __attribute__((address_space(1))) uint16_t g_u16;
typedef __attribute__((address_space(3))) i32x2 l_i32x2;
typedef __attribute__((address_space(3))) uint8_t l_u8;

constexpr int kVW = 8;                 // V waves (one 64-byte column group of the strip each)
constexpr int kRing = 3;               // source piece slots
constexpr int kPieceBytes = 64 * 512;  // 64 rows x 512 B
constexpr int kABytes = 6144 + 192;    // [slot][limb][64 lanes][16 B] + w128 rows of blocks b, b + 1, b + 2
constexpr int kAOff = kRing * kPieceBytes;
constexpr int kRecOff = kAOff + 2 * kABytes;
constexpr int kLutOff = kRecOff + 8 * 16;
constexpr int kLutSlots = 4;
constexpr int kPlanesOff = kLutOff + kLutSlots * 1024;
constexpr int kPlanePad = 176;  // 44 (mod 64) dwords: see fi_vm.hip kVmPlanePad
constexpr int kOt8Pitch = 200;  // 8-bit output tile row (<= 64 px x 3 + the row shift; 8-byte aligned rows)
static_assert(kPlanesOff % 16 == 0, "LDS layout");

// record flags (one record per piece of the stream, written by V wave 0 two
// phases ahead of the piece's compute)
constexpr int kLast = 1;    // the piece completes its block
constexpr int kEmit = 2;    // ... and the block is emitted (>= the tile's emit0)
constexpr int kFirst = 4;   // first piece of a tile
constexpr int kSlot = 8;    // plane / output-tile slot of the emitted block
constexpr int kTslotShift = 4;  // bits 4-5: LUT slot of the tile (tile sequence number mod 4)

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
__device__ __forceinline__ int32_t fold3(int32_t d0, int32_t d1, int32_t d2) {
  return (int32_t)((uint32_t)d0 + ((uint32_t)d1 << 8) + ((uint32_t)d2 << 16));
}
__device__ __forceinline__ uint32_t lds_addr(const uint8_t *p) { return (uint32_t)(uintptr_t)(const l_u8 *)p; }
// Read-only tables through the constant address space: the DMA asm clobbers
// "memory", after which hipcc no longer proves plain loads invariant and
// turns wave-uniform reads into vector loads -- whose waits (vmcnt(0)) would
// drain the DMA stream.  Constant-space loads stay scalar (lgkmcnt).
template <class T>
__device__ __forceinline__ const __attribute__((address_space(4))) T *cs(const T *p) {
  return (const __attribute__((address_space(4))) T *)p;
}
// a whole table record through the constant address space, one dword at a time
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
__device__ __forceinline__ int ufl(int x) { return __builtin_amdgcn_readfirstlane(x); }

// LDS-DMA, saddr form: lane i's 16 bytes at sbase + voff land at LDS m0 + 16 i.
// Invisible to hipcc's waitcnt pass: the V loop waits for it explicitly.
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
// the phase barrier without hipcc's vmcnt(0): LDS (and scalar) accesses
// drained, the DMAs stay in flight
__device__ __forceinline__ void phase_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }
__device__ __forceinline__ void wait_vm0() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

struct Rec {  // 16 B in LDS
  int32_t t, piece, blk, flags;
};
}  // namespace

// per-wave phase sums of MODE 9 (fi_debug_vp_stamps, tools/vp_timing.py):
// [workgroup][wave][6]: up to 5 phase sums (by role: V / H / L), [5] = phases
constexpr int kVpStampSlots = 256;
constexpr int kVpStampN = 16 * 6;
__device__ uint64_t g_vp_stamps[kVpStampSlots * kVpStampN];

constexpr int kHW = 6;                  // H waves 8-13
constexpr int kLW = 2;                  // L (loader) waves 14-15
constexpr int kLDma = 32 / kLW;         // piece DMAs per L wave (1 KB = rows 2 i, 2 i + 1 each)
static_assert(kVW + kHW + kLW == 16, "16 waves");

// MODE (profiling ablations, FI_VP_VARIANT; wrong pixels): 0 production,
// 1 DMA stream only, 2 no H role (vertical pass + planes only), 3 no stores,
// 4 H waves take one horizontal item each (the rest skipped), 5 V waves skip
// their piece reads, 6 H waves skip their plane reads, 7 V waves skip the MFMAs, 8 H role idle
// (stores kept), 9 H without its epilogue, 20 L prio 3 / H prio 0, 21 H prio 0, 9 production +
// per-phase s_memtime sums of V wave 0, H wave 8, L wave 14.
template <int MODE>
__global__ __launch_bounds__(1024, 1) void k_rs_vp(const VDesc *__restrict__ descs, const MStrip *__restrict__ strips,
                                                   const VTile *__restrict__ tiles, int ntiles,
                                                   const int32_t *__restrict__ nphase, const int32_t *__restrict__ ai,
                                                   VpLayout Lo) {
  constexpr int M = MODE >= 10 ? MODE - 10 : MODE;  // 10 + k: ablation k with the MODE 9 stamps
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wv = ufl(tid >> 6);
  const int G = (int)gridDim.x, g = (int)blockIdx.x;
  const int N = cs(nphase)[g];  // pieces of this workgroup's stream
  Rec *recs = reinterpret_cast<Rec *>(lds + kRecOff);
  const int32_t *lut = reinterpret_cast<const int32_t *>(lds + kLutOff);  // [kLutSlots][256]
  uint8_t *planes = lds + kPlanesOff;                           // [2][6][plane]
  uint8_t *otiles = lds + Lo.otile_off;                         // [2][otile_bytes]
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
  auto stamp_out = [&](int, int n) {
    if (kStamp && lane == 0 && g < kVpStampSlots) {
      uint64_t *o = g_vp_stamps + g * kVpStampN + 6 * wv;
      for (int k = 0; k < 5; k++) o[k] = k < n ? tsum[k] : 0;
      o[5] = (uint64_t)N;
    }
  };
  auto read_rec = [&](int s) -> Rec {
    const Rec x = recs[s & 7];
    return Rec{ufl(x.t), ufl(x.piece), ufl(x.blk), ufl(x.flags)};
  };

  if (wv >= kVW + kHW) {
    // ============ L role: the stream cursor, all DMAs, the records ============
    const int li = wv - (kVW + kHW);
    const int h = lane >> 5;  // half-wave: the two rows of one 1-KB DMA
    int ck = 0, ct = g, cp = 0, cp1 = 0, cp0 = 0, c_emit0 = 0, nemit = 0;
    const uint8_t *c_src = nullptr;
    int64_t c_stride = 0;
    int c_b0 = 0, c_nbytes = 0, c_rows = 0, c_nrows = 0, c_row0 = 0, c_rstep = 0, c_pmeta = 0, c_frag = 0,
        c_w128 = 0, c_lut = 0, c_lut_n = 0;
    auto load_tile = [&]() {
      const VTile T = ldc(tiles + ct);
      const VDesc D = ldc(descs + T.img);
      const MStrip S = ldc(strips + T.strip);
      cp = cp0 = T.p0;
      cp1 = T.p1;
      c_emit0 = T.emit0;
      c_src = D.src;
      c_stride = D.src_stride;
      c_b0 = S.b0;
      c_nbytes = S.nbytes;
      c_rows = D.rows;
      c_nrows = D.nrows;
      c_row0 = D.row0;
      c_rstep = D.rstep;
      c_pmeta = D.pmeta;
      c_frag = D.frag;
      c_w128 = D.w128;
      c_lut = S.lut;
      c_lut_n = S.lut_n;
    };
    // per-lane 16-byte chunk offsets of this wave's DMAs (k_rs_vp's chunk
    // swizzle, chunks past the strip clamped to 0), four patterns by DMA index
    // j: (j & 1) and ((j >> 2) & 1) fix the row's f (fast path below); the
    // second half-wave's row-gap offset folded in
    uint32_t patv[4] = {0, 0, 0, 0};
    int64_t c_gap = 0;  // bytes between consecutive touched rows (rstep > 0)
    auto tile_pats = [&]() {
      c_gap = c_rstep > 0 ? (int64_t)c_rstep * c_stride : 0;
#pragma unroll
      for (int k = 0; k < 4; k++) {
        const int j = (k & 1) | ((k >> 1) << 2);
        const int rr = 2 * (li + 2 * j) + h;
        const int f = (rr & 7) | (((rr >> 4) & 1) << 3);
        int lc = (lane & 31) ^ f;
        if (16 * lc >= c_nbytes) lc = 0;
        patv[k] = (h ? (uint32_t)c_gap : 0u) + 16u * (uint32_t)lc;
      }
    };
    if (ct < ntiles) {
      load_tile();
      tile_pats();
    }
    struct PI {
      int piece, blk, frag, w128;
    };
    // the cursor's piece -> ring slot `slot` (this wave's kLDma DMAs), its record; advance
    auto issue = [&](int s, int slot) -> PI {
      const int4 m = ldc(reinterpret_cast<const int4 *>(ai + c_pmeta + 4 * cp));  // {lo, n, blk, last}
      PI r{cp, m.z, c_frag, c_w128};
      if (li == 0 && lane == 0) {
        int fl = 0;
        if (m.w) fl |= kLast;
        if (m.w && m.z >= c_emit0) fl |= kEmit | ((nemit & 1) ? kSlot : 0);
        if (cp == cp0) fl |= kFirst;
        fl |= (ck & (kLutSlots - 1)) << kTslotShift;
        recs[s & 7] = Rec{ct, cp, m.z, fl};
      }
      if (cp == cp0 && li == 0 && lane < (c_lut_n + 3) / 4) {
        // the tile's px -> compact-column LUT (int32, <= 256 entries) with its first
        // piece, ahead of the piece's DMAs: the end-of-phase vmcnt covers it
        dma16(lds_addr(lds) + (uint32_t)(kLutOff + (ck & (kLutSlots - 1)) * 1024),
              reinterpret_cast<const uint8_t *>(ai + c_lut), 16u * lane);
      }
      if (m.w && m.z >= c_emit0) nemit++;
      const int lo = m.x, nl = m.y > 0 ? m.y - 1 : 0;
      const uint32_t m0 = lds_addr(lds) + (uint32_t)(slot * kPieceBytes);
      if (c_rstep > 0 && lo + 63 < c_nrows) {
        // fast path: evenly spaced rows and all 64 list rows inside the image
        // (rows past the piece carry zero weights): the DMA bases are linear
        // in the DMA index, the lane offsets come from patv
        const uint8_t *b = c_src + (int64_t)(c_row0 + c_rstep * lo) * c_stride + c_b0 + 2 * li * c_gap;
#pragma unroll
        for (int j = 0; j < kLDma; j++) {
          dma16(m0 + 1024 * (li + kLW * j), b, patv[(j & 1) | (((j >> 2) & 1) << 1)]);
          b += 2 * kLW * c_gap;
        }
      } else
#pragma unroll 4
      for (int j = 0; j < kLDma; j++) {
        const int i = li + kLW * j;  // DMA instruction i: rows 2 i (half 0) and 2 i + 1 (half 1)
        const int ra = 2 * i;
        const int k0 = min(lo + min(ra, nl), c_nrows - 1), k1 = min(lo + min(ra + 1, nl), c_nrows - 1);
        const int r0 = c_rstep > 0 ? c_row0 + c_rstep * k0 : cs(ai)[c_rows + k0];
        const int r1 = c_rstep > 0 ? c_row0 + c_rstep * k1 : cs(ai)[c_rows + k1];
        const uint8_t *base = c_src + (int64_t)r0 * c_stride + c_b0;
        const int rr = ra + h;
        const int f = (rr & 7) | (((rr >> 4) & 1) << 3);  // chunk swizzle of row rr
        int lc = (lane & 31) ^ f;
        if (16 * lc >= c_nbytes) lc = 0;
        const uint32_t voff = (h ? (uint32_t)((int64_t)(r1 - r0) * c_stride) : 0u) + 16u * (uint32_t)lc;
        dma16(m0 + 1024 * i, base, voff);
      }
      cp++;
      if (cp >= cp1) {
        ck++;
        ct = g + ck * G;
        if (ct < ntiles) {
          load_tile();
          tile_pats();
        }
      }
      return r;
    };
    // A record of piece r (fragments + w128 rows of blocks blk .. blk + 2) into A slot `slot`
    auto issue_a = [&](const PI &r, int slot) {
      const uint32_t m0 = lds_addr(lds) + (uint32_t)(kAOff + slot * kABytes);
      for (int i = li; i < 7; i += kLW) {
        if (i < 6)
          dma16(m0 + 1024 * i, reinterpret_cast<const uint8_t *>(ai + r.frag) + (size_t)r.piece * 6144 + 1024 * i,
                16u * lane);
        else if (lane < 12)
          dma16(m0 + 6144, reinterpret_cast<const uint8_t *>(ai + r.w128) + 64 * r.blk, 16u * lane);
      }
    };
    // the loader's few instructions go first on its SIMD: a starved loader
    // starves the whole pipeline
    if (M == 20)
      __builtin_amdgcn_s_setprio(3);
    else
      __builtin_amdgcn_s_setprio(2);
    PI P1{};
    if (N > 0) {
      const PI P0 = issue(0, 0);
      if (M != 1) issue_a(P0, 0);
    }
    if (N > 1) P1 = issue(1, 1);
    if (N > 1)
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(kLDma) : "memory");
    else
      wait_vm0();
    phase_barrier();  // records 0 / 1 and the first tile's LUT visible
    phase_barrier();
    int rslot = 0;    // ring slot of piece p
    if (kStamp) tprev = __builtin_amdgcn_s_memtime();
    int stile = -1;  // tile of the cached store descriptors
    struct StoreD {
      uint8_t *dst;
      int64_t dst_stride;
      int32_t ew, eh, rot, gray;
    } sD{};
    int sx0 = 0, sx1 = 0;
    for (int p = 0; p < N + 2; p++) {
      // stores of the block completed in phase p - 2 (the other output tile), by
      // the loader waves: their vector-memory issue already waits on HBM, the
      // compute waves' would not.  Dword-aligned 8-bit segments (the common
      // case) go after this phase's DMAs, a fixed small number of 8-byte-unit
      // stores whose count the end-of-phase vmcnt takes into account; the other
      // output kinds go before the DMAs, covered by that vmcnt as it is.
      bool st_fast = false;
      uint8_t *st_row0 = nullptr;
      int64_t st_stride = 0;
      int st_nb = 0, st_nrow = 0;
      const uint8_t *st_ot = nullptr;
      if (p >= 2 && p - 2 < N && M != 3 && M != 1 && M != 2) {
        const Rec rs = read_rec(p - 2);
        if (rs.flags & kEmit) {
          if (stile != rs.t) {
            stile = rs.t;
            const VTile T = ldc(tiles + rs.t);
            const VDesc D0 = ldc(descs + T.img);
            const MStrip S0 = ldc(strips + T.strip);
            sD = StoreD{D0.dst, D0.dst_stride, D0.ew, D0.eh, D0.rot, D0.gray};
            sx0 = S0.x0;
            sx1 = S0.x1;
          }
          const StoreD &D = sD;
          struct {
            int x0, x1;
          } S{sx0, sx1};
          const int b = rs.blk;
          const int nx = S.x1 - S.x0;
          const int oc = D.gray ? 1 : 3;
          const int rows_here = min(16, D.eh - 16 * b);
          const int nb = nx * oc;
          uint8_t *ot = otiles + ((rs.flags & kSlot) ? Lo.otile_bytes : 0);
          const uint16_t *otile = reinterpret_cast<const uint16_t *>(ot);
          const bool fastA = !D.gray && D.rot == 0 && (((uintptr_t)D.dst + (uint64_t)S.x0 * 3) & 3u) == 0 &&
                             (D.dst_stride & 3) == 0 && (nb & 3) == 0;
          if (fastA) {
            st_fast = true;
            st_row0 = D.dst + (int64_t)(16 * b + li) * D.dst_stride + (int64_t)S.x0 * 3;
            st_stride = (int64_t)kLW * D.dst_stride;
            st_nb = nb;
            st_nrow = (rows_here - li + kLW - 1) / kLW;
            st_ot = ot + li * kOt8Pitch;
          }
          auto out_byte = [&](int yl, int k) -> uint32_t {
            const uint16_t *o = otile + yl * kVmOtilePitch;
            if (!D.gray) return q16_to_u8(o[k]);
            return q16_to_u8(gray_q16(o[3 * k], o[3 * k + 1], o[3 * k + 2]));
          };
          if (D.gray == 2) {
            for (int it = tid - 64 * (kVW + kHW); it < rows_here * nx; it += 64 * kLW) {
              const int yl = it / nx, x = it - yl * nx;
              const uint16_t *o = otile + yl * kVmOtilePitch + 3 * x;
              ((g_u16 *)(D.dst + (int64_t)(16 * b + yl) * D.dst_stride))[S.x0 + x] = (uint16_t)gray_q16(o[0], o[1], o[2]);
            }
          } else if (fastA) {
            // dword-aligned fast8 segments: stored after this phase's DMAs (below)
          } else if (!D.gray && D.rot == 0) {
            // fast8: L wave li copies rows li, li + 2, ..., one destination dword per lane
            const uint32_t sh0 = (uint32_t)(((uintptr_t)D.dst + (uint64_t)S.x0 * 3) & 3u);
            const uint32_t shs = (uint32_t)(D.dst_stride & 3);
            constexpr int kRows = 16 / kLW;
            uint32_t wd[kRows];
#pragma unroll
            for (int r = 0; r < kRows; r++) wd[r] = *reinterpret_cast<const uint32_t *>(ot + (li + kLW * r) * kOt8Pitch + 4 * lane);
#pragma unroll
            for (int r = 0; r < kRows; r++) {
              const int yl = li + kLW * r;
              if (yl >= rows_here) break;
              const int sh = (int)((sh0 + (uint32_t)(16 * b + yl) * shs) & 3u);
              const int k0 = 4 * lane - sh;
              uint8_t *a0 = D.dst + (int64_t)(16 * b + yl) * D.dst_stride + (int64_t)S.x0 * 3;
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
            for (int it = tid - 64 * (kVW + kHW); it < rows_here * ndw; it += 64 * kLW) {
              const int yl = (int)(((float)it + 0.5f) * inv), d = it - yl * ndw;
              uint8_t *a0 = D.dst + (int64_t)(16 * b + yl) * D.dst_stride + (int64_t)S.x0 * oc;
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
            for (int it = tid - 64 * (kVW + kHW); it < rows_here * nx; it += 64 * kLW) {
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
              g_u8 *out = (g_u8 *)(D.dst + (int64_t)dy * D.dst_stride) + dx * oc;
              for (int c = 0; c < oc; c++) out[c] = (uint8_t)out_byte(yl, x * oc + c);
            }
          }
        }
      }
      if (M == 22 && st_fast) {  // ablation: the fast stores at the top of the phase
        const int U = st_nb >> 2;
        const float invU = 1.0f / (float)U;
        for (int it0 = 0; it0 < st_nrow * U; it0 += 64) {
          const int it = it0 + lane;
          if (it < st_nrow * U) {
            const int r = (int)(((float)it + 0.5f) * invU), u = it - r * U;
            *(g_u32 *)(st_row0 + r * st_stride + 4 * u) =
                *reinterpret_cast<const uint32_t *>(st_ot + r * kLW * kOt8Pitch + 4 * u);
          }
        }
      }
      if (M != 1 && p + 1 < N) issue_a(P1, (p + 1) & 1);
      stamp(0);
      const bool more = p + 2 < N;
      PI P2{};
      if (more) P2 = issue(p + 2, rslot == 0 ? 2 : rslot - 1);
      stamp(1);
      // dword-aligned fast8 stores of block p - 2: this wave's rows li, li + 2, ...
      // as dwords (lane -> row, dword), ns = store instructions issued
      int ns = 0;
      if (st_fast && M != 22) {
        const int U = st_nb >> 2;
        const float invU = 1.0f / (float)U;
        for (int it0 = 0; it0 < st_nrow * U; it0 += 64, ns++) {
          const int it = it0 + lane;
          if (it < st_nrow * U) {
            const int r = (int)(((float)it + 0.5f) * invU), u = it - r * U;
            *(g_u32 *)(st_row0 + r * st_stride + 4 * u) =
                *reinterpret_cast<const uint32_t *>(st_ot + r * kLW * kOt8Pitch + 4 * u);
          }
        }
      }
      // piece p + 1 and A(p + 1) landed; this wave's DMAs of piece p + 2 and the
      // ns stores after them may stay in flight (vmcnt counts in issue order)
      if (!more)
        wait_vm0();
      else if (ns == 0)
        asm volatile("s_waitcnt vmcnt(%0)" ::"n"(kLDma) : "memory");
      else if (ns == 1)
        asm volatile("s_waitcnt vmcnt(%0)" ::"n"(kLDma + 1) : "memory");
      else if (ns == 2)
        asm volatile("s_waitcnt vmcnt(%0)" ::"n"(kLDma + 2) : "memory");
      else if (ns == 3)
        asm volatile("s_waitcnt vmcnt(%0)" ::"n"(kLDma + 3) : "memory");
      else if (ns == 4)
        asm volatile("s_waitcnt vmcnt(%0)" ::"n"(kLDma + 4) : "memory");
      else if (ns == 5)
        asm volatile("s_waitcnt vmcnt(%0)" ::"n"(kLDma + 5) : "memory");
      else
        asm volatile("s_waitcnt vmcnt(%0)" ::"n"(kLDma + 6) : "memory");
      stamp(2);
      phase_barrier();
      stamp(3);
      P1 = P2;
      rslot = rslot == kRing - 1 ? 0 : rslot + 1;
    }
    stamp_out(10, 4);
    return;
  }

  if (wv < kVW) {
    // =================== V role: vertical MFMA + Q16 planes ===================
    // Waves 0-3 and 4-7 cover the same four 128-byte column groups (8 tiles of
    // 16 B each) and split the two accumulator slots: at any time one group
    // holds the current block (slot 0) and the other the next one (slot 1).
    // When a piece completes the current block its group converts it to the
    // Q16 planes and takes up block + 2, while the other group's block becomes
    // current -- so on every SIMD one V wave converts while its partner issues
    // MFMAs, instead of both doing the same thing at the same time.
    const int w = wv, grp = w >> 2, cg = w & 3;
    constexpr int kT = 8;  // tiles per wave
    const int rA = 16 * (lane >> 4) + ((lane & 15) >> 1);
    const int fA = (rA & 7) | (((rA >> 4) & 1) << 3);
    // transposing-read offset of tile j: chunk (8 cg + j) ^ fA = (8 cg ^ (fA & 8)) + (j ^ (fA & 7))
    const int offA0 = rA * 512 + 16 * ((kT * cg) ^ (fA & 8)) + 8 * (lane & 1), fA7 = fA & 7;
    uint32_t vcolp[kT / 2] = {0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu};
    i32x4 acc[kT];
#pragma unroll
    for (int j = 0; j < kT; j++) acc[j] = i32x4{0, 0, 0, 0};
    int own = grp;  // slot this wave's accumulators belong to (0: the current block)
    phase_barrier();
    phase_barrier();
    int rslot = 0;
    // this phase's record (piece p), read one phase early so its LDS latency
    // hides in the barrier wait
    Rec rC = N > 0 ? read_rec(0) : Rec{};
    if (kStamp) tprev = __builtin_amdgcn_s_memtime();
    for (int p = 0; p < N + 2; p++) {
      if (p < N && M != 1) {
        const Rec C = rC;
        const uint8_t *sp = lds + rslot * kPieceBytes;
        const i32x4 *al = reinterpret_cast<const i32x4 *>(lds + kAOff + (p & 1) * kABytes);
        if (C.flags & kFirst) {
          // new tile: group 0 starts the first block, group 1 the second, each at
          // its weight correction; Q16-plane offsets of this lane's columns from
          // the staged LUT
          own = grp;
          const VTile T = ldc(tiles + C.t);
          const MStrip S = ldc(strips + T.strip);
          const int32_t *lt = lut + 256 * ((C.flags >> kTslotShift) & (kLutSlots - 1));
#pragma unroll
          for (int j = 0; j < kT; j++) {
            acc[j] = al[384 + 4 * own + (lane >> 4)];
            const int col = 128 * cg + 16 * j + (lane & 15);
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
        i32x4 A[3];
#pragma unroll
        for (int q = 0; q < 3; q++) A[q] = al[(own * 3 + q) * 64 + lane];
        // two halves of four tiles; in each, limb 2 of every tile first, then
        // limb 1, then limb 0: each dependent MFMA issues 4 MFMAs after its producer
#pragma unroll
        for (int hf = 0; hf < 2; hf++) {
          i32x4 B[4], d[4];
#pragma unroll
          for (int jj = 0; jj < 4; jj++) {
            const int o = offA0 + 16 * ((4 * hf + jj) ^ fA7);
            const i32x2 lo = M == 5 ? i32x2{lane ^ p, o} : tr8(sp + o), hi = M == 5 ? i32x2{o, lane + jj} : tr8(sp + o + 8 * 512);
            B[jj] = i32x4{lo.x, lo.y, hi.x, hi.y} ^
                    i32x4{(int)0x80808080, (int)0x80808080, (int)0x80808080, (int)0x80808080};
          }
#pragma unroll
          for (int jj = 0; jj < 4; jj++) d[jj] = M == 7 ? (A[2] ^ B[jj]) : mfma(A[2], B[jj], i32x4{0, 0, 0, 0});
#pragma unroll
          for (int jj = 0; jj < 4; jj++) d[jj] = M == 7 ? (A[1] + B[jj] + (d[jj] << 8)) : mfma(A[1], B[jj], d[jj] << 8);
#pragma unroll
          for (int jj = 0; jj < 4; jj++)
            acc[4 * hf + jj] = (M == 7 ? (A[0] + B[jj] + acc[4 * hf + jj]) : mfma(A[0], B[jj], acc[4 * hf + jj])) + (d[jj] << 8);
        }
        stamp(1);
        if (C.flags & kLast) {
          if (own == 0) {
            if (C.flags & kEmit) {
              // block done: ClampToQuantum(257 acc / 2^22) -> Q16 hi / lo signed-byte planes
              uint8_t *vpl = planes + ((C.flags & kSlot) ? 6 * plane : 0);
#pragma unroll
              for (int j = 0; j < kT; j++) {
                const uint32_t o = (vcolp[j >> 1] >> (16 * (j & 1))) & 0xFFFFu;
                uint32_t q[4];
#pragma unroll
                for (int i = 0; i < 4; i++) q[i] = __float2uint_rz(fmaf((float)acc[j][i], 257.0f / 4194304.0f, 0.5f));
                const auto p01 = __builtin_amdgcn_cvt_pk_u16(q[0], q[1]);
                const auto p23 = __builtin_amdgcn_cvt_pk_u16(q[2], q[3]);
                const uint32_t x01 = __builtin_bit_cast(uint32_t, p01) ^ 0x80808080u;
                const uint32_t x23 = __builtin_bit_cast(uint32_t, p23) ^ 0x80808080u;
                if (o != 0xFFFFu) {
                  *reinterpret_cast<uint32_t *>(vpl + o) = __builtin_amdgcn_perm(x23, x01, 0x07050301u);
                  *reinterpret_cast<uint32_t *>(vpl + o + 3 * plane) = __builtin_amdgcn_perm(x23, x01, 0x06040200u);
                }
              }
            }
            // this group takes up block + 2 at its weight correction
            const i32x4 W2 = al[392 + (lane >> 4)];
#pragma unroll
            for (int j = 0; j < kT; j++) acc[j] = W2;
            own = 1;
          } else {
            own = 0;  // the other group's block completed: ours is now the current one
          }
        }
      }
      stamp(2);
      if (p + 1 < N) rC = read_rec(p + 1);
      phase_barrier();
      stamp(3);
      rslot = rslot == kRing - 1 ? 0 : rslot + 1;
    }
    stamp_out(0, 4);
    return;
  }

  // ============ H role: horizontal MFMA + stores + LUT staging ============
  const int hw = wv - kVW;  // 0 .. kHW - 1
  // horizontal weight fragments of the current tile (items hw, hw + kHW)
  int ftile = -1, h_nx = 0, h_items = 0;
  bool h_fast8 = false;
  uint32_t h_sh0 = 0, h_shs = 0;
  i32x4 hb[2][2][3];
  int hw0k[2] = {0, 0}, hksk[2] = {0, 0};
  float hwsk[2] = {0.f, 0.f};

  // the horizontal pass of the previous block is the longest chain of a phase:
  // it issues ahead of the vertical waves (the loader still goes first)
  if (M != 20 && M != 21) __builtin_amdgcn_s_setprio(1);
  phase_barrier();
  phase_barrier();
  Rec rH{};  // record of the block this phase's horizontal pass takes (piece p - 1), read a phase early
  if (kStamp) tprev = __builtin_amdgcn_s_memtime();
  for (int p = 0; p < N + 2; p++) {
    if (M != 1 && M != 2 && M != 18) {
      stamp(0);
      // horizontal pass of the block completed in phase p - 1
      if (p >= 1 && p - 1 < N) {
        const Rec rh = rH;
        if (rh.flags & kEmit) {
          const int b = rh.blk;
          if (ftile != rh.t) {
            // a new tile: its strip's horizontal fragments and epilogue constants
            ftile = rh.t;
            const VTile T = ldc(tiles + rh.t);
            const VDesc D = ldc(descs + T.img);
            const MStrip S = ldc(strips + T.strip);
            h_nx = S.x1 - S.x0;
            h_items = 3 * S.nocb;
            h_fast8 = !D.gray && D.rot == 0;
            h_sh0 = (uint32_t)(((uintptr_t)D.dst + (uint64_t)S.x0 * 3) & 3u);
            h_shs = (uint32_t)(D.dst_stride & 3);
            const int nx = h_nx;
            const g_i32x4 *hf = (const g_i32x4 *)(ai + S.frag);
#pragma unroll
            for (int k = 0; k < 2; k++) {
              const int it = hw + kHW * k, ob = it / 3;
              const bool ok = it < 3 * S.nocb;
              hw0k[k] = ok ? cs(ai)[S.s0 + 2 * ob] : 0;
              hksk[k] = ok ? cs(ai)[S.s0 + 2 * ob + 1] : 0;
              const int hx = 16 * ob + (lane & 15);
              hwsk[k] = (ok && hx < nx) ? 32896.0f * (float)ai[D.hwsum + S.x0 + hx] : 0.0f;
#pragma unroll
              for (int t = 0; t < 2; t++)
#pragma unroll
                for (int q = 0; q < 3; q++)
                  hb[k][t][q] = (ok && t < S.ks) ? hf[((ob * S.ks + t) * 3 + q) * 64 + lane] : i32x4{0, 0, 0, 0};
            }
          }
          stamp(1);
          const uint8_t *vpl = planes + ((rh.flags & kSlot) ? 6 * plane : 0);
          uint8_t *ot = otiles + ((rh.flags & kSlot) ? Lo.otile_bytes : 0);
          uint16_t *otile = reinterpret_cast<uint16_t *>(ot);
          const int nx = h_nx;
          const bool fast8 = h_fast8;
          const uint32_t sh0 = h_sh0, shs = h_shs;
#pragma unroll
          for (int k = 0; k < 2; k++) {
            const int it = hw + kHW * k;
            if (it >= h_items || (M == 4 && k > 0)) break;
            const int ob = it / 3, chn = it - 3 * ob;
            const int hw0 = hw0k[k], hks = hksk[k];
            i32x4 hh[3], hl[3];
#pragma unroll
            for (int q = 0; q < 3; q++) hh[q] = hl[q] = i32x4{0, 0, 0, 0};
            const uint8_t *ph = vpl + chn * plane, *pl = ph + 3 * plane;
#pragma unroll
            for (int t = 0; t < 2; t++) {
              if (t >= hks) break;
              const int cA = hw0 + 64 * t + 16 * (lane >> 4) + ((lane & 15) >> 1);
              const int o0 = col_off(cA) + 8 * (lane & 1), o1 = col_off(cA + 8) + 8 * (lane & 1);
              const i32x2 h0 = M == 6 ? i32x2{lane, o0} : tr8(ph + o0), h1 = M == 6 ? i32x2{o1, lane} : tr8(ph + o1);
              const i32x2 l0 = M == 6 ? i32x2{lane ^ o1, b} : tr8(pl + o0), l1 = M == 6 ? i32x2{b, o0} : tr8(pl + o1);
              const i32x4 Ah = {h0.x, h0.y, h1.x, h1.y}, Al = {l0.x, l0.y, l1.x, l1.y};
#pragma unroll
              for (int q = 0; q < 3; q++) {
                hh[q] = mfma(Ah, hb[k][t][q], hh[q]);
                hl[q] = mfma(Al, hb[k][t][q], hl[q]);
              }
            }
            const int hx = 16 * ob + (lane & 15);
            if (hx < nx && M != 19) {
              const float hws = hwsk[k];
#pragma unroll
              for (int i = 0; i < 4; i++) {
                const float tot = 256.0f * (float)fold3(hh[0][i], hh[1][i], hh[2][i]) +
                                  (float)fold3(hl[0][i], hl[1][i], hl[2][i]) + hws;
                const uint32_t q = min(__float2uint_rz(fmaf(tot, 1.0f / 4194304.0f, 0.5f)), 65535u);
                const int yl = 4 * (lane >> 4) + i;
                if (fast8) {
                  const int sh = (int)((sh0 + (uint32_t)(16 * b + yl) * shs) & 3u);
                  ot[yl * kOt8Pitch + sh + 3 * hx + chn] = (uint8_t)q16_to_u8(q);
                } else {
                  otile[yl * kVmOtilePitch + 3 * hx + chn] = (uint16_t)q;
                }
              }
            }
          }
        }
      }
      stamp(2);
    }
    stamp(3);
    if (p < N) rH = read_rec(p);
    phase_barrier();
    stamp(4);
  }
  stamp_out(5, 5);
}

int vp_read_stamps(uint64_t *out, int slots) {
  if (slots > kVpStampSlots) slots = kVpStampSlots;
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_vp_stamps), (size_t)slots * kVpStampN * sizeof(uint64_t)) == hipSuccess
             ? 0
             : -1;
}

VpLayout vp_lds_layout(int vpitch, bool q16) {
  VpLayout L{};
  L.plane = 16 * vpitch + kPlanePad;
  L.otile_off = kPlanesOff + 12 * L.plane;
  L.otile_off = (L.otile_off + 15) & ~15;
  L.otile_bytes = q16 ? kVmOtileBytes : 16 * kOt8Pitch;
  L.otile_bytes = (L.otile_bytes + 15) & ~15;
  L.total = L.otile_off + 2 * L.otile_bytes;
  return L;
}

int launch_vp(hipStream_t s, const VDesc *descs, const MStrip *strips, const VTile *tiles, int ntiles,
              const int32_t *nphase, int G, const int32_t *ai, VpLayout L) {
  if (ntiles <= 0 || G <= 0) return 0;
  if (L.total > kVpMaxLds) return -1;
  static const char *variant = getenv("FI_VP_VARIANT");  // profiling ablations only
  const int v = variant ? atoi(variant) : 0;
  if (v == 1)
    hipLaunchKernelGGL((k_rs_vp<1>), dim3(G), dim3(1024), L.total, s, descs, strips, tiles, ntiles, nphase, ai, L);
  else if (v == 2)
    hipLaunchKernelGGL((k_rs_vp<2>), dim3(G), dim3(1024), L.total, s, descs, strips, tiles, ntiles, nphase, ai, L);
  else if (v == 3)
    hipLaunchKernelGGL((k_rs_vp<3>), dim3(G), dim3(1024), L.total, s, descs, strips, tiles, ntiles, nphase, ai, L);
  else if (v == 4)
    hipLaunchKernelGGL((k_rs_vp<4>), dim3(G), dim3(1024), L.total, s, descs, strips, tiles, ntiles, nphase, ai, L);
  else if (v == 15)
    hipLaunchKernelGGL((k_rs_vp<15>), dim3(G), dim3(1024), L.total, s, descs, strips, tiles, ntiles, nphase, ai, L);
  else if (v == 16)
    hipLaunchKernelGGL((k_rs_vp<16>), dim3(G), dim3(1024), L.total, s, descs, strips, tiles, ntiles, nphase, ai, L);
  else if (v == 17)
    hipLaunchKernelGGL((k_rs_vp<17>), dim3(G), dim3(1024), L.total, s, descs, strips, tiles, ntiles, nphase, ai, L);
  else if (v == 28)
    hipLaunchKernelGGL((k_rs_vp<28>), dim3(G), dim3(1024), L.total, s, descs, strips, tiles, ntiles, nphase, ai, L);
  else if (v == 29)
    hipLaunchKernelGGL((k_rs_vp<29>), dim3(G), dim3(1024), L.total, s, descs, strips, tiles, ntiles, nphase, ai, L);
  else if (v == 30)
    hipLaunchKernelGGL((k_rs_vp<30>), dim3(G), dim3(1024), L.total, s, descs, strips, tiles, ntiles, nphase, ai, L);
  else if (v == 31)
    hipLaunchKernelGGL((k_rs_vp<31>), dim3(G), dim3(1024), L.total, s, descs, strips, tiles, ntiles, nphase, ai, L);
  else if (v == 13)
    hipLaunchKernelGGL((k_rs_vp<13>), dim3(G), dim3(1024), L.total, s, descs, strips, tiles, ntiles, nphase, ai, L);
  else if (v == 32)
    hipLaunchKernelGGL((k_rs_vp<32>), dim3(G), dim3(1024), L.total, s, descs, strips, tiles, ntiles, nphase, ai, L);
  else if (v == 11)
    hipLaunchKernelGGL((k_rs_vp<11>), dim3(G), dim3(1024), L.total, s, descs, strips, tiles, ntiles, nphase, ai, L);
  else if (v == 12)
    hipLaunchKernelGGL((k_rs_vp<12>), dim3(G), dim3(1024), L.total, s, descs, strips, tiles, ntiles, nphase, ai, L);
  else if (v == 9)
    hipLaunchKernelGGL((k_rs_vp<9>), dim3(G), dim3(1024), L.total, s, descs, strips, tiles, ntiles, nphase, ai, L);
  else
    hipLaunchKernelGGL((k_rs_vp<0>), dim3(G), dim3(1024), L.total, s, descs, strips, tiles, ntiles, nphase, ai, L);
  return 0;
}

}  // namespace fi
