// fi_vb.hip -- ImageMagick ResizeImage, vertical pass first (the
// ThumbnailImage sample pre-step folded into the tap tables), as a persistent
// streaming exact-integer matrix-core kernel: v_mfma_i32_16x16x64_i8.
//
// Arithmetic as k_rs_vm (fi_vm.hip): weights W = rint(w 2^22) in three
// signed-byte limbs, pixels as p - 128, exact int32 products, one float
// conversion per pass -> within +-1 LSB of IM's f64, bit-identical to k_rs_vm.
//
// Dataflow (fi_internal.h kVb*):
//  * one 1024-thread workgroup per CU, persistent; work item (image, 512-byte
//    column strip, output blocks [b0, b1)) k of workgroup g is record
//    k * gridDim.x + g (the host balances and XCD-orders them), so every
//    cursor is plain arithmetic -- no atomics, no queues;
//  * the touched source rows stream through an LDS ring of 6 groups of 32 rows
//    (32 KB-row slots, LDS-DMA global_load_lds_dwordx4, 16-byte chunks swizzled
//    for the transposing reads); the group sequence runs on across items, so
//    the next item's rows arrive while the current one finishes;
//  * one iteration = one 16-row output block b, computed in one pass over its
//    own window [K0(b), K0(b) + 64 ks(b)) (ks <= 2): 3 weight limbs x 2 column
//    tiles x ks MFMAs per wave into separate limb accumulators (no per-piece
//    folds, no carried slots), one fold, Q16 planes, horizontal pass, output
//    tile; the stores run after the next block's top barrier;
//  * per iteration the A record of block n + 1, then every group block n + 1's
//    window touches that is not issued yet (mandatory), then up to 3 more
//    (prefetch, bounded by the ring: never past the next window's first
//    group + 5).  The top wait leaves exactly the prefetch DMAs in flight
//    (vmcnt(p), p <= 3, uniform): everything the block reads has landed
//    whatever the window advance.  All DMAs and every vmcnt wait of the loop
//    are explicit; the loop holds no compiler-visible vector load.
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>
#include <stdlib.h>

#include "fi_internal.h"

namespace fi {

namespace {
typedef int32_t i32x4 __attribute__((ext_vector_type(4)));
typedef int32_t i32x2 __attribute__((ext_vector_type(2)));
typedef __attribute__((address_space(1))) uint8_t g_u8;
typedef __attribute__((address_space(1))) uint16_t g_u16;
typedef __attribute__((address_space(1))) uint32_t g_u32;
typedef __attribute__((address_space(3))) i32x2 l_i32x2;
typedef __attribute__((address_space(3))) uint8_t l_u8;
typedef __attribute__((address_space(4))) const int32_t c_i32;  // scalar loads (uniform, read-only tables)

constexpr int kWaves = kVbThreads / 64;  // 16
constexpr int kTiles = 2;                // 16-byte column tiles per wave
constexpr int kAWaves = kVbABytes / 1024;
static_assert(kWaves * kTiles == 32 && kAWaves <= kWaves, "k_rs_vb lane maps");
constexpr int kRingOff = 0;
constexpr int kAOff = kVbGroups * kVbGroupBytes;
constexpr int kSinkOff = kAOff + kVbARing * kVbABytes;
constexpr int kHfOff = kSinkOff + kVbSinkBytes;
static_assert(kHfOff + kVbHfBytes == kVbPlaneOff, "LDS layout");
constexpr int kOtilePitch = 64 * 3 + 4;  // u16 units (nx <= 64)
constexpr int kOtileBytes = 16 * kOtilePitch * 2;
constexpr int kOtile8Pitch = 64 * 3 + 4;
constexpr int kRec = sizeof(VbRec) / 4;
#define FI_VB_F(name) ((int)(offsetof(VbRec, name) / 4))

template <class T>
__device__ __forceinline__ __attribute__((address_space(3))) T *lp(const uint8_t *p) {  // LDS access: ds_* only
  return (__attribute__((address_space(3))) T *)(p);
}
__device__ __forceinline__ uint32_t lds_off(const uint8_t *p) { return (uint32_t)(uintptr_t)(const l_u8 *)p; }
__device__ __forceinline__ i32x2 tr8(const uint8_t *p) {
  return __builtin_amdgcn_ds_read_tr8_b64_v2i32((l_i32x2 *)(p));
}
__device__ __forceinline__ i32x4 mfma(i32x4 a, i32x4 b, i32x4 c) {
  return __builtin_amdgcn_mfma_i32_16x16x64_i8(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ int col_off(int ci) { return (ci * 16) ^ (((ci >> 4) & 1) << 7); }
__device__ __forceinline__ uint32_t q16_to_u8(uint32_t q) {  // ScaleQuantumToChar
  return ((q + 128u) - ((q + 128u) >> 8)) >> 8;
}
__device__ __forceinline__ uint32_t clamp_gray(double gv) {  // ClampToQuantum of Rec709Luma
  return !(gv > 0.0) ? 0u : (gv >= 65535.0 ? 65535u : (uint32_t)(gv + 0.5));
}
__device__ __forceinline__ uint32_t gray8(uint32_t r, uint32_t g, uint32_t b) {
  return q16_to_u8(clamp_gray(0.212656 * (double)r + 0.715158 * (double)g + 0.072186 * (double)b));
}
__device__ __forceinline__ int32_t fold3(int32_t d0, int32_t d1, int32_t d2) {  // modular limb fold
  return (int32_t)((uint32_t)d0 + ((uint32_t)d1 << 8) + ((uint32_t)d2 << 16));
}
__device__ __forceinline__ int rfl(int x) { return __builtin_amdgcn_readfirstlane(x); }
__device__ __forceinline__ const uint8_t *rflp(const uint8_t *p) {
  const uint64_t v = (uint64_t)(uintptr_t)p;
  return reinterpret_cast<const uint8_t *>(
      (uintptr_t)(((uint64_t)(uint32_t)rfl((int)(uint32_t)(v >> 32)) << 32) | (uint32_t)rfl((int)(uint32_t)v)));
}
// LDS-DMA, per-lane 64-bit source addresses: the wave's active lanes x 16 B
// land at LDS m0 + 16 lane.  Not counted by hipcc: see the waits.
__device__ __forceinline__ void dma16v(uint32_t m0, const uint8_t *src) {
  unsigned keep;
  m0 = (uint32_t)rfl((int)m0);
  asm volatile(
      "s_mov_b32 %0, m0\n\t"
      "s_mov_b32 m0, %2\n\t"
      "s_nop 0\n\t"
      "global_load_lds_dwordx4 %1, off\n\t"
      "s_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(src), "s"(m0)
      : "memory");
}
// LDS-DMA, saddr form: lane i's source is sbase + voff.
__device__ __forceinline__ void dma16(uint32_t m0, const uint8_t *sbase, uint32_t voff) {
  unsigned keep;
  sbase = rflp(sbase);
  m0 = (uint32_t)rfl((int)m0);
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
// the workgroup barrier without hipcc's vmcnt(0) (the DMAs stay in flight):
// LDS and scalar loads drained, then s_barrier
__device__ __forceinline__ void barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }
__device__ __forceinline__ void wait_vm0() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }
// all but this wave's last p DMAs (p uniform, <= 3)
__device__ __forceinline__ void wait_vm_keep(int p) {
  if (p >= 3)
    asm volatile("s_waitcnt vmcnt(3)" ::: "memory");
  else if (p == 2)
    asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
  else if (p == 1)
    asm volatile("s_waitcnt vmcnt(1)" ::: "memory");
  else
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

}  // namespace

// per-workgroup phase sums of MODE 9 (read by fi_debug_vb_stamps, tools/vb_timing.py)
constexpr int kVbStampSlots = 1024;
constexpr int kVbStampN = 12;  // 10 phase sums, blocks, items
__device__ uint64_t g_vb_stamps[kVbStampSlots * kVbStampN];

// MODE (profiling ablations, FI_VB_VARIANT; wrong pixels): 0 production,
// 1 stream only (no MFMA, no block phase), 3 no stores, 9 production +
// per-phase s_memtime sums of wave 0.
template <int MODE>
__global__ __launch_bounds__(kVbThreads) void k_rs_vb(const VbRec *__restrict__ recs_g,
                                                      const int32_t *__restrict__ nitem_g,  // [grid] items per workgroup
                                                      const int32_t *__restrict__ ai_g, int32_t otile_off) {
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  c_i32 *R = (c_i32 *)recs_g;  // record k: R[kRec * k + field]
  c_i32 *ca = (c_i32 *)ai_g;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wv = rfl(tid >> 6);
  const int G = gridDim.x, gid = blockIdx.x;
  uint8_t *vpl = lds + kVbPlaneOff;
  const uint32_t lds0 = lds_off(lds);
  const int nrec_wg = ((c_i32 *)nitem_g)[gid];
  // this workgroup's k-th item (valid iff k < nrec_wg); a record index past
  // every valid one stands for "none" below
  const int nrec = 0x7FFFFFFF;
  auto rec_of = [&](int k) { return k < nrec_wg ? k * G + gid : nrec; };
  auto fld = [&](int rec, int f) -> int32_t { return R[kRec * rec + f]; };
  auto fptr = [&](int rec, int f) -> uint8_t * {
    return reinterpret_cast<uint8_t *>(
        (uintptr_t)(((uint64_t)(uint32_t)R[kRec * rec + f + 1] << 32) | (uint32_t)R[kRec * rec + f]));
  };
  if (rec_of(0) >= nrec) return;

  constexpr bool kStamp = MODE == 9;
  uint64_t tsum[10] = {}, tprev = 0, n_blk = 0, n_items = 0;
  auto stamp = [&](int k) {
    if (kStamp) {
      const uint64_t t = __builtin_amdgcn_s_memtime();
      tsum[k] += t - tprev;
      tprev = t;
    }
  };

  // ---- group issue cursor: item kI, group gI (list rows 32 gI ..); group
  // sequence number sq (ring slot sq % 6) runs on across items.  The item's
  // fields are held in registers (loaded when the cursor enters it).
  int kI = 0, recI = rec_of(0), gI = 0, sq = 0;
  bool liveI = true;
  const uint8_t *iSrc = nullptr;
  int iStride = 0, iNbytes = 0, iLast = 0, iRows = 0, iRow0 = 0, iRstep = 0, iGend = 0;
  auto load_issue_item = [&]() {
    iSrc = fptr(recI, FI_VB_F(src));
    iStride = fld(recI, FI_VB_F(src_stride));
    iNbytes = fld(recI, FI_VB_F(nbytes));
    iLast = fld(recI, FI_VB_F(nrows)) - 1;
    iRows = fld(recI, FI_VB_F(rows));
    iRow0 = fld(recI, FI_VB_F(row0));
    iRstep = fld(recI, FI_VB_F(rstep));
    gI = fld(recI, FI_VB_F(g0));
    iGend = fld(recI, FI_VB_F(gend));
  };
  load_issue_item();
  // per-lane source chunk of a group DMA: lanes 32 h + c of wave w write group
  // row r = 2 w + h, chunk position c; chunk swizzle f(r) = (r & 7) | 8 ((r >> 4) & 1)
  const int hrow = lane >> 5;
  const int rDma = 2 * wv + hrow;
  const uint32_t chunk16 = 16u * (uint32_t)((lane & 31) ^ ((rDma & 7) | (((rDma >> 4) & 1) << 3)));
  auto issue_group = [&]() {  // the cursor's group -> ring slot sq % 6, then advance
    const int l0 = min(32 * gI + 2 * wv, iLast), l1 = min(l0 + 1, iLast);
    int r0, r1;
    if (iRstep > 0) {
      r0 = iRow0 + iRstep * l0;
      r1 = iRow0 + iRstep * l1;
    } else {
      r0 = ca[iRows + l0];
      r1 = ca[iRows + l1];
    }
    const int row = hrow ? r1 : r0;
    dma16v(lds0 + kRingOff + (sq % kVbGroups) * kVbGroupBytes + wv * 1024,
           iSrc + (int64_t)row * iStride + (chunk16 < (uint32_t)iNbytes ? chunk16 : 0u));
    sq++;
    if (++gI >= iGend) {
      kI++;
      recI = rec_of(kI);
      if (recI >= nrec)
        liveI = false;
      else
        load_issue_item();
    }
  };
  // ---- A-record cursor: block stream, one block ahead of the compute cursor ----
  int kA = 0, recA = rec_of(0), bA = fld(recA, FI_VB_F(b0));
  int aArec = fld(recA, FI_VB_F(arec)), aB1 = fld(recA, FI_VB_F(b1));
  bool liveA = true;
  auto issue_a = [&](int n) {  // A record of the cursor's block -> A slot n % 3, then advance
    if (liveA) {
      if (wv < kAWaves)
        dma16(lds0 + kAOff + (n % kVbARing) * kVbABytes + wv * 1024,
              reinterpret_cast<const uint8_t *>(ai_g + aArec) + (size_t)bA * kVbABytes + wv * 1024, 16u * lane);
      if (++bA >= aB1) {
        kA++;
        recA = rec_of(kA);
        if (recA >= nrec) {
          liveA = false;
        } else {
          bA = fld(recA, FI_VB_F(b0));
          aArec = fld(recA, FI_VB_F(arec));
          aB1 = fld(recA, FI_VB_F(b1));
        }
      }
    }
  };

  // ---- compute cursor --------------------------------------------------------------
  int kC = 0, recC = rec_of(0), bC = 0;
  int sC = 0;  // group sequence number of the current item's first group g0
  // the compute item's fields (registers; loaded when the cursor enters it)
  struct Item {
    uint8_t *dst;
    int dst_stride, gray, rot, x0, nx, eh, ew, nocb, vpitch, ks, arec, b1, g0, gend;
  };
  Item C;
  auto load_item = [&](int rec, Item &I) {
    I.dst = fptr(rec, FI_VB_F(dst));
    I.dst_stride = fld(rec, FI_VB_F(dst_stride));
    I.gray = fld(rec, FI_VB_F(gray));
    I.rot = fld(rec, FI_VB_F(rot));
    I.x0 = fld(rec, FI_VB_F(x0));
    I.nx = fld(rec, FI_VB_F(nx));
    I.eh = fld(rec, FI_VB_F(eh));
    I.ew = fld(rec, FI_VB_F(ew));
    I.nocb = fld(rec, FI_VB_F(nocb));
    I.vpitch = fld(rec, FI_VB_F(vpitch));
    I.ks = fld(rec, FI_VB_F(ks));
    I.arec = fld(rec, FI_VB_F(arec));
    I.b1 = fld(rec, FI_VB_F(b1));
    I.g0 = fld(rec, FI_VB_F(g0));
    I.gend = fld(rec, FI_VB_F(gend));
  };
  load_item(recC, C);
  bC = fld(recC, FI_VB_F(b0));
  // the first group sequence number the block after (kC, bC) still needs
  // and the last one its window touches (-1: no next block)
  int nlast0 = -1;  // the next item's last0 (-1: none)
  auto load_next_last0 = [&]() {
    const int rn = rec_of(kC + 1);
    nlast0 = rn < nrec ? fld(rn, FI_VB_F(last0)) : -1;
  };
  load_next_last0();
  auto next_window = [&](int &first, int &last) {
    if (bC + 1 < C.b1) {
      const int K0n = ca[C.arec + (bC + 1) * (kVbABytes / 4) + kVbMeta];
      const int Rn = ca[C.arec + (bC + 1) * (kVbABytes / 4) + kVbMeta + 2];
      first = sC + K0n / 32 - C.g0;
      last = sC + (Rn - 1) / 32 - C.g0;
    } else {
      first = sC + C.gend - C.g0;  // the next item's first group
      last = nlast0 < 0 ? -1 : first + nlast0;
    }
  };
  // per-item lane constants (loaded when the compute cursor enters an item)
  uint32_t vcolp = 0;
  float hws = 0.0f;
  int hw0 = 0, hks = 0;
  auto enter_item = [&]() {
    const int nocb = C.nocb, ks = C.ks;
    const int s0 = fld(recC, FI_VB_F(s0)), frag = fld(recC, FI_VB_F(frag));
    const i32x4 lt = *(const i32x4 *)(ai_g + fld(recC, FI_VB_F(lanes)) + 4 * tid);
    const int it = wv < 3 * nocb ? wv : 0, ob = it / 3;
    hw0 = ca[s0 + 2 * ob];
    hks = ca[s0 + 2 * ob + 1];
    // the strip's horizontal B fragments [ob][t][limb] -> LDS (read by this
    // item's horizontal passes, after their planes barrier)
    {
      const int n16 = nocb * ks * 3 * 64;  // 16-byte fragment rows, [ob][t][limb][lane] as in the table
      auto hfl = lp<i32x4>(lds + kHfOff);
      for (int i = tid; i < n16; i += kVbThreads) hfl[i] = *(const i32x4 *)(ai_g + frag + 4 * i);
    }
    vcolp = (uint32_t)lt.x;
    hws = __int_as_float(lt.z);
    // consume the loaded values here, so hipcc's vmcnt wait for them sits
    // before this iteration's DMAs are issued (it also waits for the previous
    // iteration's: once per item)
    asm volatile("" : "+v"(vcolp), "+v"(hws));
    n_items++;
  };

  // transposing-read geometry (see fi_vm.hip): lane reads window rows
  // 16 (l >> 4) + (l & 15) / 2 (+ 8) of a K-step, bytes 8 (l & 1) of chunk tile ^ f(row)
  const int rA = 16 * (lane >> 4) + ((lane & 15) >> 1);

  // pending stores: the block completed at the previous iteration
  bool pend = false, entered = false;
  int pend_b = 0, pend_buf = 0;
  Item P = C;  // the item of the pending block
  auto store_block = [&](const Item &I, int b, int buf) {
    uint8_t *dst = I.dst;
    const int64_t dst_stride = I.dst_stride;
    const int gray = I.gray, rot = I.rot;
    const int x0 = I.x0, nx = I.nx;
    const int eh = I.eh, ew = I.ew;
    const int oc = gray ? 1 : 3;
    const bool fast8 = !gray && rot == 0;
    const uint8_t *ot = lds + otile_off + buf * kOtileBytes;
    const uint16_t *otile = reinterpret_cast<const uint16_t *>(ot);
    const int rows_here = min(16, eh - 16 * b);
    const int nb = nx * oc;
    auto out_byte = [&](int yl, int kk) -> uint32_t {
      const uint16_t *o = otile + yl * kOtilePitch;
      if (!gray) return q16_to_u8(o[kk]);
      return gray8(o[3 * kk], o[3 * kk + 1], o[3 * kk + 2]);
    };
    if (gray == 2) {  // -monochrome input: Q16 gray (u16, rot = 0) for fi_mono.hip
#pragma clang loop unroll(disable)
      for (int it2 = tid; it2 < rows_here * nx; it2 += kVbThreads) {
        const int yl = it2 / nx, x = it2 - yl * nx;
        const uint16_t *o = otile + yl * kOtilePitch + 3 * x;
        const uint32_t q = clamp_gray(0.212656 * (double)o[0] + 0.715158 * (double)o[1] + 0.072186 * (double)o[2]);
        ((g_u16 *)(dst + (int64_t)(16 * b + yl) * dst_stride))[x0 + x] = (uint16_t)q;
      }
      return;
    }
    if (rot == 0) {
      // items = (row, destination dword): interior dwords stored whole, the
      // partial first / last dword of a row byte by byte
      const int ndw = (nb + 3) / 4 + 1;
      const float inv = 1.0f / (float)ndw;
      const uint32_t sh0 = (uint32_t)(((uintptr_t)dst + (uint64_t)x0 * 3) & 3u);
      const uint32_t shs = (uint32_t)(dst_stride & 3);
#pragma clang loop unroll(disable)
      for (int it2 = tid; it2 < rows_here * ndw; it2 += kVbThreads) {
        const int yl = (int)(((float)it2 + 0.5f) * inv), d = it2 - yl * ndw;
        uint8_t *a0 = dst + (int64_t)(16 * b + yl) * dst_stride + (int64_t)x0 * oc;
        const int sh = fast8 ? (int)((sh0 + (uint32_t)(16 * b + yl) * shs) & 3u) : (int)((uintptr_t)a0 & 3u);
        const int k0 = 4 * d - sh;  // segment byte of the dword's first byte
        if (k0 >= nb) continue;
        if (fast8) {
          const uint8_t *o = ot + yl * kOtile8Pitch;
          if (k0 >= 0 && k0 + 4 <= nb)
            *(g_u32 *)(a0 + k0) = *reinterpret_cast<const uint32_t *>(o + 4 * d);
          else
            for (int kk = max(k0, 0); kk < min(k0 + 4, nb); kk++) *(g_u8 *)(a0 + kk) = o[sh + kk];
        } else {
          if (k0 >= 0 && k0 + 4 <= nb)
            *(g_u32 *)(a0 + k0) = out_byte(yl, k0) | (out_byte(yl, k0 + 1) << 8) | (out_byte(yl, k0 + 2) << 16) |
                                  (out_byte(yl, k0 + 3) << 24);
          else
            for (int kk = max(k0, 0); kk < min(k0 + 4, nb); kk++) *(g_u8 *)(a0 + kk) = (uint8_t)out_byte(yl, kk);
        }
      }
      return;
    }
#pragma clang loop unroll(disable)
    for (int it2 = tid; it2 < rows_here * nx; it2 += kVbThreads) {
      const int yl = it2 / nx, x = it2 - yl * nx, y = 16 * b + yl;
      const int ox = x0 + x;
      int dx, dy;
      if (rot == 90) {
        dx = eh - 1 - y;
        dy = ox;
      } else if (rot == 180) {
        dx = ew - 1 - ox;
        dy = eh - 1 - y;
      } else {  // 270
        dx = y;
        dy = ew - 1 - ox;
      }
      g_u8 *out = (g_u8 *)(dst + (int64_t)dy * dst_stride) + dx * oc;
      for (int c = 0; c < oc; c++) out[c] = (uint8_t)out_byte(yl, x * oc + c);
    }
  };

  // ---- prologue: the ring's first 6 groups, the A record of block 0 --------------
  for (int i = 0; i < kVbGroups && liveI; i++) issue_group();
  issue_a(0);
  wait_vm0();
  int keep = 0;  // prefetch DMAs the top wait leaves in flight
  enter_item();
  if (kStamp) tprev = __builtin_amdgcn_s_memtime();

  for (int n = 0;; n++) {  // n: block number of this workgroup's stream
    stamp(9);
    wait_vm_keep(keep);  // all but this wave's trailing prefetch DMAs
    stamp(0);
    barrier();  // block n's window rows and A record landed for every wave
    stamp(1);
    n_blk++;
    if (entered) {  // the compute cursor entered a new item last iteration
      enter_item();
      entered = false;
    }
    // ---- stores of the block completed at the previous iteration
    if (pend) {
      if (MODE != 3) store_block(P, pend_b, pend_buf);
      pend = false;
    }
    stamp(2);
    const uint8_t *pa = lds + kAOff + (n % kVbARing) * kVbABytes;
    const int K0 = rfl(lp<int32_t>(pa)[kVbMeta + 0]), ks = rfl(lp<int32_t>(pa)[kVbMeta + 1]);
    const int g0C = C.g0;
    // ---- vertical: B operands of the window (transposing reads from the ring)
    i32x4 B[2][kTiles];
    {
      const int f8 = ((K0 >> 4) + (lane >> 4)) & 1;  // (row >> 4) & 1 of the lane's rows
      const int fA = (rA & 7) | (f8 << 3);
#pragma unroll
      for (int t = 0; t < 2; t++) {
        if (t >= ks) break;
        const int rw = K0 + 64 * t + rA;  // list row of the lane's first read
        const int slot = (sC + (rw >> 5) - g0C) % kVbGroups;
        const uint8_t *base = lds + kRingOff + slot * kVbGroupBytes + (rw & 31) * 512 + 8 * (lane & 1);
#pragma unroll
        for (int j = 0; j < kTiles; j++) {
          const uint8_t *p = base + 16 * ((kTiles * wv + j) ^ fA);
          const i32x2 lo = tr8(p), hi = tr8(p + 8 * 512);
          B[t][j] = i32x4{lo.x, lo.y, hi.x, hi.y} ^
                    i32x4{(int)0x80808080, (int)0x80808080, (int)0x80808080, (int)0x80808080};
        }
      }
    }
    i32x4 acc[3][kTiles];  // limb accumulators (t = 0 starts them at zero)
    if (MODE != 1) {
      auto af = lp<i32x4>(pa) + lane;
#pragma unroll
      for (int t = 0; t < 2; t++) {
        if (t >= ks) break;
#pragma unroll
        for (int q = 0; q < 3; q++) {
          const i32x4 A = af[(t * 3 + q) * 64];
#pragma unroll
          for (int j = 0; j < kTiles; j++) acc[q][j] = mfma(A, B[t][j], t == 0 ? i32x4{0, 0, 0, 0} : acc[q][j]);
        }
      }
    }
    stamp(3);
    // ---- block bC complete: fold the limbs (+ the p - 128 correction), Q16 planes
    const int nocb = C.nocb;
    const int plane = 16 * C.vpitch;
    if (MODE != 1) {
      const i32x4 w128 = lp<i32x4>(pa + 4 * kVbW128)[lane >> 4];
#pragma unroll
      for (int j = 0; j < kTiles; j++) {
        const uint32_t o = (vcolp >> (16 * j)) & 0xFFFFu;
        if (o == 0xFFFFu) continue;
        uint32_t qv[4];
#pragma unroll
        for (int i = 0; i < 4; i++) {  // ClampToQuantum: +0.5 truncated; the conversions saturate
          const int32_t a = fold3(acc[0][j][i], acc[1][j][i], acc[2][j][i]) + w128[i];
          qv[i] = __float2uint_rz(fmaf((float)a, 257.0f / 4194304.0f, 0.5f));
        }
        const auto p01 = __builtin_amdgcn_cvt_pk_u16(qv[0], qv[1]);
        const auto p23 = __builtin_amdgcn_cvt_pk_u16(qv[2], qv[3]);
        const uint32_t x01 = __builtin_bit_cast(uint32_t, p01) ^ 0x80808080u;  // signed limbs (hi - 128, lo - 128)
        const uint32_t x23 = __builtin_bit_cast(uint32_t, p23) ^ 0x80808080u;
        *lp<uint32_t>(vpl + o) = __builtin_amdgcn_perm(x23, x01, 0x07050301u);
        *lp<uint32_t>(vpl + o + 3 * plane) = __builtin_amdgcn_perm(x23, x01, 0x06040200u);
      }
    } else {  // ablation: keep the loads alive
      uint32_t z = 0;
#pragma unroll
      for (int j = 0; j < kTiles; j++) z ^= (uint32_t)B[0][j][0] ^ (uint32_t)B[1][j][1];
      if (z == 0x9E3779B9u) lds[kSinkOff + tid % 1024] = (uint8_t)z;
    }
    stamp(4);
    // the next block's window groups [flive, fneed]
    int flive, fneed;
    next_window(flive, fneed);
    barrier();  // planes complete; every wave is done with the ring rows below the next window
    stamp(5);
    // ---- the A record of block n + 1; the window groups still missing; up to 3 prefetch groups
    issue_a(n + 1);
    while (liveI && sq <= fneed) issue_group();
    keep = 0;
#pragma unroll
    for (int i = 0; i < 3; i++)
      if (liveI && sq < flive + kVbGroups) {
        issue_group();
        keep++;
      }
    stamp(6);
    // ---- horizontal: item (16-px output block ob, channel) = wave wv
    const int buf = n & 1;
    if (MODE != 1 && wv < 3 * nocb) {
      const bool fast8 = !C.gray && C.rot == 0;
      const int nx = C.nx;
      const uint32_t sh0 = (uint32_t)(((uintptr_t)C.dst + (uint64_t)C.x0 * 3) & 3u);
      const uint32_t shs = (uint32_t)(C.dst_stride & 3);
      const int ob = wv / 3, chn = wv - 3 * ob;
      const int hks_all = C.ks;  // the strip's k-steps (fragment table stride)
      i32x4 hh[3], hl[3];
#pragma unroll
      for (int q = 0; q < 3; q++) hh[q] = hl[q] = i32x4{0, 0, 0, 0};
      const uint8_t *ph = vpl + chn * plane, *pl = ph + 3 * plane;
#pragma unroll
      for (int t = 0; t < 2; t++) {
        if (t >= hks) break;
        // A: column hw0 + 64 t + 16 (l >> 4) + (l & 15) / 2 (+8), rows 8 (l & 1)
        const int cA = hw0 + 64 * t + 16 * (lane >> 4) + ((lane & 15) >> 1);
        const int o0 = col_off(cA) + 8 * (lane & 1), o1 = col_off(cA + 8) + 8 * (lane & 1);
        const i32x2 h0 = tr8(ph + o0), h1 = tr8(ph + o1);
        const i32x2 l0 = tr8(pl + o0), l1 = tr8(pl + o1);
        const i32x4 Ah = {h0.x, h0.y, h1.x, h1.y}, Al = {l0.x, l0.y, l1.x, l1.y};
        auto hfl = lp<i32x4>(lds + kHfOff) + ((ob * hks_all + t) * 3) * 64 + lane;
#pragma unroll
        for (int q = 0; q < 3; q++) {
          const i32x4 Bq = hfl[q * 64];
          hh[q] = mfma(Ah, Bq, hh[q]);
          hl[q] = mfma(Al, Bq, hl[q]);
        }
      }
      const int hx = 16 * ob + (lane & 15);
      if (hx < nx) {
        // V = 256 (h - 128) + (l - 128) + 32896; ClampToQuantum
        uint8_t *o8 = lds + otile_off + buf * kOtileBytes;
        uint16_t *o = reinterpret_cast<uint16_t *>(o8) + (4 * (lane >> 4)) * kOtilePitch + 3 * hx + chn;
#pragma unroll
        for (int i = 0; i < 4; i++) {
          const float tot = 256.0f * (float)fold3(hh[0][i], hh[1][i], hh[2][i]) +
                            (float)fold3(hl[0][i], hl[1][i], hl[2][i]) + hws;
          const uint32_t qv = min(__float2uint_rz(fmaf(tot, 1.0f / 4194304.0f, 0.5f)), 65535u);
          const int yl = 4 * (lane >> 4) + i;
          if (fast8)
            *lp<uint8_t>(o8 + yl * kOtile8Pitch + (int)((sh0 + (uint32_t)(16 * bC + yl) * shs) & 3u) + 3 * hx + chn) =
                (uint8_t)q16_to_u8(qv);
          else
            *lp<uint16_t>(reinterpret_cast<uint8_t *>(o + i * kOtilePitch)) = (uint16_t)qv;
        }
      }
    }
    pend = true;
    P = C;
    pend_b = bC;
    pend_buf = buf;
    stamp(7);
    // ---- advance the compute cursor
    if (++bC >= C.b1) {
      sC += C.gend - C.g0;
      kC++;
      recC = rec_of(kC);
      if (recC >= nrec) break;
      bC = fld(recC, FI_VB_F(b0));
      load_item(recC, C);
      load_next_last0();
      entered = true;
    }
    stamp(8);
  }
  // drain: the last block's stores
  barrier();
  if (pend && MODE != 3) store_block(P, pend_b, pend_buf);
  wait_vm0();  // no DMA may outlive the workgroup's LDS
  if (kStamp && tid == 0 && blockIdx.x < kVbStampSlots) {
    for (int k = 0; k < 10; k++) g_vb_stamps[blockIdx.x * kVbStampN + k] = tsum[k];
    g_vb_stamps[blockIdx.x * kVbStampN + 10] = n_blk;
    g_vb_stamps[blockIdx.x * kVbStampN + 11] = n_items;
  }
}
#undef FI_VB_F

int vb_read_stamps(uint64_t *out, int slots) {
  if (slots > kVbStampSlots) slots = kVbStampSlots;
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_vb_stamps), (size_t)slots * kVbStampN * sizeof(uint64_t)) == hipSuccess
             ? 0
             : -1;
}

bool vb_strip_ok(int nocb, int ks) { return nocb * ks * 3 * 1024 <= kVbHfBytes; }
size_t vb_lds_bytes(int vpitch_max) {
  return (size_t)kVbPlaneOff + (size_t)6 * 16 * vpitch_max + 2 * (size_t)kOtileBytes;
}
int vb_otile_off(int vpitch_max) { return kVbPlaneOff + 6 * 16 * vpitch_max; }

int launch_vb(hipStream_t s, int grid, const VbRec *recs, const int32_t *nitem, const int32_t *ai, int vpitch_max) {
  const size_t lds = vb_lds_bytes(vpitch_max);
  if (lds > (size_t)kVbMaxLds || grid <= 0) return -1;
  static const char *variant = getenv("FI_VB_VARIANT");  // profiling ablations only
  const int v = variant ? atoi(variant) : 0;
  const int oo = vb_otile_off(vpitch_max);
  if (v == 1)
    hipLaunchKernelGGL(k_rs_vb<1>, dim3(grid), dim3(kVbThreads), lds, s, recs, nitem, ai, oo);
  else if (v == 3)
    hipLaunchKernelGGL(k_rs_vb<3>, dim3(grid), dim3(kVbThreads), lds, s, recs, nitem, ai, oo);
  else if (v == 9)
    hipLaunchKernelGGL(k_rs_vb<9>, dim3(grid), dim3(kVbThreads), lds, s, recs, nitem, ai, oo);
  else
    hipLaunchKernelGGL(k_rs_vb<0>, dim3(grid), dim3(kVbThreads), lds, s, recs, nitem, ai, oo);
  return 0;
}

}  // namespace fi
