// fi_internal.h -- structures shared by the host planner (fi_plan.cpp), the
// runtime (fi_api.cpp) and the gfx950 kernels (fi_kernels.hip).
//
// Data layout in HBM (see DESIGN.md "Data layout"):
//   * images: RGB8 HWC rows, caller stride;
//   * one "arena" per batch holding every device-side table: tap tables
//     (int32 start/count/offset + fp32 weights), Pillow int32 coefficient
//     tables, crop lists and f64 importance tables -- uploaded with one copy;
//   * one "workspace" per batch: Q16 intermediates of the generic two-pass
//     path, resized images feeding smartcrop, prescale scratch, packed maps,
//     per-crop score slots.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/flyimg_hip.h"

namespace fi {

constexpr int kMaxChannels = 3;

// One separable axis in the *source* index domain (the ImageMagick sample
// pre-step is folded in by merging taps that map to one source index).
struct DevAxis {
  int32_t n;      // output indices covered
  int32_t start;  // arena offset (int32 units) of start[n]
  int32_t count;  // arena offset of count[n]
  int32_t woff;   // arena offset of woff[n] (float units in weight area)
  int32_t maxtaps;
  int32_t src_lo;   // min over start
  int32_t src_hi;   // max over start+count (exclusive)
  int32_t touched;  // source indices with a non-zero merged weight
  int32_t wbase;    // af offset the woff entries are relative to
  int32_t wd;       // ad offset of the f64 weights (RGBA path; -1 = not placed):
                    // weight (o, j) = ad[wd + ai[woff + o] - wbase + j]
};

// Per-image descriptor of the resample path (the generic two-pass kernels and
// the copy / epilogue kernel; the streaming kernels take VDesc / HvDesc).
struct ResizeDesc {
  const uint8_t *src;
  int64_t src_stride;  // bytes
  int32_t C;           // 3, or 4 (RGBA: IM's matte path, fi_kernels.hip k_rs4_*)
  int32_t mode;        // 0 = copy/epilogue only, 1 = V then H, 2 = H then V
  DevAxis v;           // output rows  (extent window) <- source rows
  DevAxis h;           // output cols  (extent window) <- source cols
  uint16_t *mid;       // Q16 intermediate of the generic path
  int64_t mid_stride;  // elements per row
  int32_t mid_rows, mid_cols;  // rows x pixels of the intermediate
  int32_t mid_r0, mid_c0;      // source row/col of intermediate origin
  int32_t ex0, ey0;            // extent offset (copy mode only)
  int32_t ew, eh;              // extent (= pre-rotate output) dims
  int32_t gray, rot;           // epilogue
  uint8_t *dst;
  int64_t dst_stride;
  int32_t out_w, out_h, out_c;  // post-rotate dims
  int32_t q16out;               // 1: the epilogue writes rotated Q16 (u16) for the convolution stage
};

// One step of the forwarded convolutions (fi_conv.hip) on one image's rotated
// Q16 HWC buffer: mode 0 horizontal 1-D pass, 1 vertical 1-D pass, 2 vertical
// pass + unsharp combine with `orig` (written in place), 3 2-D pass, 4 Q16 ->
// 8-bit dst.
struct ConvStep {
  const uint16_t *in;
  uint16_t *out;
  const uint16_t *orig;  // mode 2
  uint8_t *dst8;         // mode 4
  int64_t dst_stride;    // mode 4, bytes
  int32_t W, H, C;
  int32_t kw, kh;        // kernel extent
  int32_t k;             // ad offset of the kernel values
  double gain, thr;      // mode 2: unsharp gain, QuantumRange * threshold
};

// smartcrop crop window in the analysed image (smartcrop.py crops()).
struct DevCrop {
  double fx, fy, fw, fh;  // as Python holds them
  int32_t x0, y0;         // integer origin
  int32_t nin_x, nin_y;   // inside extents (x < fl(x0+fw))
  int32_t table;          // arena offset (double units) of importance table
  int32_t table_w;        // row pitch of the table
  int32_t rx, ry, rw, rh; // rescaled ints (crop() :184-190)
  double imax;            // max |importance| over the table (fast-pass error bound)
  double imax2;           // max |importance - outside_importance| over the table2
  int32_t table2;         // arena offset (double units): fl(importance - outside_importance), rows of
  int32_t table2_w;       //   table2_w = table_w rounded up to 64 (zeros past table_w)
  int32_t sg, sm, sj;     // k_sc_score3: group (within the image's), M row (x origin), y slot
  int32_t pad;
};

struct ScDesc {
  const uint8_t *img;  // smartcrop input (resized output or user image)
  int64_t stride;
  int32_t W, H, C;     // C = 1 (gray, pasted into RGB) or 3
  int32_t fx, fy;      // reduce factors (1 = none)
  int32_t rw, rh;      // reduced dims
  int32_t need_h, need_v;
  int32_t aw, ah;      // analysed dims
  int32_t ybox_first, hrows;
  int32_t hb, hk, ksh; // arena offsets: H bounds (pairs), H coeffs (int32), ksize
  int32_t vb, vk, ksv;
  int32_t hkT;         // H coeffs transposed [ksh][aw] (k_sc_prep: lanes read consecutive x)
  int32_t prep;        // 1: per-image MFMA kernels (k_sc_fz, or k_sc_hmfma + k_sc_vq; hbuf pitch apitch), 0: generic kernels
  int32_t hm;          // 1: horizontal pass by k_sc_hmfma / k_sc_fz (tables below)
  int32_t hm_rows, hm_ks, hm_pitch, hm_nb;
  int32_t hmB, hmC, hmS0;  // arena offsets (int32 units; hmB 16-B aligned)
  int32_t vq;              // 1: vertical pass + maps by k_sc_vq (tables below)
  int32_t fz;              // 1: both passes + maps by k_sc_fz (hm + vq tables, one workgroup per image)
  int32_t fd;              // 1 (with fz): rows readable to fd_rp(W) bytes, so k_sc_fd may take it
  int32_t vqA, vqC, vqK0;  // arena offsets (int32 units; vqA 16-B aligned)
  int32_t cx;              // 1: k_sc_hx + k_sc_vx take it (tables below, tbuf)
  int32_t cx_kv, cx_tp;    // their vertical k-steps, transposed H-stage row pitch (ScPlan::cx_*)
  int32_t cxA, cxK0;       // arena offsets (int32 units; cxA 16-B aligned)
  int32_t cx_pad;
  uint8_t *tbuf;       // k_sc_hx's H stage: 256-B tiles [hm_nb][C][cx_tp / 16][16 columns][16 rows]
  uint8_t *red;        // reduce scratch rw*rh*3
  uint8_t *hbuf;       // H-pass scratch aw*hrows*3
  uint8_t *pre;        // prescaled image aw*ah*3
  uint32_t *maps;      // packed skin | edge<<8 | sat<<16
  int32_t crop0, ncrops;  // into the batch crop array (shared by images of one plan)
  int32_t score0;         // into the batch CropScore array (per image)
  double prescale;
  double T[3];         // unused on host; device scratch
  int32_t result;      // index into result array
  int32_t exact_all;
  int32_t sg0, ngrp;   // k_sc_score3 groups (batch group array); ngrp = 0: k_sc_score2
  int32_t sg_lds, sg_pad;  // its dynamic LDS
};

// smartcrop prescale planning (fi_plan.cpp plan_sc_prep): kPrepRows rows per
// chunk; apitch = 16-B rounded aw*3 (hbuf and LDS row pitch), spitch = 16-B
// rounded source width*3.  LDS per workgroup <= kPrepMaxLds (host-checked).
constexpr int kPrepRows = 16;
constexpr int kVqRows = 14;  // k_sc_vq: analysed rows per workgroup (16 prescaled rows with the edge halo)
constexpr int kPrepMaxLds = 64 * 1024;
// k_sc_hx (fi_smartcrop.hip): 16-row blocks of the H stage one wave walks (a
// tile = image x 4 column blocks x kHxRb row blocks)
constexpr int kHxRb = 8;
// k_sc_fz (fi_smartcrop.hip): the fused per-image prescale + maps; LDS =
// kFzRing (80) H-stage rows + max(3 source planes of 16 rows, 16 prescaled rows
// + luma); <= 80 KB keeps two workgroups per CU
constexpr int kFzMaxLds = 80 * 1024;
// k_sc_fd (fi_smartcrop.hip): k_sc_fz's passes with the source rows streamed
// by LDS-DMA, one 16-wave workgroup per CU.  LDS: kFdSlots raw blocks of 16
// source rows (row pitch fd_rp = 16-B rounded W * 3; a slot rounded up to the
// DMA's 1 KB steps), a tail that the horizontal pass's last window may read
// past the last slot (zero weights there), then the kFzRing H-stage rows, 16
// prescaled rows and their luma.
// k_sc_skinsat's table of all 2^24 colours is laid out in Z-order of the
// channel bits (r2 g2 b2 r1 g1 b1 ...): a 128-byte line holds a 4x4x4 colour
// cube, so the maps pass's gathers for a noisy or smooth neighbourhood of
// colours touch ~1/4 of the lines an r-major table does
__host__ __device__ inline uint32_t sc_spread3(uint32_t x) {  // bit i -> bit 3 i (8 bits)
  x = (x | (x << 8)) & 0x0000F00Fu;
  x = (x | (x << 4)) & 0x000C30C3u;
  return (x | (x << 2)) & 0x00249249u;
}
__host__ __device__ inline uint32_t sc_colour_key(uint32_t r, uint32_t g, uint32_t b) {
  return (sc_spread3(r) << 2) | (sc_spread3(g) << 1) | sc_spread3(b);
}
constexpr int kFdSlots = 3;
constexpr int kFdCWaves = 14;  // compute waves (one 16-px column block each: aw <= 224); 14, 15 load
constexpr int kFdMaxLds = 160 * 1024;
__host__ __device__ inline int fd_rp(int W) { return (W * 3 + 15) & ~15; }
__host__ __device__ inline int fd_slot_bytes(int W) { return (16 * fd_rp(W) + 1023) & ~1023; }
__host__ __device__ inline int fd_ring_off(int W, int PP) {
  const int tail = 3 * PP - fd_rp(W);
  return kFdSlots * fd_slot_bytes(W) + (tail > 0 ? (tail + 15) & ~15 : 0);
}
// then the vertical pass's A fragments of every analysed-row chunk (3 limbs x
// 64 lanes x 16 B each) and its per-row bias (int32)
__host__ __device__ inline int fd_tab_off(int W, int PP, int aw) {
  const int apitch = (aw * 3 + 15) & ~15, lpitch = (aw + 3) & ~3;
  return fd_ring_off(W, PP) + 80 * apitch + 16 * apitch + 16 * lpitch;
}
__host__ __device__ inline int fd_lds(int W, int PP, int aw, int ah) {
  return fd_tab_off(W, PP, aw) + (ah + kVqRows - 1) / kVqRows * 3072 + 4 * ah;
}
// k_sc_score2: maps resident in LDS when aw*ah*4 <= this; crops whose totals /
// bounds / candidate list stay in LDS (more: the image's CropScore slots).
constexpr int kScoreLdsMaps = 112 * 1024;
constexpr int kScoreMaxCrops = 1024;
// k_sc_score3: the fast pass as exact-integer MFMA (v_mfma_i32_16x16x64_i8).
// Crops of one importance table form groups: up to 16 x origins (the M rows)
// x up to kSgSlots y origins `step` apart (N columns = kSgDigits balanced
// base-256 digits of Tq = rint((importance - oi) 2^q) per slot).  The image's
// maps enter as seven signed-byte planes (value - 128) in LDS: edge, skin,
// sat, and the low / high bytes of skin * edge and sat * edge; per row of the
// group's rows and 64-column k-step, D[limb] += A(16 x origins x 64 px of
// that plane) B(64 px x 16 (digit, slot)).  Every sum is an exact int32; the
// host B fragments are [nrows][ks][64 lanes][16 B].
constexpr int kSgSlots = 3;
constexpr int kSgDigits = 5;
constexpr int kSgPlanes = 7;
constexpr int kSgMax = 2;          // groups per image (accumulators in registers)
constexpr int kSgMaxKs = 2;        // 64-px k-steps per window row
constexpr int kSgMaxCrops = kSgMax * 16 * kSgSlots;
constexpr int kScore3Lds = 160 * 1024 - 4608;  // dynamic LDS cap (k_sc_score3 has 4384 B of static LDS)
__host__ __device__ inline int sg_pitch(int aw) { return (aw + 7) & ~7; }
struct ScGroup {
  int32_t bfrag;                // ai offset (16-B aligned) of the B fragments
  int32_t nrows, ks, ybase;     // analysed rows [ybase, ybase + nrows)
  int32_t nm, nslot, q, step;   // x origins used, y slots, Tq = rint((imp - oi) 2^q), slot spacing
  int32_t x0[16];               // x origin of M row m (rows >= nm repeat the last)
  int32_t S[kSgDigits];         // sum of each digit over the window (the p - 128 bias)
  int32_t pad[3];
};

// v_mfma_i32_16x16x64_i8 operand map (pinned by tools/mfma_probe.hip): lane l
// holds A[l & 15][k] and B[k][l & 15] for its 16 fragment bytes j, with
// k = mfma_i8_k(l, j); D[4 (l >> 4) + i][l & 15], i = 0..3.
#ifndef FI_MFMA_I8_MAP
#define FI_MFMA_I8_MAP 1
#endif
__host__ __device__ inline int mfma_i8_k(int l, int j) {
#if FI_MFMA_I8_MAP == 1
  return 16 * (l >> 4) + j;
#else
  return j < 8 ? 8 * (l >> 4) + j : 32 + 8 * (l >> 4) + (j - 8);
#endif
}
struct MStrip {               // one column strip (fi_plan.h MfmaStrip) placed in the arena
  int32_t x0, x1, b0, nbytes;
  int32_t c_lo, ncols, pitch, nocb, ks;
  int32_t lut_px0, lut_n;
  int32_t frag, s0, lut;      // arena offsets (int32 units; frag 16-B aligned)
  int32_t vpitch;             // k_rs_vm: Q16 plane columns (multiple of 16)
  int32_t frag2;              // k_rs_vr: arena offset of the two-limb fragments (fi_plan.h MfmaH::frag2)
};
// k_sc_hmfma (fi_smartcrop.hip): Pillow's horizontal pass as exact integer
// MFMA.  Per 16-column output block b: source window [s0(b), s0(b) + 64 KS),
// coefficient limbs L0 + 256 L1 + 65536 L2 (signed i8) in fragment order;
// s0(b) is 8-B aligned (two 8-byte fragment reads), ks <= 2.
constexpr int kHmMaxLds = 64 * 1024;

// k_rs_vm (fi_vm.hip): streaming exact-integer MFMA resample, vertical first.
struct VDesc {                // one image
  const uint8_t *src;
  int64_t src_stride;
  uint8_t *dst;
  int64_t dst_stride;
  int32_t ew, eh, rot, gray;
  int32_t rows, nrows, row0, rstep;  // touched-row list (ai offset) / rows[k] = row0 + rstep k when rstep > 0
  int32_t plo, pn, pblk, plast;      // ai offsets of the piece tables (fi_plan.h VmV)
  int32_t pmeta;                     // ai offset (16-B aligned): per piece {plo, pn, pblk, plast}
  int32_t frag;                      // ai offset (16-B aligned) of the piece fragments [p][2][3][64 lanes][16 B]
  int32_t w128;                      // ai offset (16-B aligned): 128 * sum of quantized weights per output row
  int32_t hwsum;                     // ai offset of the horizontal per-px weight sums
  int32_t nblk;
  int32_t vsh, hsh;                  // k_rs_vr: weight shifts of the two-limb tables (fi_plan.h VrV)
};
struct VTile {                // one workgroup: image x strip x pieces [p0, p1); blocks < emit0 are halo only
  int32_t img, strip, p0, p1, emit0, pad;
};
constexpr int kVmThreads = 512;      // 8 waves x 4 column tiles of 16 B = 512-B strips
// piece buffer: 64 rows x 512 B; 16-byte chunk c of row r at r * 512 + 16 (c ^ f(r)),
// f(r) = (r & 7) | 8 ((r >> 4) & 1): the 8 rows of a ds_read_b64_tr_b8 quarter
// wave hit 8 different chunk columns and the two 8-row groups of a half-wave
// (rows 16 apart) the two halves of the banks
constexpr int kVmChunkBytes = 64 * 512;
constexpr int kVmABytes = 6 * 1024 + 64;  // the piece's A fragments [slot][limb][64 lanes][16 B] + 16 w128 rows
constexpr int kVmMaxLds = 80 * 1024;      // two workgroups per CU
constexpr int kVmOtilePitch = 64 * 3 + 4;      // Q16 output tile row, u16 units (nx <= kVmMaxNx = 64)
constexpr int kVmOtileBytes = 16 * kVmOtilePitch * 2;
constexpr int kVmOtile8Pitch = 64 * 3 + 4;     // 8-bit tile row (fast RGB path)
constexpr int kVmOtile8Bytes = 16 * kVmOtile8Pitch;
constexpr int kVrMaxLds = 160 * 1024;  // k_rs_vr: one 1024-thread workgroup per CU
// k_rs_vr (fi_vr.hip): a persistent, warp-specialised resample with a block-major vertical pass over a
// ring of R touched source rows (fi_plan.h VrV).  The VDesc fields rows /
// nrows / row0 / rstep / w128 / frag / hwsum are VrV's, pmeta the per-block
// {K0, ks, Rend, 0}.  A workgroup walks tiles g, g + G, ...; their touched rows
// form one stream: tile t's list rows [kbase, kbase + glen) at stream
// positions [g0, g0 + glen) (kbase, g0, glen multiples of 16), ring slot of
// stream row G = G mod R.
// k_rs_vr's uneven touched-row list (rows[nrows], a 32-entry pad) is followed
// by two copies in per-wave pair classes, one per loader-wave count NL (a
// wave's own pairs are C = 2 NL rows apart): class rho = k mod C, entry j = the
// pair (rows[C j + rho], rows[C j + rho + 1]) of J_C = ceil(nrows / C) + 16
// entries; the C = 4 copy first, then the C = 8 one.  Offset (int32 units,
// from the list start) of the pair starting at row k:
__host__ __device__ inline int vr_pair_cls_len(int nrows, int C) { return (nrows + C - 1) / C + 16; }
__host__ __device__ inline int vr_pair_off(int nrows, int k, int C) {
  const int base = nrows + 32 + (C == 8 ? 8 * vr_pair_cls_len(nrows, 4) : 0);
  return base + 2 * ((k & (C - 1)) * vr_pair_cls_len(nrows, C) + k / C);
}
struct VrTile {
  int32_t img, strip, b0, b1, g0, kbase, glen, pad;
};
struct VrLayout {
  int32_t R;            // ring rows (multiple of 32)
  int32_t plane;        // bytes of one limb plane of one channel (16 vpitch + pad)
  int32_t otile_off;    // output tiles [2][otile_bytes]
  int32_t otile_bytes;
  int32_t total;        // dynamic LDS of the launch
  int32_t nl;           // loader waves (2 or 4; the H waves are the other 7 - nl of waves 8-14)
  int32_t pbuf;         // Q16 plane buffers (1: the V waves wait for the H waves' reads; 2: by block parity)
};

// k_rs_hv (fi_hv.hip): streaming exact-integer MFMA resample, horizontal first
// (fi_plan.h HvH / HvV).
struct HvDesc {               // one image
  const uint8_t *src;
  int64_t src_stride;
  uint8_t *dst;
  int64_t dst_stride;
  int32_t ew, eh, rot, gray;
  int32_t W;                  // source width (the staging's right edge)
  int32_t row0, nrows, nblk;  // source rows [row0, row0 + nrows); 16-row output blocks
  int32_t vk;                 // ai offset: per block (K0, ks)
  int32_t vfrag;              // ai offset (16-B aligned): A fragments [block][t][limb][64 lanes][16 B]
  int32_t vws;                // ai offset (16-B aligned): weight sum per output row
  int32_t hw128;              // ai offset: 128 * horizontal weight sum per output px
};
struct HvStripD {             // fi_plan.h HvStrip placed in the arena
  int32_t x0, x1, px0, pp, nocb;
  int32_t frag, s0, pad;      // ai offsets (frag 16-B aligned)
};
struct HvTile {               // one workgroup: image x strip x output blocks [b0, b1)
  int32_t img, strip, b0, b1;
};
constexpr int kHvThreads = 512;
constexpr int kHvRing = 144;          // intermediate rows: a 128-row window at any production phase
constexpr int kHvOpitch = 144;        // ring row bytes (48 px x 3 channels; 9 16-byte groups, odd)
constexpr int kHvOtPitch = 48 * 3 + 4;  // Q16 output tile row, u16 units

// fi_pixelate.hip: one ScaleImage pass of a face box (face-blur pixelation)
struct PixPass {
  const uint8_t *src8;    // MODE 0: the crop's first byte in the 8-bit image
  const uint16_t *src16;  // MODE 1: the 10% image (Q16, pitch iw * C)
  int64_t sstride;        // MODE 0: image row stride
  int32_t iw, ih;         // input dims
  uint16_t *dst16;        // MODE 0: the 10% image
  uint8_t *dst8;          // MODE 1: the image at (X, Y)
  int64_t dstride;
  int32_t ow, oh, C;
  int32_t clip_w, clip_h;  // MODE 1: writable extent right / below (X, Y)
  int32_t yoff, yidx, xoff, xidx;  // ai offsets of the row / column lists (fi_plan.h ScaleList)
  int32_t yw, xw;                  // ad offsets of their weights
};
struct ScParamsDev {
  double detail_weight, edge_radius, edge_weight, outside_importance;
  double saturation_bias, saturation_brightness_max, saturation_brightness_min,
      saturation_threshold, saturation_weight;
  double skin_bias, skin_brightness_max, skin_brightness_min;
  double skin_color[3];
  double skin_threshold, skin_weight;
  int32_t rule_of_thirds;
  int32_t pad;
};

struct ScResult {
  int32_t top;          // index within the image's crops, -1 on failure
  int32_t n_candidates;
  double total;
};

// convert -crop of the smartcrop box (SmartCropProcessor.php:30-34)
struct ApplyDesc {
  const uint8_t *src;
  int64_t src_stride;
  int32_t W, H, C;
  int32_t result, crop0;
  uint8_t *dst;
  int32_t *out_wh;  // [2] written by the kernel
};

// -monochrome (fi_mono.hip): per-image quantize state
// written by k_mono_stats, read by k_mono_dither
struct MonoState {
  int32_t bilevel;         // 1: the gray image is already black/white (no quantize)
  int32_t black, white;    // NormalizeImage stretch points
  int32_t ncol;            // colormap entries (<= 2)
  uint16_t mean[8];        // cluster means (the dither's colormap)
  uint16_t bil[8];         // thresholded bilevel colours (0 / 65535)
  uint8_t cand[256];       // per 8-bit value: colours of its closest-colour search subtree (bit i = colour i)
};
struct MonoDesc {
  const uint16_t *g;       // Q16 gray of the extent window (row stride w), written by the resample epilogue
  int32_t w, h, rot;
  int32_t pad;
  uint8_t *dst;            // final 8-bit output, rotated (IntegralRotateImage after -monochrome)
  int64_t dst_stride;
  MonoState *st;
};

struct CropScore {  // per crop (batch-global index)
  double detail, saturation, skin, total;
  double bound;
  int32_t exact;
  int32_t pad;
};

// ---- GPU JPEG decode (fi_jpeg.hip): baseline sequential Huffman, 8-bit, one
// scan (gray, or YCbCr with luma sampling 1x1 / 2x1 / 2x2 and 1x1 chroma),
// libjpeg-turbo's islow IDCT, fancy upsampling and YCbCr->RGB bit for bit.
struct JpegHuff {        // one Huffman table (jdhuff.c canonical decoding)
  uint16_t look[512];    // 9-bit lookahead: (length << 8) | symbol; 0 = code longer than 9 bits
  int32_t maxcode[18];   // largest code of each length (-1: none); [17] sentinel
  int32_t valoff[18];    // huffval index = code + valoff[length]
  uint8_t huffval[256];
  int16_t fast_ac[512];  // AC tables: code + value bits within the 9-bit lookahead:
                         // (value << 8) | (run << 4) | total length; 0 = not this fast path
};
struct JpegDesc {        // one image of a decode batch
  const uint8_t *ecs;    // entropy-coded segment (device)
  int32_t ecs_len;
  int32_t W, H, ncomp;
  int32_t hmax, vmax, mcux, mcuy;  // MCUs per row / per column
  int32_t h[3], v[3];              // sampling factors
  int32_t tq[3], td[3], ta[3];     // quant / DC / AC table of each component
  int32_t bw[3], bh[3];            // component block grid (whole MCUs)
  int32_t dw[3], dh[3];            // downsampled width / height (jdmaster.c)
  int64_t coef[3];                 // byte offsets in the work buffer: int16 blocks [bh][bw][64], zigzag order
  int64_t plane[3];                // u8 samples [bh * 8][bw * 8]
  int32_t qt;                      // index of the image's 4 quant tables (u16 [4][64], natural order)
  int32_t ht[4];                   // its Huffman tables DC0, DC1, AC0, AC1 (batch table index, -1: none)
  uint8_t *dst;                    // HWC: 3 channels (YCbCr sources, or gray replicated) or 1 (gray)
  int64_t dst_stride;
  int32_t dst_c;
};
struct JpegInterval {    // one restart interval: its MCUs and where its bits start
  int32_t img, mcu0, mcu1, byte0;
};

}  // namespace fi
