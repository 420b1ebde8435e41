// fi_plan.h -- host-side planning: ImageMagick geometry and tap tables,
// Pillow prescale geometry and coefficients, smartcrop crop windows and
// importance tables.  Pure integer/IEEE-double host code (built with
// -ffp-contract=off), no GPU calls.
#pragma once
#include <stdint.h>

#include <string>
#include <vector>

#include "fi_internal.h"

namespace fi {

enum Filter { kFilterLanczos = 1, kFilterMitchell = 2 };

// Resample geometry of one image, ImageMagick 6 semantics.
struct ImPlan {
  int status = FI_OK;
  std::string err;
  int W = 0, H = 0, C = 3;
  int tw = 0, th = 0;       // -thumbnail / -resize target (ParseMetaGeometry)
  bool resize = false;      // false: ResizeImage returns a clone
  bool sample = false;      // ThumbnailImage 5x SampleImage pre-step
  int sw = 0, sh = 0;       // sampled dims (= W, H when !sample)
  int filter = kFilterLanczos;
  bool hfirst = false;      // HorizontalFilter first iff x_factor > y_factor
  double xf = 1, yf = 1;
  int ex0 = 0, ey0 = 0, ew = 0, eh = 0;  // extent window in the resized image
  bool gray = false;
  bool mono = false;        // -monochrome: Q16 gray of the extent window -> fi_mono.hip -> rotate
  int rot = 0;
  int out_w = 0, out_h = 0, out_c = 3;   // after rotate
  // forwarded convolutions on the rotated Q16 image (bit 0 unsharp, 1 sharpen, 2 blur)
  unsigned conv = 0;
  double cv[8] = {0, 0, 0, 0, 0, 0, 0, 0};  // unsharp r, s, gain, thr; sharpen r, s; blur r, s
};
int plan_im(const fi_image &img, ImPlan *p);
// IM 6.9 kernels of the forwarded convolutions (morphology.c BlurKernel,
// effect.c SharpenImage): width, values (f64) -- the same arithmetic as the
// oracle's or_im_blur_kernel / or_im_sharpen_kernel.
int im_blur_kernel(double radius, double sigma, std::vector<double> *k);
int im_sharpen_kernel(double radius, double sigma, std::vector<double> *k);
constexpr int kConvMaxBlur = 1023;   // 1-D taps
constexpr int kConvMaxSharpen = 63;  // 2-D kernel side

// One resample axis in the source index domain.
struct AxisTable {
  std::vector<int32_t> start, count, woff;
  std::vector<float> w;
  std::vector<double> wd;  // the same weights in f64 (the RGBA path accumulates in f64 as IM does)
  int32_t maxtaps = 0, src_lo = 0, src_hi = 0, touched = 0;
};

// Exact-integer MFMA resample tables (k_rs_vm, fi_vm.hip; k_sc_hmfma).
// Weights are quantized to W = rint(w * 2^kMfmaWBits) and split into three
// signed-byte limbs; fragments are in the v_mfma_i32_16x16x64_i8 lane order
// (fi_internal.h mfma_i8_k), 256 int32 (1 KB) each.
constexpr int kMfmaWBits = 22;
constexpr int kMfmaStripBytes = 512;   // source bytes per column strip
constexpr int kMfmaMaxNx = 168;        // output px per strip
constexpr int kMfmaMaxPitch = 232;     // widest strip window (touched columns incl. fragment padding)
struct MfmaStrip {                     // one column strip of the horizontal pass
  int32_t x0, x1;                      // output px [x0, x1)
  int32_t b0, nbytes;                  // source bytes loaded (16-B aligned)
  int32_t c_lo, ncols, pitch;          // compacted touched columns of the strip, LDS plane pitch
  int32_t vpitch;                      // k_rs_vm plane columns: covers every fragment window, multiple of 16
  int32_t nocb, ks;                    // 16-px output blocks, k-steps of 64 columns
  int32_t lut_px0, lut_n;              // px -> compact column LUT over [lut_px0, lut_px0 + lut_n)
  size_t frag, s0, lut;                // offsets into MfmaH::frag / s0 / lut
  size_t frag2;                        // offset into MfmaH::frag2 (two-limb fragments of k_rs_vr)
};
struct MfmaH {
  std::vector<int32_t> cols;           // touched source columns, ascending
  std::vector<MfmaStrip> strips;
  std::vector<int32_t> frag, s0, lut;  // B fragments [strip][nocb][ks][3]; (w0, ks) per block; LUTs
  std::vector<int32_t> wsum;           // [ew] sum of quantized weights per output px
  // k_rs_vr's horizontal pass: W = rint(w * 2^shift2) in TWO signed-byte limbs
  // (vr_quant), fragments [strip][nocb][ks][2]; shift2 = 0: no two-limb form
  int32_t shift2 = 0;
  std::vector<int32_t> frag2, wsum2;
};
bool build_mfma_h(const AxisTable &h, MfmaH *m, int max_nx = kMfmaMaxNx);

// Streaming vertical tables of k_rs_vm (fi_vm.hip).  The touched-row list is
// cut into pieces of <= 64 rows aligned to the 16-row output blocks: the
// pieces of block b hold the rows first needed by b, [R(b-1), R(b)), with
// R(b) = one past the last tap row of block b.  A piece feeds two
// accumulator slots: slot 0 = its own block b, slot 1 = block b + 1 (whose
// window starts inside it).  Block b is complete after its last piece.
// Requires every tap of block b to lie in the pieces of b - 1 and b
// (checked: taps span <= 21 output rows' worth of rows for Lanczos/Mitchell
// at any downscale).
constexpr int kVmMaxNx = 64;           // output px per strip: 4 16-px blocks, one per wave
struct VmV {
  std::vector<int32_t> rows;           // touched source rows, ascending
  int nblk = 0;                        // 16-row output blocks
  std::vector<int32_t> plo, pn, pblk, plast;  // per piece: list start, rows, block, block completes
  std::vector<int32_t> frag;           // [piece][slot 0/1][limb 0..2] fragments (256 int32 each)
  std::vector<int32_t> w128;           // [16 nblk] 128 * sum of quantized weights of each output row
  int32_t row0 = 0, rstep = 0;         // rstep > 0: rows[k] == row0 + rstep * k
};
bool build_vm_v(const AxisTable &v, VmV *m);

// Tables of k_rs_hv (fi_hv.hip): the horizontal-first streaming kernel.  Both
// axes must touch a contiguous range of source rows / columns (always the case
// without the ThumbnailImage sample pre-step, and a horizontal-first geometry
// never has one: the sampled factors are equal).
//   horizontal  column strips of <= kHvMaxNx output px; the strip's source
//               window [px0, px0 + pp) starts on a 16-px boundary (48 bytes:
//               whole pixels, 16-byte aligned loads); per 16-px output block a
//               window start w0 (8-aligned, relative to px0) and <= 2 k-steps
//               of 64 columns, B fragments [block][t][limb] (t < 2, zero past ks);
//   vertical    per 16-row output block a window start K0 (touched-row list
//               index, nondecreasing) and <= 2 k-steps of 64 rows, A fragments
//               [block][t][limb], and the weight sum of every output row.
constexpr int kHvMaxNx = 48;     // output px per strip: 3 16-px blocks (32-px strips measured slower: 21.7 vs 18.7 ms, cfg4 8192-image run)
constexpr int kHvMaxPP = 256;    // source px of a strip window
struct HvStrip {
  int32_t x0, x1, px0, pp, nocb;
  size_t frag, s0;               // offsets into HvH::frag / s0
};
struct HvH {
  int32_t col0 = 0;              // touched columns = [col0, col0 + ncols)
  std::vector<HvStrip> strips;
  std::vector<int32_t> frag, s0, w128;  // w128: 128 * weight sum per output px
};
bool build_hv_h(const AxisTable &h, HvH *m);
struct HvV {
  int32_t row0 = 0, nrows = 0, nblk = 0;
  std::vector<int32_t> k0ks;     // per block: K0, ks
  std::vector<int32_t> frag;     // [block][t < 2][limb][256]
  std::vector<int32_t> wsum;     // [16 nblk] weight sum per output row
};
bool build_hv_v(const AxisTable &v, HvV *m);

// Block-major vertical tables of k_rs_vr (fi_vr.hip): the vertical-first pass
// with each 16-row output block computed in one go from a ring of touched
// source rows.  Per block b: window start K0(b) (touched-row list index, a
// multiple of 16, nondecreasing), ks(b) <= 2 k-steps of 64 list rows, Rend(b) =
// one past its last non-zero tap, A fragments [b][t][limb] (zero past ks and
// past the taps) and 128 * the quantized weight sum of every output row (pixels
// enter the MFMA as p - 128).
//
// Two weight limbs, not k_rs_vm's three: W = rint(w * 2^shift) with the largest
// shift <= kVrMaxShift whose W all fit two signed bytes (vr_quant; the shift
// follows the largest weight, so the precision relative to it is ~15 bits at
// any factor), each output's W adjusted to keep its sum (quant_axis), so a
// block costs 4 MFMAs per column tile instead of 6.  shift >= kVrMinShift,
// else no k_rs_vr.  tests/native/vr_quant_bound.cpp rebuilds every table of the
// BASELINE geometries and 200 random ones from its fragments and bounds the
// worst case over all 8-bit inputs against IM's f64 weights: <= 0.1 LSB before
// the final rounding (so within +-1 LSB); tests/test_gpu_vr.py checks every
// k_rs_vr class against k_rs_vm's 22-bit path and the oracle.
constexpr int kVrMaxShift = 22;
constexpr int kVrMinShift = 15;
struct VrV {
  std::vector<int32_t> rows;           // touched source rows, ascending
  int32_t row0 = 0, rstep = 0;         // rstep > 0: rows[k] == row0 + rstep * k
  int nblk = 0;
  int32_t shift = 0;                   // W = rint(w * 2^shift)
  std::vector<int32_t> bmeta;          // [nblk][4] {K0, ks, Rend, 0}
  std::vector<int32_t> frag;           // [nblk][2][2][256]
  std::vector<int32_t> w128;           // [16 nblk]
  int32_t maxgap = 0;                  // widest gap between consecutive touched rows
};
// the largest shift in [kVrMinShift, kVrMaxShift] at which every sum-kept
// quantised weight of the axis fits two signed-byte limbs (hi * 256 + lo, both
// in [-128, 127]), the weights in *wq (AxisTable::w order); 0 if none
int vr_quant(const AxisTable &t, std::vector<int32_t> *wq);
// k_rs_vm's 2^22-scaled weights (AxisTable::w order): vr_quant's times
// 2^(22 - shift) when the axis has two-limb weights, else rint(w 2^22); returns
// the shift they carry (22 for the latter)
int axis_q22(const AxisTable &t, std::vector<int32_t> *q);
bool build_vr_v(const AxisTable &v, VrV *m);

// Output indices [o0, o1) of a filter pass from `in_sampled` (sampled domain)
// to `out_size`; taps mapped back to the `in_src` source indices through the
// SampleImage offsets (identity when !sample) and merged.
void build_axis(int filter, double factor, int in_sampled, int out_size, int o0, int o1,
                bool sample, int in_src, AxisTable *t);

// ----------------------------------------------------------------------
struct CropHost {
  double fx, fy, fw, fh;
  int32_t x0, y0, nin_x, nin_y;
  int32_t rx, ry, rw, rh;
};
struct ScPlan {
  int status = FI_OK;
  std::string err;
  int W = 0, H = 0;
  double prescale = 1;
  int cw = 0, ch = 0;                   // crop dims in the analysed image
  bool thumb = false;                   // Pillow thumbnail runs
  int fx = 1, fy = 1, rw = 0, rh = 0;   // reduce
  int aw = 0, ah = 0;                   // analysed dims
  bool need_h = false, need_v = false;
  int ksh = 0, ksv = 0, ybox_first = 0, hrows = 0;
  std::vector<int32_t> hb, hk, vb, vk;  // bounds pairs and int32 coeffs
  std::vector<int32_t> hkT;             // hk transposed [ksh][aw]
  bool prep_ok = false;                 // k_sc_hrows/k_sc_vmaps fit LDS (else generic kernels)
  int h_chunks = 0, h_lds = 0, v_chunks = 0, v_lds = 0;
  // k_sc_hmfma: exact-integer MFMA horizontal pass (fi_internal.h mfma_i8_k)
  bool hm_ok = false;
  int hm_ks = 0, hm_pitch = 0, hm_rows = 0, hm_nb = 0, hm_lds = 0, hm_chunks = 0;
  std::vector<int32_t> hmB;   // [nb][ks][3 limbs] fragments of 64 lanes x 16 B (256 int32)
  std::vector<int32_t> hmC;   // [aw] 2^21 + 128 * sum_j k[x][j]  (pixels enter as p - 128)
  std::vector<int32_t> hmS0;  // [nb] first source column of the block's window (multiple of 16)
  // k_sc_vq: Pillow's vertical pass as exact integer MFMA fused with the maps;
  // one workgroup per kVqRows analysed rows (+1 halo row each side = one
  // 16-row MFMA block), its H-stage window starts at vqK0[chunk] (<= 64 rows)
  bool vq_ok = false;
  int vq_chunks = 0, vq_lds = 0;
  // k_sc_hx + k_sc_vx (co-resident with the next batch's resample: no LDS,
  // <= 64 VGPRs): the H-stage goes to HBM as 256-B tiles [block][channel][row
  // block][16 columns][16 rows] of p - 128 bytes, cx_tp / 16 row blocks, of
  // which k_sc_hx writes all but the last (source rows clamped to the last;
  // the last block is read only as zero-weight straddle).  Per chunk the vertical window
  // starts at cxK0 (vqK0 rounded down to 4: dword loads) and spans cx_kv
  // 64-row k-steps; cxA = [chunk][kv][3 limbs] fragments (256 int32 each).
  bool cx_ok = false;
  int cx_kv = 0, cx_tp = 0;
  std::vector<int32_t> cxA, cxK0;
  bool fz_ok = false;  // k_sc_fz (fused per-image prescale + maps)
  int fz_lds = 0;
  std::vector<int32_t> vqA;   // [chunk][3 limbs] fragments of 64 lanes x 16 B (256 int32)
  std::vector<int32_t> vqC;   // [ah] 2^21 + 128 * sum_j k[y][j]
  std::vector<int32_t> vqK0;  // [chunk] first H-stage row of the window
  std::vector<CropHost> crops;
};
void plan_sc_prep(ScPlan *p);
int plan_sc(int W, int H, int target_w, int target_h, const fi_smartcrop_options &o, ScPlan *p);
void sc_importance_table(const fi_smartcrop_params &P, double fw, double fh, int nx, int ny,
                         std::vector<double> *out);
// k_sc_score3's B fragments of one importance table (fi_internal.h ScGroup):
// Tq(u, v) = rint((imp(u, v) - oi) 2^q) as kSgDigits balanced signed base-256
// digits, q the largest that keeps |Tq| < 2^38.9; rows r of a group with
// `nslot` y origins `step` apart hold window row r - step j in slot j.
struct ScoreBTab {
  bool ok = false;
  int q = 0, nrows = 0, ks = 0;
  int32_t S[5] = {0, 0, 0, 0, 0};  // sum over the window of each digit
  std::vector<int32_t> frag;       // [nrows][ks][64 lanes][16 B]
};
void sc_score_btab(const std::vector<double> &imp, int nx, int ny, double oi, int nslot, int step, ScoreBTab *out);
// or_pil_coeffs equivalent (Resample.c precompute_coeffs + normalize_coeffs_8bpc)
int pil_coeffs(int in_size, float in0, float in1, int out_size, std::vector<int32_t> *bounds,
               std::vector<int32_t> *kk);

// IM 6 ScaleImage (resize.c) as per-output contribution lists: output o is
// sum_k w[k] * in[idx[k]], k in [off[o], off[o + 1]), accumulated from 0 in
// list order -- exactly the additions ScaleImage makes (rows: the y_vector /
// span.y loop; columns: the pixel / span.x loop, including which partial sums
// it keeps).  Used by the face-blur pixelation (fi_pixelate.hip).
struct ScaleList {
  std::vector<int32_t> off, idx;
  std::vector<double> w;
};
void im_scale_rows(int in_size, int out_size, ScaleList *L);
void im_scale_cols(int in_size, int out_size, ScaleList *L);
// ParseMetaGeometry's percentage size: floor(percent * size / 100 + 0.5)
int im_percent_size(int size, double percent);

}  // namespace fi
