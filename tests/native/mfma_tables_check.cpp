// CPU check of the k_rs_vm / k_sc_hmfma host tables (fi_plan.cpp): the
// weight matrices rebuilt from the fragment bytes through mfma_i8_k must give,
// with the kernel's integer algebra, exactly sum(quant(w) * p) for every
// output -- for the vertical pass over the touched-row list, the horizontal
// pass over each strip's compacted columns (plus the px -> column LUT and
// byte ranges), and the Pillow horizontal pass (exact int32 of Resample.c).
// Built and run by tests/test_native_cpu.py (hipcc, host only).
#include <math.h>
#include <stdio.h>
#include <stdlib.h>

#include <random>
#include <vector>

#include "../../flyimg_amd/csrc/fi_plan.h"

using namespace fi;

static int g_fail = 0;
#define CHECK(c, ...)                 \
  do {                                \
    if (!(c)) {                       \
      if (g_fail < 20) {              \
        printf("FAIL %s:%d ", __FILE__, __LINE__); \
        printf(__VA_ARGS__);          \
        printf("\n");                 \
      }                               \
      g_fail++;                       \
    }                                 \
  } while (0)

static int32_t qw(float w) { return (int32_t)lrint((double)w * (double)(1 << kMfmaWBits)); }
static int8_t frag_byte(const std::vector<int32_t> &f, size_t base, int q, int lane, int j) {
  return (int8_t)reinterpret_cast<const uint8_t *>(&f[base + (size_t)q * 256])[lane * 16 + j];
}
static int64_t limb_w(const std::vector<int32_t> &f, size_t base, int lane, int j) {
  return (int64_t)frag_byte(f, base, 0, lane, j) + 256 * (int64_t)frag_byte(f, base, 1, lane, j) +
         65536 * (int64_t)frag_byte(f, base, 2, lane, j);
}

static bool g_required = false;  // the geometry must take the MFMA path
// k_rs_vm: stream the pieces in order with two accumulator slots exactly as
// the kernel does (slot 0 = the piece's block, slot 1 = the next block,
// started at its w128 correction) and compare every completed block.
static void check_vm(const AxisTable &v, const char *name) {
  VmV m;
  if (!build_vm_v(v, &m)) {
    printf("  %s: streaming vertical tables not built, skipped\n", name);
    CHECK(!g_required, "%s: streaming vertical tables required", name);
    return;
  }
  const int ny = (int)v.start.size(), np = (int)m.plo.size();
  std::vector<int32_t> q22;  // k_rs_vm carries k_rs_vr's two-limb weights scaled to 2^22 (axis_q22)
  axis_q22(v, &q22);
  std::mt19937 rng(4321);
  std::vector<int> px(v.src_hi);
  for (auto &x : px) x = (int)(rng() & 255);
  auto w128 = [&](int b, int r) -> int64_t { return b < m.nblk ? m.w128[16 * b + r] : 0; };
  std::vector<int64_t> acc0(16), acc1(16);
  int b0 = m.pblk[0], done = 0;
  for (int r = 0; r < 16; r++) {
    acc0[r] = w128(b0, r);
    acc1[r] = w128(b0 + 1, r);
  }
  for (int p = 0; p < np; p++) {
    CHECK(m.pn[p] >= 0 && m.pn[p] <= 64, "%s: piece %d has %d rows", name, p, m.pn[p]);
    CHECK(p == 0 || m.plo[p] == m.plo[p - 1] + m.pn[p - 1], "%s: pieces not contiguous at %d", name, p);
    for (int s = 0; s < 2; s++)
      for (int l = 0; l < 64; l++)
        for (int j = 0; j < 16; j++) {
          const int k = mfma_i8_k(l, j);
          const int64_t w = limb_w(m.frag, (size_t)(p * 2 + s) * 3 * 256, l, j);
          if (k >= m.pn[p]) {
            CHECK(w == 0, "%s: weight past the piece", name);
            continue;
          }
          const int64_t add = w * (px[m.rows[m.plo[p] + k]] - 128);
          (s == 0 ? acc0 : acc1)[l & 15] += add;
        }
    if (m.plast[p]) {
      const int b = m.pblk[p];
      CHECK(b == done, "%s: block %d completes out of order", name, b);
      for (int r = 0; r < 16; r++) {
        const int y = 16 * b + r;
        if (y >= ny) continue;
        int64_t ref = 0;
        for (int j = 0; j < v.count[y]; j++) ref += (int64_t)q22[v.woff[y] + j] * px[v.start[y] + j];
        CHECK(acc0[r] == ref, "%s: streaming vertical y=%d %lld != %lld", name, y, (long long)acc0[r],
              (long long)ref);
        CHECK(llabs(acc0[r]) < (1ll << 31), "%s: accumulator exceeds int32", name);
      }
      done++;
      acc0 = acc1;
      for (int r = 0; r < 16; r++) acc1[r] = w128(b + 2, r);
    }
  }
  CHECK(done == m.nblk, "%s: %d of %d blocks completed", name, done, m.nblk);
  printf("  %s: streaming vertical %d blocks, %d pieces, rstep %d ok\n", name, m.nblk, np, m.rstep);
}

// k_rs_vs: stream the uniform 64-row pieces with three rotating slots exactly
// as the kernel does (new slots start at the record's w128 rows, completed
// slots retire from the bottom) and compare every completed block.
static void check_h(const AxisTable &h, const char *name) {
  MfmaH m;
  if (!build_mfma_h(h, &m)) {
    printf("  %s: horizontal tables not built, skipped\n", name);
    CHECK(!g_required, "%s: horizontal MFMA tables required", name);
    return;
  }
  const int nx = (int)h.start.size();
  std::vector<int32_t> q22;
  axis_q22(h, &q22);
  std::mt19937 rng(99);
  std::vector<int> V(h.src_hi);
  for (auto &x : V) x = (int)(rng() % 65536);
  int covered = 0;
  for (const MfmaStrip &S : m.strips) {
    CHECK(S.b0 % 16 == 0 && S.nbytes % 16 == 0 && S.nbytes <= kMfmaStripBytes, "%s: strip bytes", name);
    // compact column c (relative) -> source px, through the LUT
    std::vector<int> colpx(S.pitch, -1);
    for (int k = 0; k < S.lut_n; k++) {
      const int ci = m.lut[S.lut + k];
      if (ci < 0) continue;
      const int px = S.lut_px0 + k;
      CHECK(3 * px >= S.b0 && 3 * px + 3 <= S.b0 + S.nbytes, "%s: px %d outside strip bytes", name, px);
      CHECK(ci < S.ncols && colpx[ci] < 0, "%s: LUT column %d", name, ci);
      if (ci < S.ncols) colpx[ci] = px;
    }
    for (int c = 0; c < S.ncols; c++) CHECK(colpx[c] == m.cols[S.c_lo + c], "%s: column %d not mapped", name, c);
    for (int ob = 0; ob < S.nocb; ob++) {
      const int w0 = m.s0[S.s0 + 2 * ob], ksob = m.s0[S.s0 + 2 * ob + 1];
      CHECK(w0 % 8 == 0 && ksob >= 1 && ksob <= S.ks && w0 + 64 * ksob <= S.pitch, "%s: window", name);
      for (int t = ksob; t < S.ks; t++)
        for (int l = 0; l < 64; l++)
          for (int j = 0; j < 16; j++)
            CHECK(limb_w(m.frag, S.frag + (size_t)(ob * S.ks + t) * 3 * 256, l, j) == 0, "%s: weight past ks", name);
      std::vector<int64_t> W((size_t)16 * 64 * S.ks, 0);
      for (int t = 0; t < S.ks; t++)
        for (int l = 0; l < 64; l++)
          for (int j = 0; j < 16; j++)
            W[(size_t)(l & 15) * 64 * S.ks + 64 * t + mfma_i8_k(l, j)] =
                limb_w(m.frag, S.frag + (size_t)(ob * S.ks + t) * 3 * 256, l, j);
      for (int n = 0; n < 16; n++) {
        const int x = S.x0 + 16 * ob + n;
        if (x >= S.x1) continue;
        covered++;
        // kernel: 256 sum W (Vh - 128) + sum W (Vl - 128) + 32896 wsum
        int64_t sh = 0, sl = 0;
        for (int k = 0; k < 64 * S.ks; k++) {
          const int64_t w = W[(size_t)n * 64 * S.ks + k];
          const int c = w0 + k;
          if (w == 0) continue;
          CHECK(c < S.ncols, "%s: weight on padding column", name);
          const int v = V[colpx[c]];
          sh += w * ((v >> 8) - 128);
          sl += w * ((v & 255) - 128);
        }
        const int64_t s = 256 * sh + sl + 32896 * (int64_t)m.wsum[x];
        int64_t ref = 0;
        for (int j = 0; j < h.count[x]; j++) ref += (int64_t)q22[h.woff[x] + j] * V[h.start[x] + j];
        CHECK(s == ref, "%s: horizontal x=%d %lld != %lld", name, x, (long long)s, (long long)ref);
        CHECK(llabs(sh) < (1ll << 31) && llabs(sl) < (1ll << 31), "%s: horizontal limb sum exceeds int32", name);
      }
    }
  }
  CHECK(covered == nx, "%s: strips cover %d of %d px", name, covered, nx);
  printf("  %s: horizontal %zu strips ok\n", name, m.strips.size());
}

// k_rs_hv: the horizontal pass over each strip's plane window and the
// vertical pass over each block's ring window, with the kernel's algebra
// (H: sum W (p - 128) + 128 sum W; V: 256 sum W (Vh - 128) + sum W (Vl - 128)
// + 32896 sum W) against sum(quant(w) * value).
static void check_hv(const AxisTable &h, const AxisTable &v, const char *name) {
  HvH mh;
  HvV mv;
  if (!build_hv_h(h, &mh) || !build_hv_v(v, &mv)) {
    printf("  %s: horizontal-first tables not built, skipped\n", name);
    CHECK(!g_required, "%s: horizontal-first tables required", name);
    return;
  }
  std::mt19937 rng(77);
  std::vector<int> P(h.src_hi + kHvMaxPP), V(v.src_hi);
  for (auto &x : P) x = (int)(rng() & 255);
  for (auto &x : V) x = (int)(rng() % 65536);
  const int nx = (int)h.start.size(), ny = (int)v.start.size();
  int covered = 0;
  for (const HvStrip &S : mh.strips) {
    CHECK(S.px0 % 16 == 0 && S.pp % 16 == 0 && S.pp <= kHvMaxPP && S.x1 - S.x0 <= kHvMaxNx, "%s: strip", name);
    for (int ob = 0; ob < S.nocb; ob++) {
      const int w0 = mh.s0[S.s0 + 2 * ob], ks = mh.s0[S.s0 + 2 * ob + 1];
      CHECK(w0 % 8 == 0 && ks >= 1 && ks <= 2 && w0 + 64 * ks <= S.pp, "%s: horizontal window", name);
      for (int n = 0; n < 16; n++) {
        const int x = S.x0 + 16 * ob + n;
        if (x >= S.x1) continue;
        covered++;
        int64_t acc = mh.w128[x];
        for (int t = 0; t < 2; t++)
          for (int l = 0; l < 64; l++) {
            if ((l & 15) != n) continue;
            for (int j = 0; j < 16; j++) {
              const int64_t w = limb_w(mh.frag, S.frag + (size_t)(ob * 2 + t) * 3 * 256, l, j);
              if (w == 0) continue;
              CHECK(t < ks, "%s: horizontal weight past ks", name);
              acc += w * (P[S.px0 + w0 + 64 * t + mfma_i8_k(l, j)] - 128);
            }
          }
        int64_t ref = 0;
        for (int j = 0; j < h.count[x]; j++) ref += (int64_t)qw(h.w[h.woff[x] + j]) * P[h.start[x] + j];
        CHECK(acc == ref, "%s: hv horizontal x=%d %lld != %lld", name, x, (long long)acc, (long long)ref);
      }
    }
  }
  CHECK(covered == nx, "%s: hv strips cover %d of %d px", name, covered, nx);
  for (int b = 0; b < mv.nblk; b++) {
    const int K0 = mv.k0ks[2 * b], ks = mv.k0ks[2 * b + 1];
    CHECK(ks >= 1 && ks <= 2 && (b == 0 || K0 >= mv.k0ks[2 * b - 2]), "%s: vertical window %d", name, b);
    for (int n = 0; n < 16; n++) {
      const int y = 16 * b + n;
      if (y >= ny) continue;
      int64_t sh = 0, sl = 0;
      for (int t = 0; t < 2; t++)
        for (int l = 0; l < 64; l++) {
          if ((l & 15) != n) continue;
          for (int j = 0; j < 16; j++) {
            const int64_t w = limb_w(mv.frag, (size_t)(b * 2 + t) * 3 * 256, l, j);
            if (w == 0) continue;
            const int k = K0 + 64 * t + mfma_i8_k(l, j);
            CHECK(t < ks && k < mv.nrows, "%s: vertical weight outside the window", name);
            const int val = V[mv.row0 + k];
            sh += w * ((val >> 8) - 128);
            sl += w * ((val & 255) - 128);
          }
        }
      const int64_t s = 256 * sh + sl + 32896 * (int64_t)mv.wsum[y];
      int64_t ref = 0;
      for (int j = 0; j < v.count[y]; j++) ref += (int64_t)qw(v.w[v.woff[y] + j]) * V[v.start[y] + j];
      CHECK(s == ref, "%s: hv vertical y=%d %lld != %lld", name, y, (long long)s, (long long)ref);
      CHECK(llabs(sh) < (1ll << 31) && llabs(sl) < (1ll << 31), "%s: vertical limb sum exceeds int32", name);
    }
  }
  printf("  %s: horizontal-first %zu strips, %d blocks ok\n", name, mh.strips.size(), mv.nblk);
}

static void check_pillow(int W, int H, int tw, int th, const char *name) {
  fi_smartcrop_options o;
  o.prescale = 1;
  o.max_scale = 1;
  o.min_scale = 0.9;
  o.scale_step = 0.1;
  o.step = 8;
  o.exact_all = 0;
  ScPlan p;
  if (plan_sc(W, H, tw, th, o, &p) != FI_OK || !p.hm_ok) {
    printf("  %s: no MFMA prescale plan, skipped\n", name);
    return;
  }
  std::mt19937 rng(5);
  const int sw = p.rw;
  std::vector<int> px(sw);
  for (auto &x : px) x = (int)(rng() & 255);
  for (int b = 0; b < p.hm_nb; b++)
    for (int n = 0; n < 16; n++) {
      const int x = 16 * b + n;
      if (x >= p.aw) continue;
      int64_t s = p.hmC[x];
      for (int t = 0; t < p.hm_ks; t++)
        for (int l = 0; l < 64; l++) {
          if ((l & 15) != n) continue;
          for (int j = 0; j < 16; j++) {
            const int col = p.hmS0[b] + 64 * t + mfma_i8_k(l, j);
            const int64_t w = limb_w(p.hmB, (size_t)((b * p.hm_ks + t) * 3) * 256, l, j);
            if (w == 0) continue;
            CHECK(col < sw, "%s: Pillow weight beyond the row", name);
            s += w * (px[col] - 128);
          }
        }
      int64_t ref = 1 << 21;
      for (int j = 0; j < p.hb[2 * x + 1]; j++) ref += (int64_t)p.hk[(size_t)x * p.ksh + j] * px[p.hb[2 * x] + j];
      CHECK(s == ref, "%s: Pillow x=%d %lld != %lld", name, x, (long long)s, (long long)ref);
    }
  printf("  %s: Pillow horizontal %d blocks ok\n", name, p.hm_nb);
}

static void geometry(int W, int H, int tw, int th, uint32_t flags, const char *name) {
  fi_image im{};
  im.src_w = W;
  im.src_h = H;
  im.src_stride = W * 3;
  im.src_channels = 3;
  im.target_w = tw;
  im.target_h = th;
  im.flags = flags;
  ImPlan P;
  if (plan_im(im, &P) != FI_OK || !P.resize) {
    printf("  %s: no resize\n", name);
    return;
  }
  AxisTable v, h;
  build_axis(P.filter, P.yf, P.sh, P.th, P.ey0, P.ey0 + P.eh, P.sample, P.H, &v);
  build_axis(P.filter, P.xf, P.sw, P.tw, P.ex0, P.ex0 + P.ew, P.sample, P.W, &h);
  if (P.hfirst) {
    CHECK(!P.sample, "%s: horizontal-first with the sample pre-step", name);
    check_hv(h, v, name);
  } else {
    check_h(h, name);
    check_vm(v, name);
  }
}

int main() {
  const uint32_t T = FI_OP_THUMBNAIL, F = FI_GEOM_FILL, X = FI_OP_EXTENT, S = FI_GEOM_SHRINK_ONLY;
  g_required = true;  // the BASELINE configurations run on the MFMA kernel
  geometry(1920, 1080, 500, 0, T | S, "cfg2 1920x1080 w_500");
  geometry(3840, 2160, 512, 512, T | F | X, "cfg3 3840x2160 512x512 c_1");
  geometry(6000, 4000, 400, 400, T | F | X, "cfg5 6000x4000 400x400 c_1");
  geometry(3000, 2000, 300, 250, T | F | X, "cfg1 3000x2000 300x250 c_1");
  g_required = false;
  geometry(1200, 800, 400, 400, T | F | X, "1200x800 400x400 c_1");
  geometry(300, 200, 150, 100, T | S, "300x200 -> 150");
  geometry(900, 600, 250, 300, FI_OP_RESIZE | F | X, "resize 900x600 250x300");
  geometry(120, 90, 300, 0, T, "enlarge 120x90 -> 300");
  geometry(1000, 600, 0, 300, T | S, "h_300 on 1000x600 (factor 2)");
  geometry(4000, 3000, 0, 300, T | S, "h_300 on 4000x3000");
  geometry(1600, 1200, 400, 400, T | F | X, "1600x1200 400x400 c_1");
  geometry(6000, 400, 60, 0, T | S, "factor 0.01 no sample");
  // horizontal-first (tests/test_gpu_parity.py HV_CASES): k_rs_hv tables required
  const uint32_t R = FI_OP_RESIZE;
  g_required = true;
  geometry(1000, 702, 640, 0, R | S, "hv 1000x702 -> 640");
  geometry(1500, 1000, 500, 0, R | S, "hv 1500x1000 -> 500 (1/3)");
  geometry(2000, 1497, 500, 0, R | S, "hv 2000x1497 -> 500 (1/4)");
  geometry(2500, 1497, 500, 0, R | S, "hv 2500x1497 -> 500 (1/5)");
  geometry(901, 600, 250, 300, R | F | X, "hv fill 901x600 250x300");
  geometry(125, 91, 300, 0, T, "hv enlarge 125x91 -> 300");
  geometry(4000, 702, 2600, 0, R | S, "hv 4000x702 -> 2600");
  g_required = false;
  geometry(3000, 2001, 450, 0, R | S, "hv 3000x2001 -> 450 (0.15: two-pass)");
  check_pillow(500, 281, 100, 100, "smartcrop 500x281");
  check_pillow(400, 400, 100, 100, "smartcrop 400x400");
  check_pillow(512, 512, 100, 100, "smartcrop 512x512");
  check_pillow(1000, 750, 100, 100, "smartcrop 1000x750 (reduce)");
  printf("%s (%d failures)\n", g_fail ? "FAILED" : "OK", g_fail);
  return g_fail ? 1 : 0;
}
