// k_rs_vr's two-limb weight quantisation, proved on the host.
//
// For every geometry below, the vertical (VrV) and horizontal (MfmaH::frag2)
// tables of k_rs_vr are rebuilt from their fragment bytes and checked against
// vr_quant / quant_axis: two signed-byte limbs W = lo + 256 hi, every output
// row summing to exactly 2^shift (so the kernel's constant MFMA bias
// 128 * 2^shift turns sum W (p - 128) into sum W p), the horizontal bias
// 32896 * wsum2 of the Q16 hi / lo byte split.  Then the worst case over ALL
// 8-bit inputs of |kernel - ImageMagick| is bounded, output by output:
//
//   vertical   v = 257 sum_j W_j p_j / 2^s  vs  IM's 257 sum_j wd_j p_j (f64):
//              E_V = 65535 sum_j |W_j 2^-s - wd_j| + eps_f32 (the kernel's
//              float(tot) and fmaf(tot, 257 2^-s, 0.5)); both sides round to
//              a Q16 integer (ClampToQuantum): |dq| <= E_V + 1
//   horizontal h = sum_k W2_k q_k / 2^s2  vs  sum_k wd_k q_IM_k:
//              |dh| <= A1 (E_V + 1) + 65535 sum_k |W2_k 2^-s2 - wd_k| + eps_f32,
//              A1 = sum_k |W2_k| 2^-s2; the Q16 results differ by <= |dh| + 1
//   8 bit      ScaleQuantumToChar maps Q16 values less than 257 apart to bytes
//              at most 1 apart: the bound in 8-bit LSB is (|dh| + 1) / 257,
//              asserted < 1 for every table (and < 1 after -colorspace Gray's
//              Rec709 sum, whose coefficients sum to 1, plus its rounding).
//
// wd_j are the f64 weights of the host's ImageMagick restatement (fi_plan.cpp
// build_axis: resize.c's filter, support and density normalisation, the
// ThumbnailImage sample step merged) -- IM's own f64 accumulation error
// (~1e-12 of a Q16 unit) is covered by a 1e-6 margin.
// Built and run by tests/test_native_cpu.py (host only).
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <map>
#include <random>
#include <vector>

#include "../../flyimg_amd/csrc/fi_plan.h"

using namespace fi;

static int g_fail = 0;
#define CHECK(c, ...)                                \
  do {                                               \
    if (!(c)) {                                      \
      if (g_fail < 20) {                             \
        printf("FAIL %s:%d ", __FILE__, __LINE__);   \
        printf(__VA_ARGS__);                         \
        printf("\n");                                \
      }                                              \
      g_fail++;                                      \
    }                                                \
  } while (0)

static int64_t limb2(const std::vector<int32_t> &f, size_t base, int l, int j) {
  const uint8_t *b = reinterpret_cast<const uint8_t *>(&f[base]);
  return (int64_t)(int8_t)b[l * 16 + j] + 256 * (int64_t)(int8_t)b[256 * 4 + l * 16 + j];
}

static double g_worst = 0;  // over every table checked
static int g_tables = 0;
static long g_cmp_taps = 0;  // weights compared with the oracle's
static int g_cmp_tables = 0;
extern "C" int or_im_axis_taps(int W, int H, int ow, int oh, int thumbnail, int matte, int axis, int o, int *start,
                               double *w, int cap);

// returns false when the geometry does not take k_rs_vr
static bool check(int W, int H, int tw, int th, uint32_t flags, const char *name, bool verbose) {
  fi_image im{};
  im.src_w = W;
  im.src_h = H;
  im.src_stride = W * 3;
  im.src_channels = 3;
  im.target_w = tw;
  im.target_h = th;
  im.flags = flags;
  ImPlan P;
  if (plan_im(im, &P) != FI_OK || !P.resize || P.hfirst) return false;
  AxisTable v, h;
  build_axis(P.filter, P.yf, P.sh, P.th, P.ey0, P.ey0 + P.eh, P.sample, P.H, &v);
  build_axis(P.filter, P.xf, P.sw, P.tw, P.ex0, P.ex0 + P.ew, P.sample, P.W, &h);
  // the f64 weights bounded below ARE the oracle's: every output's taps (first
  // source index, count, each weight bit for bit) equal or_im_axis_taps, the
  // oracle's resample on the same geometry
  {
    const int thumb = (flags & FI_OP_THUMBNAIL) ? 1 : 0;
    std::vector<double> ow(8192);
    for (int axis = 0; axis < 2; axis++) {
      const AxisTable &t = axis ? v : h;
      const int o0 = axis ? P.ey0 : P.ex0, o1 = o0 + (axis ? P.eh : P.ew);
      for (int o = o0; o < o1; o++) {
        const size_t k = (size_t)(o - o0);
        int s = -1;
        const int n = or_im_axis_taps(W, H, P.tw, P.th, thumb, 0, axis, o, &s, ow.data(), (int)ow.size());
        CHECK(n == t.count[k] && s == t.start[k], "%s: axis %d out %d: oracle %d taps at %d, planner %d at %d", name,
              axis, o, n, s, t.count[k], t.start[k]);
        if (n != t.count[k]) continue;
        int same = 0;
        for (int j = 0; j < n; j++) same += memcmp(&ow[j], &t.wd[t.woff[k] + j], sizeof(double)) == 0;
        CHECK(same == n, "%s: axis %d out %d: %d of %d weights differ from the oracle's", name, axis, o, n - same, n);
        g_cmp_taps += n;
      }
    }
    g_cmp_tables++;
  }
  VrV m;
  MfmaH mh;
  if (!build_vr_v(v, &m) || !build_mfma_h(h, &mh) || mh.shift2 == 0) return false;
  const int ny = (int)v.start.size(), nx = (int)h.start.size(), nl = (int)m.rows.size();
  // ---- vertical: fragments -> W(y, list row) ----
  std::vector<int32_t> wq;
  const int s = vr_quant(v, &wq);
  CHECK(s == m.shift && s >= kVrMinShift && s <= kVrMaxShift, "%s: shift %d / %d", name, s, m.shift);
  std::map<std::pair<int, int>, int64_t> Wv;
  for (int b = 0; b < m.nblk; b++) {
    const int K0 = m.bmeta[4 * b], ks = m.bmeta[4 * b + 1];
    CHECK(ks >= 1 && ks <= 2 && K0 % 16 == 0, "%s: block %d window", name, b);
    for (int t = 0; t < 2; t++)
      for (int l = 0; l < 64; l++)
        for (int j = 0; j < 16; j++) {
          const int64_t w = limb2(m.frag, (size_t)(b * 2 + t) * 2 * 256, l, j);
          if (w == 0) continue;
          const int y = 16 * b + (l & 15), k = K0 + 64 * t + mfma_i8_k(l, j);
          CHECK(t < ks && y < ny && k < nl, "%s: vertical weight outside block %d", name, b);
          Wv[{y, k}] += w;
        }
  }
  std::vector<double> EV(ny);
  std::mt19937 rng(1234 + W + 7 * H);
  for (int y = 0; y < ny; y++) {
    int64_t sum = 0, exact = 0, biased = 0;
    double dev = 0, aw = 0;
    for (int j = 0; j < v.count[y]; j++) {
      const int row = v.start[y] + j;
      const int32_t q = wq[v.woff[y] + j];
      const auto it = std::lower_bound(m.rows.begin(), m.rows.end(), row);
      const int li = (it != m.rows.end() && *it == row) ? (int)(it - m.rows.begin()) : -1;
      const int64_t got = li >= 0 && Wv.count({y, li}) ? Wv[{y, li}] : 0;
      CHECK(got == q, "%s: vertical y=%d row %d: fragment %lld vs vr_quant %d", name, y, row, (long long)got, q);
      CHECK(q >= -32896 && q <= 32639, "%s: vertical weight %d beyond two limbs", name, q);
      sum += q;
      const int p = (int)(rng() & 255);
      exact += (int64_t)q * p;
      biased += (int64_t)q * (p - 128);
      dev += fabs(ldexp((double)q, -s) - v.wd[v.woff[y] + j]);
      aw += fabs((double)q);
    }
    CHECK(sum == ((int64_t)1 << s), "%s: vertical row %d sums to %lld, not 2^%d", name, y, (long long)sum, s);
    CHECK(biased + ((int64_t)128 << s) == exact, "%s: vertical bias algebra y=%d", name, y);
    CHECK(255.0 * aw < 2147483647.0, "%s: vertical int32 range y=%d", name, y);
    // float(tot) and fmaf(tot, 257 2^-s, 0.5): |tot| <= 255 sum |W|
    const double eps = ldexp(1.0, -23) * 65535.0 * ldexp(aw, -s) + ldexp(1.0, -24);
    EV[y] = 65535.0 * dev + eps;
  }
  // ---- horizontal two-limb fragments per strip ----
  std::vector<int32_t> wq2;
  const int s2 = vr_quant(h, &wq2);
  CHECK(s2 == mh.shift2, "%s: horizontal shift %d / %d", name, s2, mh.shift2);
  std::vector<double> EH(nx, -1), A1(nx, 0);
  for (const MfmaStrip &S : mh.strips) {
    std::vector<int> colpx(S.pitch, -1);
    for (int k = 0; k < S.lut_n; k++) {
      const int ci = mh.lut[S.lut + k];
      if (ci >= 0 && ci < S.pitch) colpx[ci] = S.lut_px0 + k;
    }
    for (int ob = 0; ob < S.nocb; ob++) {
      const int w0 = mh.s0[S.s0 + 2 * ob];
      std::map<std::pair<int, int>, int64_t> Wh;  // (x, source px)
      for (int t = 0; t < S.ks; t++)
        for (int l = 0; l < 64; l++)
          for (int j = 0; j < 16; j++) {
            const int64_t w = limb2(mh.frag2, S.frag2 + (size_t)(ob * S.ks + t) * 2 * 256, l, j);
            if (w == 0) continue;
            const int x = S.x0 + 16 * ob + (l & 15), c = w0 + 64 * t + mfma_i8_k(l, j);
            CHECK(x < S.x1 && c < S.ncols && colpx[c] >= 0, "%s: horizontal weight off the strip", name);
            if (c < S.ncols && colpx[c] >= 0) Wh[{x, colpx[c]}] += w;
          }
      for (int n = 0; n < 16; n++) {
        const int x = S.x0 + 16 * ob + n;
        if (x >= S.x1) continue;
        int64_t sum = 0;
        double dev = 0, aw = 0;
        for (int j = 0; j < h.count[x]; j++) {
          const int px = h.start[x] + j;
          const int32_t q = wq2[h.woff[x] + j];
          const int64_t got = Wh.count({x, px}) ? Wh[{x, px}] : 0;
          CHECK(got == q, "%s: horizontal x=%d px %d: fragment %lld vs vr_quant %d", name, x, px, (long long)got, q);
          sum += q;
          dev += fabs(ldexp((double)q, -s2) - h.wd[h.woff[x] + j]);
          aw += fabs((double)q);
        }
        CHECK(sum == mh.wsum2[x], "%s: horizontal weight sum x=%d", name, x);
        CHECK(128.0 * aw < 2147483647.0, "%s: horizontal limb sums beyond int32 x=%d", name, x);
        A1[x] = ldexp(aw, -s2);
        // 256 float(sum W hi') + float(sum W lo') + float(32896 wsum2), fmaf(., 2^-s2, 0.5)
        const double eps = 6.0 * ldexp(1.0, -24) * 65664.0 * A1[x] + ldexp(1.0, -24) * 65536.0;
        EH[x] = 65535.0 * dev + eps;
      }
    }
  }
  double worst = 0;
  for (int x = 0; x < nx; x++) CHECK(EH[x] >= 0, "%s: output px %d in no strip", name, x);
  const double evmax = *std::max_element(EV.begin(), EV.end());
  for (int x = 0; x < nx; x++) {
    const double dh = A1[x] * (evmax + 1.0) + EH[x] + 1e-6;
    // RGB: Q16 results differ by <= dh + 1; Gray: + Rec709 sum (coefficients sum to 1) + its rounding
    worst = std::max(worst, (dh + 2.0) / 257.0);
  }
  CHECK(worst < 1.0, "%s: bound %.4f LSB", name, worst);
  g_worst = std::max(g_worst, worst);
  g_tables++;
  if (verbose)
    printf("  %s: shifts %d / %d, E_V %.2f Q16, bound %.4f LSB (8-bit)\n", name, s, s2, evmax, worst);
  return true;
}

int main() {
  const uint32_t T = FI_OP_THUMBNAIL, F = FI_GEOM_FILL, X = FI_OP_EXTENT, S = FI_GEOM_SHRINK_ONLY, R = FI_OP_RESIZE;
  // BASELINE.json configs (cfg4's ops on its size classes below)
  CHECK(check(3000, 2000, 300, 250, T | F | X, "cfg1 3000x2000 w_300,h_250,c_1", true), "cfg1 not on k_rs_vr");
  CHECK(check(1920, 1080, 500, 0, T | S, "cfg2 1920x1080 w_500", true), "cfg2 not on k_rs_vr");
  CHECK(check(3840, 2160, 512, 512, T | F | X, "cfg3 3840x2160 w_512,h_512,c_1", true), "cfg3 not on k_rs_vr");
  CHECK(check(6000, 4000, 400, 400, T | F | X, "cfg5 6000x4000 w_400,h_400,c_1", true), "cfg5 not on k_rs_vr");
  // 200 random geometries: cfg4's size law (0.5-24 MP, six aspects) and ops,
  // plus -resize and enlargements
  std::mt19937 rng(20250112);
  const double asp[6] = {4.0 / 3, 1.5, 16.0 / 9, 1.0, 2.0 / 3, 9.0 / 16};
  struct Op {
    int tw, th;
    uint32_t f;
  } ops[8] = {{300, 250, T | F | X}, {500, 0, T | S}, {512, 512, T | F | X}, {0, 300, T | S},
              {400, 400, T | F | X}, {640, 0, R | S}, {250, 300, R | F | X}, {900, 0, T}};
  int taken = 0;
  for (int i = 0; i < 200; i++) {
    const double mp = exp(log(0.5) + (log(24.0) - log(0.5)) * (rng() / 4294967296.0));
    const double a = asp[rng() % 6];
    const int W = std::max(16, (int)lrint(sqrt(mp * 1e6 * a))), H = std::max(16, (int)lrint(W / a));
    const Op &o = ops[rng() % 8];
    char name[96];
    snprintf(name, sizeof name, "random %d: %dx%d -> %dx%d flags %x", i, W, H, o.tw, o.th, o.f);
    taken += check(W, H, o.tw, o.th, o.f, name, false) ? 1 : 0;
  }
  printf("  %d of 200 random geometries on k_rs_vr\n", taken);
  CHECK(taken >= 100, "only %d random geometries took k_rs_vr", taken);
  printf("planner tap tables == oracle's: %ld weights of %d geometries compared bit for bit\n", g_cmp_taps,
         g_cmp_tables);
  CHECK(g_cmp_tables >= 100 && g_cmp_taps > 0, "too few geometries compared with the oracle");
  printf("worst bound %.4f LSB over %d tables\n", g_worst, g_tables);
  printf("%s (%d failures)\n", g_fail ? "FAILED" : "OK", g_fail);
  return g_fail ? 1 : 0;
}
