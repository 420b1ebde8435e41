// fi_mono.hip -- ImageMagick -monochrome (flyimg emits it
// for mnchr_1 at src/Core/Processor/ImageProcessor.php:90-92), after the
// resample/extent/gray epilogue and before -rotate.
//
// IM 6 SetImageType(BilevelType) on the Q16 gray extent window:
//   already bilevel -> unchanged;
//   NormalizeImage  = ContrastStretchImageChannel(0.15 %, 99.95 %);
//   QuantizeImage(2 colours, GRAY): octree classification (depth 8 for gray
//                     images), rapid reduction + Reduce/PruneChild passes,
//                     DefineImageColormap;
//   Riemersma dither along the Hilbert curve (16-entry exponentially weighted
//                     error queue, 6-bit closest-colour cache);
//   monochrome colormap threshold at QuantumRange / 2, SyncImage.
// The arithmetic follows oracle/fi_oracle.c or_im_monochrome bit for bit
// (same deterministic reformulation of IM's raster-order sums, documented
// there); tests/test_gpu_parity.py checks the two are identical.
//
// Two kernels per batch:
//   k_mono_stats   one 1024-thread workgroup per image: coarse + fine
//                  histograms for the stretch points (LDS), the stretched
//                  Q16 histogram in four 16384-bin LDS passes feeding the
//                  per-(tree level, 8-bit bin) quantize-error partials (one
//                  thread per pair), then thread 0 builds / reduces the
//                  <= 511-node tree and writes the MonoState.
//   k_mono_dither  one wave per image: the walk itself is sequential (each
//                  pixel's value depends on the previous 16 errors), so the
//                  wave computes 64 curve positions and their stretched
//                  pixels at once (d2xy per lane, one gather), compacts the
//                  ones inside the image, runs the serial error chain on them
//                  (wave-uniform), and scatters the 64 results rotated.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "fi_internal.h"

namespace fi {

constexpr int kMonoThreads = 1024;
constexpr int kMonoQuarter = 16384;  // stretched-histogram bins per LDS pass
constexpr double kMonoQScale = 1.0 / 65535.0;

__device__ __forceinline__ unsigned mono_q2c(unsigned q) { return ((q + 128u) - ((q + 128u) >> 8)) >> 8; }

__device__ __forceinline__ unsigned mono_stretch(unsigned q, int black, int white) {
  if (black == white) return q;
  if ((int)q < black) return 0;
  if ((int)q > white) return 65535;
  const double v = 65535.0 * ((double)((int)q - black)) / ((double)(white - black));  // ScaleMapToQuantum
  if (v <= 0.0) return 0;
  if (v >= 65535.0) return 65535;
  return (unsigned)(v + 0.5);
}

__device__ __forceinline__ double mono_mid(int L, unsigned c) {
  double mid = 65535.0 / 2.0, bisect = (65535.0 + 1.0) / 2.0;
  for (int l = 1; l <= L; l++) {
    bisect *= 0.5;
    mid += ((c >> (8 - l)) & 1) ? bisect : -bisect;
  }
  return mid;
}

__device__ __forceinline__ double mono_term(double count, unsigned q, double mid) {
  const double e = kMonoQScale * ((double)q - mid);
  double d = e * e + e * e;
  d = d + e * e;
  return count * sqrt(d);
}

// heap-indexed binary trie: node k at level floor(log2(k + 1)), children 2k+1 (id 0), 2k+2 (id 7)
constexpr int kMonoNodes = 511;
__device__ __forceinline__ int mono_level(int k) { return 31 - __clz(k + 1); }

struct MonoLds {
  uint32_t hist[kMonoQuarter];   // coarse/fine histograms, then the stretched-histogram quarters
  double part[8][256];           // quantize-error partials per (level, 8-bit bin)
  uint64_t bnu[256], btot[256];  // leaf pixel counts / Q16 sums per 8-bit bin
  uint32_t lo[257];              // first Q16 value of each 8-bit bin
  double qerr[kMonoNodes];
  uint64_t nu[kMonoNodes], tot[kMonoNodes];
  int16_t order[kMonoNodes];
  int8_t color[kMonoNodes];
  uint8_t exist[kMonoNodes];
  int32_t nonbilevel, black, white, cb, cw;
  uint64_t accb, accw;
};

// post-order of the existing nodes (children id 0, id 7, then the node)
__device__ int mono_postorder(MonoLds &S) {
  int n = 0, sp = 0;
  int stk[10];
  int st[10];
  stk[0] = 0;
  st[0] = 0;
  while (sp >= 0) {
    const int k = stk[sp];
    if (st[sp] < 2) {
      const int ch = 2 * k + 1 + st[sp];
      st[sp]++;
      if (ch < kMonoNodes && S.exist[ch]) {
        sp++;
        stk[sp] = ch;
        st[sp] = 0;
      }
    } else {
      S.order[n++] = (int16_t)k;
      sp--;
    }
  }
  return n;
}

// PruneChild(k): k's remaining subtree merged into its parent
__device__ int mono_prune(MonoLds &S, int k) {
  const int parent = k == 0 ? 0 : (k - 1) / 2;
  uint64_t snu = 0, stot = 0;
  int removed = 0;
  for (int l = 0; l <= 8 - mono_level(k); l++) {
    const int first = ((k + 1) << l) - 1;
    for (int j = 0; j < (1 << l); j++) {
      const int m = first + j;
      if (m >= kMonoNodes || !S.exist[m]) continue;
      snu += S.nu[m];
      stot += S.tot[m];
      S.exist[m] = 0;
      removed++;
    }
  }
  S.nu[parent] += snu;
  S.tot[parent] += stot;
  return removed;
}

// the tree part of QuantizeImage, thread 0 only (<= 511 nodes)
__device__ void mono_tree(MonoLds &S, MonoState &st) {
  for (int k = 0; k < kMonoNodes; k++) {
    S.exist[k] = 0;
    S.qerr[k] = 0.0;
    S.nu[k] = S.tot[k] = 0;
    S.color[k] = -1;
  }
  S.exist[0] = 1;
  S.qerr[0] = 1.79769313486231570815e+308;  // the root: larger than any node
  long colors = 0;
  int nodes = 1;
  for (int c = 0; c < 256; c++) {
    if (!S.bnu[c]) continue;
    for (int L = 1; L <= 8; L++) {
      const int k = (1 << L) - 1 + (c >> (8 - L));
      if (!S.exist[k]) {
        S.exist[k] = 1;
        nodes++;
        if (L == 8) colors++;
      }
    }
    const int leaf = 255 + c;
    S.nu[leaf] = S.bnu[c];
    S.tot[leaf] = S.btot[c];
  }
  for (int L = 1; L <= 8; L++)
    for (int c = 0; c < 256; c++)
      if (S.bnu[c]) S.qerr[(1 << L) - 1 + (c >> (8 - L))] += S.part[L - 1][c];
  // ReduceImageColors: rapid reduction threshold = errs[nodes - 3] (ascending)
  const long maxc = 2;
  double next = 0.0, pruning;
  if (colors > maxc && nodes > (int)(110 * (maxc + 1) / 100)) {
    double t0 = -1.0, t1 = -1.0, t2 = -1.0;  // the three largest (with multiplicity)
    for (int k = 0; k < kMonoNodes; k++) {
      if (!S.exist[k]) continue;
      const double e = S.qerr[k];
      if (e >= t0) {
        t2 = t1;
        t1 = t0;
        t0 = e;
      } else if (e >= t1) {
        t2 = t1;
        t1 = e;
      } else if (e > t2) {
        t2 = e;
      }
    }
    next = t2;
  }
  while (colors > maxc) {
    pruning = next;
    next = S.qerr[0] - 1;
    colors = 0;
    const int n = mono_postorder(S);
    for (int i = 0; i < n; i++) {
      const int k = S.order[i];
      if (!S.exist[k]) continue;
      if (S.qerr[k] <= pruning) {
        nodes -= mono_prune(S, k);
      } else {
        if (S.nu[k] > 0) colors++;
        if (S.qerr[k] < next) next = S.qerr[k];
      }
    }
  }
  // DefineImageColormap (post-order)
  const int n = mono_postorder(S);
  int ncol = 0;
  for (int i = 0; i < n; i++) {
    const int k = S.order[i];
    if (S.nu[k] == 0 || ncol >= 8) continue;
    const double total = (double)S.tot[k] * kMonoQScale;
    const double alpha = 1.0 / (double)S.nu[k];
    const double val = alpha * 65535.0 * total;
    st.mean[ncol] = val <= 0.0 ? 0 : (val >= 65535.0 ? 65535 : (uint16_t)(val + 0.5));
    const double cv = (double)st.mean[ncol];
    const double luma = 0.212656 * cv + 0.715158 * cv + 0.072186 * cv;
    st.bil[ncol] = luma < 65535.0 / 2.0 ? 0 : 65535;
    S.color[k] = (int8_t)ncol++;
  }
  st.ncol = ncol;
  // closest-colour search subtree of every 8-bit value
  for (int c = 0; c < 256; c++) {
    int k = 0;
    for (int index = 7; index > 0; index--) {
      const int ch = 2 * k + 1 + ((c >> index) & 1);
      if (!S.exist[ch]) break;
      k = ch;
    }
    const int s = k == 0 ? 0 : (k - 1) / 2, ls = mono_level(s);
    uint32_t mask = 0;
    for (int i = 0; i < n; i++) {
      const int m = S.order[i];
      if (S.color[m] < 0) continue;
      const int lm = mono_level(m);
      if (lm >= ls && ((m + 1) >> (lm - ls)) == s + 1) mask |= 1u << S.color[m];
    }
    st.cand[c] = (uint8_t)mask;
  }
}

__global__ __launch_bounds__(kMonoThreads) void k_mono_stats(const MonoDesc *__restrict__ descs) {
  extern __shared__ __attribute__((aligned(16))) uint8_t lds_raw[];
  MonoLds &S = *reinterpret_cast<MonoLds *>(lds_raw);
  const MonoDesc D = descs[blockIdx.x];
  MonoState &st = *D.st;
  const int tid = threadIdx.x;
  const long n = (long)D.w * D.h;
  // ---- pass 1: coarse histogram (q >> 8) and the bilevel test
  for (int i = tid; i < 768; i += kMonoThreads) S.hist[i] = 0;
  if (tid == 0) S.nonbilevel = 0;
  __syncthreads();
  int nb = 0;
  for (long i = tid; i < n; i += kMonoThreads) {
    const unsigned q = D.g[i];
    nb |= (q != 0 && q != 65535);
    atomicAdd(&S.hist[q >> 8], 1u);
  }
  if (nb) S.nonbilevel = 1;
  __syncthreads();
  if (!S.nonbilevel) {
    if (tid == 0) st.bilevel = 1;
    return;
  }
  // ---- NormalizeImage black / white points: coarse bin, then its fine bins
  if (tid == 0) {
    const double bp = (double)n * 0.0015, wp = (double)n * 0.9995;
    double acc = 0.0;
    int C = 0;
    for (; C < 256; C++) {
      if (acc + (double)S.hist[C] > bp) break;
      acc += (double)S.hist[C];
    }
    S.cb = C;
    S.accb = (uint64_t)acc;
    acc = 0.0;
    C = 255;
    for (; C >= 0; C--) {
      if (acc + (double)S.hist[C] > ((double)n - wp)) break;
      acc += (double)S.hist[C];
    }
    S.cw = C;  // -1: never exceeded above q = 0 (the fine scan below stops at q = 1)
    S.accw = (uint64_t)acc;
  }
  __syncthreads();
  const int cb = S.cb, cw = S.cw;
  for (int i = tid; i < 512; i += kMonoThreads) S.hist[256 + i] = 0;
  __syncthreads();
  for (long i = tid; i < n; i += kMonoThreads) {
    const unsigned q = D.g[i];
    if ((int)(q >> 8) == cb) atomicAdd(&S.hist[256 + (q & 255)], 1u);
    if ((int)(q >> 8) == cw) atomicAdd(&S.hist[512 + (q & 255)], 1u);
  }
  __syncthreads();
  if (tid == 0) {
    const double bp = (double)n * 0.0015, wp = (double)n * 0.9995;
    int black = 65535;
    if (cb < 256) {
      double acc = (double)S.accb;
      for (int k = 0; k < 256; k++) {
        acc += (double)S.hist[256 + k];
        if (acc > bp) {
          black = 256 * cb + k;
          break;
        }
      }
    }
    int white = 0;
    if (cw >= 0) {
      double acc = (double)S.accw;
      for (int k = 255; k >= 0; k--) {
        const int q = 256 * cw + k;
        if (q == 0) break;
        acc += (double)S.hist[512 + k];
        if (acc > ((double)n - wp)) {
          white = q;
          break;
        }
      }
    }
    S.black = black;
    S.white = white;
    st.bilevel = 0;
    st.black = black;
    st.white = white;
  }
  for (int c = tid; c <= 256; c += kMonoThreads) {
    unsigned q = c == 0 ? 0u : (c >= 256 ? 65536u : (unsigned)max(0, 257 * c - 300));
    if (c > 0 && c < 256)
      while (mono_q2c(q) < (unsigned)c) q++;
    S.lo[c] = q;
  }
  __syncthreads();
  const int black = S.black, white = S.white;
  // ---- stretched histogram in four quarters; per (level, bin) partials
  // pairs k = tid, tid + 1024: level L = k / 256 + 1, bin c = k % 256
  double part[2] = {0.0, 0.0};
  uint64_t lnu = 0, ltot = 0;  // leaf stats of the L = 8 pair
  for (int qb = 0; qb < 65536; qb += kMonoQuarter) {
    for (int i = tid; i < kMonoQuarter; i += kMonoThreads) S.hist[i] = 0;
    __syncthreads();
    for (long i = tid; i < n; i += kMonoThreads) {
      const unsigned s = mono_stretch(D.g[i], black, white);
      if (s >= (unsigned)qb && s < (unsigned)(qb + kMonoQuarter)) atomicAdd(&S.hist[s - qb], 1u);
    }
    __syncthreads();
#pragma unroll
    for (int r = 0; r < 2; r++) {
      const int k = tid + r * kMonoThreads, L = k / 256 + 1;
      const unsigned c = (unsigned)(k & 255);
      const unsigned q0 = max(S.lo[c], (unsigned)qb), q1 = min(S.lo[c + 1], (unsigned)(qb + kMonoQuarter));
      if (q0 >= q1) continue;
      const double mid = mono_mid(L, c);
      for (unsigned q = q0; q < q1; q++) {
        const uint32_t h = S.hist[q - qb];
        if (!h) continue;
        part[r] += mono_term((double)h, q, mid);
        if (L == 8) {
          lnu += h;
          ltot += (uint64_t)h * q;
        }
      }
    }
    __syncthreads();
  }
#pragma unroll
  for (int r = 0; r < 2; r++) {
    const int k = tid + r * kMonoThreads;
    S.part[k / 256][k & 255] = part[r];
    if (k / 256 == 7) {
      S.bnu[k & 255] = lnu;
      S.btot[k & 255] = ltot;
    }
  }
  __syncthreads();
  if (tid == 0) mono_tree(S, st);
}

// -------------------------------------------------------------------------
__device__ __forceinline__ void mono_d2xy(int L, long d, int *x_, int *y_) {
  long x = 0, y = 0, t = d;
  for (int l = 0; l < L; l++) {
    const long s = 1L << l;
    const long rx = 1 & (t / 2), ry = 1 & (t ^ rx);
    if (ry == 0) {
      if (rx == 1) {
        x = s - 1 - x;
        y = s - 1 - y;
      }
      const long tmp = x;
      x = y;
      y = tmp;
    }
    x += s * rx;
    y += s * ry;
    t /= 4;
  }
  *x_ = (int)x;
  *y_ = (int)y;
}

__device__ __forceinline__ void mono_store(const MonoDesc &D, int x, int y, uint8_t v) {
  int dx = x, dy = y;
  if (D.rot == 90) {
    dx = D.h - 1 - y;
    dy = x;
  } else if (D.rot == 180) {
    dx = D.w - 1 - x;
    dy = D.h - 1 - y;
  } else if (D.rot == 270) {
    dx = y;
    dy = D.w - 1 - x;
  }
  D.dst[(int64_t)dy * D.dst_stride + dx] = v;
}

__device__ __forceinline__ double mono_readlane(double v, int j) {
  const uint64_t b = __builtin_bit_cast(uint64_t, v);
  const uint32_t lo = __builtin_amdgcn_readlane((uint32_t)b, j), hi = __builtin_amdgcn_readlane((uint32_t)(b >> 32), j);
  return __builtin_bit_cast(double, ((uint64_t)hi << 32) | lo);
}

// one wave per image; wts = the 16 error-queue weights (host-computed, as the oracle)
__global__ __launch_bounds__(64) void k_mono_dither(const MonoDesc *__restrict__ descs, const double *__restrict__ wts) {
  __shared__ int32_t cache[64];
  __shared__ int32_t cx[64], cy[64];
  __shared__ uint16_t cv[64];
  const MonoDesc D = descs[blockIdx.x];
  const MonoState &st = *D.st;
  const int lane = threadIdx.x;
  const long n = (long)D.w * D.h;
  if (st.bilevel) {
    for (long i = lane; i < n; i += 64) {
      const int y = (int)(i / D.w), x = (int)(i - (long)y * D.w);
      mono_store(D, x, y, D.g[i] ? 255 : 0);
    }
    return;
  }
  const int black = st.black, white = st.white, ncol = st.ncol;
  double mean[2] = {(double)st.mean[0], ncol > 1 ? (double)st.mean[1] : 0.0};
  const uint32_t bil = (st.bil[0] ? 1u : 0u) | (ncol > 1 && st.bil[1] ? 2u : 0u);
  double w[16], err[16];
#pragma unroll
  for (int i = 0; i < 16; i++) {
    w[i] = wts[i];
    err[i] = 0.0;
  }
  cache[lane] = -1;
  __syncthreads();
  // curve level (DitherImage depth - 1)
  int L;
  {
    long i = D.w > D.h ? D.w : D.h, m = i;
    int depth;
    for (depth = 1; i != 0; depth++) i >>= 1;
    if ((1L << depth) < m) depth++;
    L = depth - 1;
  }
  const long steps = 1L << (2 * L);
  for (long base = 0; base < steps; base += 64) {
    int x, y;
    mono_d2xy(L, base + lane, &x, &y);
    const bool inside = base + lane < steps && x < D.w && y < D.h;
    const uint64_t mask = __ballot(inside);
    if (mask == 0) continue;
    const int pos = __builtin_amdgcn_mbcnt_hi((uint32_t)(mask >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)mask, 0));
    if (inside) {
      cx[pos] = x;
      cy[pos] = y;
      cv[pos] = (uint16_t)mono_stretch(D.g[(long)y * D.w + x], black, white);
    }
    __syncthreads();
    const int cnt = __popcll(mask);
    const double mine = lane < cnt ? (double)cv[lane] : 0.0;
    uint32_t res = 0;
    for (int j = 0; j < cnt; j++) {
      double pv = mono_readlane(mine, j);
#pragma unroll
      for (int i = 0; i < 16; i++) pv += w[i] * err[i];
      pv = pv < 0.0 ? 0.0 : (pv >= 65535.0 ? 65535.0 : (double)(uint16_t)(pv + 0.5));
      const unsigned c8 = mono_q2c((unsigned)pv);
      const int key = (int)(c8 >> 2);
      int idx = cache[key];
      if (idx < 0) {
        double best = 4.0 * (65535.0 + 1.0) * (65535.0 + 1.0) + 1.0;
        int pick = 0;
        const uint32_t cm = st.cand[c8];
        for (int i = 0; i < ncol && i < 2; i++) {
          if (!((cm >> i) & 1)) continue;
          const double px = 1.0 * mean[i] - 1.0 * pv;
          double d = px * px;
          if (d <= best) {
            d += px * px;
            if (d <= best) {
              d += px * px;
              if (d <= best && d < best) {
                best = d;
                pick = i;
              }
            }
          }
        }
        idx = pick;
        cache[key] = pick;  // every lane writes the same value
      }
      if (lane == j) res = (bil >> idx) & 1u;
#pragma unroll
      for (int i = 0; i < 15; i++) err[i] = err[i + 1];
      err[15] = pv - mean[idx];
    }
    if (lane < cnt) mono_store(D, cx[lane], cy[lane], res ? 255 : 0);
    __syncthreads();
  }
}

size_t mono_lds_bytes() { return sizeof(MonoLds); }

int launch_mono(hipStream_t s, const MonoDesc *descs, int n, const double *wts) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(k_mono_stats, dim3(n), dim3(kMonoThreads), sizeof(MonoLds), s, descs);
  hipLaunchKernelGGL(k_mono_dither, dim3(n), dim3(64), 0, s, descs, wts);
  return 0;
}

}  // namespace fi
