// stream_probe: HBM read rate of the fused resample kernel's access pattern
// (column strips of a pitched image batch, rows streamed top to bottom),
// without any arithmetic.  Answers "how many bytes in flight per CU does
// this pattern need" before the kernel is restructured.
//
//   hipcc --offload-arch=gfx950 -O3 -o /tmp/stream_probe tools/stream_probe.hip
//   ./stream_probe [images]
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#define CK(x)                                                                  \
  do {                                                                         \
    hipError_t e_ = (x);                                                       \
    if (e_ != hipSuccess) {                                                    \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                 \
    }                                                                          \
  } while (0)

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
typedef __attribute__((address_space(1))) const u32x4 g_u32x4;
typedef __attribute__((address_space(1))) const u32x2 g_u32x2;

template <int LW>
struct Vec;
typedef __attribute__((address_space(1))) const uint32_t g_u32;
template <>
struct Vec<4> {
  typedef uint32_t T;
  static __device__ T ld(const uint8_t *p) { return *(g_u32 *)p; }
  static __device__ uint32_t red(T v) { return v; }
};
template <>
struct Vec<8> {
  typedef u32x2 T;
  static __device__ T ld(const uint8_t *p) { return *(g_u32x2 *)p; }
  static __device__ uint32_t red(T v) { return v.x ^ v.y; }
};
template <>
struct Vec<16> {
  typedef u32x4 T;
  static __device__ T ld(const uint8_t *p) { return *(g_u32x4 *)p; }
  static __device__ uint32_t red(T v) { return v.x ^ v.y ^ v.z ^ v.w; }
};

// one WG = one strip (blockDim.x * LW bytes) of one image, all H rows.
template <int LW, int D>
__global__ void k_strips(const uint8_t *base, int64_t img_bytes, int64_t stride, int W3, int H, int nstrips,
                         uint32_t *sink) {
  extern __shared__ uint32_t lds_pad[];
  const int img = blockIdx.x / nstrips, s = blockIdx.x % nstrips;
  const int b0 = s * blockDim.x * LW;
  int off = b0 + threadIdx.x * LW;
  if (off + LW > W3) off = b0;
  const uint8_t *p = base + img * img_bytes + off;
  typedef typename Vec<LW>::T V;
  V pf[D];
#pragma unroll
  for (int d = 0; d < D; d++) {
    pf[d] = Vec<LW>::ld(p + (int64_t)d * stride);
    __builtin_amdgcn_sched_barrier(0);
  }
  uint32_t acc = 0;
  for (int r = 0; r < H; r += D) {
#pragma unroll
    for (int d = 0; d < D; d++) {
      acc += Vec<LW>::red(pf[d]);
      int rr = r + d + D;
      rr = rr < H ? rr : H - 1;
      pf[d] = Vec<LW>::ld(p + (int64_t)rr * stride);
    }
  }
  if (acc == 0x12345678u) sink[0] = acc + lds_pad[0];
}

// the k_rs_mfma pattern: one WG (8 waves) = (image, 1 KB strip, block of 16
// output rows) reading a window of WIN rows starting at 61 * block; each wave
// loads its column chunks of CW bytes (CW / 16 lanes per row, 64 * 16 / CW
// rows per instruction), 2 chunks... all as k_rs_mfma (no compute)
template <int CW>
__global__ __launch_bounds__(512) void k_windows(const uint8_t *base, int64_t img_bytes, int64_t stride,
                                                 int nstrips, int nblocks, int win, uint32_t *sink) {
  extern __shared__ uint32_t lds_w[];
  const int t = blockIdx.x;
  const int img = t / (nstrips * nblocks), rem = t % (nstrips * nblocks);
  const int strip = rem / nblocks, blk = rem % nblocks;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  constexpr int LPR = CW / 16;          // lanes per row
  constexpr int RPI = 64 / LPR;         // rows per instruction
  const uint8_t *p = base + img * img_bytes + (int64_t)(61 * blk) * stride + strip * 1024;
  uint32_t acc = 0;
  for (int ch = wave; ch < 1024 / CW; ch += 8) {
    u32x4 v[128 / RPI];
#pragma unroll
    for (int i = 0; i < 128 / RPI; i++) {
      int row = RPI * i + lane / LPR;
      row = row < win ? row : 0;
      v[i] = *(g_u32x4 *)(p + (int64_t)row * stride + ch * CW + 16 * (lane % LPR));
    }
#pragma unroll
    for (int i = 0; i < 128 / RPI; i++) acc += v[i].x ^ v[i].w;
  }
  if (acc == 0x12345678u) sink[0] = acc + lds_w[0];
}

// k_rs_mfma's loop: one WG per (image, 1 KB strip) walking down its blocks
// (window WIN rows at 61 * block), a barrier per block, each wave 2 chunks
// of 64 B; PREF: the next block's first chunk is loaded before the barrier.
template <int PREF, int BAR>
__global__ __launch_bounds__(512) void k_loop(const uint8_t *base, int64_t img_bytes, int64_t stride, int nstrips,
                                              int nblocks, int win, uint32_t *sink) {
  extern __shared__ uint32_t lds_w[];
  const int img = blockIdx.x / nstrips, strip = blockIdx.x % nstrips;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const uint8_t *p0 = base + img * img_bytes + strip * 1024;
  uint32_t acc = 0;
  u32x4 v[8];
  auto issue = [&](int blk, int ch) {
    const uint8_t *p = p0 + (int64_t)(61 * blk) * stride + ch * 64 + 16 * (lane & 3);
#pragma unroll
    for (int i = 0; i < 8; i++) {
      int row = 16 * i + (lane >> 2);
      row = row < win ? row : 0;
      v[i] = *(g_u32x4 *)(p + (int64_t)row * stride);
    }
  };
  if (PREF) issue(0, wave);
  for (int blk = 0; blk < nblocks; blk++) {
    for (int u = 0; u < 2; u++) {
      const int ch = wave + 8 * u;
      if (!PREF || u == 1) issue(blk, ch);
#pragma unroll
      for (int i = 0; i < 8; i++) acc += v[i].x ^ v[i].w;
      if (PREF && u == 1 && blk + 1 < nblocks) issue(blk + 1, wave);
    }
    if (BAR) __syncthreads();
  }
  if (acc == 0x12345678u) sink[0] = acc + lds_w[0];
}

// reference: each WG reads a contiguous chunk (memcpy-like read)
__global__ void k_linear(const u32x4 *base, int64_t n16, uint32_t *sink) {
  uint32_t acc = 0;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n16; i += (int64_t)gridDim.x * blockDim.x) {
    u32x4 v = ((g_u32x4 *)base)[i];
    acc += v.x ^ v.y ^ v.z ^ v.w;
  }
  if (acc == 0x12345678u) sink[0] = acc;
}

template <typename F>
static float timeit(F f, int reps) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  f();
  CK(hipDeviceSynchronize());
  CK(hipEventRecord(a));
  for (int i = 0; i < reps; i++) f();
  CK(hipEventRecord(b));
  CK(hipEventSynchronize(b));
  float ms;
  CK(hipEventElapsedTime(&ms, a, b));
  return ms / reps;
}

int main(int argc, char **argv) {
  const int nimg = argc > 1 ? atoi(argv[1]) : 1024;
  const int W = 1920, H = 1080, W3 = W * 3;
  const int64_t stride = W3, img_bytes = stride * H;
  const int64_t total = img_bytes * nimg;
  uint8_t *buf;
  uint32_t *sink;
  CK(hipMalloc(&buf, total));
  CK(hipMalloc(&sink, 64));
  CK(hipMemset(buf, 1, total));
  const double gb = total / 1e9;
  {
    float ms = timeit([&] { hipLaunchKernelGGL(k_linear, dim3(256 * 32), dim3(256), 0, 0, (const u32x4 *)buf, total / 16, sink); }, 5);
    printf("linear read                      %8.3f ms %8.1f GB/s\n", ms, gb / ms * 1e3);
  }
  // lds_kb limits WGs per CU (the fused kernel holds ~48 KB -> 2-3 WGs/CU)
  int lds_opts[] = {0, 48, 80};
#define RUN(LW, D, TH)                                                                                   \
  for (int li = 0; li < 3; li++) {                                                                       \
    const int sw = (TH) * (LW);                                                                          \
    const int ns = (W3 + sw - 1) / sw;                                                                   \
    const size_t lds = (size_t)lds_opts[li] * 1024;                                                      \
    float ms = timeit([&] { hipLaunchKernelGGL((k_strips<LW, D>), dim3(nimg * ns), dim3(TH), lds, 0, buf, img_bytes, \
                                               stride, W3, H, ns, sink); }, 5);                           \
    printf("strips LW=%2d D=%2d threads=%4d lds=%2dKB %8.3f ms %8.1f GB/s\n", LW, D, TH, lds_opts[li], ms, \
           gb / ms * 1e3);                                                                               \
  }
  {
    const int nstrips = 5, nblocks = 17, win = 82;  // 5 KB of each row, rows 0 .. 61*16+82
    const double wgb = (double)nimg * nstrips * nblocks * win * 1024 / 1e9;
    {
      const double lgb = (double)nimg * 5 * 17 * win * 1024 / 1e9;  // 5 strips x 17 blocks; rows < 61*16+82 < 1080
      float a = timeit([&] { hipLaunchKernelGGL((k_loop<0, 1>), dim3(nimg * 5), dim3(512), 78 * 1024, 0, buf, img_bytes, stride, 5, 17, win, sink); }, 5);
      float b = timeit([&] { hipLaunchKernelGGL((k_loop<1, 1>), dim3(nimg * 5), dim3(512), 78 * 1024, 0, buf, img_bytes, stride, 5, 17, win, sink); }, 5);
      float c = timeit([&] { hipLaunchKernelGGL((k_loop<1, 0>), dim3(nimg * 5), dim3(512), 78 * 1024, 0, buf, img_bytes, stride, 5, 17, win, sink); }, 5);
      float d = timeit([&] { hipLaunchKernelGGL((k_loop<1, 1>), dim3(nimg * 5), dim3(512), 0, 0, buf, img_bytes, stride, 5, 17, win, sink); }, 5);
      printf("loop per strip (%.2f GB req): no-pref+bar %.3f ms | pref+bar %.3f ms | pref no-bar %.3f ms | pref+bar lds0 %.3f ms\n",
             lgb, a, b, c, d);
    }
    for (int kb : {40, 60, 78}) {
      float m = timeit([&] { hipLaunchKernelGGL(k_windows<64>, dim3(nimg * nstrips * nblocks), dim3(512), kb * 1024, 0, buf,
                                                img_bytes, stride, nstrips, nblocks, win, sink); }, 5);
      printf("windows 64 B/row with %d KB LDS: %.3f ms %.0f GB/s\n", kb, m, wgb / m * 1e3);
    }
    float ms64 = timeit([&] { hipLaunchKernelGGL(k_windows<64>, dim3(nimg * nstrips * nblocks), dim3(512), 0, 0, buf,
                                                 img_bytes, stride, nstrips, nblocks, win, sink); }, 5);
    float ms128 = timeit([&] { hipLaunchKernelGGL(k_windows<128>, dim3(nimg * nstrips * nblocks), dim3(512), 0, 0, buf,
                                                  img_bytes, stride, nstrips, nblocks, win, sink); }, 5);
    float ms256 = timeit([&] { hipLaunchKernelGGL(k_windows<256>, dim3(nimg * nstrips * nblocks), dim3(512), 0, 0, buf,
                                                  img_bytes, stride, nstrips, nblocks, win, sink); }, 5);
    printf("windows (k_rs_mfma pattern, %.2f GB requested): 64 B/row %.3f ms %.0f GB/s | 128 B/row %.3f ms %.0f GB/s | 256 B/row %.3f ms %.0f GB/s\n",
           wgb, ms64, wgb / ms64 * 1e3, ms128, wgb / ms128 * 1e3, ms256, wgb / ms256 * 1e3);
  }
  RUN(8, 8, 256);
  RUN(8, 16, 256);
  RUN(8, 32, 256);
  RUN(16, 8, 256);
  RUN(16, 16, 256);
  RUN(8, 8, 512);
  RUN(16, 8, 128);
  RUN(4, 16, 512);
  CK(hipFree(buf));
  return 0;
}
