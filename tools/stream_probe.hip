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
