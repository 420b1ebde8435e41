// ring_probe: the ceiling of k_rs_vr's row stream (fi_vr.hip) without any
// arithmetic, barriers or phase waits: loader waves stream the cfg2 batch
// (1024 images of 1920x1080 RGB, rows 5760 B) by LDS-DMA into a ring, strip by
// strip (512-B column strips, rows in pairs: lanes 0-31 row r, lanes 32-63 row
// r + 1), with a sliding window of D DMAs in flight per wave.  Tiles are handed
// out as the kernel does (tile t = image t / S, strip t % S, workgroup t % G),
// so the workgroups on one image's strips run side by side.
//
//   hipcc --offload-arch=gfx950 -O3 -o /tmp/ring_probe tools/ring_probe.hip && /tmp/ring_probe
//
// Walks: 0 strips (the kernel's), 1 whole rows (1-KB pieces of a row-major
// sweep of each image: the contiguous ceiling of the same bytes).
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

typedef __attribute__((address_space(3))) uint8_t l_u8;

template <int NT>
__device__ __forceinline__ void dma16(uint32_t m0, const uint8_t *sbase, uint32_t voff) {
  unsigned keep;
  const uint64_t sb = (uint64_t)(uintptr_t)sbase;
  sbase = reinterpret_cast<const uint8_t *>(
      (uintptr_t)(((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(sb >> 32)) << 32) |
                  (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)sb)));
  m0 = (uint32_t)__builtin_amdgcn_readfirstlane((int)m0);
  if (NT)
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, %2 nt\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "v"(voff), "s"(sbase), "s"(m0) : "memory");
  else
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, %2\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "v"(voff), "s"(sbase), "s"(m0) : "memory");
}
template <int D>
__device__ __forceinline__ void wait_d() {
  if (D == 8) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
  if (D == 16) asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
  if (D == 32) asm volatile("s_waitcnt vmcnt(32)" ::: "memory");
  if (D == 48) asm volatile("s_waitcnt vmcnt(48)" ::: "memory");
}

template <int D, int NT>
__global__ __launch_bounds__(1024, 1) void k_ring(const uint8_t *buf, int nimg, int rowb, int H, int S, int walk,
                                                  int nw, uint32_t *sink) {
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  const int tid = threadIdx.x, lane = tid & 63, w = __builtin_amdgcn_readfirstlane(tid >> 6);
  if (w >= nw) return;
  const int G = gridDim.x, g = blockIdx.x, h = lane >> 5;
  const uint32_t l0 = (uint32_t)(uintptr_t)(const l_u8 *)lds;
  const int64_t imgb = (int64_t)rowb * H;
  int slot = w;
  if (walk == 0) {
    const int ntiles = nimg * S;
    for (int t = g; t < ntiles; t += G) {
      const int img = t / S, s = t - img * S;
      const int nb = min(512, rowb - 512 * s);
      const uint8_t *base = buf + img * imgb + 512 * s;
      uint32_t lc = (uint32_t)(lane & 31);
      if (16 * (int)lc >= nb) lc = 0;
      const uint32_t voff = (h ? (uint32_t)rowb : 0u) + 16u * lc;
      for (int pr = w; 2 * pr < H; pr += nw) {
        dma16<NT>(l0 + (uint32_t)(slot * 1024), base + (int64_t)(2 * pr) * rowb, voff);
        slot += nw;
        if (slot >= 128) slot -= 128;
        wait_d<D>();
      }
    }
  } else {
    // each workgroup sweeps whole images (1-KB pieces), images t = g, g + G, ...
    const int per = (int)(imgb / 1024);
    for (int img = g; img < nimg; img += G) {
      const uint8_t *base = buf + img * imgb;
      for (int i = w; i < per; i += nw) {
        dma16<NT>(l0 + (uint32_t)(slot * 1024), base + (int64_t)i * 1024, 16u * lane);
        slot += nw;
        if (slot >= 128) slot -= 128;
        wait_d<D>();
      }
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if (lds[tid] == 0x5a && tid == 12345) sink[0] = 1;
}

int main(int argc, char **argv) {
  hipDeviceProp_t prop;
  CK(hipGetDeviceProperties(&prop, 0));
  const int ncu = prop.multiProcessorCount;
  const int nimg = argc > 1 ? atoi(argv[1]) : 1024, W = 1920, H = 1080, rowb = 3 * W;
  const int S = (rowb + 511) / 512;
  const int64_t total = (int64_t)nimg * rowb * H;
  uint8_t *buf;
  uint32_t *sink;
  CK(hipMalloc(&buf, total));
  CK(hipMalloc(&sink, 4096));
  CK(hipMemset(buf, 1, total));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const int lds = 136 * 1024;  // one workgroup per CU
  printf("%d images %dx%d (%.2f GB), %d strips, %d workgroups\n", nimg, W, H, total / 1e9, S, ncu);
  for (int walk = 0; walk < 2; walk++)
    for (int nt = 0; nt < 2; nt++)
      for (int d : {16, 32, 48})
        for (int nw : {1, 2, 4, 8}) {
          auto launch = [&]() {
#define L_(DD, NN) hipLaunchKernelGGL((k_ring<DD, NN>), dim3(ncu), dim3(1024), lds, 0, buf, nimg, rowb, H, S, walk, nw, sink)
            if (d == 16) { if (nt) L_(16, 1); else L_(16, 0); }
            if (d == 32) { if (nt) L_(32, 1); else L_(32, 0); }
            if (d == 48) { if (nt) L_(48, 1); else L_(48, 0); }
#undef L_
          };
          launch();
          CK(hipDeviceSynchronize());
          CK(hipEventRecord(e0));
          for (int k = 0; k < 3; k++) launch();
          CK(hipEventRecord(e1));
          CK(hipEventSynchronize(e1));
          float ms = 0;
          CK(hipEventElapsedTime(&ms, e0, e1));
          ms /= 3;
          printf("%-6s nt %d inflight %2d waves %d: %7.3f ms %7.1f GB/s\n", walk ? "rows" : "strips", nt, d, nw, ms,
                 (double)total / (ms * 1e-3) / 1e9);
          fflush(stdout);
        }
  return 0;
}
