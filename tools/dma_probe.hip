// dma_probe: LDS-DMA (global_load_lds_dwordx4) streaming rate on gfx950 as a
// function of issuing waves per CU and the per-instruction address pattern --
// the loader design question of k_rs_vp (fi_vp.hip).
//
//   hipcc --offload-arch=gfx950 -O3 -o /tmp/dma_probe tools/dma_probe.hip && /tmp/dma_probe
//
// One 1024-thread workgroup per CU streams its share of a 8 GB buffer in
// "pieces" of 32 x 1 KB DMAs (rows of 512 B, as k_rs_vp's pieces), PIPE
// pieces in flight, through a 3-slot LDS ring.  The issuing waves are the
// first NW waves; every wave joins the per-piece barrier.  Patterns:
//   0  contiguous: DMA i = 1 KB at piece base + 1 KB i (lane l: +16 l)
//   1  two rows: DMA i = rows 2i, 2i+1 (512 B each of rows 5632 B apart: an
//      11-strip image walked strip by strip, 64-row pieces down each strip)
//   2  two rows, k_rs_vp's XOR chunk swizzle within each row
//   3  register staging: global_load_dwordx4 + ds_write_b128 (pattern 1)
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
typedef __attribute__((address_space(3))) uint8_t l_u8;
typedef __attribute__((address_space(1))) const u32x4 g_u32x4;

__device__ __forceinline__ void dma16(uint32_t m0, const uint8_t *sbase, uint32_t voff) {
  unsigned keep;
  const uint64_t sb = (uint64_t)(uintptr_t)sbase;
  sbase = reinterpret_cast<const uint8_t *>(
      (uintptr_t)(((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(sb >> 32)) << 32) |
                  (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)sb)));
  m0 = (uint32_t)__builtin_amdgcn_readfirstlane((int)m0);
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

template <int PAT>
__global__ __launch_bounds__(1024, 1) void k_stream(const uint8_t *buf, int64_t per_wg, int nw, uint32_t *sink) {
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  const int tid = threadIdx.x, lane = tid & 63, w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const uint8_t *base = buf + (int64_t)blockIdx.x * per_wg;
  const int npieces = (int)(per_wg / 32768);
  const uint32_t l0 = (uint32_t)(uintptr_t)(const l_u8 *)lds;
  const int h = lane >> 5;
  u32x4 r[32];
  int per = 32 / nw;  // DMAs per issuing wave per piece
  auto row_of = [&](int p, int row) {  // strip-major walk of an image of 5632-B rows
    const int strip = p % 11, prow = ((p / 11) * 64 + row) % 5800;
    return base + (int64_t)prow * 5632 + 512 * strip;
  };
  uint32_t acc = 0;
  for (int p = 0; p < npieces; p++) {
    const int slot = p % 3;
    if (w < nw) {
      const uint8_t *pb = base + (int64_t)p * 32768;
      for (int j = 0; j < per; j++) {
        const int i = w * per + j;
        if (PAT == 0) {
          dma16(l0 + slot * 32768 + 1024 * i, pb + 1024 * i, 16u * lane);
        } else if (PAT == 1 || PAT == 2) {
          const int rr = 2 * i + h;
          int lc = lane & 31;
          if (PAT == 2) lc ^= (rr & 7) | (((rr >> 4) & 1) << 3);
          dma16(l0 + slot * 32768 + 1024 * i, row_of(p, 2 * i), (uint32_t)(h * 5632 + 16 * lc));
        } else {
          r[j] = *(g_u32x4 *)(row_of(p, 2 * i) + h * 5632 + 16 * (lane & 31));
        }
      }
      if (PAT == 3) {
        for (int j = 0; j < per; j++) *reinterpret_cast<u32x4 *>(lds + slot * 32768 + 1024 * (w * per + j) + 16 * lane) = r[j];
      } else {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    acc ^= *reinterpret_cast<const uint32_t *>(lds + slot * 32768 + 4 * (tid & 1023));
  }
  if (acc == 0x12345678u) sink[tid] = acc;
}

template <int PAT>
__global__ __launch_bounds__(1024, 1) void k_stream_pipe(const uint8_t *buf, int64_t per_wg, int nw, uint32_t *sink) {
  // the same with the DMAs of piece p + 2 in flight while piece p is "consumed"
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  const int tid = threadIdx.x, lane = tid & 63, w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const uint8_t *base = buf + (int64_t)blockIdx.x * per_wg;
  const int npieces = (int)(per_wg / 32768);
  const uint32_t l0 = (uint32_t)(uintptr_t)(const l_u8 *)lds;
  const int h = lane >> 5;
  const int per = 32 / nw;
  uint32_t acc = 0;
  auto row_of = [&](int p, int row) {
    const int strip = p % 11, prow = ((p / 11) * 64 + row) % 5800;
    return base + (int64_t)prow * 5632 + 512 * strip;
  };
  auto issue = [&](int p) {
    const int slot = p % 3;
    const uint8_t *pb = base + (int64_t)p * 32768;
    for (int j = 0; j < per; j++) {
      const int i = w * per + j;
      if (PAT == 0) {
        dma16(l0 + slot * 32768 + 1024 * i, pb + 1024 * i, 16u * lane);
      } else {
        const int rr = 2 * i + h;
        int lc = lane & 31;
        if (PAT == 2) lc ^= (rr & 7) | (((rr >> 4) & 1) << 3);
        dma16(l0 + slot * 32768 + 1024 * i, row_of(p, 2 * i), (uint32_t)(h * 5632 + 16 * lc));
      }
    }
  };
  if (w < nw) {
    issue(0);
    issue(1);
  }
  for (int p = 0; p < npieces; p++) {
    if (w < nw) {
      if (p + 2 < npieces) issue(p + 2);
      // wait for piece p + 1 (this wave's DMAs of p + 2 may stay in flight)
      if (p + 2 < npieces) {
        if (per == 32) asm volatile("s_waitcnt vmcnt(32)" ::: "memory");
        else if (per == 16) asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
        else if (per == 8) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
        else if (per == 4) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
        else asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
      } else {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    acc ^= *reinterpret_cast<const uint32_t *>(lds + (p % 3) * 32768 + 4 * (tid & 1023));
  }
  if (acc == 0x12345678u) sink[tid] = acc;
}

int main() {
  int ncu = 0;
  hipDeviceProp_t prop;
  CK(hipGetDeviceProperties(&prop, 0));
  ncu = prop.multiProcessorCount;
  const int64_t per_wg = (int64_t)32 << 20;  // 32 MB per CU: 8 GB total
  const int64_t total = per_wg * ncu;
  uint8_t *buf;
  uint32_t *sink;
  CK(hipMalloc(&buf, total));
  CK(hipMalloc(&sink, 4096));
  CK(hipMemset(buf, 1, total));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const char *names[4] = {"contig 1KB", "two rows", "two rows swz", "regs+ds_write"};
  for (int pipe = 0; pipe < 2; pipe++) {
    for (int pat = 0; pat < 4; pat++) {
      if (pipe && pat == 3) continue;
      for (int nw : {1, 2, 4, 8, 16}) {
        auto launch = [&]() {
          if (!pipe) {
            if (pat == 0) hipLaunchKernelGGL(k_stream<0>, dim3(ncu), dim3(1024), 3 * 32768, 0, buf, per_wg, nw, sink);
            if (pat == 1) hipLaunchKernelGGL(k_stream<1>, dim3(ncu), dim3(1024), 3 * 32768, 0, buf, per_wg, nw, sink);
            if (pat == 2) hipLaunchKernelGGL(k_stream<2>, dim3(ncu), dim3(1024), 3 * 32768, 0, buf, per_wg, nw, sink);
            if (pat == 3) hipLaunchKernelGGL(k_stream<3>, dim3(ncu), dim3(1024), 3 * 32768, 0, buf, per_wg, nw, sink);
          } else {
            if (pat == 0) hipLaunchKernelGGL(k_stream_pipe<0>, dim3(ncu), dim3(1024), 3 * 32768, 0, buf, per_wg, nw, sink);
            if (pat == 1) hipLaunchKernelGGL(k_stream_pipe<1>, dim3(ncu), dim3(1024), 3 * 32768, 0, buf, per_wg, nw, sink);
            if (pat == 2) hipLaunchKernelGGL(k_stream_pipe<2>, dim3(ncu), dim3(1024), 3 * 32768, 0, buf, per_wg, nw, sink);
          }
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
        printf("%s %-14s waves %2d: %8.3f ms  %7.1f GB/s\n", pipe ? "pipe2" : "sync ", names[pat], nw, ms,
               (double)total / (ms * 1e-3) / 1e9);
        fflush(stdout);
      }
    }
  }
  return 0;
}
