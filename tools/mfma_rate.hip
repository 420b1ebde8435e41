// mfma_rate: cycles per back-to-back MFMA (one wave per SIMD, 4 independent
// accumulators) for the i8 shapes k_rs_vm can use.  s_memtime around the loop.
//   hipcc --offload-arch=gfx950 -O3 -o /tmp/mfma_rate tools/mfma_rate.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

typedef int32_t i32x4 __attribute__((ext_vector_type(4)));
typedef int32_t i32x16 __attribute__((ext_vector_type(16)));

template <int SHAPE>
__global__ void k(int32_t *out, uint64_t *cyc, int iters) {
  const int tx = (int)threadIdx.x;
  i32x4 a = {tx, 1, 2, 3}, b = {3, tx, 1, 2};
  i32x4 c0 = {0, 0, 0, 0}, c1 = c0, c2 = c0, c3 = c0;
  long a2 = tx, b2 = 7;
  i32x16 d0 = {}, d1 = {};
  const uint64_t t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < iters; i++) {
    if (SHAPE == 0) {  // 16x16x64 i8
      c0 = __builtin_amdgcn_mfma_i32_16x16x64_i8(a, b, c0, 0, 0, 0);
      c1 = __builtin_amdgcn_mfma_i32_16x16x64_i8(a, b, c1, 0, 0, 0);
      c2 = __builtin_amdgcn_mfma_i32_16x16x64_i8(a, b, c2, 0, 0, 0);
      c3 = __builtin_amdgcn_mfma_i32_16x16x64_i8(a, b, c3, 0, 0, 0);
    } else if (SHAPE == 1) {  // 16x16x32 i8
      c0 = __builtin_amdgcn_mfma_i32_16x16x32_i8(a2, b2, c0, 0, 0, 0);
      c1 = __builtin_amdgcn_mfma_i32_16x16x32_i8(a2, b2, c1, 0, 0, 0);
      c2 = __builtin_amdgcn_mfma_i32_16x16x32_i8(a2, b2, c2, 0, 0, 0);
      c3 = __builtin_amdgcn_mfma_i32_16x16x32_i8(a2, b2, c3, 0, 0, 0);
    } else {  // 32x32x32 i8
      d0 = __builtin_amdgcn_mfma_i32_32x32x32_i8(a, b, d0, 0, 0, 0);
      d1 = __builtin_amdgcn_mfma_i32_32x32x32_i8(a, b, d1, 0, 0, 0);
    }
  }
  const uint64_t t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
  out[blockIdx.x * 64 + threadIdx.x] = c0[0] + c1[1] + c2[2] + c3[3] + d0[0] + d1[5];
}

int main() {
  int32_t *out;
  uint64_t *cyc;
  hipMalloc(&out, 1024 * 64 * 4);
  hipMalloc(&cyc, 1024 * 8);
  const int iters = 4096;
  const char *names[3] = {"16x16x64_i8 (4 acc)", "16x16x32_i8 (4 acc)", "32x32x32_i8 (2 acc)"};
  for (int s = 0; s < 3; s++) {
    for (int rep = 0; rep < 2; rep++) {
      if (s == 0) hipLaunchKernelGGL(k<0>, dim3(1), dim3(64), 0, 0, out, cyc, iters);
      if (s == 1) hipLaunchKernelGGL(k<1>, dim3(1), dim3(64), 0, 0, out, cyc, iters);
      if (s == 2) hipLaunchKernelGGL(k<2>, dim3(1), dim3(64), 0, 0, out, cyc, iters);
      hipDeviceSynchronize();
    }
    uint64_t c;
    hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost);
    const int per = s == 2 ? 2 : 4;
    printf("%-22s %.2f cycles/MFMA\n", names[s], (double)c / (iters * per));
  }
  return 0;
}
