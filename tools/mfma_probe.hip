// mfma_probe: pin the lane maps of v_mfma_i32_16x16x64_i8 on gfx950 with
// exact integer data (the guide documents the bf16 maps only).
//   hypothesis H1: lane l holds A[l&15][16(l>>4) + j] and B[16(l>>4) + j][l&15], j = 0..15
//   hypothesis H2: lane l holds A[l&15][8(l>>4) + j] (j < 8) and A[l&15][32 + 8(l>>4) + j-8] (j >= 8), same for B
//   D: lane l holds D[4(l>>4) + i][l&15], i = 0..3
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

typedef int32_t i32x4 __attribute__((ext_vector_type(4)));

__device__ int kidx(int hyp, int l, int j) {
  if (hyp == 1) return 16 * (l >> 4) + j;
  return j < 8 ? 8 * (l >> 4) + j : 32 + 8 * (l >> 4) + (j - 8);
}

__global__ void k_probe(const int8_t *A, const int8_t *B, int32_t *D, int hyp) {
  const int l = threadIdx.x;
  int8_t a[16], b[16];
  for (int j = 0; j < 16; j++) {
    const int k = kidx(hyp, l, j);
    a[j] = A[(l & 15) * 64 + k];  // A [16][64]
    b[j] = B[k * 16 + (l & 15)];  // B [64][16]
  }
  i32x4 av, bv;
  __builtin_memcpy(&av, a, 16);
  __builtin_memcpy(&bv, b, 16);
  i32x4 c = {0, 0, 0, 0};
  c = __builtin_amdgcn_mfma_i32_16x16x64_i8(av, bv, c, 0, 0, 0);
  for (int i = 0; i < 4; i++) D[(4 * (l >> 4) + i) * 16 + (l & 15)] = c[i];
}

int main() {
  int8_t hA[16 * 64], hB[64 * 16];
  srand(7);
  for (int i = 0; i < 16 * 64; i++) hA[i] = (int8_t)(rand() % 256 - 128);
  for (int i = 0; i < 64 * 16; i++) hB[i] = (int8_t)(rand() % 256 - 128);
  int32_t ref[256];
  for (int m = 0; m < 16; m++)
    for (int n = 0; n < 16; n++) {
      int32_t s = 0;
      for (int k = 0; k < 64; k++) s += (int32_t)hA[m * 64 + k] * hB[k * 16 + n];
      ref[m * 16 + n] = s;
    }
  int8_t *dA, *dB;
  int32_t *dD;
  hipMalloc(&dA, sizeof hA);
  hipMalloc(&dB, sizeof hB);
  hipMalloc(&dD, 1024);
  hipMemcpy(dA, hA, sizeof hA, hipMemcpyHostToDevice);
  hipMemcpy(dB, hB, sizeof hB, hipMemcpyHostToDevice);
  for (int hyp = 1; hyp <= 2; hyp++) {
    hipMemset(dD, 0, 1024);
    hipLaunchKernelGGL(k_probe, dim3(1), dim3(64), 0, 0, dA, dB, dD, hyp);
    int32_t hD[256];
    hipMemcpy(hD, dD, 1024, hipMemcpyDeviceToHost);
    int bad = 0;
    for (int i = 0; i < 256; i++) bad += hD[i] != ref[i];
    printf("i8 16x16x64 hypothesis H%d: %d / 256 mismatches\n", hyp, bad);
  }
  return 0;
}
