// tr8_probe: semantics of gfx950 ds_read_b64_tr_b8 (the guide documents the
// 16-bit form only).  LDS holds a [64 rows][16 cols] byte tile, value =
// row * 16 + col encoded as (row, col) through two runs (row in one, col in
// the other).  Each lane supplies an address under a few candidate patterns;
// the program prints, per lane, the (row, col) of each of the 8 bytes it got.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

typedef int v2i __attribute__((ext_vector_type(2)));

// pattern 0: lane i of each 16-lane group g -> row 8g' + (i >> 1), cols 8 (i & 1) .. +7
//            (tile rows 8 per group; groups use rows 8g .. 8g+7)
// pattern 1: lane i -> row 8g + (i & 7), cols 8 (i >> 3) .. +7
__global__ void k_probe(int pattern, int what, uint8_t *out) {
  __shared__ __attribute__((aligned(16))) uint8_t t[64 * 16];
  for (int i = threadIdx.x; i < 64 * 16; i += 64) {
    const int row = i / 16, col = i % 16;
    t[i] = what == 0 ? (uint8_t)row : (uint8_t)col;
  }
  __syncthreads();
  const int l = threadIdx.x, g = l >> 4, i = l & 15;
  int row, col;
  if (pattern == 0) {
    row = 8 * g + (i >> 1);
    col = 8 * (i & 1);
  } else {
    row = 8 * g + (i & 7);
    col = 8 * (i >> 3);
  }
  v2i r = __builtin_amdgcn_ds_read_tr8_b64_v2i32((__attribute__((address_space(3))) v2i *)(t + row * 16 + col));
  uint8_t b[8];
  __builtin_memcpy(b, &r, 8);
  for (int k = 0; k < 8; k++) out[l * 8 + k] = b[k];
}

int main() {
  uint8_t *d;
  hipMalloc(&d, 512);
  for (int pattern = 0; pattern < 2; pattern++) {
    uint8_t rows[512], cols[512];
    hipLaunchKernelGGL(k_probe, dim3(1), dim3(64), 0, 0, pattern, 0, d);
    hipMemcpy(rows, d, 512, hipMemcpyDeviceToHost);
    hipLaunchKernelGGL(k_probe, dim3(1), dim3(64), 0, 0, pattern, 1, d);
    hipMemcpy(cols, d, 512, hipMemcpyDeviceToHost);
    printf("pattern %d (lane: (row,col) of bytes 0..7)\n", pattern);
    for (int l = 0; l < 64; l++) {
      if (l >= 20 && l < 60) continue;
      printf("  lane %2d:", l);
      for (int k = 0; k < 8; k++) printf(" (%2d,%2d)", rows[l * 8 + k], cols[l * 8 + k]);
      printf("\n");
    }
  }
  return 0;
}
