/* Oracle driver for the sanitizer test (tests/test_sanitize_cpu.py): the C
 * restatement (oracle/fi_oracle.c, included as one translation unit) over a
 * grid of ImageMagick convert geometries -- RGB and RGBA, thumbnail / resize,
 * fill + extent with every gravity, gray, monochrome, rotations, forwarded
 * convolutions, degenerate 1-px sizes -- and SmartCrop.crop() on synthetic
 * images of many shapes and targets.  Built with
 * -fsanitize=address,undefined: any out-of-bounds access or UB aborts. */
#include "../../oracle/fi_oracle.c"

#include <stdio.h>

static uint32_t g_seed = 12345;
static uint8_t rnd8(void) {
  g_seed = g_seed * 1664525u + 1013904223u;
  return (uint8_t)(g_seed >> 24);
}
static uint8_t *synth(int W, int H, int C) {
  uint8_t *p = (uint8_t *)malloc((size_t)W * H * C);
  for (int y = 0; y < H; y++)
    for (int x = 0; x < W; x++)
      for (int c = 0; c < C; c++) {
        const int v = ((x * (c + 3)) ^ (y * 5)) & 255;
        p[((size_t)y * W + x) * C + c] = (uint8_t)((v + (rnd8() & 31)) & 255);
      }
  return p;
}

int main(void) {
  static const int sizes[][2] = {{1, 1}, {2, 3}, {7, 5}, {64, 48}, {100, 100}, {301, 199}, {640, 161}, {161, 640}};
  static const int targets[][2] = {{1, 1}, {50, 0}, {0, 40}, {100, 100}, {317, 0}, {150, 150}, {333, 222}};
  const unsigned geo_flags[] = {1, 1 | 4, 1 | 2 | 8, 0, 2 | 8, 1 | 2 | 8 | 16, 1 | 2 | 8 | 16 | 32,
                                1 | 64, 1 | 2 | 8 | 32, 1 | 128};
  int n = 0, fails = 0;
  double conv[8] = {2, 1.0, 1.5, 0.02, 1, 0.8, 1, 1.2};
  for (size_t s = 0; s < sizeof sizes / sizeof sizes[0]; s++) {
    const int W = sizes[s][0], H = sizes[s][1];
    for (int C = 3; C <= 4; C++) {
      uint8_t *src = synth(W, H, C);
      for (size_t t = 0; t < sizeof targets / sizeof targets[0]; t++)
        for (size_t f = 0; f < sizeof geo_flags / sizeof geo_flags[0]; f++) {
          const unsigned fl = geo_flags[f];
          if (C == 4 && (fl & 64)) continue; /* monochrome of a matte image: not restated */
          const int rw = targets[t][0], rh = targets[t][1];
          const int cap = 4 * (W + 400) * (H + 400) + 64;
          uint8_t *out = (uint8_t *)malloc(cap);
          int ow, oh, oc;
          const int grav = 1 + (int)((s + t + f) % 9);
          const int rot = (fl & 32) ? 90 * (int)((s + t) % 4) : 0;
          const unsigned cops = (C == 3 && !(fl & 64) && (s + t) % 3 == 0) ? (unsigned)(1 + (t % 7)) : 0u;
          const int rc = or_im_convert_ex(src, W, H, C, W * C, rw, rh, fl, grav, rot, cops ? conv : NULL, cops, out,
                                          cap, &ow, &oh, &oc);
          n++;
          if (rc != 0 && rc != OR_EINVAL) fails++;
          free(out);
        }
      free(src);
    }
  }
  /* SmartCrop.crop(): shapes x targets, default and non-square */
  static const int scs[][4] = {{500, 281, 100, 100}, {281, 500, 100, 100}, {400, 400, 100, 100},
                               {150, 100, 100, 100}, {64, 48, 100, 100}, {8, 1000, 100, 100},
                               {1000, 101, 100, 100}, {500, 281, 100, 56}, {3, 3, 100, 100},
                               {1, 1, 100, 100}, {1000, 750, 100, 100}};
  or_sc_params P;
  or_sc_default_params(&P);
  for (size_t k = 0; k < sizeof scs / sizeof scs[0]; k++) {
    const int W = scs[k][0], H = scs[k][1];
    uint8_t *rgb = synth(W, H, 3);
    const int capc = or_sc_max_crops(W, H, 8) + 16;
    or_sc_crop_t *crops = (or_sc_crop_t *)malloc(sizeof(or_sc_crop_t) * (size_t)capc);
    int top = -1, aw = 0, ah = 0;
    double ps = 0;
    uint8_t *maps = (uint8_t *)malloc((size_t)W * H * 3 + 16);
    uint8_t *pre = (uint8_t *)malloc((size_t)W * H * 3 + 16);
    const int rc = or_sc_crop(&P, rgb, W, H, W * 3, scs[k][2], scs[k][3], 1, 1.0, 0.9, 0.1, 8, crops, capc, &top,
                              &aw, &ah, &ps, maps, pre);
    n++;
    if (rc < 0 && rc != OR_ENOCROP) fails++;
    free(rgb);
    free(crops);
    free(maps);
    free(pre);
  }
  /* -monochrome of Q16 gray */
  for (int k = 0; k < 4; k++) {
    const int w = 3 + 97 * k, h = 2 + 61 * k;
    uint16_t *g = (uint16_t *)malloc(sizeof(uint16_t) * (size_t)w * h);
    for (int i = 0; i < w * h; i++) g[i] = (uint16_t)(rnd8() * 257);
    uint8_t *o = (uint8_t *)malloc((size_t)w * h);
    if (or_im_monochrome(g, w, h, o) != 0) fails++;
    n++;
    free(g);
    free(o);
  }
  printf("DONE %d runs, %d unexpected errors\n", n, fails);
  return fails != 0;
}
