// Host-only driver for the GPU JPEG decoder's header parser
// (fi_jpeg_parse.cpp: jpeg_parse + jpeg_build_huff through jpeg_info) under ASan/UBSan: every
// file named on the command line, all its truncations (every 7th length) and
// seeded random byte mutations.  Prints "DONE <n> parses".
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include <vector>

#include "../../flyimg_amd/csrc/fi_jpeg.h"

int main(int argc, char **argv) {
  long n = 0;
  uint64_t rng = 0x9E3779B97F4A7C15ull;
  auto next = [&]() {
    rng ^= rng << 13;
    rng ^= rng >> 7;
    rng ^= rng << 17;
    return rng;
  };
  for (int a = 1; a < argc; a++) {
    FILE *f = fopen(argv[a], "rb");
    if (!f) return 2;
    std::vector<uint8_t> d;
    int ch;
    while ((ch = fgetc(f)) != EOF) d.push_back((uint8_t)ch);
    fclose(f);
    int w, h, c;
    for (size_t L = 0; L <= d.size(); L += (L < 1024 ? 1 : 7)) {
      std::vector<uint8_t> t(d.begin(), d.begin() + L);  // exact-size copy: overreads trip ASan
      fi::jpeg_info(t.data(), t.size(), &w, &h, &c);
      n++;
    }
    for (int m = 0; m < 3000; m++) {
      std::vector<uint8_t> t = d;
      const int k = 1 + (int)(next() % 8);
      for (int j = 0; j < k; j++) {
        // mutate mostly the headers (the first 1 KB), sometimes anywhere
        const size_t lim = (next() & 3) ? (t.size() < 1024 ? t.size() : 1024) : t.size();
        t[next() % lim] = (uint8_t)next();
      }
      fi::jpeg_info(t.data(), t.size(), &w, &h, &c);
      n++;
    }
  }
  printf("DONE %ld parses\n", n);
  return 0;
}
