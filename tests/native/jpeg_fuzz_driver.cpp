// Host-only driver for the GPU JPEG decoder's header parser
// (fi_jpeg_parse.cpp: jpeg_parse + jpeg_build_huff through jpeg_info) under ASan/UBSan: every
// file named on the command line, all its truncations (every 7th length) and
// seeded random byte mutations.  Prints "DONE <n> parses".
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include <string>
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
  // crafted seeds: an SOS whose length field is 2 at the very end
  // of the data, and over-subscribed / all-ones / DC > 15 Huffman tables
  {
    int w, h, c;
    const uint8_t sof[] = {0xFF, 0xD8, 0xFF, 0xC0, 0, 11, 8, 0, 8, 0, 8, 1, 1, 0x11, 0, 0xFF, 0xDA, 0x00, 0x02};
    std::vector<uint8_t> t(sof, sof + sizeof(sof));
    fi::jpeg_info(t.data(), t.size(), &w, &h, &c);
    n++;
    const int lens[3][2] = {{0, 40}, {0, 2}, {0, 1}};
    for (int k = 0; k < 3; k++) {
      std::vector<uint8_t> d2 = {0xFF, 0xD8, 0xFF, 0xC4};
      const int cnt = lens[k][1];
      const int L = 2 + 1 + 16 + cnt;
      d2.push_back((uint8_t)(L >> 8));
      d2.push_back((uint8_t)L);
      d2.push_back(0x00);
      for (int l = 0; l < 16; l++) d2.push_back((uint8_t)(l == 0 ? cnt : 0));
      for (int v = 0; v < cnt; v++) d2.push_back((uint8_t)(k == 2 ? 200 : v));
      std::vector<uint8_t> t2(d2.begin(), d2.end());
      fi::jpeg_info(t2.data(), t2.size(), &w, &h, &c);
      std::string dht((const char *)d2.data() + 7, d2.size() - 7);
      fi::JpegHuff hf;
      if (fi::jpeg_build_huff(dht, true, &hf)) return 3;  // every crafted table is invalid
      n++;
    }
  }
  printf("DONE %ld parses\n", n);
  return 0;
}
