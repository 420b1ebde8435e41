// fi_jpeg.h -- host side of the GPU JPEG decoder (fi_jpeg_parse.cpp): the
// header summary the batch planner in fi_jpeg.hip works from.  Host C++ only,
// so the parser can be built and fuzzed under ASan/UBSan on its own
// (tests/native/jpeg_fuzz_driver.cpp).
#pragma once
#include <stddef.h>
#include <stdint.h>

#include <string>

#include "fi_internal.h"

namespace fi {

struct JpegHdr {
  int W = 0, H = 0, ncomp = 0, restart = 0;
  int id[3] = {}, h[3] = {}, v[3] = {}, tq[3] = {}, td[3] = {}, ta[3] = {};
  uint16_t qt[4][64] = {};  // natural order
  bool qt_ok[4] = {};
  std::string dht[4];       // DC0, DC1, AC0, AC1: bits[16] + huffval
  size_t ecs0 = 0, ecs1 = 0;  // entropy-coded segment [ecs0, ecs1)
};

// 0 = OK; FI_EUNSUPPORTED for streams the GPU decoder does not handle;
// FI_EINVAL for malformed data
int jpeg_parse(const uint8_t *d, size_t n, JpegHdr *o);
// jdhuff.c jpeg_make_d_derived_tbl (+ the fast-AC entries); false when the
// code lengths are over-subscribed, the value count does not match, or (dc) a
// DC symbol exceeds 15 -- the tables libjpeg rejects with JERR_BAD_HUFF_TABLE
bool jpeg_build_huff(const std::string &dht, bool dc, JpegHuff *t);
// dimensions and output channels of a stream the GPU decoder takes
int jpeg_info(const uint8_t *data, size_t len, int *w, int *h, int *c);

}  // namespace fi
