// fi_jpeg_parse.cpp -- the GPU JPEG decoder's host-side header parser and
// Huffman table builder (restating libjpeg-turbo jdmarker.c / jdhuff.c for
// the streams fi_jpeg.hip decodes).  Host C++ only: no HIP calls.
#include <string.h>

#include "fi_jpeg.h"

namespace fi {

static int be16(const uint8_t *p) { return (p[0] << 8) | p[1]; }

// 0 = OK; FI_EUNSUPPORTED for streams the GPU decoder does not handle;
// FI_EINVAL for malformed data
int jpeg_parse(const uint8_t *d, size_t n, JpegHdr *o) {
  if (!d || n < 4 || d[0] != 0xFF || d[1] != 0xD8) return FI_EINVAL;
  static const uint8_t zz[64] = {0,  1,  8,  16, 9,  2,  3,  10, 17, 24, 32, 25, 18, 11, 4,  5,
                                 12, 19, 26, 33, 40, 48, 41, 34, 27, 20, 13, 6,  7,  14, 21, 28,
                                 35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23, 30, 37, 44, 51,
                                 58, 59, 52, 45, 38, 31, 39, 46, 53, 60, 61, 54, 47, 55, 62, 63};
  size_t p = 2;
  bool sof = false;
  // jdmarker.c examine_app0 / examine_app14: what default_decompress_parms
  // (jdapimin.c) reads to pick the colour space of a 3-component stream
  bool jfif = false, adobe = false;
  int adobe_transform = 0;
  while (p + 4 <= n) {
    if (d[p] != 0xFF) return FI_EINVAL;
    const int m = d[p + 1];
    if (m == 0xFF) {  // fill byte
      p++;
      continue;
    }
    if (m == 0xD8 || (m >= 0xD0 && m <= 0xD7) || m == 0x01) {
      p += 2;
      continue;
    }
    const size_t L = (size_t)be16(d + p + 2);
    if (L < 2 || p + 2 + L > n) return FI_EINVAL;
    const uint8_t *s = d + p + 4, *e = d + p + 2 + L;
    switch (m) {
      case 0xC0:
      case 0xC1: {  // baseline / extended sequential, Huffman
        if (sof || L < 8 || s[0] != 8) return FI_EUNSUPPORTED;
        sof = true;
        o->H = be16(s + 1);
        o->W = be16(s + 3);
        o->ncomp = s[5];
        if (o->W <= 0 || o->H <= 0) return FI_EUNSUPPORTED;  // DNL-defined height
        if (o->ncomp != 1 && o->ncomp != 3) return FI_EUNSUPPORTED;
        if (L != 8 + 3 * (size_t)o->ncomp) return FI_EINVAL;
        for (int c = 0; c < o->ncomp; c++) {
          o->id[c] = s[6 + 3 * c];
          o->h[c] = s[7 + 3 * c] >> 4;
          o->v[c] = s[7 + 3 * c] & 15;
          o->tq[c] = s[8 + 3 * c];
          if (o->tq[c] > 3 || o->h[c] < 1 || o->v[c] < 1) return FI_EINVAL;
        }
        break;
      }
      case 0xC2: case 0xC3: case 0xC5: case 0xC6: case 0xC7: case 0xC9: case 0xCA: case 0xCB:
      case 0xCD: case 0xCE: case 0xCF:
        return FI_EUNSUPPORTED;  // progressive, lossless, hierarchical, arithmetic
      case 0xDB: {  // DQT
        for (const uint8_t *q = s; q < e;) {
          const int pq = q[0] >> 4, tq = q[0] & 15;
          if (tq > 3 || pq > 1 || q + 1 + 64 * (pq + 1) > e) return FI_EINVAL;
          for (int k = 0; k < 64; k++)
            o->qt[tq][zz[k]] = (uint16_t)(pq ? be16(q + 1 + 2 * k) : q[1 + k]);
          o->qt_ok[tq] = true;
          q += 1 + 64 * (pq + 1);
        }
        break;
      }
      case 0xC4: {  // DHT
        for (const uint8_t *q = s; q < e;) {
          if (q + 17 > e) return FI_EINVAL;
          const int tc = q[0] >> 4, th = q[0] & 15;
          if (tc > 1 || th > 1) return FI_EUNSUPPORTED;  // baseline: two tables per class
          int cnt = 0;
          for (int l = 0; l < 16; l++) cnt += q[1 + l];
          if (cnt > 256 || q + 17 + cnt > e) return FI_EINVAL;
          o->dht[2 * tc + th].assign((const char *)q + 1, 16 + cnt);
          q += 17 + cnt;
        }
        break;
      }
      case 0xDD:  // DRI
        if (L != 4) return FI_EINVAL;
        o->restart = be16(s);
        break;
      case 0xDA: {  // SOS: the one scan, then the entropy-coded data up to EOI
        if (!sof || L < 3) return FI_EINVAL;
        const int ns = s[0];
        if (ns != o->ncomp || L != 6 + 2 * (size_t)ns) return FI_EUNSUPPORTED;  // one interleaved scan
        for (int k = 0; k < ns; k++) {
          const int cs = s[1 + 2 * k];
          if (cs != o->id[k]) return FI_EUNSUPPORTED;
          o->td[k] = s[2 + 2 * k] >> 4;
          o->ta[k] = s[2 + 2 * k] & 15;
          if (o->td[k] > 1 || o->ta[k] > 1) return FI_EUNSUPPORTED;
        }
        const uint8_t *t = s + 1 + 2 * ns;
        if (t[0] != 0 || t[1] != 63 || t[2] != 0) return FI_EUNSUPPORTED;
        o->ecs0 = (size_t)(e - d);
        // end of the scan: the first marker other than RSTn (stuffed 0xFF00 and fill bytes skipped)
        size_t q = o->ecs0;
        for (;;) {
          const void *f = memchr(d + q, 0xFF, n - q);
          if (!f) {
            q = n;
            break;
          }
          q = (size_t)((const uint8_t *)f - d);
          if (q + 1 >= n) {
            q = n;
            break;
          }
          const int b = d[q + 1];
          if (b == 0x00 || b == 0xFF || (b >= 0xD0 && b <= 0xD7)) {
            q += b == 0xFF ? 1 : 2;
            continue;
          }
          break;
        }
        o->ecs1 = q;
        // the scan must end at EOI: a truncated stream (no marker before the
        // end of the data) or one with markers after the scan goes to the host
        // decoder, which reports truncation as libjpeg / Pillow do
        if (q + 1 >= n || d[q + 1] != 0xD9) return FI_EUNSUPPORTED;
        // libjpeg decodes a 3-component stream as RGB (no colour conversion) when
        // it has no JFIF marker and either an Adobe marker with transform 0 or,
        // with no Adobe marker, the component ids 'R', 'G', 'B'; the GPU path
        // converts YCbCr only
        if (o->ncomp == 3 && !jfif) {
          if (adobe && adobe_transform == 0) return FI_EUNSUPPORTED;
          if (!adobe && o->id[0] == 82 && o->id[1] == 71 && o->id[2] == 66) return FI_EUNSUPPORTED;
        }
        for (int c = 0; c < o->ncomp; c++) {
          if (!o->qt_ok[o->tq[c]] || o->dht[o->td[c]].empty() || o->dht[2 + o->ta[c]].empty()) return FI_EINVAL;
        }
        if (o->ncomp == 1) {
          o->h[0] = o->v[0] = 1;  // non-interleaved scan: one block per MCU
        } else {
          // YCbCr with luma 1x1 / 2x1 / 2x2 over 1x1 chroma (jdsample.c fullsize / h2v1 / h2v2)
          if (o->h[1] != 1 || o->v[1] != 1 || o->h[2] != 1 || o->v[2] != 1) return FI_EUNSUPPORTED;
          const int hv = o->h[0] * 10 + o->v[0];
          if (hv != 11 && hv != 21 && hv != 22) return FI_EUNSUPPORTED;
        }
        return 0;
      }
      case 0xE0:  // APP0 "JFIF\0" (examine_app0: at least 14 data bytes)
        if (L >= 16 && memcmp(s, "JFIF\0", 5) == 0) jfif = true;
        break;
      case 0xEE:  // APP14 "Adobe" (examine_app14: at least 12 data bytes); it may precede SOF
        if (L >= 14 && memcmp(s, "Adobe", 5) == 0) {
          adobe = true;
          adobe_transform = s[11];
        }
        break;
      default:
        break;  // APPn, COM, ...
    }
    p += 2 + L;
  }
  return FI_EINVAL;
}

// jdhuff.c jpeg_make_d_derived_tbl: canonical codes, maxcode / valoffset,
// 9-bit lookahead
bool jpeg_build_huff(const std::string &dht, bool dc, JpegHuff *t) {
  memset(t, 0, sizeof(*t));
  if (dht.size() < 16 || dht.size() > 16 + 256) return false;
  const uint8_t *bits = (const uint8_t *)dht.data();
  const int nv = (int)dht.size() - 16;
  int cnt = 0;
  for (int l = 0; l < 16; l++) cnt += bits[l];
  if (cnt != nv) return false;
  memcpy(t->huffval, bits + 16, nv);
  // jdhuff.c: DC symbols are coefficient sizes, 0..15 (JERR_BAD_HUFF_TABLE)
  if (dc)
    for (int k = 0; k < nv; k++)
      if (t->huffval[k] > 15) return false;
  int p = 0;
  uint32_t code = 0;
  for (int l = 1; l <= 16; l++) {
    // jdhuff.c: the codes of length l, and the next code after them, must fit
    // in l bits (no code is all ones); checked before any lookahead entry is
    // written, so an over-subscribed table never writes past look[]
    if ((uint64_t)code + bits[l - 1] >= ((uint64_t)1 << l)) return false;
    if (bits[l - 1]) {
      t->valoff[l] = p - (int)code;
      for (int i = 0; i < bits[l - 1]; i++, p++, code++) {
        if (l <= 9) {
          const uint32_t lo = code << (9 - l), cnt = 1u << (9 - l);
          for (uint32_t k = 0; k < cnt; k++) t->look[lo + k] = (uint16_t)((l << 8) | t->huffval[p]);
        }
      }
      t->maxcode[l] = (int32_t)code - 1;
    } else {
      t->maxcode[l] = -1;
    }
    code <<= 1;
  }
  t->maxcode[17] = 0x7FFFFFFF;
  // fast AC entries (as stb_image's fast_ac): run/size symbols whose code and
  // value bits both fit the 9-bit lookahead and whose value fits a signed byte
  for (int l = 0; l < 512; l++) {
    const int lk = t->look[l];
    if (!lk) continue;
    const int len = lk >> 8, rs = lk & 255, run = rs >> 4, sz = rs & 15;
    if (sz == 0 || len + sz > 9) continue;
    const int v = (l >> (9 - len - sz)) & ((1 << sz) - 1);
    const int val = v < (1 << (sz - 1)) ? v - (1 << sz) + 1 : v;  // HUFF_EXTEND
    if (val < -128 || val > 127) continue;
    t->fast_ac[l] = (int16_t)((val * 256) | (run << 4) | (len + sz));
  }
  return p == nv;
}


int jpeg_info(const uint8_t *data, size_t len, int *w, int *h, int *c) {
  JpegHdr hd;
  const int rc = jpeg_parse(data, len, &hd);
  if (rc) return rc;
  for (int t = 0; t < 4; t++) {  // the Huffman tables must build (jdhuff.c rejects bad ones too)
    JpegHuff hf;
    if (!hd.dht[t].empty() && !jpeg_build_huff(hd.dht[t], t < 2, &hf)) return FI_EINVAL;
  }
  *w = hd.W;
  *h = hd.H;
  *c = hd.ncomp == 1 ? 1 : 3;
  return 0;
}

}  // namespace fi
