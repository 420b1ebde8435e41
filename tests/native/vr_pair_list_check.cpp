// The pair-class copies of k_rs_vr's uneven touched-row list (fi_internal.h
// vr_pair_off, laid out by fi_api.cpp build_vr_tiles, read by the loader waves
// in fi_vr.hip): for 2 and 4 loader waves (C = 2 NL rows between a wave's own
// pairs) every pair start k has its own two slots, inside the copy, the C = 8
// copy after the C = 4 one, and a wave's own pairs k, k + C, k + 2C, ... at
// consecutive entries (what one scalar load of PL pairs relies on).
#include <cstdio>
#include <set>

#include "fi_internal.h"

int main() {
  int fails = 0;
  for (int n : {1, 2, 3, 7, 8, 9, 15, 16, 17, 63, 64, 65, 250, 1250, 2000, 4097}) {
    const int J4 = fi::vr_pair_cls_len(n, 4), J8 = fi::vr_pair_cls_len(n, 8);
    const int lo = n + 32, hi = n + 32 + 8 * J4 + 16 * J8;  // the two copies after the list and its pad
    for (int C : {4, 8}) {
      const int J = C == 4 ? J4 : J8;
      const int clo = C == 4 ? lo : lo + 8 * J4, chi = C == 4 ? lo + 8 * J4 : hi;
      std::set<int> seen;
      for (int k = 0; k < C * J; k++) {
        const int o = fi::vr_pair_off(n, k, C);
        if (o < clo || o + 2 > chi || (o - clo) % 2 != 0 || !seen.insert(o).second) {
          std::printf("n %d C %d k %d: offset %d outside [%d, %d) or shared\n", n, C, k, o, clo, chi);
          fails++;
        }
        if (k + C < C * J && fi::vr_pair_off(n, k + C, C) != o + 2) {
          std::printf("n %d C %d k %d: own pairs not consecutive\n", n, C, k);
          fails++;
        }
      }
      // every pair a wave can start (k < n) and the PL - 1 entries a scalar
      // load may read past the wave's last pair stay inside the class
      for (int k = 0; k < n; k++)
        if (k / C + 16 > J) {
          std::printf("n %d C %d k %d: class too short for the 16-entry read ahead\n", n, C, k);
          fails++;
        }
    }
  }
  std::printf("%s (%d failures)\n", fails ? "FAIL" : "OK", fails);
  return fails ? 1 : 0;
}
