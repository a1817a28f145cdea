// Host harness for handel_amd/csrc/bn256_inv.h (the product's Bernstein-Yang
// inversion, compiled for the host): reads 8 hex LE words per line, prints the
// inverse mod p. Driven by tests/test_inverse.py against Python's pow(a, -1, p).
#include <stdio.h>

#include "bn256_inv.h"

int main(int argc, char** argv) {
  const bool use62 = argc > 1;  // the signed62 form for comparison
  uint32_t w[8];
  for (;;) {
    for (int i = 0; i < 8; i++)
      if (scanf("%x", &w[i]) != 1) return 0;
    if (use62) hg::inv::inv_words62(w);
    else hg::inv::inv_words(w);
    for (int i = 0; i < 8; i++) printf("%08x ", w[i]);
    printf("\n");
  }
}
