// Host harness for handel_amd/csrc/bn256_inv.h (the product's Bernstein-Yang
// inversion, compiled for the host): reads 8 hex LE words per line, prints the
// inverse mod p. Driven by tests/test_inverse.py against Python's pow(a, -1, p).
#include <stdio.h>

#include "bn256_inv.h"

int main() {
  uint32_t w[8];
  for (;;) {
    for (int i = 0; i < 8; i++)
      if (scanf("%x", &w[i]) != 1) return 0;
    hg::inv::inv_words(w);
    for (int i = 0; i < 8; i++) printf("%08x ", w[i]);
    printf("\n");
  }
}
