/* TEST INFRASTRUCTURE (tools/gen_npmath.py).  Evaluates the two instructions
 * SVML's __svml_log8_ha (numpy's np.log on AVX512_SKX hosts) uses for its
 * table reciprocal -- vrcp14pd then vrndscalepd imm 0x58 (round to 1/32) -- for
 * every 16-bit leading mantissa u of m in [1, 2), checks that the lower 36
 * mantissa bits never change the result and that it never increases with u,
 * and prints the u at which it falls by 1/32 (16 values). */
#include <immintrin.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

static double from_bits(uint64_t b) { double d; memcpy(&d, &b, 8); return d; }
static double rcp_grid(double m) {
  return _mm512_cvtsd_f64(_mm512_roundscale_pd(_mm512_rcp14_pd(_mm512_set1_pd(m)), 0x58));
}

int main(void) {
  double prev = 2.0;
  for (uint32_t u = 0; u < 65536; ++u) {
    const uint64_t b = 0x3ff0000000000000ull | ((uint64_t)u << 36);
    const double r = rcp_grid(from_bits(b));
    if (rcp_grid(from_bits(b | 0xfffffffffull)) != r || rcp_grid(from_bits(b | 0x5a5a5a5a5ull)) != r) {
      fprintf(stderr, "low mantissa bits change rcp14 at u=%u\n", u);
      return 1;
    }
    if (r > prev) { fprintf(stderr, "not monotone at u=%u\n", u); return 1; }
    if (u > 0 && r < prev) printf("%u\n", u);
    prev = r;
  }
  return 0;
}
