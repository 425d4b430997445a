// Host check that the two forms of the Hamming algebra in codec_math.h agree:
// the v_perm table form the gfx950 kernels use (run here through byte_perm's
// host emulation) and the shift/XOR form of the host backend.  Every byte value
// in every byte lane of a word (with several fillers in the other lanes) for
// decode; every 16-bit pattern in both halves of a word for encode.  Also the
// injection draw: the kernels' add+compare BER test and per-element flip masks
// against plain per-bit Philox draws with the fold+compare test.
// Built and run by tests/test_codec_math_native.py; prints "mismatches N".
#include <cstdio>
#include <initializer_list>
#include "codec_math.h"

using namespace kvecc;

static long g_bad = 0;

static void expect(bool ok, const char *what, uint32_t w) {
  if (!ok && g_bad++ < 8) std::printf("%s mismatch at %08x\n", what, w);
}

int main() {
  // the host emulation of v_perm_b32 on known selectors
  expect(byte_perm(0x77665544u, 0x33221100u, 0x07050301u) == 0x77553311u, "byte_perm", 0);
  const uint32_t fills[] = {0x00u, 0x5Au, 0xFFu, 0x33u, 0x80u, 0x0Fu};
  for (uint32_t lane = 0; lane < 4; ++lane)
    for (uint32_t fill : fills)
      for (uint32_t b = 0; b < 256; ++b) {
        const uint32_t w = ((fill * 0x01010101u) & ~(0xFFu << (8 * lane))) | b << (8 * lane);
        const HammingTables t(w);
        const HammingSyndrome s(w);
        const uint32_t pe = byte_parity4(w);
        expect(t.nz() == s.nz, "nz", w);
        expect(t.pe() == pe, "pe", w);
        expect(((w ^ (t.fx & t.pe_rep)) & 0x0F0F0F0Fu) == ((w ^ (s.fix & (pe * 0x0Fu))) & 0x0F0F0F0Fu),
               "h84 data", w);
        expect(((w ^ t.fx) & 0x0F0F0F0Fu) == ((w ^ s.fix) & 0x0F0F0F0Fu), "h74 data", w);
      }
  for (uint32_t v = 0; v < (1u << 16); ++v) {
    const uint32_t w = v | v << 16;
    expect(h_encode4_tables<true>(w) == h_encode4_shifts<true>(w), "h84 encode", w);
    expect(h_encode4_tables<false>(w) == h_encode4_shifts<false>(w), "h74 encode", w);
  }
  // Injection: the add+compare BER test equals the fold+compare test (windows
  // around every boundary of the flip set; the full 2^32 sweep was run once
  // offline), and the per-element masks (shared sign word, bits shifted in
  // high to low, thr == 2^31 short cut) equal plain per-bit draws, also for
  // key runs that cross 2^31 and 2^32.
  const uint32_t thrs[] = {0u, 1u, 2u, 3u, 2147484u, 21474837u, 1073741824u, 2147483646u,
                           2147483647u, 2147483648u};
  for (uint32_t t : thrs) {
    const uint32_t centres[] = {0u, t, 0u - t, 0x7FFFFFFFu, 0x80000000u, t * 2, 0xFFFFFFFFu};
    for (uint32_t c : centres)
      for (uint32_t d = 0; d < 4096; ++d) {
        const uint32_t x = c + d - 2048;
        const bool want = philox_below(x, t);
        const bool got = t > 0x7FFFFFFFu ? true : philox_below2(x, t, 2 * t) != 0;
        expect(want == got, "ber test", x);
      }
  }
  const uint32_t bases[] = {0u, 8u, 0x7FFFFFF8u, 0x7FFFFFF9u, 0x7FFFFFFEu, 0xFFFFFFF0u,
                            0xFFFFFFFCu, 0x12345678u, 0x80000000u};
  for (uint32_t t : {1073741824u, 21474837u, 2147483647u, 2147483648u, 0u})
    for (uint32_t kb : bases)
      for (uint32_t ctr = 0; ctr < 64; ++ctr) {
        const uint32_t key = kb + ctr * 7u;
        auto plain = [&](int nb) {
          uint32_t m = 0;
          for (int b = 0; b < nb; ++b) m |= (uint32_t)philox_below(philox_word0(ctr, key + b), t) << b;
          return m;
        };
        expect(philox_flip_mask<8>(key, ctr, t, 8) == plain(8), "mask nb8", key);
        expect(philox_flip_mask<24>(key, ctr, t, 24) == plain(24), "mask nb24", key);
        expect(philox_flip_mask<7>(key, ctr, t, 7) == plain(7), "mask nb7", key);
        for (int nb : {0, 1, 5, 12})
          expect(philox_flip_mask<-1>(key, ctr, t, nb) == plain(nb), "mask runtime", key);
      }
  std::printf("mismatches %ld\n", g_bad);
  return g_bad != 0;
}
