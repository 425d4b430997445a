// Host check that the two forms of the Hamming algebra in codec_math.h agree:
// the v_perm table form the gfx950 kernels use (run here through byte_perm's
// host emulation) and the shift/XOR form of the host backend.  Every byte value
// in every byte lane of a word (with several fillers in the other lanes) for
// decode; every 16-bit pattern in both halves of a word for encode.
// Built and run by tests/test_codec_math_native.py; prints "mismatches N".
#include <cstdio>
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
  std::printf("mismatches %ld\n", g_bad);
  return g_bad != 0;
}
