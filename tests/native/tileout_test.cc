// tileout_test.cc — raw_emit.h's TileOut on the CPU (built by
// tests/test_raw_emit.py with hipcc, host side only): random byte runs fed as
// the scan feeds them (put4 of 1..4 bytes, single bytes, the absent / SEP /
// REST pairs) must come out as the string's 16-byte units, each byte through
// the code map, the last unit's bytes past the string zero, nothing stored
// past the last unit, units 64 uint4 apart (one tile row each).
#include <cstdio>
#include <cstring>
#include <random>
#include <vector>

#include "raw_emit.h"

int main() {
  std::mt19937 rng(20261017);
  uint8_t lut[256];
  for (int b = 0; b < 256; ++b) lut[b] = (uint8_t)(rng() | 1);  // never 0: padding stays visible
  int bad = 0;
  for (int iter = 0; iter < 20000; ++iter) {
    std::vector<uint8_t> want;  // the uncoded string
    const int nseg = (int)(rng() % 24);
    std::vector<std::pair<uint32_t, uint32_t>> calls;  // (v, nb)
    for (int k = 0; k < nseg; ++k) {
      switch (rng() % 4) {
        case 0:  // absent field pair, or two of them
          if (rng() & 1) calls.push_back({1u, 2});
          else calls.push_back({0x00010001u, 4});
          break;
        case 1:  // SEP or REST
          calls.push_back({(rng() & 1) ? 0u : 2u, 1});
          break;
        default: {  // a value: quads, the last one short
          const uint32_t L = rng() % 70;
          for (uint32_t o = 0; o < L; o += 4) {
            const uint32_t nb = L - o < 4 ? L - o : 4;
            uint32_t q = (uint32_t)rng();
            if (nb < 4) q &= (1u << (8 * nb)) - 1u;
            calls.push_back({q, nb});
          }
        }
      }
    }
    for (auto& c : calls)
      for (uint32_t j = 0; j < c.second; ++j) want.push_back((uint8_t)(c.first >> (8 * j)));
    const size_t len = want.size(), units = (len + 15) / 16;
    std::vector<uint4> buf((units + 1) * 64);
    memset(buf.data(), 0xAB, buf.size() * sizeof(uint4));
    // even iterations: coded (the default path's bytes); odd: raw bytes
    // (TileOut<false>, the device-layout scan's: http_kernel codes them)
    const bool coded = (iter & 1) == 0;
    auto feed = [&](auto& o) {
      for (auto& c : calls) {
        if (c.second == 1 && (rng() & 1)) o.put(c.first);
        else o.put4(c.first, c.second);
      }
      o.finish();
    };
    if (coded) {
      cg::TileOut<true> o(buf.data() + 3, lut);  // lane 3 of the tile row
      feed(o);
    } else {
      cg::TileOut<false> o(buf.data() + 3, nullptr);
      feed(o);
    }
    for (size_t u = 0; u <= units; ++u) {
      uint8_t got[16];
      memcpy(got, &buf[u * 64 + 3], 16);
      for (int j = 0; j < 16; ++j) {
        const size_t at = u * 16 + j;
        const uint8_t exp = u == units ? 0xAB : at < len ? (coded ? lut[want[at]] : want[at]) : 0;
        if (got[j] != exp) {
          if (bad++ < 5)
            fprintf(stderr, "iter %d len %zu unit %zu byte %d: got %02x want %02x\n", iter, len, u, j, got[j], exp);
        }
      }
      // the other lanes' bytes of the row are never touched
      uint8_t other[16];
      memcpy(other, &buf[u * 64 + 4], 16);
      for (int j = 0; j < 16; ++j)
        if (other[j] != 0xAB && bad++ < 5) fprintf(stderr, "iter %d: lane 4 of unit %zu written\n", iter, u);
    }
  }
  if (bad) {
    fprintf(stderr, "%d mismatches\n", bad);
    return 1;
  }
  printf("tileout ok\n");
  return 0;
}
