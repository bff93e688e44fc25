// kwz_test.cc — cilium_amd/csrc/kw_inflate.h (the GPU Kafka decoder's gzip /
// snappy payload decoding) built for the host and driven by
// tests/test_kw_inflate.py: cases from argv[1], results to argv[2].
//   case:   u8 codec (1 gzip, 2 snappy), u32 n, n bytes
//   result: u8 status (kKwz*), u32 cap, u32 out_len, out bytes (status ok)
// The output buffer is sized as the kernel sizes it (kernels_kafka.hip
// DevInflate): gzip from the trailing ISIZE, snappy from kwz::snappy_size.
#include <cstdio>
#include <cstring>
#include <vector>

#include "kafka_wire.h"
#include "kw_inflate.h"

namespace {
uint32_t g_crc[256];
struct Crc {
  uint32_t operator()(const uint8_t* p, uint32_t n) const {
    uint32_t c = 0xFFFFFFFFu;
    for (uint32_t i = 0; i < n; ++i) c = g_crc[(c ^ p[i]) & 0xFF] ^ (c >> 8);
    return ~c;
  }
};
}  // namespace

int main(int argc, char** argv) {
  if (argc < 3) return 2;
  for (uint32_t i = 0; i < 256; ++i) {
    uint32_t c = i;
    for (int k = 0; k < 8; ++k) c = (c & 1) ? 0xEDB88320u ^ (c >> 1) : c >> 1;
    g_crc[i] = c;
  }
  FILE* in = fopen(argv[1], "rb");
  FILE* out = fopen(argv[2], "wb");
  if (!in || !out) return 2;
  for (;;) {
    uint8_t codec;
    uint32_t n;
    if (fread(&codec, 1, 1, in) != 1) break;
    if (fread(&n, 4, 1, in) != 1) return 2;
    std::vector<uint8_t> b(n + 1);
    if (n && fread(b.data(), 1, n, in) != n) return 2;
    uint64_t need = 0;
    bool sized = true;
    if (codec == 1) {
      need = n >= 4 ? (uint64_t)b[n - 4] | (uint64_t)b[n - 3] << 8 | (uint64_t)b[n - 2] << 16 | (uint64_t)b[n - 1] << 24
                    : 0;
    } else {
      sized = cg::kwz::snappy_size(b.data(), n, &need);
    }
    uint8_t st;
    uint32_t got = 0;
    const bool fits = sized && need <= cg::kKafkaMaxParseBuf;
    std::vector<uint8_t> dst(fits ? need + 1 : 1);
    if (!fits) {
      st = cg::kwz::kKwzMore;
    } else {
      st = (uint8_t)(codec == 1 ? cg::kwz::gunzip_one(b.data(), n, dst.data(), (uint32_t)need, &got, Crc{})
                                : cg::kwz::snappy_go(b.data(), n, dst.data(), (uint32_t)need, &got));
    }
    const uint32_t cap = (uint32_t)need;
    fwrite(&st, 1, 1, out);
    fwrite(&cap, 4, 1, out);
    const uint32_t ol = st == cg::kwz::kKwzOk ? got : 0;
    fwrite(&ol, 4, 1, out);
    if (ol) fwrite(dst.data(), 1, ol, out);
  }
  fclose(out);
  printf("kwz ok\n");
  return 0;
}
