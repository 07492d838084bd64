// Host-side I/O helpers for the checkpoint / record formats.
//
// CRC32C (Castagnoli) is the checksum of TF's tensor-bundle entries, LevelDB
// table block trailers, TFRecord framing and event files (SURVEY §5,
// checkpoint/resume + metrics rows).  On x86 it maps onto the SSE4.2 `crc32`
// instruction (8 bytes per instruction), so checksumming a multi-hundred-MB
// ResNet-101 checkpoint is a ~0.1 s affair instead of minutes in Python; other
// hosts use a slicing-by-8 table.
#include <stddef.h>
#include <stdint.h>
#include <string.h>

// DTR_CRC32C_PORTABLE forces the table path (tested under ASan on x86 too)
#if defined(__x86_64__) && !defined(DTR_CRC32C_PORTABLE)
#define DTR_CRC32C_SSE42 1
#include <nmmintrin.h>
#endif

namespace dtr {

#if defined(DTR_CRC32C_SSE42)
__attribute__((target("sse4.2"))) uint32_t crc32c_extend(uint32_t crc, const uint8_t* p,
                                                        size_t n) {
  uint64_t c = ~crc;
  while (n >= 8) {
    uint64_t v;
    memcpy(&v, p, 8);
    c = _mm_crc32_u64(c, v);
    p += 8;
    n -= 8;
  }
  uint32_t c32 = (uint32_t)c;
  while (n--) c32 = _mm_crc32_u8(c32, *p++);
  return ~c32;
}
#else
namespace {
struct Tables {
  uint32_t t[8][256];
  Tables() {
    for (uint32_t i = 0; i < 256; ++i) {
      uint32_t c = i;
      for (int k = 0; k < 8; ++k) c = (c >> 1) ^ (0x82F63B78u & (0u - (c & 1u)));
      t[0][i] = c;
    }
    for (int s = 1; s < 8; ++s)
      for (uint32_t i = 0; i < 256; ++i) t[s][i] = (t[s - 1][i] >> 8) ^ t[0][t[s - 1][i] & 0xff];
  }
};
const Tables& tables() {
  static const Tables tb;
  return tb;
}
}  // namespace

uint32_t crc32c_extend(uint32_t crc, const uint8_t* p, size_t n) {
  const Tables& tb = tables();
  uint32_t c = ~crc;
  while (n >= 8) {
    uint32_t lo, hi;
    memcpy(&lo, p, 4);
    memcpy(&hi, p + 4, 4);
    lo ^= c;
    c = tb.t[7][lo & 0xff] ^ tb.t[6][(lo >> 8) & 0xff] ^ tb.t[5][(lo >> 16) & 0xff] ^
        tb.t[4][lo >> 24] ^ tb.t[3][hi & 0xff] ^ tb.t[2][(hi >> 8) & 0xff] ^
        tb.t[1][(hi >> 16) & 0xff] ^ tb.t[0][hi >> 24];
    p += 8;
    n -= 8;
  }
  while (n--) c = (c >> 8) ^ tb.t[0][(c ^ *p++) & 0xff];
  return ~c;
}
#endif

}  // namespace dtr
