// Host-side I/O helpers for the checkpoint / record formats.
//
// CRC32C (Castagnoli) is the checksum of TF's tensor-bundle entries, LevelDB
// table block trailers, TFRecord framing and event files (SURVEY §5,
// checkpoint/resume + metrics rows).  On x86 it maps onto the SSE4.2 `crc32`
// instruction (8 bytes per instruction), so checksumming a multi-hundred-MB
// ResNet-101 checkpoint is a ~0.1 s affair instead of minutes in Python.
#include <nmmintrin.h>
#include <stddef.h>
#include <stdint.h>
#include <string.h>

namespace dtr {

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

}  // namespace dtr
