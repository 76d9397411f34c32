#include "crc32.hpp"

#include <cstring>

namespace ecamd {
namespace {

struct Tables {
  uint32_t t[8][256];
  Tables() {
    for (uint32_t n = 0; n < 256; ++n) {
      uint32_t c = n;
      for (int b = 0; b < 8; ++b) c = (c & 1) ? (0xEDB88320u ^ (c >> 1)) : (c >> 1);
      t[0][n] = c;
    }
    for (uint32_t n = 0; n < 256; ++n)
      for (int s = 1; s < 8; ++s) t[s][n] = (t[s - 1][n] >> 8) ^ t[0][t[s - 1][n] & 0xFF];
  }
};

const Tables& tables() {
  static const Tables tb;
  return tb;
}

}  // namespace

// Slicing-by-8 over little-endian 64-bit words.
uint32_t crc32(uint32_t crc, const void* buf, size_t len) {
  const Tables& tb = tables();
  const uint8_t* p = static_cast<const uint8_t*>(buf);
  uint32_t c = ~crc;
  while (len && (reinterpret_cast<uintptr_t>(p) & 7)) {
    c = tb.t[0][(c ^ *p++) & 0xFF] ^ (c >> 8);
    --len;
  }
  while (len >= 8) {
    uint64_t w;
    std::memcpy(&w, p, 8);
    const uint32_t lo = static_cast<uint32_t>(w) ^ c;
    const uint32_t hi = static_cast<uint32_t>(w >> 32);
    c = tb.t[7][lo & 0xFF] ^ tb.t[6][(lo >> 8) & 0xFF] ^ tb.t[5][(lo >> 16) & 0xFF] ^
        tb.t[4][lo >> 24] ^ tb.t[3][hi & 0xFF] ^ tb.t[2][(hi >> 8) & 0xFF] ^
        tb.t[1][(hi >> 16) & 0xFF] ^ tb.t[0][hi >> 24];
    p += 8;
    len -= 8;
  }
  while (len--) c = tb.t[0][(c ^ *p++) & 0xFF] ^ (c >> 8);
  return ~c;
}

uint32_t crc32_legacy(uint32_t crc, const void* buf, size_t len) {
  const Tables& tb = tables();
  const uint8_t* p = static_cast<const uint8_t*>(buf);
  int32_t c = static_cast<int32_t>(crc ^ ~0u);
  while (len--)
    c = static_cast<int32_t>(tb.t[0][(c ^ *p++) & 0xFF]) ^ (c >> 8);  // arithmetic shift
  return static_cast<uint32_t>(c) ^ ~0u;
}

}  // namespace ecamd
