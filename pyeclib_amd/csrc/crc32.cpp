#include "crc32.hpp"

#include <cstring>
#include <utility>

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

namespace ecamd {
namespace {

// 32x32 GF(2) matrices: column b = image of bit b.
struct Mat {
  uint32_t col[32];
};

uint32_t apply(const Mat& m, uint32_t r) {
  uint32_t a = 0;
  for (int b = 0; b < 32; ++b)
    if (r >> b & 1) a ^= m.col[b];
  return a;
}

Mat compose(const Mat& f, const Mat& g) {  // f(g(x))
  Mat h;
  for (int b = 0; b < 32; ++b) h.col[b] = apply(f, g.col[b]);
  return h;
}

Mat identity() {
  Mat m;
  for (int b = 0; b < 32; ++b) m.col[b] = 1u << b;
  return m;
}

// Z_n: append n zero bytes to the (reflected) CRC register.
Mat zeros(uint64_t n) {
  const Tables& tb = tables();
  Mat one;
  for (int b = 0; b < 32; ++b) {
    const uint32_t r = 1u << b;
    one.col[b] = tb.t[0][r & 0xFF] ^ (r >> 8);
  }
  Mat acc = identity();
  while (n) {
    if (n & 1) acc = compose(one, acc);
    one = compose(one, one);
    n >>= 1;
  }
  return acc;
}

bool inverse(const Mat& m, Mat& out) {
  // rows[i] bit j = m[i][j]; augment with identity, Gauss-Jordan over GF(2)
  uint64_t rows[32];
  for (int i = 0; i < 32; ++i) {
    uint32_t r = 0;
    for (int j = 0; j < 32; ++j) r |= (m.col[j] >> i & 1u) << j;
    rows[i] = r | (uint64_t(1) << (32 + i));
  }
  for (int c = 0; c < 32; ++c) {
    int p = c;
    while (p < 32 && !(rows[p] >> c & 1)) ++p;
    if (p == 32) return false;
    std::swap(rows[p], rows[c]);
    for (int r = 0; r < 32; ++r)
      if (r != c && (rows[r] >> c & 1)) rows[r] ^= rows[c];
  }
  for (int j = 0; j < 32; ++j) {
    uint32_t col = 0;
    for (int i = 0; i < 32; ++i) col |= static_cast<uint32_t>(rows[i] >> (32 + j) & 1) << i;
    out.col[j] = col;
  }
  return true;
}

void nibble_tables(const Mat& m, uint32_t (*t)[16]) {
  for (int q = 0; q < 8; ++q)
    for (uint32_t v = 0; v < 16; ++v) t[q][v] = apply(m, v << (4 * q));
}

}  // namespace

void build_crc_tables(uint32_t bs, uint32_t steps, CrcTables* out) {
  const Tables& tb = tables();
  std::memset(out, 0, sizeof(*out));
  // raw CRC of a 16-byte chunk with byte i = v << 4h and zeros elsewhere:
  // T0[byte] after byte i, then 15 - i zero bytes
  Mat tail[16];
  for (int i = 0; i < 16; ++i) tail[i] = zeros(15 - i);
  for (int p = 0; p < 32; ++p) {
    const int i = p / 2, h = p % 2;
    for (uint32_t v = 0; v < 16; ++v) out->raw16[p][v] = apply(tail[i], tb.t[0][(v << (4 * h)) & 0xFF]);
  }
  nibble_tables(zeros(4096), out->z4096);
  for (int l = 0; l < 8; ++l) nibble_tables(zeros(uint64_t(16) << l), out->level[l]);
  nibble_tables(zeros(8192), out->z8192);
  nibble_tables(zeros(12288), out->z12288);
  nibble_tables(zeros(16384), out->z16384);
  Mat inv;
  const uint64_t pad = uint64_t(steps) * 4096 - bs;
  if (!inverse(zeros(pad), inv)) inv = identity();  // Z_n is always invertible (x is a unit mod P)
  nibble_tables(inv, out->unshift);
  for (int i = 0; i < 256; ++i) out->t0[i] = tb.t[0][i];
  out->init_term = apply(zeros(bs), 0xFFFFFFFFu) ^ 0xFFFFFFFFu;
}

void build_crc_finish_tables(uint32_t bs, uint32_t tiles_total, CrcFinishTables* out) {
  const Tables& tb = tables();
  std::memset(out, 0, sizeof(*out));
  Mat z = zeros(4096);
  for (int i = 0; i < kCrcPowBits; ++i) {
    nibble_tables(z, out->pow[i]);
    z = compose(z, z);
  }
  Mat inv;
  const uint64_t pad = uint64_t(tiles_total) * 4096 - bs;
  if (!inverse(zeros(pad), inv)) inv = identity();  // Z_n is always invertible
  nibble_tables(inv, out->unshift);
  for (int i = 0; i < 256; ++i) out->t0[i] = tb.t[0][i];
  out->init_term = apply(zeros(bs), 0xFFFFFFFFu) ^ 0xFFFFFFFFu;
}

}  // namespace ecamd
