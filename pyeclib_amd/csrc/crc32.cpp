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

// One zero byte appended to the CRC register: zlib's step, or the legacy
// one whose right shift is arithmetic (crc32_legacy).
Mat zero_byte(bool legacy) {
  const Tables& tb = tables();
  Mat one;
  for (int b = 0; b < 32; ++b) {
    const uint32_t r = 1u << b;
    const uint32_t sh = legacy ? static_cast<uint32_t>(static_cast<int32_t>(r) >> 8) : r >> 8;
    one.col[b] = tb.t[0][r & 0xFF] ^ sh;
  }
  return one;
}

// Z_n: append n zero bytes to the (reflected) CRC register.
Mat zeros(uint64_t n, bool legacy) {
  Mat one = zero_byte(legacy);
  Mat acc = identity();
  while (n) {
    if (n & 1) acc = compose(one, acc);
    one = compose(one, one);
    n >>= 1;
  }
  return acc;
}

void nibble_tables(const Mat& m, uint32_t (*t)[16]) {
  for (int q = 0; q < 8; ++q)
    for (uint32_t v = 0; v < 16; ++v) t[q][v] = apply(m, v << (4 * q));
}

}  // namespace

void build_crc_lane_tables(bool legacy, CrcLaneTables* out) {
  const Tables& tb = tables();
  std::memset(out, 0, sizeof(*out));
  // raw CRC of a 16-byte piece with byte i = v << 4h and zeros elsewhere: the
  // byte's step from a zero register (T0[byte] in both variants), then 15 - i
  // zero bytes
  for (int i = 0; i < 16; ++i) {
    const Mat tail = zeros(15 - i, legacy);
    for (int h = 0; h < 2; ++h)
      for (uint32_t v = 0; v < 16; ++v) out->raw16[2 * i + h][v] = apply(tail, tb.t[0][(v << (4 * h)) & 0xFF]);
  }
  // Matrix-core form.  A operand of v_mfma_i32_32x32x32_i8, plane b: lane L
  // holds its piece's 16 bytes masked to bit b (value 2^b or 0), row L mod 32,
  // K block L / 32 -- so row r sums lanes r and r + 32, the latter 512 bytes
  // nearer the chunk's end.  B, plane b: lane L = n + 32 g, byte e = bit n of
  // Z_{512 (1 - g)}(raw16 of bit b of byte e), times 2^(7 - b): every product
  // is then 128 (mod 256) times a 0/1 term, and bit 7 of the i32 sum is its
  // parity (+-128 alike: -128 = 128 mod 256).
  const Mat shift[2] = {zeros(512, legacy), identity()};
  Mat tails[16], rows[32];
  for (int e = 0; e < 16; ++e) tails[e] = zeros(15 - e, legacy);
  for (int r = 0; r < 32; ++r) rows[r] = zeros(uint64_t(16) * (31 - r), legacy);
  for (int b = 0; b < 8; ++b)
    for (int L = 0; L < 64; ++L)
      for (int e = 0; e < 16; ++e) {
        const uint32_t v = apply(shift[L / 32], apply(tails[e], tb.t[0][1u << b]));
        out->mfb[b][L][e] = (v >> (L % 32) & 1) ? static_cast<int8_t>(static_cast<uint8_t>(0x80u >> b)) : 0;
      }
  // Second stage.  Accumulator j of lane l holds C[8 (j / 4) + 4 (l / 32) +
  // j mod 4][l mod 32]: row r's sum for output bit n = l mod 32, i.e. bit n of
  // u_r, and raw(chunk) = XOR_r Z_{16 (31 - r)}(u_r).  Nibble q of lane l =
  // the parities of its accumulators 4q .. 4q + 3.
  for (int l = 0; l < 64; ++l)
    for (int q = 0; q < 4; ++q)
      for (uint32_t v = 0; v < 16; ++v) {
        uint32_t a = 0;
        for (int i = 0; i < 4; ++i)
          if (v >> i & 1) a ^= rows[8 * q + 4 * (l / 32) + i].col[l % 32];
        out->mst[q][v][l] = a;
      }
  for (int l = 0; l < 64; ++l) {
    uint32_t t[8][16];
    nibble_tables(zeros(uint64_t(16) * (63 - l), legacy), t);
    for (int q = 0; q < 8; ++q)
      for (int v = 0; v < 16; ++v) out->lane[q][v][l] = t[q][v];
  }
}

void build_crc_finish_tables(uint32_t bs, bool legacy, CrcFinishTables* out) {
  const Tables& tb = tables();
  std::memset(out, 0, sizeof(*out));
  Mat z = zeros(1024, legacy);
  for (int i = 0; i < kCrcPowBits; ++i) {
    nibble_tables(z, out->pow[i]);
    z = compose(z, z);
  }
  nibble_tables(zeros(bs % 1024, legacy), out->zr);
  // metadata checksum change: the raw CRC of chksum[0]'s 4 bytes (header
  // bytes 21..24), followed by the 34 bytes to the end of the 59-byte block
  Mat meta;
  for (int b = 0; b < 32; ++b) {
    const uint32_t c = 1u << b;
    uint32_t r = 0;
    for (int i = 0; i < 4; ++i) {
      const uint32_t x = (r ^ (c >> (8 * i))) & 0xFF;
      const uint32_t sh = legacy ? static_cast<uint32_t>(static_cast<int32_t>(r) >> 8) : r >> 8;
      r = tb.t[0][x] ^ sh;
    }
    meta.col[b] = apply(zeros(59 - 25, legacy), r);
  }
  nibble_tables(meta, out->meta);
  for (int k = 0; k < 6; ++k) nibble_tables(zeros(uint64_t(16) << k, legacy), out->z16[k]);
  out->init_term = apply(zeros(bs, legacy), 0xFFFFFFFFu) ^ 0xFFFFFFFFu;
}

}  // namespace ecamd
