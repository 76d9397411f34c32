#include "gf16.hpp"

#include <cstring>

namespace ecamd {

Gf16::Gf16() : log_(65536, 0), exp_(2 * 65535, 0) {
  uint32_t x = 1;
  for (uint32_t i = 0; i < 65535; ++i) {
    exp_[i] = exp_[i + 65535] = static_cast<uint16_t>(x);
    log_[x] = i;
    x <<= 1;
    if (x & 0x10000u) x ^= kGfPoly;
  }
}

const Gf16& Gf16::get() {
  static const Gf16 field;  // C++11 magic static: thread-safe init
  return field;
}

bool invert(const GfMatrix& a, GfMatrix& out, int n) {
  const Gf16& gf = Gf16::get();
  const int w = 2 * n;
  std::vector<uint16_t> t(static_cast<size_t>(n) * w, 0);
  for (int i = 0; i < n; ++i) {
    std::memcpy(&t[i * w], &a[i * n], sizeof(uint16_t) * n);
    t[i * w + n + i] = 1;
  }
  for (int col = 0; col < n; ++col) {
    int piv = col;
    while (piv < n && t[piv * w + col] == 0) ++piv;
    if (piv == n) return false;
    if (piv != col)
      for (int c = 0; c < w; ++c) std::swap(t[piv * w + c], t[col * w + c]);
    const uint16_t s = gf.inv(t[col * w + col]);
    for (int c = 0; c < w; ++c) t[col * w + c] = gf.mul(t[col * w + c], s);
    for (int r = 0; r < n; ++r) {
      const uint16_t f = t[r * w + col];
      if (r == col || f == 0) continue;
      for (int c = 0; c < w; ++c) t[r * w + c] ^= gf.mul(f, t[col * w + c]);
    }
  }
  out.assign(static_cast<size_t>(n) * n, 0);
  for (int i = 0; i < n; ++i) std::memcpy(&out[i * n], &t[i * w + n], sizeof(uint16_t) * n);
  return true;
}

GfMatrix make_generator(int k, int m) {
  const Gf16& gf = Gf16::get();
  const int rows = k + m;
  GfMatrix v(static_cast<size_t>(rows) * k, 0);
  for (int i = 0; i < rows; ++i) {
    uint16_t acc = 1;  // i^0 = 1, including 0^0 for row 0
    for (int j = 0; j < k; ++j) {
      v[i * k + j] = (i == 0 && j > 0) ? 0 : acc;
      acc = gf.mul(acc, static_cast<uint16_t>(i));
    }
  }
  GfMatrix top(v.begin(), v.begin() + static_cast<size_t>(k) * k), top_inv;
  invert(top, top_inv, k);  // Vandermonde on distinct points: never singular
  GfMatrix g(static_cast<size_t>(rows) * k, 0);
  for (int i = 0; i < rows; ++i)
    for (int j = 0; j < k; ++j) {
      uint16_t acc = 0;
      for (int t = 0; t < k; ++t) acc ^= gf.mul(v[i * k + t], top_inv[t * k + j]);
      g[i * k + j] = acc;
    }
  for (int j = 0; j < k; ++j) {
    const uint16_t s = gf.inv(g[k * k + j]);
    for (int i = k; i < rows; ++i) g[i * k + j] = gf.mul(g[i * k + j], s);
  }
  return g;
}

void build_nibble_tables(const uint16_t* rows, int nrows, int ncols, uint64_t* out) {
  // Products are GF(2)-linear in the nibble, so entry v is the XOR of the
  // entries of v's bits: 4 multiplications per (column, position) instead of
  // 16 (decode builds one set per new erasure pattern, inside the call).
  const Gf16& gf = Gf16::get();
  for (int c = 0; c < ncols; ++c)
    for (int q = 0; q < 4; ++q) {
      uint64_t basis[4] = {0, 0, 0, 0};
      for (int b = 0; b < 4; ++b) {
        const uint16_t x = static_cast<uint16_t>(1u << (4 * q + b));
        for (int r = 0; r < nrows && r < 4; ++r)
          basis[b] |= static_cast<uint64_t>(gf.mul(rows[r * ncols + c], x)) << (16 * r);
      }
      uint64_t* t = out + c * 64 + (q >> 1) * 32 + (q & 1);
      for (int v = 0; v < 16; ++v)
        t[v * 2] = ((v & 1) ? basis[0] : 0) ^ ((v & 2) ? basis[1] : 0) ^ ((v & 4) ? basis[2] : 0) ^
                   ((v & 8) ? basis[3] : 0);
    }
}

void build_nibble_tables_x8(const uint16_t* rows, int nrows, int ncols, uint16_t* out) {
  const Gf16& gf = Gf16::get();
  for (int c = 0; c < ncols; ++c)
    for (int q = 0; q < 4; ++q) {
      uint16_t basis[4][kRowsWide] = {};
      for (int b = 0; b < 4; ++b) {
        const uint16_t x = static_cast<uint16_t>(1u << (4 * q + b));
        for (int r = 0; r < nrows && r < kRowsWide; ++r) basis[b][r] = gf.mul(rows[r * ncols + c], x);
      }
      uint16_t* t = out + (c * 4 + q) * 16 * kRowsWide;
      for (int v = 0; v < 16; ++v)
        for (int r = 0; r < kRowsWide; ++r)
          t[v * kRowsWide + r] = static_cast<uint16_t>(
              ((v & 1) ? basis[0][r] : 0) ^ ((v & 2) ? basis[1][r] : 0) ^
              ((v & 4) ? basis[2][r] : 0) ^ ((v & 8) ? basis[3][r] : 0));
    }
}

}  // namespace ecamd
