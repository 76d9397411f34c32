#include "gf8.hpp"

#include <cstring>
#include <utility>

namespace ecamd {

Gf8::Gf8() {
  uint32_t x = 1;
  for (uint32_t i = 0; i < 255; ++i) {
    exp_[i] = exp_[i + 255] = static_cast<uint16_t>(x);
    log_[x] = static_cast<uint16_t>(i);
    x <<= 1;
    if (x & 0x100u) x ^= kGf8Poly;
  }
  exp_[510] = exp_[511] = 0;
  log_[0] = 0;
}

const Gf8& Gf8::get() {
  static const Gf8 field;
  return field;
}

namespace {

GfMatrix identity_top(int k, int m) {
  GfMatrix a(static_cast<size_t>(k + m) * k, 0);
  for (int i = 0; i < k; ++i) a[i * k + i] = 1;
  return a;
}

}  // namespace

GfMatrix make_isal_rs_matrix(int k, int m) {
  const Gf8& gf = Gf8::get();
  GfMatrix a = identity_top(k, m);
  uint16_t gen = 1;
  for (int i = k; i < k + m; ++i) {
    uint16_t p = 1;
    for (int j = 0; j < k; ++j) {
      a[i * k + j] = p;
      p = gf.mul(p, gen);
    }
    gen = gf.mul(gen, 2);
  }
  return a;
}

GfMatrix make_isal_cauchy_matrix(int k, int m) {
  const Gf8& gf = Gf8::get();
  GfMatrix a = identity_top(k, m);
  for (int i = k; i < k + m; ++i)
    for (int j = 0; j < k; ++j) a[i * k + j] = gf.inv(static_cast<uint16_t>(i ^ j));
  return a;
}

bool invert8(const GfMatrix& a, GfMatrix& out, int n) {
  const Gf8& gf = Gf8::get();
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

void build_nibble_tables8(const uint16_t* rows, int nrows, int ncols, uint32_t* out) {
  // linear in the nibble: 4 products per (column, position), XOR-combined
  const Gf8& gf = Gf8::get();
  for (int c = 0; c < ncols; ++c)
    for (int q = 0; q < 2; ++q) {
      uint32_t basis[4] = {0, 0, 0, 0};
      for (int b = 0; b < 4; ++b) {
        const uint16_t x = static_cast<uint16_t>(1u << (4 * q + b));
        for (int r = 0; r < nrows && r < 4; ++r)
          basis[b] |= static_cast<uint32_t>(gf.mul(rows[r * ncols + c], x)) << (8 * r);
      }
      for (int v = 0; v < 16; ++v)
        out[(c * 2 + q) * 16 + v] = ((v & 1) ? basis[0] : 0) ^ ((v & 2) ? basis[1] : 0) ^
                                    ((v & 4) ? basis[2] : 0) ^ ((v & 8) ? basis[3] : 0);
    }
}

}  // namespace ecamd
