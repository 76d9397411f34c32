// Host restatement of the GPU inline-CRC scheme (crc_device.hpp chunk_crc,
// ec_crc.hip crc_finish_kernel -- finish_tree, round 5; finish, the round-4
// form), checked against the byte-serial CRCs.
// Built and run by tests/test_crc_math.py with g++ against
// pyeclib_amd/csrc/crc32.cpp -- no GPU, no HIP.
//
// For payload sizes around the chunk and tile boundaries, in both variants
// (zlib and liberasurecode's legacy CRC) and for several interior chunk
// counts: the 1 KiB chunks' raw CRCs from the lane tables, shifted to the
// payload's end as the finishing pass does, plus the end-aligned edge
// chunks, plus the init term, must equal crc32 / crc32_legacy of the
// payload; and the metadata checksum patched by the linear delta must equal
// the checksum recomputed over the patched header.
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <random>
#include <vector>

#include "crc32.hpp"

using namespace ecamd;

static uint32_t zmap(const uint32_t (*t)[16], uint32_t r) {
  uint32_t a = 0;
  for (int q = 0; q < 8; ++q) a ^= t[q][(r >> (4 * q)) & 15];
  return a;
}

static uint32_t raw16(const CrcLaneTables& L, const uint8_t* b) {
  uint32_t a = 0;
  for (int i = 0; i < 16; ++i) a ^= L.raw16[2 * i][b[i] & 15] ^ L.raw16[2 * i + 1][b[i] >> 4];
  return a;
}

static uint32_t lane_map(const CrcLaneTables& L, uint32_t r, int lane) {
  uint32_t a = 0;
  for (int q = 0; q < 8; ++q) a ^= L.lane[q][(r >> (4 * q)) & 15][lane];
  return a;
}

// chunk_crc: 64 lanes x 16 bytes
static uint32_t chunk_crc(const CrcLaneTables& L, const uint8_t* c) {
  uint32_t a = 0;
  for (int l = 0; l < 64; ++l) a ^= lane_map(L, raw16(L, c + 16 * l), l);
  return a;
}

// the matrix-core form (crc_device.hpp mfma_plane / mfma_finish), with the
// operand layout of v_mfma_i32_32x32x32_i8 (tools/mfma_probe.hip checks it
// on the GPU): row r of A = lanes r and r + 32, B's lane n + 32 g holds
// column n of K block g, accumulator j of lane l = C[8 (j / 4) + 4 (l / 32) +
// j % 4][l % 32]; plane b keeps the bits at and above b (those above land
// on multiples of 256).  Every sum must have bits 0..6 clear (*bad counts those).
static uint32_t mfma_chunk_crc(const CrcLaneTables& L, const uint8_t* c, int* bad) {
  int32_t C[32][32] = {};
  for (int b = 0; b < 8; ++b)
    for (int r = 0; r < 32; ++r)
      for (int n = 0; n < 32; ++n)
        for (int g = 0; g < 2; ++g)
          for (int e = 0; e < 16; ++e) {
            const int8_t a = static_cast<int8_t>(c[16 * (r + 32 * g) + e] & (0xFFu << b));
            C[r][n] += int32_t(a) * int32_t(L.mfb[b][n + 32 * g][e]);
          }
  uint32_t acc = 0;
  for (int l = 0; l < 64; ++l)
    for (int q = 0; q < 4; ++q) {
      uint32_t v = 0;
      for (int i = 0; i < 4; ++i) {
        const int32_t x = C[8 * q + 4 * (l / 32) + i][l % 32];
        *bad += (x & 0x7F) != 0;
        v |= ((static_cast<uint32_t>(x) >> 7) & 1u) << i;
      }
      acc ^= L.mst[q][v][l];
    }
  return acc;
}

static uint32_t shift_chunks(const CrcFinishTables& F, uint32_t r, uint32_t d) {
  for (int i = 0; d; ++i, d >>= 1)
    if (d & 1) r = zmap(F.pow[i], r);
  return r;
}

// the finishing pass for one payload, interior = chunks [0, chunks)
static uint32_t finish(const CrcLaneTables& L, const CrcFinishTables& F, const uint8_t* pay,
                       uint32_t bs, uint32_t chunks) {
  const uint32_t nfull = bs / 1024;
  uint32_t acc = 0;
  for (uint32_t c = 0; c < chunks; ++c) acc ^= shift_chunks(F, chunk_crc(L, pay + 1024 * c), nfull - 1 - c);
  const int64_t e0 = int64_t(chunks) * 1024;
  const uint32_t n_edge = static_cast<uint32_t>((int64_t(bs) - e0 + 1023) / 1024);
  uint32_t edge = 0;
  for (uint32_t j = 0; j < n_edge; ++j) {
    uint8_t buf[1024];
    const int64_t start = int64_t(bs) - 1024 * int64_t(j + 1);
    for (int b = 0; b < 1024; ++b) {
      const int64_t at = start + b;
      buf[b] = (at >= e0 && at < int64_t(bs)) ? pay[at] : 0;
    }
    edge ^= shift_chunks(F, chunk_crc(L, buf), j);
  }
  return zmap(F.zr, acc) ^ edge ^ F.init_term;
}

// 64 lanes' values joined by the level maps tab(k) (ec_crc.hip lane_tree;
// lanes below 2^k take their own value, as __shfl_up gives them)
template <class Tab>
static uint32_t lane_tree(std::vector<uint32_t> v, Tab tab) {
  for (int k = 0; k < 6; ++k) {
    std::vector<uint32_t> n(64);
    for (int l = 0; l < 64; ++l) n[l] = zmap(tab(k), v[l >= (1 << k) ? l - (1 << k) : l]) ^ v[l];
    v = n;
  }
  return v[63];
}

// the round-5 finishing pass: runs of L chunks per thread (Horner by
// Z_1024), the lane tree by Z_{1024 L 2^k}, the waves by Z_{1024 64 L}, the
// shift from chunk n's end to nfull's; edge chunks by the Z_{16 2^k} tree
static uint32_t finish_tree(const CrcLaneTables& L, const CrcFinishTables& F, const uint8_t* pay,
                            uint32_t bs, uint32_t n) {
  const uint32_t nfull = bs / 1024;
  uint32_t lg = 0;
  while ((256u << lg) < n) ++lg;
  const uint32_t run = 1u << lg;
  const int64_t lead = int64_t(256u << lg) - n;
  uint32_t red[4];
  for (int w = 0; w < 4; ++w) {
    std::vector<uint32_t> v(64);
    for (int l = 0; l < 64; ++l) {
      uint32_t acc = 0;
      for (uint32_t j = 0; j < run; ++j) {
        const int64_t c = int64_t(64 * w + l) * run + j - lead;
        const uint32_t x = c >= 0 ? chunk_crc(L, pay + 1024 * c) : 0u;
        acc = (j == 0 ? 0u : zmap(F.pow[0], acc)) ^ x;
      }
      v[l] = acc;
    }
    red[w] = lane_tree(v, [&](int k) { return F.pow[lg + k]; });
  }
  uint32_t a = red[0];
  for (int w = 1; w < 4; ++w) a = zmap(F.pow[lg + 6], a) ^ red[w];
  a = shift_chunks(F, a, nfull - n);
  const int64_t e0 = int64_t(n) * 1024;
  const uint32_t n_edge = static_cast<uint32_t>((int64_t(bs) - e0 + 1023) / 1024);
  uint32_t edge = 0;
  for (uint32_t j = 0; j < n_edge; ++j) {
    uint8_t buf[1024];
    const int64_t start = int64_t(bs) - 1024 * int64_t(j + 1);
    for (int b = 0; b < 1024; ++b) {
      const int64_t at = start + b;
      buf[b] = (at >= e0 && at < int64_t(bs)) ? pay[at] : 0;
    }
    std::vector<uint32_t> v(64);
    for (int l = 0; l < 64; ++l) v[l] = raw16(L, buf + 16 * l);
    edge ^= shift_chunks(F, lane_tree(v, [&](int k) { return F.z16[k]; }), j);
  }
  return zmap(F.zr, a) ^ edge ^ F.init_term;
}

int main() {
  std::mt19937_64 rng(20261018);
  int failures = 0, checks = 0;
  CrcLaneTables* L = new CrcLaneTables;
  CrcFinishTables* F = new CrcFinishTables;
  const uint32_t sizes[] = {1, 2, 15, 16, 17, 1000, 1023, 1024, 1025, 2048, 4095, 4096, 4097,
                            12287, 12288, 12289, 16384, 20000, 104864, 419432};
  for (int legacy = 0; legacy < 2; ++legacy) {
    build_crc_lane_tables(legacy != 0, L);
    for (uint32_t bs : sizes) {
      build_crc_finish_tables(bs, legacy != 0, F);
      std::vector<uint8_t> pay(bs);
      for (auto& b : pay) b = static_cast<uint8_t>(rng());
      const uint32_t want = legacy ? crc32_legacy(0, pay.data(), bs) : crc32(0, pay.data(), bs);
      // interior chunk counts: none, one, all 4 KiB tiles, every full chunk
      const uint32_t cands[] = {0u, bs >= 1024 ? 1u : 0u, bs / 4096 * 4, bs / 1024};
      for (uint32_t chunks : cands) {
        ++checks;
        const uint32_t got = finish(*L, *F, pay.data(), bs, chunks);
        if (got != want) {
          ++failures;
          std::printf("FAIL legacy=%d bs=%u chunks=%u got %08x want %08x\n", legacy, bs, chunks, got, want);
        }
        ++checks;
        const uint32_t got2 = finish_tree(*L, *F, pay.data(), bs, chunks);
        if (got2 != want) {
          ++failures;
          std::printf("FAIL tree legacy=%d bs=%u chunks=%u got %08x want %08x\n", legacy, bs, chunks, got2, want);
        }
      }
      // metadata checksum: delta from chksum[0] = 0 to chksum[0] = want
      uint8_t h[80];
      for (auto& b : h) b = static_cast<uint8_t>(rng());
      std::memset(h + 21, 0, 4);
      const uint32_t m0 = legacy ? crc32_legacy(0, h, 59) : crc32(0, h, 59);
      std::memcpy(h + 21, &want, 4);
      const uint32_t m1 = legacy ? crc32_legacy(0, h, 59) : crc32(0, h, 59);
      ++checks;
      if ((m0 ^ zmap(F->meta, want)) != m1) {
        ++failures;
        std::printf("FAIL meta legacy=%d bs=%u\n", legacy, bs);
      }
    }
  }
  // the matrix-core form against the lookup form, random and extreme chunks
  for (int legacy = 0; legacy < 2; ++legacy) {
    build_crc_lane_tables(legacy != 0, L);
    for (int t = 0; t < 40; ++t) {
      uint8_t c[1024];
      for (auto& b : c) b = t == 0 ? 0xFF : t == 1 ? 0x80 : t == 2 ? 0 : static_cast<uint8_t>(rng());
      int bad = 0;
      ++checks;
      const uint32_t got = mfma_chunk_crc(*L, c, &bad), want = chunk_crc(*L, c);
      if (got != want || bad) {
        ++failures;
        std::printf("FAIL mfma legacy=%d t=%d got %08x want %08x (low bits set %d)\n", legacy, t, got, want, bad);
      }
    }
  }
  std::printf("%d checks, %d failures\n", checks, failures);
  return failures ? 1 : 0;
}
