// Device side of the GPU payload CRC-32: GF(2)-linear maps applied by
// nibble-table lookups in LDS (tables built by crc32.cpp, layout
// [q 0..7][v 0..15] u32 per 32-bit map; [p 0..31][v 0..15] for raw16;
// CrcLaneTables::lane [q][v][lane]).  Shared by the region kernels, which
// take each 1 KiB chunk's raw CRC as they write it (ec_kernels_impl.hpp), and
// the finishing pass (ec_crc.hip).
#pragma once

#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdint>

#include "crc32.hpp"

namespace ecamd {
namespace crcdev {

typedef __attribute__((address_space(3))) char lds_char;

__device__ __forceinline__ uint32_t lds32(uint32_t byte) {
  return *reinterpret_cast<const __attribute__((address_space(3))) uint32_t*>(
      reinterpret_cast<const lds_char*>(static_cast<uintptr_t>(byte)));
}

__device__ __forceinline__ uint32_t byte_of(uint32_t x, int b) { return (x >> (8 * b)) & 0xFFu; }

// map(r) = XOR over the 8 nibbles of r of the map's table at LDS byte `tab`.
__device__ __forceinline__ uint32_t zmap(uint32_t r, uint32_t tab) {
  const uint32_t lo = (r << 2) & 0x3C3C3C3Cu, hi = (r >> 2) & 0x3C3C3C3Cu;
  uint32_t a = 0;
#pragma unroll
  for (int b = 0; b < 4; ++b)
    a ^= lds32(tab + 128 * b + byte_of(lo, b)) ^ lds32(tab + 128 * b + 64 + byte_of(hi, b));
  asm volatile("" : "+v"(a));  // materialised here (see raw16)
  return a;
}

// Raw CRC (zero start, no final XOR) of one 16-byte piece: 32 nibble lookups
// in the raw16 table at LDS byte `tab`.
__device__ __forceinline__ uint32_t raw16(const uint4& x, uint32_t tab) {
  const uint32_t w[4] = {x.x, x.y, x.z, x.w};
  uint32_t a = 0;
#pragma unroll
  for (int d = 0; d < 4; ++d) {
    const uint32_t lo = (w[d] << 2) & 0x3C3C3C3Cu, hi = (w[d] >> 2) & 0x3C3C3C3Cu;
#pragma unroll
    for (int b = 0; b < 4; ++b) {
      const uint32_t p = 8 * d + 2 * b;  // nibble position of the byte's low nibble
      a ^= lds32(tab + 64 * p + byte_of(lo, b)) ^ lds32(tab + 64 * (p + 1) + byte_of(hi, b));
    }
    // one dword's 8 lookups at a time: otherwise hipcc hoists all 32 (and
    // those of the next call) ahead of the XORs, one VGPR each.  The pin
    // keeps the XORs from sinking, the memory clobber the lookups from
    // rising, at the IR level (ec_kernels_impl.hpp lookup_fence).
    asm volatile("" : "+v"(a));
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("" ::: "memory");
  }
  return a;
}

// raw16 without the per-dword fences: the 32 lookups of a piece may all be
// in flight at once (for kernels with registers to spare -- the loader /
// consumer encode -- where the fenced form's 4 dependent LDS round trips
// per row and chunk left the CRC latency-bound).
__device__ __forceinline__ uint32_t raw16_free(const uint4& x, uint32_t tab) {
  const uint32_t w[4] = {x.x, x.y, x.z, x.w};
  uint32_t a = 0;
#pragma unroll
  for (int d = 0; d < 4; ++d) {
    const uint32_t lo = (w[d] << 2) & 0x3C3C3C3Cu, hi = (w[d] >> 2) & 0x3C3C3C3Cu;
#pragma unroll
    for (int b = 0; b < 4; ++b) {
      const uint32_t p = 8 * d + 2 * b;
      a ^= lds32(tab + 64 * p + byte_of(lo, b)) ^ lds32(tab + 64 * (p + 1) + byte_of(hi, b));
    }
  }
  return a;
}

// Dword d's share of raw16 (raw16(x) = XOR of raw_dword(x[d], d) over d):
// 8 nibble lookups, for callers that spread a piece's CRC over time.
__device__ __forceinline__ uint32_t raw_dword(uint32_t w, int d, uint32_t tab) {
  const uint32_t lo = (w << 2) & 0x3C3C3C3Cu, hi = (w >> 2) & 0x3C3C3C3Cu;
  uint32_t a = 0;
#pragma unroll
  for (int b = 0; b < 4; ++b) {
    const uint32_t p = 8 * d + 2 * b;
    a ^= lds32(tab + 64 * p + byte_of(lo, b)) ^ lds32(tab + 64 * (p + 1) + byte_of(hi, b));
  }
  asm volatile("" : "+v"(a));
  return a;
}

// Z_{16 (63 - l)}(r) for this lane: the lane-minor tables at LDS byte
// `tab`, lane4 = 4 * lane.
__device__ __forceinline__ uint32_t lane_map(uint32_t r, uint32_t tab, uint32_t lane4) {
  uint32_t a = 0;
#pragma unroll
  for (int q = 0; q < 8; ++q) a ^= lds32(tab + 4096u * q + (((r >> (4 * q)) & 15u) << 8) + lane4);
  asm volatile("" : "+v"(a));
  return a;
}

// XOR of a over the 64 lanes of the wave (wave-uniform): DPP within each row
// of 16 lanes, then the four rows' values read out.
__device__ __forceinline__ uint32_t wave_xor(uint32_t a) {
  a ^= static_cast<uint32_t>(__builtin_amdgcn_update_dpp(0, static_cast<int>(a), 0xB1, 0xF, 0xF, false));
  a ^= static_cast<uint32_t>(__builtin_amdgcn_update_dpp(0, static_cast<int>(a), 0x4E, 0xF, 0xF, false));
  a ^= static_cast<uint32_t>(__builtin_amdgcn_update_dpp(0, static_cast<int>(a), 0x141, 0xF, 0xF, false));
  a ^= static_cast<uint32_t>(__builtin_amdgcn_update_dpp(0, static_cast<int>(a), 0x140, 0xF, 0xF, false));
  return __builtin_amdgcn_readlane(a, 0) ^ __builtin_amdgcn_readlane(a, 16) ^
         __builtin_amdgcn_readlane(a, 32) ^ __builtin_amdgcn_readlane(a, 48);
}

// ---- matrix-core form (CrcLaneTables::mst / mfb; crc32.cpp builds them) ----
// raw(chunk) is a GF(2)-linear map of its 8192 bits.  Over the integers,
// with the bits as 0/1 values, each output bit is the parity of a sum of
// products -- a matrix product, which v_mfma_i32_32x32x32_i8 takes 32 K at a
// time.  Plane b of the lane's piece (its 16 bytes masked to bit b, 2^b or 0)
// times B (the map's 0/1 entries scaled by 2^(7 - b)) puts every term at
// 128 (mod 256), so bit 7 of each i32 sum is the parity: 8 instructions (one
// per plane) give C[r][n] = bit n of u_r, row r = lanes r and r + 32 (the
// second one's Z_512 folded into its B rows), and raw(chunk) = XOR_r
// Z_{16 (31 - r)}(u_r): per lane 16 parities of one column, 4 nibble
// lookups, the wave XOR.  Against the 40 lookups of raw16 + lane_map.
typedef int mfma_v4i __attribute__((ext_vector_type(4)));
typedef int mfma_v16i __attribute__((ext_vector_type(16)));

// This lane's B operands of the 8 planes, from the tables in device memory.
__device__ __forceinline__ void mfma_load_b(const void* lanes, uint32_t lane, mfma_v4i (&b)[8]) {
  const mfma_v4i* t = reinterpret_cast<const mfma_v4i*>(static_cast<const char*>(lanes) +
                                                        offsetof(CrcLaneTables, mfb));
#pragma unroll
  for (int s = 0; s < 8; ++s) b[s] = t[s * 64 + lane];
}

// Plane s of the piece x into the row sums (s a constant after unrolling).
// Only the bits BELOW s need clearing: a bit above it lands on a multiple of
// 256 (2^(7 - s) times 2^(s + 1) or more), which leaves bit 7 alone -- so
// plane 0 takes the bytes as they are.
__device__ __forceinline__ mfma_v16i mfma_plane(const uint4& x, int s, const mfma_v4i& b, const mfma_v16i& acc) {
  const uint32_t m = (0xFFu << s & 0xFFu) * 0x01010101u;
  const mfma_v4i a = s == 0 ? mfma_v4i{static_cast<int>(x.x), static_cast<int>(x.y), static_cast<int>(x.z),
                                       static_cast<int>(x.w)}
                            : mfma_v4i{static_cast<int>(x.x & m), static_cast<int>(x.y & m),
                                       static_cast<int>(x.z & m), static_cast<int>(x.w & m)};
  return __builtin_amdgcn_mfma_i32_32x32x32_i8(a, b, acc, 0, 0, 0);
}

// This lane's share of the chunk's raw CRC from its row sums (mst at LDS
// byte `tab`): the parities of accumulators 4q .. 4q + 3 (byte 0 is 0x00 or
// 0x80) weighted into nibble q's table offset by v_dot4, one lookup per
// nibble.  The 4 lookups are independent (one wait).
__device__ __forceinline__ uint32_t mfma_lanes(const mfma_v16i& c, uint32_t tab, uint32_t lane4) {
  uint32_t x[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    x[q] = tab + 4096u * q + lane4;
    x[q] = __builtin_amdgcn_udot4(static_cast<uint32_t>(c[4 * q]), 0x02u, x[q], false);
    x[q] = __builtin_amdgcn_udot4(static_cast<uint32_t>(c[4 * q + 1]), 0x04u, x[q], false);
    x[q] = __builtin_amdgcn_udot4(static_cast<uint32_t>(c[4 * q + 2]), 0x08u, x[q], false);
    x[q] = __builtin_amdgcn_udot4(static_cast<uint32_t>(c[4 * q + 3]), 0x10u, x[q], false);
  }
  const uint32_t a = lds32(x[0]) ^ lds32(x[1]) ^ lds32(x[2]) ^ lds32(x[3]);
  uint32_t r = a;
  asm volatile("" : "+v"(r));
  return r;
}

// Raw CRC of the chunk (wave-uniform).
__device__ __forceinline__ uint32_t mfma_finish(const mfma_v16i& c, uint32_t tab, uint32_t lane4) {
  return wave_xor(mfma_lanes(c, tab, lane4));
}

// Each lane keeps one of a, b and hands the other to its partner (DPP CTRL),
// which keeps that one: the XOR is then over the pair of lanes, a in the
// lanes where `odd` is false, b in the others.
template <int CTRL>
__device__ __forceinline__ uint32_t fold_pair(bool odd, uint32_t a, uint32_t b) {
  const uint32_t keep = odd ? b : a, give = odd ? a : b;
  return keep ^ static_cast<uint32_t>(__builtin_amdgcn_update_dpp(0, static_cast<int>(give), CTRL, 0xF, 0xF, false));
}

// XOR over the wave of four per-lane values at once: lane l returns the
// total of value l mod 4 (lanes 0..3 hold the four totals).  Two DPP
// exchanges that halve the values while doubling the lanes each total
// covers, then two rotations within 16 lanes and the two permlane swaps:
// 15 instructions for the four, against 4 x 8 for wave_xor.
__device__ __forceinline__ uint32_t wave_xor4(uint32_t v0, uint32_t v1, uint32_t v2, uint32_t v3, uint32_t lane) {
  const bool o1 = lane & 1, o2 = lane & 2;
  const uint32_t u0 = fold_pair<0xB1>(o1, v0, v1);  // quad_perm [1,0,3,2]: lane ^ 1
  const uint32_t u1 = fold_pair<0xB1>(o1, v2, v3);
  uint32_t w = fold_pair<0x4E>(o2, u0, u1);          // quad_perm [2,3,0,1]: lane ^ 2
  w ^= static_cast<uint32_t>(__builtin_amdgcn_update_dpp(0, static_cast<int>(w), 0x124, 0xF, 0xF, false));  // row_ror:4
  w ^= static_cast<uint32_t>(__builtin_amdgcn_update_dpp(0, static_cast<int>(w), 0x128, 0xF, 0xF, false));  // row_ror:8
  const auto h = __builtin_amdgcn_permlane16_swap(w, w, false, false);
  w = h[0] ^ h[1];
  const auto f = __builtin_amdgcn_permlane32_swap(w, w, false, false);
  return f[0] ^ f[1];
}

// Raw CRC of the wave's 1 KiB chunk, lane l holding bytes [16 l, 16 l + 16)
// in v (CrcLaneTables at LDS byte `tab`): wave-uniform.  FREE: raw16_free.
template <bool FREE = false>
__device__ __forceinline__ uint32_t chunk_crc(const uint4& v, uint32_t tab, uint32_t lane4) {
  const uint32_t r = FREE ? raw16_free(v, tab) : raw16(v, tab);
  return wave_xor(lane_map(r, tab + offsetof(CrcLaneTables, lane), lane4));
}

// Set chksum[0] (header bytes 21..24) of the fragment header at `frag` to
// `crc` (it was 0) and update the metadata checksum (bytes 67..70) by the
// change that makes (CrcFinishTables::meta at LDS byte `meta`).
__device__ __forceinline__ void patch_header(uint8_t* frag, uint32_t crc, uint32_t meta) {
  const uint32_t d = zmap(crc, meta);
  for (int b = 0; b < 4; ++b) {
    frag[21 + b] = static_cast<uint8_t>(crc >> (8 * b));
    frag[67 + b] = static_cast<uint8_t>(frag[67 + b] ^ (d >> (8 * b)));
  }
}

}  // namespace crcdev
}  // namespace ecamd
