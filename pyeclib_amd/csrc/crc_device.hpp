// Device side of the GPU payload CRC-32: GF(2)-linear maps applied by
// nibble-table lookups in LDS (tables built by crc32.cpp, layout
// [q 0..7][v 0..15] u32 per 32-bit map; [p 0..31][v 0..15] for raw16).
// Shared by the CRC pass (ec_crc.hip) and the fused parity CRC of the encode
// kernel (ec_kernels_impl.hpp).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

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

// zlib crc32 of the 59-byte metadata block of a header held as 16 dwords
// (bytewise table t0 at LDS byte `t0`).
__device__ __forceinline__ uint32_t meta_crc(const uint32_t (&h)[16], uint32_t t0) {
  uint32_t m = 0xFFFFFFFFu;
  for (int b = 0; b < 59; ++b) m = lds32(t0 + 4 * ((m ^ byte_of(h[b >> 2], b & 3)) & 0xFF)) ^ (m >> 8);
  return m ^ 0xFFFFFFFFu;
}

// Patch chksum[0] (header bytes 21..24) with `crc` and then the metadata
// checksum (bytes 67..70) of the fragment header at `frag`.
__device__ __forceinline__ void patch_header(uint8_t* frag, uint32_t crc, uint32_t t0) {
  uint32_t h[16];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const uint4 v = reinterpret_cast<const uint4*>(frag)[q];
    h[4 * q] = v.x;
    h[4 * q + 1] = v.y;
    h[4 * q + 2] = v.z;
    h[4 * q + 3] = v.w;
  }
  // chksum occupies bytes 21..24: bytes 21..23 in h[5] (bits 8..31), 24 in h[6]
  h[5] = (h[5] & 0x000000FFu) | (crc << 8);
  h[6] = (h[6] & 0xFFFFFF00u) | (crc >> 24);
  const uint32_t m = meta_crc(h, t0);
  for (int b = 21; b < 25; ++b) frag[b] = static_cast<uint8_t>(crc >> (8 * (b - 21)));
  for (int b = 67; b < 71; ++b) frag[b] = static_cast<uint8_t>(m >> (8 * (b - 67)));
}

}  // namespace crcdev
}  // namespace ecamd
