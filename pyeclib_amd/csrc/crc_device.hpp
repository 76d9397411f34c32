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

// Byte b of x, times 4 (a byte-indexed table's offset): one SDWA shift.
template <int B>
__device__ __forceinline__ uint32_t byte4(uint32_t x) {
  uint32_t r;
  if constexpr (B == 0)
    asm("v_lshlrev_b32_sdwa %0, %2, %1 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_0"
        : "=v"(r) : "v"(x), "v"(2u));
  else if constexpr (B == 1)
    asm("v_lshlrev_b32_sdwa %0, %2, %1 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_1"
        : "=v"(r) : "v"(x), "v"(2u));
  else if constexpr (B == 2)
    asm("v_lshlrev_b32_sdwa %0, %2, %1 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_2"
        : "=v"(r) : "v"(x), "v"(2u));
  else
    asm("v_lshlrev_b32_sdwa %0, %2, %1 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_3"
        : "=v"(r) : "v"(x), "v"(2u));
  return r;
}

// raw_dword by byte-indexed tables (CrcLaneTables::rawb; `tab` = the lane
// tables' LDS base): 4 lookups instead of 8, one SDWA shift each for the
// address.  A 256-entry table read by 64 lanes at random shares banks
// (4 entries per bank), which nibble tables never do.
__device__ __forceinline__ uint32_t raw_dword_b(uint32_t w, int d, uint32_t tab) {
  const uint32_t t = tab + static_cast<uint32_t>(offsetof(CrcLaneTables, rawb)) + 4096u * d;
  const uint32_t a = lds32(t + byte4<0>(w)) ^ lds32(t + 1024 + byte4<1>(w)) ^
                     lds32(t + 2048 + byte4<2>(w)) ^ lds32(t + 3072 + byte4<3>(w));
  uint32_t r = a;
  asm volatile("" : "+v"(r));
  return r;
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
