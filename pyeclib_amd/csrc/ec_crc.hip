// Inline CRC-32 of fragment payloads on the GPU (chksum_type 'inline_crc32').
//
// Replaces, for the batch path, what liberasurecode does on the host after
// encoding: set_checksum (zlib crc32(0, payload, size) into chksum[0]) and
// set_metadata_chksum (crc32 of the 59-byte metadata block at offset 67)
// (upstream erasurecode_helpers.c; pyeclib enables it through
// core.py:59-63 -> pyeclib_c.c:248).
//
// One workgroup per fragment.  Lane i owns the 16-B chunks i, i+256, ... of
// the payload (every step is one coalesced 4 KiB read) and keeps their raw
// CRC in Horner form acc = Z_4096(acc) ^ raw16(chunk); a tree over the 256
// lanes (Z_{16*2^l} at level l) joins them, the zero padding past the payload
// is removed with Z_pad^-1, and the init/final XORs are folded in at the end
// (crc32.hpp: CrcTables).  Every linear map is 8 nibble lookups in LDS.
#include <algorithm>
#include <cstddef>

#include "crc32.hpp"
#include "crc_device.hpp"
#include "ec_crc.hpp"

namespace ecamd {
namespace {

using crcdev::lds32;
using crcdev::zmap;

typedef unsigned int v4u __attribute__((ext_vector_type(4)));

constexpr uint32_t kRaw16 = offsetof(CrcTables, raw16);
constexpr uint32_t kZ4096 = offsetof(CrcTables, z4096);
constexpr uint32_t kLevel = offsetof(CrcTables, level);
constexpr uint32_t kUnshift = offsetof(CrcTables, unshift);
constexpr uint32_t kT0 = offsetof(CrcTables, t0);
constexpr uint32_t kInit = offsetof(CrcTables, init_term);

__device__ __forceinline__ uint32_t raw16(const uint4& x) { return crcdev::raw16(x, kRaw16); }

constexpr int kAhead = 4;

// Step s's 16-B piece of this thread: (s * 256 + thread) * 16 bytes into the
// payload; bytes past bs count as zero padding.
__device__ __forceinline__ uint4 piece(const uint8_t* pay, uint32_t s, uint32_t bs) {
  const uint32_t off = (s * 256 + threadIdx.x) * 16;
  if (off + 16 <= bs) {
    const v4u v = __builtin_nontemporal_load(reinterpret_cast<const v4u*>(pay + off));
    return make_uint4(v.x, v.y, v.z, v.w);
  }
  uint32_t w[4] = {0, 0, 0, 0};
  for (uint32_t b = 0; off + b < bs && b < 16; ++b)  // payload tail (rare)
    w[b >> 2] |= static_cast<uint32_t>(pay[off + b]) << (8 * (b & 3));
  return make_uint4(w[0], w[1], w[2], w[3]);
}

__global__ void __launch_bounds__(256) crc_kernel(CrcParams p) {
  {
    auto* dst = reinterpret_cast<__attribute__((address_space(3))) v4u*>(static_cast<uintptr_t>(0));
    const v4u* src = reinterpret_cast<const v4u*>(p.tables);
    for (uint32_t i = threadIdx.x; i < sizeof(CrcTables) / 16; i += blockDim.x) dst[i] = src[i];
  }
  __syncthreads();
  __attribute__((address_space(3))) uint32_t* partial =
      reinterpret_cast<__attribute__((address_space(3))) uint32_t*>(
          static_cast<uintptr_t>(sizeof(CrcTables)));
  const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const uint32_t total = p.n_obj * p.count;
  for (uint32_t f = blockIdx.x; f < total; f += gridDim.x) {
    const uint32_t o = f / p.count, i = p.first + (f - o * p.count);
    uint8_t* frag = p.frags + static_cast<uint64_t>(o) * p.stripe_stride + i * p.frag_stride;
    const uint8_t* pay = frag + 80;
    // kAhead pieces in flight per lane: without the prefetch every step was
    // one dependent HBM round trip per 16 B (measured round 2: inline-CRC
    // encode 455 us against 310 plain at 256 x 4 MiB, profiles/r02o)
    uint4 q[kAhead];
#pragma unroll
    for (int i = 0; i < kAhead; ++i) q[i] = piece(pay, i, p.bs);
    uint32_t acc = 0;
    for (uint32_t s0 = 0; s0 < p.steps; s0 += kAhead) {
#pragma unroll
      for (int i = 0; i < kAhead; ++i) {
        const uint4 x = q[i];
        q[i] = piece(pay, s0 + i + kAhead, p.bs);
        if (s0 + i < p.steps) acc = zmap(acc, kZ4096) ^ raw16(x);
      }
    }
    // lane tree inside the wave: level l joins lanes i and i + 2^l
#pragma unroll
    for (int l = 0; l < 6; ++l) {
      const uint32_t other = __shfl_down(acc, 1u << l, 64);
      acc = zmap(acc, kLevel + 512 * l) ^ other;
    }
    if (lane == 0) partial[wave] = acc;
    __syncthreads();
    if (threadIdx.x == 0) {
      const uint32_t a = zmap(partial[0], kLevel + 512 * 6) ^ partial[1];
      const uint32_t b = zmap(partial[2], kLevel + 512 * 6) ^ partial[3];
      const uint32_t raw = zmap(zmap(a, kLevel + 512 * 7) ^ b, kUnshift);
      crcdev::patch_header(frag, raw ^ lds32(kInit), kT0);
    }
    __syncthreads();  // partial[] is reused by the next fragment
  }
}

// LDS of the finishing pass: the CrcTables maps (raw16, z4096, level) at 0,
// then the CrcFinishTables.
constexpr uint32_t kFMaps = offsetof(CrcTables, unshift);
constexpr uint32_t kFPow = kFMaps + offsetof(CrcFinishTables, pow);
constexpr uint32_t kFUnshift = kFMaps + offsetof(CrcFinishTables, unshift);
constexpr uint32_t kFT0 = kFMaps + offsetof(CrcFinishTables, t0);
constexpr uint32_t kFInit = kFMaps + offsetof(CrcFinishTables, init_term);
constexpr uint32_t kFRed = kFMaps + sizeof(CrcFinishTables);  // 4 wave partials
constexpr uint32_t kFLds = kFRed + 16;

// Z_{4096 * d}(r) by the binary expansion of d.
__device__ __forceinline__ uint32_t shift_tiles(uint32_t r, uint32_t d) {
  for (int i = 0; d != 0 && i < kCrcPowBits; ++i, d >>= 1)
    if (d & 1u) r = zmap(r, kFPow + 512u * i);
  return r;
}

// First interior item of block b of the encode launch (encode_crc_interior).
__device__ __forceinline__ uint64_t run_begin(uint64_t n, uint32_t b, uint32_t g) {
  return n * b / g;
}

// One block per parity fragment (object o, row row0 + f % nrows).
__global__ void __launch_bounds__(256) crc_finish_kernel(CrcFinishParams p) {
  {
    auto* dst = reinterpret_cast<__attribute__((address_space(3))) v4u*>(static_cast<uintptr_t>(0));
    const v4u* maps = reinterpret_cast<const v4u*>(p.maps);
    for (uint32_t i = threadIdx.x; i < kFMaps / 16; i += blockDim.x) dst[i] = maps[i];
    const v4u* fin = reinterpret_cast<const v4u*>(p.tables);
    for (uint32_t i = threadIdx.x; i < sizeof(CrcFinishTables) / 16; i += blockDim.x)
      dst[kFMaps / 16 + i] = fin[i];
  }
  __syncthreads();
  auto* red = reinterpret_cast<__attribute__((address_space(3))) uint32_t*>(
      static_cast<uintptr_t>(kFRed));
  const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const uint32_t total = p.tiles + p.edge_tiles;
  for (uint32_t f = blockIdx.x; f < p.n_obj * p.nrows; f += gridDim.x) {
    const uint32_t o = f / p.nrows, row = p.row0 + (f - o * p.nrows);
    uint8_t* frag = p.parity + static_cast<uint64_t>(o) * p.stripe_stride + row * p.frag_stride;
    // edge tiles: their raw CRC from the payload (bytes past bs count as zero)
    uint32_t edge = 0;
    for (uint32_t e = 0; e < p.edge_tiles; ++e) {
      const uint32_t off = (p.tiles + e) * 4096 + threadIdx.x * 16;
      uint4 x = make_uint4(0, 0, 0, 0);
      if (off < p.bs) {  // off + 16 <= round16(bs): inside the fragment slot
        const v4u v = *reinterpret_cast<const v4u*>(frag + 80 + off);
        uint32_t w[4] = {v.x, v.y, v.z, v.w};
        const int64_t rem = static_cast<int64_t>(p.bs) - off;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int64_t valid = rem - 4 * i;
          w[i] &= valid >= 4 ? 0xFFFFFFFFu : (valid <= 0 ? 0u : (1u << (8 * valid)) - 1u);
        }
        x = make_uint4(w[0], w[1], w[2], w[3]);
      }
      uint32_t acc = crcdev::raw16(x, 0);
#pragma unroll
      for (int l = 0; l < 6; ++l) {
        const uint32_t other = __shfl_down(acc, 1u << l, 64);
        acc = zmap(acc, kLevel + 512 * l) ^ other;
      }
      if (lane == 0) red[wave] = acc;
      __syncthreads();
      if (threadIdx.x == 0) {
        const uint32_t a = zmap(red[0], kLevel + 512 * 6) ^ red[1];
        const uint32_t b = zmap(red[2], kLevel + 512 * 6) ^ red[3];
        edge ^= shift_tiles(zmap(a, kLevel + 512 * 7) ^ b, p.edge_tiles - 1 - e);
      }
      __syncthreads();
    }
    // the tail is thread 0's alone; every thread then meets the block-uniform
    // barrier below in the same iteration (red[] is reused next fragment)
    if (threadIdx.x == 0) {
      const uint32_t* part = p.part + static_cast<uint64_t>(o) * total * p.m + row;
      uint32_t acc = edge;
      if (p.tiles != 0) {
        // the runs of object o's interior items (tile_ch tiles each): cut at
        // the launch's block ranges
        const uint32_t ch = p.tile_ch, items = p.tiles / ch;
        const uint64_t n = static_cast<uint64_t>(p.n_obj) * items;
        const uint64_t lo = static_cast<uint64_t>(o) * items, hi = lo + items;
        uint32_t b = static_cast<uint32_t>(lo * p.grid / n);
        while (b > 0 && run_begin(n, b, p.grid) > lo) --b;
        while (b + 1 < p.grid && run_begin(n, b + 1, p.grid) <= lo) ++b;
        for (uint64_t s = lo; s < hi; ++b) {
          const uint64_t e = std::min<uint64_t>(b + 1 < p.grid ? run_begin(n, b + 1, p.grid) : n, hi);
          if (e <= s) continue;  // empty block range
          const uint32_t t0 = static_cast<uint32_t>(s - lo) * ch, t1 = static_cast<uint32_t>(e - lo) * ch;
          acc ^= shift_tiles(part[static_cast<uint64_t>(t0) * p.m], total - t1);
          s = e;
        }
      }
      crcdev::patch_header(frag, zmap(acc, kFUnshift) ^ lds32(kFInit), kFT0);
    }
    __syncthreads();
  }
}

}  // namespace

hipError_t launch_crc_finish(const CrcFinishParams& p, hipStream_t stream) {
  const uint32_t total = p.n_obj * p.nrows;
  if (total == 0) return hipSuccess;
  int dev = 0, cus = 256;
  if (hipGetDevice(&dev) == hipSuccess)
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  const uint32_t grid = std::min<uint32_t>(total, static_cast<uint32_t>(cus) * 4);
  hipLaunchKernelGGL(crc_finish_kernel, dim3(grid), dim3(256), kFLds, stream, p);
  return hipGetLastError();
}

hipError_t launch_crc(const CrcParams& p, hipStream_t stream) {
  const uint32_t total = p.n_obj * p.count;
  if (total == 0) return hipSuccess;
  int dev = 0, cus = 256;
  if (hipGetDevice(&dev) == hipSuccess)
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  const uint32_t grid = std::min<uint32_t>(total, static_cast<uint32_t>(cus) * 4);
  hipLaunchKernelGGL(crc_kernel, dim3(grid), dim3(256), sizeof(CrcTables) + 16, stream, p);
  return hipGetLastError();
}

}  // namespace ecamd
