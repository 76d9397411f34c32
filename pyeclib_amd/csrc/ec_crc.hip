// Inline CRC-32 of fragment payloads on the GPU (chksum_type 'inline_crc32'):
// the finishing pass.
//
// Replaces, for the batch paths, what liberasurecode does on the host after
// encoding or reconstructing: set_checksum (crc32(0, payload, size) into
// chksum[0]) and set_metadata_chksum (crc32 of the 59-byte metadata block at
// offset 67) (upstream erasurecode_helpers.c; pyeclib enables it through
// core.py:59-63 -> pyeclib_c.c:248), zlib's CRC or, with
// LIBERASURECODE_WRITE_LEGACY_CRC, liberasurecode's legacy one.
//
// The region kernel that wrote the payloads left one raw CRC per 1 KiB
// chunk of their interior (crc_device.hpp chunk_crc).  One block per
// fragment: its threads shift those partials to the end of the payload
// (Z_{1024 a} by the binary expansion of a, then Z_{bs mod 1024} once for
// all), its waves take the raw CRC of the payload past them -- the edge
// items' bytes, read back in 1 KiB chunks aligned to the END of the payload,
// so the leading bytes that belong to the interior count as zeros (a zero
// prefix leaves a raw CRC unchanged) and nothing past bs enters -- and
// thread 0 folds in the init / final XORs and patches the header.  Every
// linear map is 8 nibble lookups in LDS.
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

// LDS: the raw16 table (CrcLaneTables::raw16) at 0, CrcFinishTables after
// it, 8 wave partials -- 17 KiB, so eight blocks fit a CU.
constexpr uint32_t kFin = sizeof(CrcLaneTables::raw16);
constexpr uint32_t kPow = kFin + offsetof(CrcFinishTables, pow);
constexpr uint32_t kZr = kFin + offsetof(CrcFinishTables, zr);
constexpr uint32_t kMeta = kFin + offsetof(CrcFinishTables, meta);
constexpr uint32_t kZ16 = kFin + offsetof(CrcFinishTables, z16);
constexpr uint32_t kInit = kFin + offsetof(CrcFinishTables, init_term);
constexpr uint32_t kRed = kFin + sizeof(CrcFinishTables);
constexpr uint32_t kLds = kRed + 32;
constexpr uint32_t kThreads = 256;
static_assert(offsetof(CrcLaneTables, raw16) == 0 && kFin % 16 == 0, "raw16 first");

// Z_{1024 d}(r) by the binary expansion of d.
__device__ __forceinline__ uint32_t shift_chunks(uint32_t r, uint32_t d) {
  while (d != 0) {
    const uint32_t i = static_cast<uint32_t>(__builtin_ctz(d));
    r = zmap(r, kPow + 512u * i);
    d &= d - 1;
  }
  return r;
}

// 16 payload bytes at [start, start + 16), those outside [lo, hi) as zero.
__device__ __forceinline__ uint4 window16(const uint8_t* pay, int64_t start, int64_t lo, int64_t hi) {
  if (start >= lo && start + 16 <= hi) {
    uint4 x;
    __builtin_memcpy(&x, pay + start, 16);  // unaligned when bs is not a multiple of 16
    return x;
  }
  uint32_t w[4] = {0, 0, 0, 0};
  if (start + 16 > lo && start < hi)
    for (int b = 0; b < 16; ++b) {
      const int64_t at = start + b;
      if (at >= lo && at < hi) w[b >> 2] |= static_cast<uint32_t>(pay[at]) << (8 * (b & 3));
    }
  return make_uint4(w[0], w[1], w[2], w[3]);
}

// The raw CRC of 64 consecutive pieces, piece l in lane l, whose pieces are
// `unit` bytes each with tab_k = Z_{unit * 2^k} at LDS byte tab + 512 k: a
// six-level tree in which every lane applies the same map (one table per
// lookup instruction: no divergence, no bank conflicts).  Level k joins the
// halves of each group of 2^(k+1) lanes at the group's last lane:
// raw(A || B) = Z_|B|(raw A) ^ raw B.  The result is lane 63's.
__device__ __forceinline__ uint32_t lane_tree(uint32_t v, uint32_t tab) {
#pragma unroll
  for (int k = 0; k < 6; ++k) v = zmap(__shfl_up(v, 1u << k, 64), tab + 512u * k) ^ v;
  return __shfl(v, 63, 64);
}

// Round 5: the interior partials are folded by trees of uniform maps (each
// thread a run of L chunks, Horner by Z_1024; then Z_{1024 L 2^k} across the
// lanes and Z_{1024 64 L} across the waves) instead of every partial shifted
// by its own binary expansion -- divergent lookups into 22 tables 512 B
// apart, which the LDS served with 46 % bank-conflict cycles -- and an edge
// chunk's lanes by the Z_{16 2^k} tree instead of the 32 KiB lane-minor map,
// so the block's tables shrink from 46 to 17 KiB.
__global__ void __launch_bounds__(kThreads) crc_finish_kernel(CrcFinishParams p) {
  {
    auto* dst = reinterpret_cast<__attribute__((address_space(3))) v4u*>(static_cast<uintptr_t>(0));
    const v4u* raw16 = reinterpret_cast<const v4u*>(p.lanes);
    for (uint32_t i = threadIdx.x; i < kFin / 16; i += kThreads) dst[i] = raw16[i];
    const v4u* fin = reinterpret_cast<const v4u*>(p.tables);
    for (uint32_t i = threadIdx.x; i < sizeof(CrcFinishTables) / 16; i += kThreads)
      dst[kFin / 16 + i] = fin[i];
  }
  __syncthreads();
  auto* red = reinterpret_cast<__attribute__((address_space(3))) uint32_t*>(
      static_cast<uintptr_t>(kRed));
  const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const uint32_t nfull = p.bs / 1024;
  const uint32_t n = p.chunks;
  // runs of L = 2^lg chunks per thread, 256 L >= n; the 256 L - n virtual
  // chunks in front are zeros (a zero prefix leaves a raw CRC unchanged)
  uint32_t lg = 0;
  while ((kThreads << lg) < n) ++lg;
  const uint32_t L = 1u << lg;
  const int64_t lead = static_cast<int64_t>(kThreads << lg) - n;
  const int64_t e0 = static_cast<int64_t>(n) * 1024, bs = p.bs;
  const uint32_t n_edge = static_cast<uint32_t>((bs - e0 + 1023) / 1024);
  for (uint32_t f = blockIdx.x; f < p.n_obj * p.count; f += gridDim.x) {
    const uint32_t o = f / p.count, r = f - o * p.count;
    uint8_t* frag = p.frags + static_cast<uint64_t>(o) * p.stripe_stride + r * p.frag_stride;
    const uint8_t* pay = frag + 80;
    const uint32_t* part =
        p.part + static_cast<uint64_t>(o) * n * p.part_rows + p.part_row0 + r;
    // this thread's run, then the lane tree (Z_{1024 L 2^k} = pow[lg + k])
    uint32_t acc = 0;
    for (uint32_t j = 0; j < L; ++j) {
      const int64_t c = static_cast<int64_t>(threadIdx.x) * L + j - lead;
      const uint32_t x = c >= 0 ? part[static_cast<uint64_t>(c) * p.part_rows] : 0u;
      acc = (j == 0 ? 0u : zmap(acc, kPow)) ^ x;
    }
    acc = lane_tree(acc, kPow + 512u * lg);
    // the edge bytes [e0, bs) in chunks ending at bs, 1024 j before it
    uint32_t edge = 0;
    for (uint32_t j = wave; j < n_edge; j += 4) {
      const int64_t start = bs - 1024 * static_cast<int64_t>(j + 1) + 16 * lane;
      const uint32_t v = lane_tree(crcdev::raw16(window16(pay, start, e0, bs), 0), kZ16);
      edge ^= shift_chunks(v, j);
    }
    if (lane == 0) {
      red[wave] = acc;
      red[4 + wave] = edge;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      // the four waves' runs (64 L chunks each) joined by Z_{1024 64 L}, the
      // whole shifted from chunk n's end to nfull's, then by bs mod 1024
      uint32_t a = red[0];
      for (int w = 1; w < 4; ++w) a = zmap(a, kPow + 512u * (lg + 6)) ^ red[w];
      a = shift_chunks(a, nfull - n);
      const uint32_t e = red[4] ^ red[5] ^ red[6] ^ red[7];
      crcdev::patch_header(frag, zmap(a, kZr) ^ e ^ lds32(kInit), kMeta);
    }
    __syncthreads();  // red[] is reused by the next fragment
  }
}

}  // namespace

hipError_t launch_crc_finish(const CrcFinishParams& p, hipStream_t stream) {
  const uint32_t total = p.n_obj * p.count;
  if (total == 0) return hipSuccess;
  int dev = 0, cus = 256;
  if (hipGetDevice(&dev) == hipSuccess)
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  // eight blocks' LDS and waves fit a CU: one fragment per block for
  // batches up to that
  const uint32_t grid = std::min<uint32_t>(total, static_cast<uint32_t>(cus) * 8);
  hipLaunchKernelGGL(crc_finish_kernel, dim3(grid), dim3(kThreads), kLds, stream, p);
  return hipGetLastError();
}

}  // namespace ecamd
