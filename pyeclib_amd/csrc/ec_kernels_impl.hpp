// gfx950 region kernels for the Reed-Solomon codes: templates behind
// ec_kernels.hpp, instantiated per field by ec_gf16.hip and ec_gf8.hip.
//
// Hot loops replaced: liberasurecode_rs_vand's region_dot_product /
// region_multiply / region_xor (upstream src/builtin/rs_vand/
// liberasurecode_rs_vand.c), which walks one 16-bit word at a time through a
// 64 K-entry log/antilog table on one CPU thread; and ISA-L's ec_encode_data
// (GF(2^8)), behind liberasurecode's isa_l_rs_vand / isa_l_rs_cauchy.
//
// Arithmetic.  Multiplication by a constant c is GF(2)-linear, so over
// GF(2^16)
//   c * x = T[0][x & 15] ^ T[1][(x>>4) & 15] ^ T[2][(x>>8) & 15] ^ T[3][x>>12]
// with T[q][v] = c * (v << 4q), and over GF(2^8) two such tables.  One table
// entry packs the products for up to four output rows (u64 = 4 x 16 bits,
// u32 = 4 x 8 bits), so one LDS read per nibble feeds all four outputs.  A
// 16-entry table spans 32 (u64) or 16 (u32) LDS banks: the lanes of one
// ds_read lane group can never hit one bank with two different addresses, so
// every lookup is conflict-free whatever the data.
//
// Addressing (GF(2^16)).  Table entry (c, q, v) sits at byte
// 512c + 256(q >> 1) + 16v + 8(q & 1) (gf16.hpp), so the lookup address of
// a nibble is the nibble times 16 plus a compile-time offset that rides in
// the ds_read immediate (the input loop is unrolled over a compile-time k).
// Byte b of an input dword x holds nibble positions q = 2(b & 1) and
// 2(b & 1) + 1 of symbol b >> 1; their addresses are byte b of (x << 4)
// and of x, masked with 0xF0.  Encode's tables sit at LDS 0, so one
// v_and_b32_sdwa (src0_sel:BYTE_b) makes each address: 9 VALU ops for the
// eight lookups of a dword.  Decode's table set lives in one of two slots,
// so its addresses also carry the slot base: one v_perm_b32 per lookup
// assembles {masked byte, base >> 8} (11 ops per dword).  GF(2^8) uses
// 128-B tables, 4-byte entries, one byte per symbol and the v_perm form.
//
// Memory.  Each lane moves 16 B per input per step (global_load_dwordx4,
// 1 KiB contiguous per wave-instruction); inputs are read once from HBM and
// every output byte is written once.  Fragment payloads inside an object
// start at j*bs, which is only 2-byte (GF(2^16)) or 1-byte aligned: encode
// reads those slices with gfx9's unaligned loads; decode writes them as
// realigned 16-B units (see "Realigned object stores").
#pragma once

#include <algorithm>
#include <cstdlib>
#include <cstddef>
#include <type_traits>
#include <mutex>
#include <unordered_map>

#include "ec_kernels.hpp"

namespace ecamd {
namespace {

// LDS is addressed by raw byte offsets: these kernels declare no static
// __shared__ data, so the dynamic allocation (the nibble tables) starts at
// LDS address 0.  Going through an address_space(3) pointer made from the
// integer keeps hipcc from adding the symbol base to every lookup address,
// and the compile-time `tab` folds into the ds_read offset field.
typedef __attribute__((address_space(3))) char lds_char;
typedef unsigned int v2u __attribute__((ext_vector_type(2)));
typedef unsigned int v4u __attribute__((ext_vector_type(4)));
__device__ __forceinline__ uint2 lds_u64(uint32_t a, uint32_t tab) {
  const v2u v = *reinterpret_cast<const __attribute__((address_space(3))) v2u*>(
      reinterpret_cast<const lds_char*>(static_cast<uintptr_t>(a)) + tab);
  return make_uint2(v.x, v.y);
}
__device__ __forceinline__ uint32_t lds_u32(uint32_t a, uint32_t tab) {
  return *reinterpret_cast<const __attribute__((address_space(3))) uint32_t*>(
      reinterpret_cast<const lds_char*>(static_cast<uintptr_t>(a)) + tab);
}
__device__ __forceinline__ __attribute__((address_space(3))) v4u* lds_v4(uint32_t byte) {
  return reinterpret_cast<__attribute__((address_space(3))) v4u*>(static_cast<uintptr_t>(byte));
}

// Streaming global accesses: every input byte is read once and every output
// byte written once, so they bypass cache residency (nontemporal).  Measured
// on the encode stream pattern (tools/microbench.hip): 4.9 -> 5.5 TB/s.
__device__ __forceinline__ uint4 ld_stream(const void* p) {
  const v4u v = __builtin_nontemporal_load(reinterpret_cast<const v4u*>(p));
  return make_uint4(v.x, v.y, v.z, v.w);
}
__device__ __forceinline__ void st_stream(void* p, const uint4& x) {
  v4u v;
  v.x = x.x;
  v.y = x.y;
  v.z = x.z;
  v.w = x.w;
  __builtin_nontemporal_store(v, reinterpret_cast<v4u*>(p));
}

// Buffer access to the interior streams: a wave-uniform descriptor per
// object (base made provably uniform with readfirstlane, so hipcc builds it
// in SGPRs without a waterfall loop: cdna_hip_programming.md T20), the lane's
// 16*lane in voffset and every per-input / per-output offset in soffset, so
// all K loads and stores of a chunk share ONE address VGPR instead of a
// 64-bit address pair each.  aux 2 = nt (streamed once).
typedef __amdgpu_buffer_rsrc_t Rsrc;
constexpr int kNt = 2;
// `records` = bytes addressable through the descriptor; a zero-record
// descriptor turns its loads into zeros with no memory access at all (the
// range check drops them), which is how a wave's last item "prefetches"
// nothing while keeping the instruction stream -- and so hipcc's wait
// counts -- identical to every other item.
__device__ __forceinline__ Rsrc rsrc(const void* base, int records = -1) {
  const uint64_t a = reinterpret_cast<uint64_t>(base);
  const uint32_t lo = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(a));
  const uint32_t hi = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(a >> 32));
  const int n = static_cast<int>(__builtin_amdgcn_readfirstlane(static_cast<uint32_t>(records)));
  return __builtin_amdgcn_make_buffer_rsrc(
      reinterpret_cast<void*>((static_cast<uint64_t>(hi) << 32) | lo), 0, n, 0x00020000);
}
// Cache policy of the interior streams (compile time; POL bits):
// nontemporal by default, kPolLoadsCached / kPolStoresCached switch loads /
// stores to the default policy (A/B variants of the benchmark case).
constexpr int kPolLoadsCached = 1, kPolStoresCached = 2;
template <bool CACHED = false>
__device__ __forceinline__ uint4 buf_ld(Rsrc r, uint32_t voff, uint32_t soff) {
  const v4u v = __builtin_amdgcn_raw_buffer_load_b128(r, voff, soff, CACHED ? 0 : kNt);
  return make_uint4(v.x, v.y, v.z, v.w);
}
template <bool CACHED = false>
__device__ __forceinline__ void buf_st(Rsrc r, uint32_t voff, uint32_t soff, const uint4& x) {
  v4u v;
  v.x = x.x;
  v.y = x.y;
  v.z = x.z;
  v.w = x.w;
  __builtin_amdgcn_raw_buffer_store_b128(v, r, voff, soff, CACHED ? 0 : kNt);
}

// a ^ b ^ c in one VALU op (gfx950 v_bitop3_b32, truth table 0x96)
__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
  return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}

// ---------------- GF(2^16): liberasurecode_rs_vand ----------------

// x & 0xF0 with x's byte B as the source operand (SDWA, gfx9): the
// lookup address of the high nibble of byte B, times 16.
#define ECAMD_SDWA_AND_BYTE(B)                                                              \
  "v_and_b32_sdwa %0, %1, %2 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_" #B \
  " src1_sel:DWORD"
template <int B>
__device__ __forceinline__ uint32_t hi_nib16(uint32_t x) {
  uint32_t r;
  if constexpr (B == 0)
    r = x & 0xF0u;
  else if constexpr (B == 1)
    asm(ECAMD_SDWA_AND_BYTE(1) : "=v"(r) : "v"(x), "v"(0xF0u));
  else if constexpr (B == 2)
    asm(ECAMD_SDWA_AND_BYTE(2) : "=v"(r) : "v"(x), "v"(0xF0u));
  else
    asm(ECAMD_SDWA_AND_BYTE(3) : "=v"(r) : "v"(x), "v"(0xF0u));
  return r;
}
#undef ECAMD_SDWA_AND_BYTE

// NW = 2: u64 entries (up to 4 rows); NW = 1: rows <= 2, read the low dword
// only (ds_read_b32; same table layout).
template <int NW>
struct Gf16 {
  static constexpr uint32_t kW = 16;
  static constexpr uint32_t kTableBytes = 512;
  struct Acc {
    uint2 s[8];  // s[2d] / s[2d+1]: rows 0-3 of the low / high symbol of input dword d
  };
  // second byte of a lookup address: the table set's LDS base (a multiple
  // of 256, below 64 KiB)
  static __device__ __forceinline__ uint32_t kb(uint32_t base) { return base >> 8; }
  static __device__ __forceinline__ void zero(Acc& a) {
#pragma unroll
    for (int i = 0; i < 8; ++i) a.s[i] = make_uint2(0, 0);
  }
  // Materialise the accumulators here: otherwise hipcc sinks the row 2-3 XOR
  // chains into the (runtime-conditional) store blocks and keeps every
  // looked-up table word live until then.
  static __device__ __forceinline__ void pin(Acc& a) {
#pragma unroll
    for (int i = 0; i < 8; ++i) asm volatile("" : "+v"(a.s[i].x), "+v"(a.s[i].y));
  }
  // Lookup addresses of the 8 nibbles of x, in q order per symbol:
  // a[4h + q] for symbol h (0 = low half-word).  Z: table set at LDS 0.
  template <bool Z>
  static __device__ __forceinline__ void addrs(uint32_t kb, uint32_t x, uint32_t (&a)[8]) {
    const uint32_t w = x << 4;
    if constexpr (Z) {
      a[0] = hi_nib16<0>(w);
      a[1] = hi_nib16<0>(x);
      a[2] = hi_nib16<1>(w);
      a[3] = hi_nib16<1>(x);
      a[4] = hi_nib16<2>(w);
      a[5] = hi_nib16<2>(x);
      a[6] = hi_nib16<3>(w);
      a[7] = hi_nib16<3>(x);
    } else {
      const uint32_t ml = w & 0xF0F0F0F0u, mh = x & 0xF0F0F0F0u;
#pragma unroll
      for (int b = 0; b < 4; ++b) {
        a[2 * b] = __builtin_amdgcn_perm(kb, ml, 0x0C0C0400u | b);
        a[2 * b + 1] = __builtin_amdgcn_perm(kb, mh, 0x0C0C0400u | b);
      }
    }
  }
  // immediate offset of nibble position q inside an input's 512-B table
  static constexpr uint32_t qoff(int q) { return 256u * (q >> 1) + 8u * (q & 1); }
  template <bool Z>
  static __device__ __forceinline__ void mac_dword(uint32_t kb, uint32_t tab, uint32_t x,
                                                   uint2& s_lo, uint2& s_hi) {
    uint32_t a[8];
    addrs<Z>(kb, x, a);
    if constexpr (NW == 2) {
      const uint2 e0 = lds_u64(a[0], tab + qoff(0)), e1 = lds_u64(a[1], tab + qoff(1)),
                  e2 = lds_u64(a[2], tab + qoff(2)), e3 = lds_u64(a[3], tab + qoff(3));
      const uint2 e4 = lds_u64(a[4], tab + qoff(0)), e5 = lds_u64(a[5], tab + qoff(1)),
                  e6 = lds_u64(a[6], tab + qoff(2)), e7 = lds_u64(a[7], tab + qoff(3));
      s_lo.x = xor3(xor3(s_lo.x, e0.x, e1.x), e2.x, e3.x);
      s_lo.y = xor3(xor3(s_lo.y, e0.y, e1.y), e2.y, e3.y);
      s_hi.x = xor3(xor3(s_hi.x, e4.x, e5.x), e6.x, e7.x);
      s_hi.y = xor3(xor3(s_hi.y, e4.y, e5.y), e6.y, e7.y);
    } else {
      s_lo.x = xor3(xor3(s_lo.x, lds_u32(a[0], tab + qoff(0)), lds_u32(a[1], tab + qoff(1))),
                    lds_u32(a[2], tab + qoff(2)), lds_u32(a[3], tab + qoff(3)));
      s_hi.x = xor3(xor3(s_hi.x, lds_u32(a[4], tab + qoff(0)), lds_u32(a[5], tab + qoff(1))),
                    lds_u32(a[6], tab + qoff(2)), lds_u32(a[7], tab + qoff(3)));
    }
  }
  // The scheduling barriers stop hipcc from hoisting every LDS lookup of the
  // unrolled input loop ahead of the XORs that consume them (2 VGPRs each).
  template <bool Z = false>
  static __device__ __forceinline__ void mac(uint32_t kb, uint32_t tab, const uint4& x, Acc& a) {
    mac_dword<Z>(kb, tab, x.x, a.s[0], a.s[1]);
    __builtin_amdgcn_sched_barrier(0);
    mac_dword<Z>(kb, tab, x.y, a.s[2], a.s[3]);
    __builtin_amdgcn_sched_barrier(0);
    mac_dword<Z>(kb, tab, x.z, a.s[4], a.s[5]);
    __builtin_amdgcn_sched_barrier(0);
    mac_dword<Z>(kb, tab, x.w, a.s[6], a.s[7]);
    __builtin_amdgcn_sched_barrier(0);
  }
  static __device__ __forceinline__ uint32_t pack(const uint2& lo, const uint2& hi, int r) {
    const uint32_t a = (r < 2) ? lo.x : lo.y;
    const uint32_t b = (r < 2) ? hi.x : hi.y;
    return __builtin_amdgcn_perm(b, a, (r & 1) ? 0x07060302u : 0x05040100u);
  }
  // Output row r of the 8 accumulated symbols as a 16-byte chunk.
  static __device__ __forceinline__ uint4 row(const Acc& a, int r) {
    return make_uint4(pack(a.s[0], a.s[1], r), pack(a.s[2], a.s[3], r), pack(a.s[4], a.s[5], r),
                      pack(a.s[6], a.s[7], r));
  }
};

// ---------------- GF(2^8): ISA-L layout ----------------

struct Gf8 {
  static constexpr uint32_t kW = 8;
  static constexpr uint32_t kTableBytes = 128;  // [q 0..1][v 0..15] u32
  struct Acc {
    uint32_t a[16];  // a[4d + b]: rows 0-3 (bytes 0-3) for byte b of input dword d
  };
  static __device__ __forceinline__ uint32_t kb(uint32_t base) { return base >> 8; }
  static __device__ __forceinline__ void zero(Acc& a) {
#pragma unroll
    for (int i = 0; i < 16; ++i) a.a[i] = 0;
  }
  static __device__ __forceinline__ void pin(Acc& a) {
#pragma unroll
    for (int i = 0; i < 16; ++i) asm volatile("" : "+v"(a.a[i]));
  }
  static __device__ __forceinline__ void mac_dword(uint32_t kb, uint32_t tab, uint32_t x,
                                                   uint32_t* a) {
    const uint32_t ylo = (x << 2) & 0x3C3C3C3Cu;                  // low nibbles * 4
    const uint32_t yhi = ((x >> 2) & 0x3C3C3C3Cu) | 0x40404040u;  // high nibbles * 4 + 64
#pragma unroll
    for (int b = 0; b < 4; ++b) {
      const uint32_t sel = 0x0C0C0400u | static_cast<uint32_t>(b);
      a[b] = xor3(a[b], lds_u32(__builtin_amdgcn_perm(kb, ylo, sel), tab),
                  lds_u32(__builtin_amdgcn_perm(kb, yhi, sel), tab));
    }
  }
  template <bool Z = false>
  static __device__ __forceinline__ void mac(uint32_t kb, uint32_t tab, const uint4& x, Acc& a) {
    mac_dword(kb, tab, x.x, a.a + 0);
    __builtin_amdgcn_sched_barrier(0);
    mac_dword(kb, tab, x.y, a.a + 4);
    __builtin_amdgcn_sched_barrier(0);
    mac_dword(kb, tab, x.z, a.a + 8);
    __builtin_amdgcn_sched_barrier(0);
    mac_dword(kb, tab, x.w, a.a + 12);
    __builtin_amdgcn_sched_barrier(0);
  }
  // 4x4 byte transpose: byte b of the result is byte r of a[b].
  static __device__ __forceinline__ uint32_t pack(const uint32_t* a, int r) {
    const uint32_t sel = (r < 2) ? 0x05010400u : 0x07030602u;
    const uint32_t lo = __builtin_amdgcn_perm(a[1], a[0], sel);
    const uint32_t hi = __builtin_amdgcn_perm(a[3], a[2], sel);
    return __builtin_amdgcn_perm(hi, lo, (r & 1) ? 0x07060302u : 0x05040100u);
  }
  static __device__ __forceinline__ uint4 row(const Acc& a, int r) {
    return make_uint4(pack(a.a + 0, r), pack(a.a + 4, r), pack(a.a + 8, r), pack(a.a + 12, r));
  }
};

// ---------------- common helpers ----------------

constexpr uint32_t kLanes = 64;
constexpr uint32_t kChunkBytes = kLanes * 16;  // one 16-B-per-lane wave access
constexpr uint32_t kWavesPerBlock = kThreadsPerBlock / kLanes;

__device__ __forceinline__ uint32_t lane_id() { return threadIdx.x & (kLanes - 1); }
__device__ __forceinline__ uint32_t wave_in_block() {
  return __builtin_amdgcn_readfirstlane(threadIdx.x / kLanes);
}

// 16 bytes at base+off; bytes at or past `len` read as zero (encode padding).
__device__ __forceinline__ uint4 load_clamped(const uint8_t* base, uint64_t off, uint64_t len) {
  if (off + 16 <= len) return *reinterpret_cast<const uint4*>(base + off);
  uint32_t w[4] = {0, 0, 0, 0};
  for (int i = 0; i < 16; ++i)
    if (off + i < len) w[i >> 2] |= static_cast<uint32_t>(base[off + i]) << (8 * (i & 3));
  return make_uint4(w[0], w[1], w[2], w[3]);
}

__device__ __forceinline__ uint32_t byte_of(const uint4& v, uint32_t b) {
  const uint64_t lo = v.x | (static_cast<uint64_t>(v.y) << 32);
  const uint64_t hi = v.z | (static_cast<uint64_t>(v.w) << 32);
  return static_cast<uint32_t>((b < 8 ? lo >> (8 * b) : hi >> (8 * (b - 8))) & 0xFFu);
}

// Bytes [from, from + n) of v stored at p (byte stores; run ends only).
__device__ __forceinline__ void put_bytes(uint8_t* p, const uint4& v, uint32_t from, uint32_t n) {
  for (uint32_t i = 0; i < n; ++i) p[i] = static_cast<uint8_t>(byte_of(v, from + i));
}

// Store the first `n` (> 0) bytes of v at dst.
__device__ __forceinline__ void store_partial(uint8_t* dst, const uint4& v, int64_t n) {
  if (n >= 16) {
    *reinterpret_cast<uint4*>(dst) = v;
    return;
  }
  put_bytes(dst, v, 0, static_cast<uint32_t>(n));
}

// Whole block copies `bytes` of tables from global memory to LDS byte `dst`.
__device__ __forceinline__ void load_tables(const uint32_t* src, uint32_t bytes, uint32_t dst) {
  auto* d = lds_v4(dst);
  const v4u* s = reinterpret_cast<const v4u*>(src);
  for (uint32_t i = threadIdx.x; i < bytes / 16; i += blockDim.x) d[i] = s[i];
}

// Bytes of data fragment `idx` at payload offset t that belong to the object.
__device__ __forceinline__ int64_t object_bytes(uint32_t idx, uint32_t bs, uint32_t t,
                                                uint64_t len) {
  const int64_t start = static_cast<int64_t>(idx) * bs + t;
  int64_t n = static_cast<int64_t>(bs) - t;
  const int64_t left = static_cast<int64_t>(len) - start;
  if (left < n) n = left;
  return n;
}

// ---------------- work decomposition ----------------
//
// Work item = (object o, tile): the block's 4 waves each take one chunk of
// consecutive payload positions of object o.  Encode and reconstruct chunks
// are 1 KiB (64 lanes x 16 B; tile = 4 KiB).  Decode chunks advance 1008 B:
// lane 0 re-reads the previous chunk's last 16 B (the "overlap lane") so that
// lanes 1..63 can assemble 16-B-aligned object units (see "Realigned object
// stores"); tile = 4032 B.  Tiles [0, tiles) of every object are "interior":
// every lane reads 16 in-bounds bytes from every input and writes one
// 16-byte unit to every output, so they run unconditionally, unrolled over K
// and with the next item's loads in flight (register double buffering).  The
// rest of each payload -- the head and tail of decode's object slices, the
// payload tail, the zero padding -- are "edge" items (4 KiB each, per-lane
// byte bounds), run first by the highest-numbered blocks.
//
// Order (measured, round 2: tools/ab_bench.py): the waves of the grid must
// work on one compact region of memory at a time -- blocks walk the item list
// grid-stride, so consecutive blocks take neighbouring tiles.  Giving each
// wave its own contiguous range instead (every wave streaming a different
// part of the 1.5 GB batch) cost 10 % on encode and 40 % on decode.
//
// XCD placement (speed only): blocks are dealt round-robin over the 8 XCDs
// (MI355X_MICROARCH.md), so with xcd_split the item list is cut into 8
// contiguous ranges and range x is walked, grid-stride, by the blocks with
// b % 8 == x: neighbouring tiles meet in one L2.

struct ItemRange {
  uint32_t begin, end, step;
};
__device__ __forceinline__ ItemRange item_range(uint32_t items, uint32_t xcd_split) {
  if (!xcd_split) return {blockIdx.x, items, gridDim.x};
  const uint32_t x = blockIdx.x & 7u;
  const uint32_t lo = static_cast<uint32_t>(static_cast<uint64_t>(items) * x / 8);
  const uint32_t hi = static_cast<uint32_t>(static_cast<uint64_t>(items) * (x + 1) / 8);
  return {lo + (blockIdx.x >> 3), hi, gridDim.x >> 3};
}

// Whole block writes `count` 80-byte headers (fragment f at frag0 + f*stride).
__device__ __forceinline__ void block_headers(uint8_t* frag0, uint64_t stride, const uint8_t* hdr,
                                              uint32_t count) {
  for (uint32_t i = threadIdx.x; i < count * 5; i += blockDim.x) {
    const uint32_t f = i / 5, part = i - f * 5;
    reinterpret_cast<uint4*>(frag0 + f * stride)[part] =
        reinterpret_cast<const uint4*>(hdr + f * kHeaderBytes)[part];
  }
}

// Bytes [lo, hi) of a slice, of which this lane holds [pos, pos + 16) in v:
// store the overlap at base + that position (edge items; byte-exact).
__device__ __forceinline__ void store_window(uint8_t* base, uint32_t pos, const uint4& v,
                                             int64_t lo, int64_t hi) {
  const int64_t a = lo > pos ? lo - pos : 0;
  const int64_t b = hi < static_cast<int64_t>(pos) + 16 ? hi - pos : 16;
  if (a >= b) return;
  if (a == 0 && b == 16)
    *reinterpret_cast<uint4*>(base + pos) = v;
  else
    put_bytes(base + pos + a, v, static_cast<uint32_t>(a), static_cast<uint32_t>(b - a));
}

// ---------------- encode ----------------

// Interior item w: 4 KiB of payload positions starting at t0 = tile*4096;
// this wave's chunk at t0 + 1024*wave, the lane at + 16*lane (voffset).
__device__ __forceinline__ void enc_item_pos(const EncodeParams& p, uint32_t w, uint32_t& o,
                                             uint32_t& x) {
  o = w / p.tiles;
  x = (w - o * p.tiles) * (kWavesPerBlock * kChunkBytes) + wave_in_block() * kChunkBytes;
}

template <int K, int POL>
__device__ __forceinline__ void encode_load(const EncodeParams& p, uint32_t o, uint32_t x,
                                            uint4 (&v)[K], bool none = false) {
  const Rsrc r = rsrc(p.objs + static_cast<uint64_t>(o) * p.obj_stride, none ? 0 : -1);
#pragma unroll
  for (int j = 0; j < K; ++j)
    v[j] = buf_ld<(POL & kPolLoadsCached) != 0>(r, lane_id() * 16, j * p.bs + x);
}

// One interior item with its inputs in `cur`; first issues the loads of the
// block's next item into `nxt` so they are in flight while this item's table
// lookups run (the last item's "next" loads go through a zero-record
// descriptor: no memory traffic).  Every memory
// operation in the loop body is unconditional, so hipcc's s_waitcnt before
// cur[j] waits only for cur's own loads (a branch around a load or store
// makes it fall back to the shortest path's count -- measured in round 1 as
// waiting for the prefetch too, which serialised memory and compute).
template <class F, int K, int NR, int POL, bool SDWA, bool NOCOMP = false>
__device__ __forceinline__ void encode_item(const EncodeParams& p, uint32_t w, uint32_t wn,
                                            uint4 (&cur)[K], uint4 (&nxt)[K], bool none) {
  uint32_t o, x, on, xn;
  enc_item_pos(p, w, o, x);
  enc_item_pos(p, wn, on, xn);
  encode_load<K, POL>(p, on, xn, nxt, none);
  typename F::Acc s;
  F::zero(s);
  if constexpr (NOCOMP) {
    // memory-only probe (A/B, wrong parity): the inputs XORed, no lookups
    uint32_t* a = reinterpret_cast<uint32_t*>(&s);
#pragma unroll
    for (int j = 0; j < K; ++j) {
      a[0] ^= cur[j].x;
      a[2] ^= cur[j].y;
      a[4] ^= cur[j].z;
      a[6] ^= cur[j].w;
    }
  } else {
#pragma unroll
    for (int j = 0; j < K; ++j) F::template mac<SDWA>(F::kb(0), j * F::kTableBytes, cur[j], s);
  }
  F::pin(s);
  const Rsrc par = rsrc(p.parity + static_cast<uint64_t>(o) * p.stripe_stride);
  const uint32_t soff = p.row0 * p.frag_stride + kHeaderBytes + x;
#pragma unroll
  for (int q = 0; q < NR; ++q)
    buf_st<(POL & kPolStoresCached) != 0>(par, lane_id() * 16, soff + q * p.frag_stride, F::row(s, q));
}

// Edge item: payload tail and chunks reaching the zero padding past obj_len
// (liberasurecode's prepare_fragments_for_encode zero-fills).
template <class F, int K, int NR>
__device__ __forceinline__ void encode_edge_item(const EncodeParams& p, uint32_t e) {
  const uint32_t o = e / p.edge_tiles;
  const uint32_t t = (p.tiles + (e - o * p.edge_tiles)) * (kWavesPerBlock * kChunkBytes) +
                     threadIdx.x * 16;
  if (t >= p.bs) return;
  const uint8_t* obj = p.objs + static_cast<uint64_t>(o) * p.obj_stride;
  const int64_t rem = static_cast<int64_t>(p.bs) - t;
  uint4 x[K];
#pragma unroll
  for (int j = 0; j < K; ++j) x[j] = load_clamped(obj, static_cast<uint64_t>(j) * p.bs + t, p.obj_len);
  typename F::Acc s;
  F::zero(s);
#pragma unroll
  for (int j = 0; j < K; ++j) F::template mac<true>(F::kb(0), j * F::kTableBytes, x[j], s);
  F::pin(s);
  uint8_t* par = p.parity + static_cast<uint64_t>(o) * p.stripe_stride + p.row0 * p.frag_stride +
                 kHeaderBytes + t;
#pragma unroll
  for (int q = 0; q < NR; ++q) store_partial(par + q * p.frag_stride, F::row(s, q), rem);
}

// SDWA = false: the table addresses are built with v_perm (decode's form;
// A/B of the benchmark case, ECAMD_ENC_PERM=1).
template <class F, int K, int NR, int POL, bool SDWA = true, bool NOCOMP = false>
__global__ void __launch_bounds__(kThreadsPerBlock) encode_kernel(EncodeParams p) {
  load_tables(p.tables, K * F::kTableBytes, 0);
  if (p.headers != nullptr && p.row0 == 0)
    for (uint32_t o = blockIdx.x; o < p.n_obj; o += gridDim.x) {
      const uint64_t base = static_cast<uint64_t>(o) * p.stripe_stride;
      block_headers(p.parity + base, p.frag_stride, p.headers + K * kHeaderBytes, p.m);
      if (p.data != nullptr) block_headers(p.data + base, p.frag_stride, p.headers, K);
    }
  __syncthreads();
  // edge items first, on the highest-numbered blocks (those with the fewest
  // interior items)
  const uint32_t n_edge = p.n_obj * p.edge_tiles;
  for (uint32_t e = gridDim.x - 1 - blockIdx.x; e < n_edge; e += gridDim.x)
    encode_edge_item<F, K, NR>(p, e);
  const ItemRange r = item_range(p.n_obj * p.tiles, p.xcd_split);
  uint32_t w = r.begin;
  if (w < r.end) {
    uint4 xa[K], xb[K];
    uint32_t o, x;
    enc_item_pos(p, w, o, x);
    encode_load<K, POL>(p, o, x, xa);
    // two items per trip so cur / nxt stay compile-time register arrays
    while (true) {
      uint32_t wn = w + r.step < r.end ? w + r.step : w;
      encode_item<F, K, NR, POL, SDWA, NOCOMP>(p, w, wn, xa, xb, wn == w);
      if (wn == w) break;
      w = wn;
      wn = w + r.step < r.end ? w + r.step : w;
      encode_item<F, K, NR, POL, SDWA, NOCOMP>(p, w, wn, xb, xa, wn == w);
      if (wn == w) break;
      w = wn;
    }
  }
}

// Prefetch depth 2 (A/B of the benchmark case, ECAMD_ENC_DEPTH2=1): while
// item w is computed, items w + step and w + 2*step are in flight (three
// register buffers; 3 waves per SIMD).
template <class F, int K, int NR, int POL>
__global__ void __launch_bounds__(kThreadsPerBlock) __attribute__((amdgpu_waves_per_eu(3, 8)))
encode_kernel_d2(EncodeParams p) {
  load_tables(p.tables, K * F::kTableBytes, 0);
  if (p.headers != nullptr && p.row0 == 0)
    for (uint32_t o = blockIdx.x; o < p.n_obj; o += gridDim.x) {
      const uint64_t base = static_cast<uint64_t>(o) * p.stripe_stride;
      block_headers(p.parity + base, p.frag_stride, p.headers + K * kHeaderBytes, p.m);
      if (p.data != nullptr) block_headers(p.data + base, p.frag_stride, p.headers, K);
    }
  __syncthreads();
  const uint32_t n_edge = p.n_obj * p.edge_tiles;
  for (uint32_t e = gridDim.x - 1 - blockIdx.x; e < n_edge; e += gridDim.x)
    encode_edge_item<F, K, NR>(p, e);
  const ItemRange r = item_range(p.n_obj * p.tiles, p.xcd_split);
  uint32_t w = r.begin;
  if (w >= r.end) return;
  uint4 xa[K], xb[K], xc[K];
  // item w + k*step if it exists, else w itself (loaded through a
  // zero-record descriptor: no traffic)
  auto ahead = [&](uint32_t v, uint32_t k) { return v + k * r.step < r.end ? v + k * r.step : v; };
  {
    uint32_t o, x;
    enc_item_pos(p, w, o, x);
    encode_load<K, POL>(p, o, x, xa);
    const uint32_t w1 = ahead(w, 1);
    enc_item_pos(p, w1, o, x);
    encode_load<K, POL>(p, o, x, xb, w1 == w);
  }
  while (true) {
    uint32_t f = ahead(w, 2);
    encode_item<F, K, NR, POL, true>(p, w, f, xa, xc, f == w);
    if (w + r.step >= r.end) break;
    w += r.step;
    f = ahead(w, 2);
    encode_item<F, K, NR, POL, true>(p, w, f, xb, xa, f == w);
    if (w + r.step >= r.end) break;
    w += r.step;
    f = ahead(w, 2);
    encode_item<F, K, NR, POL, true>(p, w, f, xc, xb, f == w);
    if (w + r.step >= r.end) break;
    w += r.step;
  }
}

// Data fragments (optional output of encode): the k padded object slices
// copied into their fragment payloads.  Item = (object, fragment, 4 KiB).
__global__ void __launch_bounds__(kThreadsPerBlock) copy_data_kernel(EncodeParams p) {
  const uint32_t per_frag = (p.bs + kWavesPerBlock * kChunkBytes - 1) / (kWavesPerBlock * kChunkBytes);
  const uint32_t per_obj = p.k * per_frag;
  const uint32_t items = p.n_obj * per_obj;
  for (uint32_t w = blockIdx.x; w < items; w += gridDim.x) {
    const uint32_t o = w / per_obj, rest = w - o * per_obj;
    const uint32_t j = rest / per_frag, c = rest - j * per_frag;
    const uint32_t t = c * (kWavesPerBlock * kChunkBytes) + threadIdx.x * 16;
    if (t >= p.bs) continue;
    const uint8_t* obj = p.objs + static_cast<uint64_t>(o) * p.obj_stride;
    const uint4 x = load_clamped(obj, static_cast<uint64_t>(j) * p.bs + t, p.obj_len);
    store_partial(p.data + static_cast<uint64_t>(o) * p.stripe_stride + j * p.frag_stride +
                      kHeaderBytes + t,
                  x, static_cast<int64_t>(p.bs) - t);
  }
}

// ---------------- decode / reconstruct ----------------
//
// Table sets.  Each object's descriptor names a table set (its erasure
// pattern's decode rows); consecutive items of a block usually belong to
// different objects.  LDS holds two slots: a new set goes into the slot not
// in use, so one barrier per change suffices -- a wave writes slot s only
// after passing the barrier of the previous change, which every wave reaches
// only after finishing the items that read slot s.  The item loop fetches
// the next item's set into registers together with its payload loads, so a
// change costs a few ds_writes and one barrier, not an L2 round trip.
//
// Realigned object stores.  Decode writes data slice j of an object at
// j*bs + t, and bs is rarely a multiple of 16 (419,432 = 8 mod 16 at 4 MiB,
// k = 10), so a plain 16-B lane store would straddle two 16-B units (the
// memory pipeline splits it in two, and the lines at both ends of every wave
// access are written as partial lines: 448 us vs 378 us for the same stream
// line-aligned, round 1).  The shift s = (j*bs) mod 16 is uniform over the
// slice.  Decode chunks therefore advance 63 lanes (1008 B) and lane 0 holds
// the previous chunk's last 16 B; lane L >= 1 stores the aligned unit that
// starts s bytes below its own position -- the last s bytes of lane L-1
// (DPP wave_shr:1) and its own first 16 - s bytes -- and lane 0's store is
// dropped by the buffer range check (its voffset is past the descriptor's
// 2 GiB of records), so every slice costs exactly one aligned dwordx4 store
// instruction per chunk, with no carried state and no branch around it.  A
// chunk at x covers slice bytes [x + 16 - s, x + 1024 - s); the head
// [0, 16 - s) and the tail are edge items.

struct Slots {
  uint32_t table;  // set in the current slot (0xFFFFFFFF = none)
  uint32_t slot;   // 0 / 1
};

template <class F, int K>
struct TablePre {
  static constexpr int kChunks = K * F::kTableBytes / 16;
  static constexpr int kPer = (kChunks + kThreadsPerBlock - 1) / kThreadsPerBlock;
  uint4 v[kPer];
  uint32_t table;
};

template <class F, int K>
__device__ __forceinline__ void table_prefetch(const DecodeParams& p, uint32_t table,
                                               TablePre<F, K>& pre) {
  const uint4* src = reinterpret_cast<const uint4*>(
      p.tables + static_cast<uint64_t>(table) * (K * F::kTableBytes / 4));
#pragma unroll
  for (int i = 0; i < TablePre<F, K>::kPer; ++i) {
    const uint32_t c = threadIdx.x + i * kThreadsPerBlock;
    if (c < static_cast<uint32_t>(TablePre<F, K>::kChunks)) pre.v[i] = src[c];
  }
  pre.table = table;
}

// Make d's table set current; returns its kb.  Block-uniform (barrier;
// SYNC: a barrier even when the set is unchanged -- the staged stores'
// write-after-read fence on the staging area).
template <class F, int K, bool SYNC = false, class D>
__device__ __forceinline__ uint32_t ensure_tables(const DecodeParams& p, const D& d, Slots& st,
                                                  const TablePre<F, K>& pre) {
  constexpr uint32_t kSlot = table_slot_bytes(K, F::kW);
  if (d.n_out() != 0 && d.table() != st.table) {
    st.slot ^= 1u;
    const uint32_t base = st.slot * kSlot;
    if (pre.table == d.table()) {
      auto* dst = lds_v4(base);
#pragma unroll
      for (int i = 0; i < TablePre<F, K>::kPer; ++i) {
        const uint32_t c = threadIdx.x + i * kThreadsPerBlock;
        if (c < static_cast<uint32_t>(TablePre<F, K>::kChunks)) {
          v4u v;
          v.x = pre.v[i].x;
          v.y = pre.v[i].y;
          v.z = pre.v[i].z;
          v.w = pre.v[i].w;
          dst[c] = v;
        }
      }
    } else {
      load_tables(p.tables + static_cast<uint64_t>(d.table()) * (K * F::kTableBytes / 4),
                  K * F::kTableBytes, base);
    }
    __syncthreads();
    st.table = d.table();
  } else if constexpr (SYNC) {
    __syncthreads();
  }
  return F::kb(st.slot * kSlot);
}

enum DecodeMode : int {
  kDecode = 0,        // one pass holds every missing row: all k data slices stored
  kReconstruct = 1,   // one fragment per object (aligned payload)
  kDecodeGeneric = 2  // more than 4 missing data fragments (several passes)
};

// Chunk stride: decode overlaps one lane (realigned slices) unless PLAIN
// (lane stores at their natural, unaligned positions -- kept for A/B).
template <int MODE, bool PLAIN>
__host__ __device__ constexpr bool overlaps() {
  return MODE != kReconstruct && !PLAIN;
}
template <int MODE, bool PLAIN>
__host__ __device__ constexpr uint32_t chunk_stride() {
  return overlaps<MODE, PLAIN>() ? kChunkBytes - 16 : kChunkBytes;
}

// An object's descriptor held in SGPRs.  The descriptor array is read with
// vector loads (hipcc cannot prove the kernel's stores leave it untouched, so
// it will not use scalar loads), and every field feeds a buffer soffset, a
// uniform branch or the table switch: readfirstlane makes them provably
// uniform -- without it hipcc wraps every buffer op in a waterfall loop
// (measured: each load serialised behind s_waitcnt vmcnt(0);
// cdna_hip_programming.md T20).
// (Fields are extracted with shifts only: indexing w[] with a runtime value
// would put the array in scratch memory and make the results non-uniform.)
struct DescU {
  uint32_t w[sizeof(ObjDesc) / 4];
  // c: compile-time after unrolling
  __device__ __forceinline__ uint32_t in_idx(int c) const {
    return (w[c >> 2] >> (8 * (c & 3))) & 0xFFu;
  }
  // q: runtime (0..3)
  __device__ __forceinline__ uint32_t out_idx(uint32_t q) const { return (w[8] >> (8 * q)) & 0xFFu; }
  __device__ __forceinline__ uint32_t n_out() const { return w[9] & 0xFFu; }
  __device__ __forceinline__ uint32_t copy_inputs() const { return (w[9] >> 8) & 0xFFu; }
  __device__ __forceinline__ uint32_t table() const { return w[10]; }
  __device__ __forceinline__ uint32_t header() const { return w[11]; }
};
static_assert(offsetof(ObjDesc, out_idx) == 32 && offsetof(ObjDesc, n_out) == 36 &&
                  offsetof(ObjDesc, copy_inputs) == 37 && offsetof(ObjDesc, table) == 40 &&
                  offsetof(ObjDesc, header) == 44 && sizeof(ObjDesc) % 4 == 0,
              "DescU mirrors ObjDesc");
__device__ __forceinline__ DescU load_desc(const DecodeParams& p, uint32_t o) {
  const uint32_t* src = reinterpret_cast<const uint32_t*>(p.desc + o);
  DescU u;
#pragma unroll
  for (uint32_t i = 0; i < sizeof(ObjDesc) / 4; ++i) u.w[i] = __builtin_amdgcn_readfirstlane(src[i]);
  return u;
}

// Fragment group position of input c.
__device__ __forceinline__ uint32_t in_pos(const DecodeParams& p, const DescU& d, int c) {
  return p.compact ? static_cast<uint32_t>(c) : d.in_idx(c);
}

template <int MODE, bool PLAIN>
__device__ __forceinline__ void dec_item_pos(const DecodeParams& p, uint32_t w, uint32_t& o,
                                             uint32_t& x) {
  constexpr uint32_t kStride = chunk_stride<MODE, PLAIN>();
  o = w / p.tiles;
  x = (w - o * p.tiles) * (kWavesPerBlock * kStride) + wave_in_block() * kStride;
}

template <int K, int POL>
__device__ __forceinline__ void decode_load(const DecodeParams& p, uint32_t o, const DescU& d,
                                            uint32_t x, uint4 (&v)[K], bool none = false) {
  const Rsrc in = rsrc(p.frags + static_cast<uint64_t>(o) * p.stripe_stride, none ? 0 : -1);
#pragma unroll
  for (int j = 0; j < K; ++j)
    v[j] = buf_ld<(POL & kPolLoadsCached) != 0>(
        in, lane_id() * 16, in_pos(p, d, j) * p.frag_stride + kHeaderBytes + x);
}

// Output descriptor: 2 GiB - 1 records, so a voffset of kDrop (2 GiB) makes
// the buffer range check discard that lane's store.
constexpr uint32_t kDrop = 0x80000000u;
__device__ __forceinline__ Rsrc rsrc_out(const void* base) {
  const uint64_t a = reinterpret_cast<uint64_t>(base);
  const uint32_t lo = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(a));
  const uint32_t hi = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(a >> 32));
  return __builtin_amdgcn_make_buffer_rsrc(
      reinterpret_cast<void*>((static_cast<uint64_t>(hi) << 32) | lo), 0, 0x7FFFFFFF, 0x00020000);
}

__device__ __forceinline__ uint32_t shr1(uint32_t v) {
  return static_cast<uint32_t>(__builtin_amdgcn_update_dpp(
      0, static_cast<int>(v), 0x138 /* wave_shr:1 */, 0xF, 0xF, false));
}

// Store slice unit: this lane's 16 B v sits at slice position x + 16*lane,
// object offset soff + 16*lane with soff mod 16 == s; lane L >= 1 writes the
// aligned unit at soff + 16*L - s, lane 0 is dropped (vst = kDrop).  Only
// the dwords of lane L-1 that the unit uses are moved (d = (16 - s) / 4).
// Every path issues exactly one store instruction.
template <bool CACHED>
__device__ __forceinline__ void st_unit(Rsrc out, uint32_t vst, uint32_t soff, const uint4& v,
                                        uint32_t s) {
  if (s == 0) {
    buf_st<CACHED>(out, vst, soff, v);
    return;
  }
  const uint32_t r = (16u - s) & 3u;
  uint4 u;
  switch ((16u - s) >> 2) {
    case 0: {
      const uint32_t p0 = shr1(v.x), p1 = shr1(v.y), p2 = shr1(v.z), p3 = shr1(v.w);
      u = make_uint4(__builtin_amdgcn_alignbyte(p1, p0, r), __builtin_amdgcn_alignbyte(p2, p1, r),
                     __builtin_amdgcn_alignbyte(p3, p2, r), __builtin_amdgcn_alignbyte(v.x, p3, r));
      break;
    }
    case 1: {
      const uint32_t p1 = shr1(v.y), p2 = shr1(v.z), p3 = shr1(v.w);
      u = make_uint4(__builtin_amdgcn_alignbyte(p2, p1, r), __builtin_amdgcn_alignbyte(p3, p2, r),
                     __builtin_amdgcn_alignbyte(v.x, p3, r), __builtin_amdgcn_alignbyte(v.y, v.x, r));
      break;
    }
    case 2: {
      const uint32_t p2 = shr1(v.z), p3 = shr1(v.w);
      u = make_uint4(__builtin_amdgcn_alignbyte(p3, p2, r), __builtin_amdgcn_alignbyte(v.x, p3, r),
                     __builtin_amdgcn_alignbyte(v.y, v.x, r), __builtin_amdgcn_alignbyte(v.z, v.y, r));
      break;
    }
    default: {
      const uint32_t p3 = shr1(v.w);
      u = make_uint4(__builtin_amdgcn_alignbyte(v.x, p3, r), __builtin_amdgcn_alignbyte(v.y, v.x, r),
                     __builtin_amdgcn_alignbyte(v.z, v.y, r), __builtin_amdgcn_alignbyte(v.w, v.z, r));
      break;
    }
  }
  buf_st<CACHED>(out, vst, soff - s, u);
}

// Staged object stores (STAGED, kDecode).  The block's four waves hold the
// 4 KiB tile [t0, t0 + 4096) of every slice; they write it to LDS (slice c
// at stage + c * 4096), and after a barrier thread u stores the 16-B-aligned
// object unit u of each slice: slice j's tile lands at A = j*bs + t0, so with
// a = A mod 16 unit u covers tile bytes [16u - a, 16u - a + 16) -- the last
// a bytes of staged unit u - 1 and the first 16 - a of unit u (two aligned
// ds_read_b128 and a funnel shift).  Every store is a whole aligned 16-B
// unit except the two at the tile's ends (unit 0: bytes [a, 16); unit 256:
// bytes [0, a)), so a slice's lines are split only where two tiles meet
// (every 4 KiB), not at every wave's 1 KiB as with lane-natural stores.
constexpr uint32_t kStageTile = kWavesPerBlock * kChunkBytes;  // 4096

// Bytes [lo, hi) of v stored at voff + lo (naturally aligned pieces).
__device__ __forceinline__ void buf_st_bytes(Rsrc r, uint32_t voff, const uint4& v, uint32_t lo,
                                             uint32_t hi) {
  const uint64_t q0 = v.x | (static_cast<uint64_t>(v.y) << 32);
  const uint64_t q1 = v.z | (static_cast<uint64_t>(v.w) << 32);
  for (uint32_t i = lo; i < hi;) {
    const uint64_t qv = i < 8 ? q0 >> (8 * i) : q1 >> (8 * (i - 8));
    if ((i & 7) == 0 && i + 8 <= hi) {
      v2u d;
      d.x = static_cast<uint32_t>(qv);
      d.y = static_cast<uint32_t>(qv >> 32);
      __builtin_amdgcn_raw_buffer_store_b64(d, r, voff + i, 0, 0);
      i += 8;
    } else if ((i & 3) == 0 && i + 4 <= hi) {
      __builtin_amdgcn_raw_buffer_store_b32(static_cast<uint32_t>(qv), r, voff + i, 0, 0);
      i += 4;
    } else if ((i & 1) == 0 && i + 2 <= hi) {
      __builtin_amdgcn_raw_buffer_store_b16(static_cast<unsigned short>(qv), r, voff + i, 0, 0);
      i += 2;
    } else {
      __builtin_amdgcn_raw_buffer_store_b8(static_cast<unsigned char>(qv), r, voff + i, 0, 0);
      i += 1;
    }
  }
}

// Bytes [b0, b0 + 16) of the 32-byte pair (lo, hi), b0 = 16 - a in 1..15
// (wave-uniform).
__device__ __forceinline__ uint4 funnel16(const uint4& lo, const uint4& hi, uint32_t b0) {
  const uint32_t r = b0 & 3u;
  switch (b0 >> 2) {
    case 0:
      return make_uint4(__builtin_amdgcn_alignbyte(lo.y, lo.x, r), __builtin_amdgcn_alignbyte(lo.z, lo.y, r),
                        __builtin_amdgcn_alignbyte(lo.w, lo.z, r), __builtin_amdgcn_alignbyte(hi.x, lo.w, r));
    case 1:
      return make_uint4(__builtin_amdgcn_alignbyte(lo.z, lo.y, r), __builtin_amdgcn_alignbyte(lo.w, lo.z, r),
                        __builtin_amdgcn_alignbyte(hi.x, lo.w, r), __builtin_amdgcn_alignbyte(hi.y, hi.x, r));
    case 2:
      return make_uint4(__builtin_amdgcn_alignbyte(lo.w, lo.z, r), __builtin_amdgcn_alignbyte(hi.x, lo.w, r),
                        __builtin_amdgcn_alignbyte(hi.y, hi.x, r), __builtin_amdgcn_alignbyte(hi.z, hi.y, r));
    default:
      return make_uint4(__builtin_amdgcn_alignbyte(hi.x, lo.w, r), __builtin_amdgcn_alignbyte(hi.y, hi.x, r),
                        __builtin_amdgcn_alignbyte(hi.z, hi.y, r), __builtin_amdgcn_alignbyte(hi.w, hi.z, r));
  }
}

// Store one staged slice tile (LDS bytes [sb, sb + 4096), preceded by 16
// readable bytes) at object offset A.  Block-wide; after the staging barrier.
template <bool CACHED>
__device__ __forceinline__ void stage_out(Rsrc out, uint32_t sb, uint32_t A) {
  const uint32_t u = threadIdx.x;
  const uint32_t a = A & 15u, U0 = A - a;
  const v4u c = *lds_v4(sb + 16 * u);
  const uint4 cu = make_uint4(c.x, c.y, c.z, c.w);
  if (a == 0) {
    buf_st<CACHED>(out, 16 * u, U0, cu);
    return;
  }
  const v4u p = *lds_v4(sb + 16 * u - 16);
  const uint4 v = funnel16(make_uint4(p.x, p.y, p.z, p.w), cu, 16 - a);
  if (u != 0)
    buf_st<CACHED>(out, 16 * u, U0, v);
  else
    buf_st_bytes(out, U0, v, a, 16);
  if (u == kThreadsPerBlock - 1) {
    // unit 256: the last a bytes of staged unit 255
    const uint4 t = funnel16(cu, make_uint4(0, 0, 0, 0), 16 - a);
    buf_st_bytes(out, U0 + 16 * kThreadsPerBlock, t, 0, a);
  }
}

// kDecode: the k inputs are the first k available fragments in ascending
// order, so the present data fragments come first and the parity inputs --
// as many as there are missing data slices, e -- are the last e.  After the
// products, row q overwrites parity input K-e+q: cur[c] then holds data slice
// slice_of(c) for every c, and all K slices are stored unconditionally.
__device__ __forceinline__ uint32_t slice_of(const DescU& d, uint32_t e, int K, int c) {
  return c < K - static_cast<int>(e) ? d.in_idx(c) : d.out_idx(c - (K - static_cast<int>(e)));
}

template <class F, int K>
__device__ __forceinline__ void place_rows(const typename F::Acc& s, uint32_t e, uint4 (&x)[K]) {
  constexpr int L = K < 4 ? K : 4;
  switch (e) {
#define ECAMD_PLACE(E)                                                                     \
  case E:                                                                                  \
    if constexpr (E <= L) {                                                                \
      _Pragma("unroll") for (int q = 0; q < E; ++q) x[K - E + q] = F::row(s, q);           \
    }                                                                                      \
    break;
    ECAMD_PLACE(1) ECAMD_PLACE(2) ECAMD_PLACE(3) ECAMD_PLACE(4)
#undef ECAMD_PLACE
    default:
      break;
  }
}

// One interior decode / reconstruct item with inputs in `cur`; prefetches the
// block's next item (payloads into `nxt`, its table set into `pre`).
template <class F, int K, int MODE, bool PLAIN, int POL, bool STAGED, bool NOCOMP = false>
__device__ __forceinline__ void decode_item(const DecodeParams& p, uint32_t w, uint32_t wn,
                                            Slots& st, TablePre<F, K>& pre, uint4 (&cur)[K],
                                            uint4 (&nxt)[K]) {
  uint32_t o, x, on, xn;
  dec_item_pos<MODE, PLAIN>(p, w, o, x);
  dec_item_pos<MODE, PLAIN>(p, wn, on, xn);
  const DescU dn = load_desc(p, on);
  decode_load<K, POL>(p, on, dn, xn, nxt, wn == w);
  const DescU d = load_desc(p, o);
  const uint32_t kb = ensure_tables<F, K, STAGED>(p, d, st, pre);
  if (dn.n_out() != 0 && dn.table() != st.table && dn.table() != pre.table)
    table_prefetch<F, K>(p, dn.table(), pre);
  const uint32_t n_out = d.n_out();
  typename F::Acc s;
  F::zero(s);
  if (!NOCOMP && n_out != 0) {
#pragma unroll
    for (int j = 0; j < K; ++j) F::mac(kb, j * F::kTableBytes, cur[j], s);
  }
  F::pin(s);
  constexpr bool kStC = (POL & kPolStoresCached) != 0;
  uint8_t* const outp = p.out + static_cast<uint64_t>(o) * p.out_stride;
  if constexpr (MODE == kReconstruct) {
    buf_st<kStC>(rsrc(outp), lane_id() * 16, kHeaderBytes + x, F::row(s, 0));
  } else {
    // overlap: lane 0 only carries the previous chunk's bytes, its store is
    // dropped; plain: every lane stores its own 16 B where they belong
    const Rsrc out = PLAIN ? rsrc(outp) : rsrc_out(outp);
    const uint32_t vst = (!PLAIN && lane_id() == 0) ? kDrop : lane_id() * 16;
    auto put = [&](uint32_t off, const uint4& v) {
      if constexpr (PLAIN)
        buf_st<kStC>(out, vst, off + x, v);
      else
        st_unit<kStC>(out, vst, off + x, v, off & 15u);
    };
    if constexpr (MODE == kDecode && STAGED) {
      place_rows<F, K>(s, n_out, cur);
      constexpr uint32_t sb0 = 2 * table_slot_bytes(K, F::kW) + 16;
#pragma unroll
      for (int j = 0; j < K; ++j) {
        v4u v;
        v.x = cur[j].x;
        v.y = cur[j].y;
        v.z = cur[j].z;
        v.w = cur[j].w;
        *lds_v4(sb0 + j * kStageTile + wave_in_block() * kChunkBytes + lane_id() * 16) = v;
      }
      __syncthreads();
      const uint32_t t0 = x - wave_in_block() * kChunkBytes;
      const Rsrc outb = rsrc(outp);
#pragma unroll
      for (int j = 0; j < K; ++j)
        stage_out<kStC>(outb, sb0 + j * kStageTile, slice_of(d, n_out, K, j) * p.bs + t0);
    } else if constexpr (MODE == kDecode) {
      place_rows<F, K>(s, n_out, cur);
#pragma unroll
      for (int j = 0; j < K; ++j) put(slice_of(d, n_out, K, j) * p.bs, cur[j]);
    } else {
      if (d.copy_inputs()) {
#pragma unroll
        for (int j = 0; j < K; ++j) {
          const uint32_t idx = d.in_idx(j);
          if (idx < static_cast<uint32_t>(K)) put(idx * p.bs, cur[j]);
        }
      }
#pragma unroll
      for (int q = 0; q < kRowsPerPass; ++q)
        if (q < static_cast<int>(n_out)) put(d.out_idx(q) * p.bs, F::row(s, q));
    }
  }
}

// Edge item: 4 KiB of positions from q0 (+ 16 per thread), byte-exact stores
// clipped to each output's window.  Decode: head item (window [0, 16 - s))
// and tail items (window [tiles*4032 + 16 - s, object bytes of the slice)).
// Reconstruct: tail items [tiles*4096, bs).
template <class F, int K, int MODE, bool PLAIN>
__device__ __forceinline__ void decode_edge_item(const DecodeParams& p, uint32_t e, Slots& st,
                                                 const TablePre<F, K>& pre) {
  constexpr bool kOv = overlaps<MODE, PLAIN>();
  const uint32_t o = e / p.edge_tiles;
  const uint32_t ei = e - o * p.edge_tiles;
  const uint32_t tail0 = p.tiles * kWavesPerBlock * chunk_stride<MODE, PLAIN>();
  const bool head = kOv && ei == 0;
  const uint32_t q0 = head ? 0u : tail0 + (ei - (kOv ? 1u : 0u)) * 4096u;
  const DescU d = load_desc(p, o);
  const uint32_t kb = ensure_tables<F, K>(p, d, st, pre);
  const uint32_t t = q0 + threadIdx.x * 16;
  if (t >= p.bs) return;
  uint8_t* out = p.out + static_cast<uint64_t>(o) * p.out_stride;
  // t < bs and 16 | t, so t + 16 <= round16(bs) <= frag_stride - 80: in bounds
  const uint8_t* in = p.frags + static_cast<uint64_t>(o) * p.stripe_stride + kHeaderBytes + t;
  uint4 x[K];
#pragma unroll
  for (int j = 0; j < K; ++j)
    x[j] = *reinterpret_cast<const uint4*>(in + in_pos(p, d, j) * p.frag_stride);
  typename F::Acc s;
  F::zero(s);
  if (d.n_out() != 0) {
#pragma unroll
    for (int j = 0; j < K; ++j) F::mac(kb, j * F::kTableBytes, x[j], s);
  }
  F::pin(s);
  if (MODE == kReconstruct) {
    if (d.n_out() != 0) store_window(out + kHeaderBytes, t, F::row(s, 0), tail0, p.bs);
    return;
  }
  // window of slice j: [lo_j, hi_j) in slice positions
  auto window = [&](uint32_t j, int64_t& lo, int64_t& hi) {
    const uint32_t sh = (j * p.bs) & 15u;
    const int64_t valid = object_bytes(j, p.bs, 0, p.obj_len);
    lo = head ? 0 : static_cast<int64_t>(tail0) + (kOv ? 16 - sh : 0);
    hi = head ? 16 - sh : valid;
    if (hi > valid) hi = valid;
  };
  if (d.copy_inputs()) {
#pragma unroll
    for (int j = 0; j < K; ++j) {
      const uint32_t idx = d.in_idx(j);
      if (idx >= K) continue;
      int64_t lo, hi;
      window(idx, lo, hi);
      store_window(out + static_cast<uint64_t>(idx) * p.bs, t, x[j], lo, hi);
    }
  }
  for (uint32_t q = 0; q < d.n_out(); ++q) {
    const uint32_t idx = d.out_idx(q);
    int64_t lo, hi;
    window(idx, lo, hi);
    store_window(out + static_cast<uint64_t>(idx) * p.bs, t, F::row(s, q), lo, hi);
  }
}

// OCC = minimum waves per SIMD the register allocation must allow (hipcc
// left alone spends ~140 VGPRs on the decode variants: 3 waves per SIMD; 4
// fits in 128 VGPRs with a few spills around the table prefetch).
template <class F, int K, int MODE, int OCC, bool PLAIN, int POL, bool STAGED = false,
          bool NOCOMP = false>
__global__ void __launch_bounds__(kThreadsPerBlock) __attribute__((amdgpu_waves_per_eu(OCC, 8)))
decode_kernel(DecodeParams p) {
  if (MODE == kReconstruct && p.headers != nullptr)
    for (uint32_t o = blockIdx.x; o < p.n_obj; o += gridDim.x)
      block_headers(p.out + static_cast<uint64_t>(o) * p.out_stride, 0,
                    p.headers + static_cast<uint64_t>(load_desc(p, o).header()) * kHeaderBytes, 1);
  Slots st{0xFFFFFFFFu, 1u};
  TablePre<F, K> pre;
  pre.table = 0xFFFFFFFFu;
  // edge items first, on the highest-numbered blocks
  const uint32_t n_edge = p.n_obj * p.edge_tiles;
  for (uint32_t e = gridDim.x - 1 - blockIdx.x; e < n_edge; e += gridDim.x)
    decode_edge_item<F, K, MODE, PLAIN>(p, e, st, pre);
  const ItemRange r = item_range(p.n_obj * p.tiles, p.xcd_split);
  uint32_t w = r.begin;
  if (w < r.end) {
    uint4 xa[K], xb[K];
    uint32_t o, x;
    dec_item_pos<MODE, PLAIN>(p, w, o, x);
    const DescU d0 = load_desc(p, o);
    decode_load<K, POL>(p, o, d0, x, xa);
    if (d0.n_out() != 0 && d0.table() != st.table) table_prefetch<F, K>(p, d0.table(), pre);
    while (true) {
      uint32_t wn = w + r.step < r.end ? w + r.step : w;
      decode_item<F, K, MODE, PLAIN, POL, STAGED, NOCOMP>(p, w, wn, st, pre, xa, xb);
      if (wn == w) break;
      w = wn;
      wn = w + r.step < r.end ? w + r.step : w;
      decode_item<F, K, MODE, PLAIN, POL, STAGED, NOCOMP>(p, w, wn, st, pre, xb, xa);
      if (wn == w) break;
      w = wn;
    }
  }
}

// ---------------- launch ----------------

inline bool env_flag(const char* name, bool dflt) {
  const char* v = std::getenv(name);
  if (v == nullptr || *v == 0) return dflt;
  return v[0] != '0';
}

inline int grid_for(const void* kernel, size_t lds_bytes, uint32_t items) {
  int dev = 0, cus = 256, per_cu = 4;
  if (hipGetDevice(&dev) == hipSuccess) {
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    int b = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&b, kernel, kThreadsPerBlock, lds_bytes) ==
            hipSuccess &&
        b > 0)
      per_cu = b;
  }
  // The occupancy API can report one block per CU more than fits
  // (MI355X_MICROARCH.md, Residency); a grid-stride kernel must not queue
  // blocks behind the resident ones, so stay at <= 4 per CU.
  per_cu = std::min(per_cu, 4);
  const uint32_t resident = static_cast<uint32_t>(cus * per_cu);
  return static_cast<int>(items < resident ? (items ? items : 1) : resident);
}

// The kernels address LDS by raw byte offset from 0, which is only valid when
// the kernel has no static __shared__ data (the dynamic allocation then
// starts at address 0).  Checked once per kernel; a violation fails loudly.
inline bool lds_starts_at_zero(const void* kern) {
  static std::mutex mu;
  static std::unordered_map<const void*, bool> seen;
  std::lock_guard<std::mutex> lk(mu);
  auto it = seen.find(kern);
  if (it != seen.end()) return it->second;
  hipFuncAttributes attr{};
  const bool ok = hipFuncGetAttributes(&attr, kern) == hipSuccess && attr.sharedSizeBytes == 0;
  seen.emplace(kern, ok);
  return ok;
}

template <typename Kern, typename Params>
hipError_t launch(Kern kern, Params p, size_t lds, uint32_t items, hipStream_t stream) {
  if (items == 0) return hipSuccess;
  const void* k = reinterpret_cast<const void*>(kern);
  if (!lds_starts_at_zero(k)) return hipErrorInvalidKernelFile;
  const int grid = grid_for(k, lds, items);
  p.xcd_split = (grid >= 8 && grid % 8 == 0 && env_flag("ECAMD_XCD", true)) ? 1u : 0u;

  hipLaunchKernelGGL(kern, dim3(grid), dim3(kThreadsPerBlock), lds, stream, p);
  return hipGetLastError();
}

// Bytes of the last data fragment that lie inside the object (encode inputs
// and decode outputs stop there; <= bs).
inline int64_t last_room(uint32_t bs, uint64_t obj_len, uint32_t k) {
  int64_t room = static_cast<int64_t>(obj_len) - static_cast<int64_t>(k - 1) * bs;
  if (room > static_cast<int64_t>(bs)) room = bs;
  return room < 0 ? 0 : room;
}

// Cache-policy variant requested through the environment (A/B of the
// benchmark case only): ECAMD_LD_CACHED=0/1, ECAMD_ST_CACHED=0/1.
inline int env_policy(int dflt) {
  return (env_flag("ECAMD_LD_CACHED", dflt & kPolLoadsCached) ? kPolLoadsCached : 0) |
         (env_flag("ECAMD_ST_CACHED", dflt & kPolStoresCached) ? kPolStoresCached : 0);
}

// Defaults, measured on MI355X (round 2, tools/ab_bench.py, k=10 m=4,
// 256 x 4 MiB): encode reads the object slices with the default cache
// policy -- neighbouring slices share 128-B lines, which L2 then serves
// twice (303 vs 308 us); stores stay nontemporal (cached: 331 us).
// Decode stores each lane's 16 B where they belong (446 us) rather than
// through the overlap-lane realignment (456 us): the 1008-B chunks it needs
// cost 12 % more HBM reads and writes than the aligned units save.
constexpr int kEncodePolicy = kPolLoadsCached;
constexpr bool kDecodePlain = true;
constexpr bool kDecodeStaged = false;

template <class F, int K, int NR>
hipError_t launch_encode_k(EncodeParams p, hipStream_t stream) {
  // interior tiles: 4 KiB of positions ending at or before min(bs, room)
  const uint32_t tile = kWavesPerBlock * kChunkBytes;
  p.tiles = static_cast<uint32_t>(last_room(p.bs, p.obj_len, K) / tile);
  p.edge_tiles = (p.bs + tile - 1) / tile - p.tiles;
  const uint32_t items = std::max(std::max(p.n_obj * p.tiles, p.n_obj * p.edge_tiles),
                                  p.headers ? p.n_obj : 0u);
  hipError_t e = hipErrorInvalidValue;
  const int pol = (K == 10 && NR == 4) ? env_policy(kEncodePolicy) : kEncodePolicy;
  bool sdwa = true;
  if constexpr (K == 10 && NR == 4) sdwa = !env_flag("ECAMD_ENC_PERM", false);
  if constexpr (K == 10 && NR == 4) {
    if (pol == kEncodePolicy && env_flag("ECAMD_ENC_NOCOMP", false))
      return launch(encode_kernel<F, K, NR, kEncodePolicy, true, true>, p, K * F::kTableBytes,
                    items, stream);
    if (pol == kEncodePolicy && env_flag("ECAMD_ENC_DEPTH2", false)) {
      e = launch(encode_kernel_d2<F, K, NR, kEncodePolicy>, p, K * F::kTableBytes, items, stream);
      if (e != hipSuccess || p.data == nullptr || p.row0 != 0) return e;
      return launch(copy_data_kernel, p, 0, p.n_obj * K * ((p.bs + tile - 1) / tile), stream);
    }
  }
  if (pol == kEncodePolicy && !sdwa) {
    if constexpr (K == 10 && NR == 4)
      e = launch(encode_kernel<F, K, NR, kEncodePolicy, false>, p, K * F::kTableBytes, items, stream);
  } else if (pol == kEncodePolicy)
    e = launch(encode_kernel<F, K, NR, kEncodePolicy>, p, K * F::kTableBytes, items, stream);
  else if constexpr (K == 10 && NR == 4)
    e = pol == 0   ? launch(encode_kernel<F, K, NR, 0>, p, K * F::kTableBytes, items, stream)
        : pol == 2 ? launch(encode_kernel<F, K, NR, 2>, p, K * F::kTableBytes, items, stream)
                   : launch(encode_kernel<F, K, NR, 3>, p, K * F::kTableBytes, items, stream);
  else
    e = hipErrorInvalidValue;
  if (e != hipSuccess || p.data == nullptr || p.row0 != 0) return e;
  return launch(copy_data_kernel, p, 0, p.n_obj * K * ((p.bs + tile - 1) / tile), stream);
}

template <class F, int K>
hipError_t launch_encode_rows(const EncodeParams& p, hipStream_t stream) {
  switch (p.nrows) {
    case 1:
      return launch_encode_k<F, K, 1>(p, stream);
    case 2:
      return launch_encode_k<F, K, 2>(p, stream);
    case 3:
      return launch_encode_k<F, K, 3>(p, stream);
    case 4:
      return launch_encode_k<F, K, 4>(p, stream);
    default:
      return hipErrorInvalidValue;
  }
}

constexpr int kDecodeOcc = 4;

// LDS of a decode launch: two table slots (+ the staging area).
template <class F, int K, bool STAGED>
constexpr uint32_t decode_lds_bytes() {
  return 2 * table_slot_bytes(K, F::kW) + (STAGED ? 16 + K * kStageTile : 0);
}
// Staged stores need K * 4 KiB of LDS per block; used while two blocks per
// CU still fit (k <= 16 for GF(2^16)).
template <class F, int K>
constexpr bool staged_fits() {
  return decode_lds_bytes<F, K, true>() <= 80u * 1024u;
}

template <class F, int K, int MODE, int OCC, bool PLAIN, int POL = 0, bool STAGED = false,
          bool NOCOMP = false>
hipError_t launch_decode_variant(DecodeParams p, hipStream_t stream) {
  constexpr uint32_t tile = kWavesPerBlock * chunk_stride<MODE, PLAIN>();
  if constexpr (!overlaps<MODE, PLAIN>()) {
    // 4 KiB tiles over the payload (reconstruct) or up to the object's end
    const int64_t lim = MODE == kReconstruct ? static_cast<int64_t>(p.bs)
                                             : last_room(p.bs, p.obj_len, K);
    p.tiles = static_cast<uint32_t>(lim / tile);
    p.edge_tiles = (p.bs + tile - 1) / tile - p.tiles;
  } else {
    // tile T covers loads [T*4032, T*4032 + 4048) and slice bytes up to
    // T*4032 + 4048 - s; it must stay inside min(bs, room)
    const int64_t lim = last_room(p.bs, p.obj_len, K);
    p.tiles = lim >= tile + 16 ? static_cast<uint32_t>((lim - 16) / tile) : 0u;
    p.edge_tiles = 1 + (p.bs - p.tiles * tile + 4095) / 4096;  // head + tail items
  }
  const uint32_t items = std::max(std::max(p.n_obj * p.tiles, p.n_obj * p.edge_tiles),
                                  p.reconstruct ? p.n_obj : 0u);
  return launch(decode_kernel<F, K, MODE, OCC, PLAIN, POL, STAGED, NOCOMP>, p,
                decode_lds_bytes<F, K, STAGED>(), items, stream);
}

template <class F, int K, int MODE>
hipError_t launch_decode_mode(DecodeParams p, hipStream_t stream) {
  if constexpr (K == 10 && MODE == kDecode) {
    if (env_flag("ECAMD_DEC_NOCOMP", false))  // memory-only probe (wrong output)
      return env_flag("ECAMD_DEC_STAGED", kDecodeStaged)
                 ? launch_decode_variant<F, K, MODE, 3, true, 0, true, true>(p, stream)
                 : launch_decode_variant<F, K, MODE, kDecodeOcc, true, 0, false, true>(p, stream);
  }
  if constexpr (MODE == kDecode && staged_fits<F, K>()) {
    // staged, line-friendly object stores (LDS bounds occupancy to 3 blocks
    // per CU at k = 10, so the register budget is 3 waves per SIMD)
    if (env_flag("ECAMD_DEC_STAGED", kDecodeStaged))
      return launch_decode_variant<F, K, MODE, 3, true, 0, true>(p, stream);
  }
  if constexpr (K == 10 && MODE == kDecode) {
    // the benchmark configuration carries the A/B variants
    // (tools/ab_bench.py): ECAMD_DEC_OCC3=1 (3 waves per SIMD, no spills),
    // ECAMD_DEC_PLAIN=1 (unaligned lane stores, no overlap lane)
    const bool plain = env_flag("ECAMD_DEC_PLAIN", kDecodePlain);
    switch (env_policy(0)) {
      case 1:
        return plain ? launch_decode_variant<F, K, MODE, kDecodeOcc, true, 1>(p, stream)
                     : launch_decode_variant<F, K, MODE, kDecodeOcc, false, 1>(p, stream);
      case 2:
        return plain ? launch_decode_variant<F, K, MODE, kDecodeOcc, true, 2>(p, stream)
                     : launch_decode_variant<F, K, MODE, kDecodeOcc, false, 2>(p, stream);
      case 3:
        return plain ? launch_decode_variant<F, K, MODE, kDecodeOcc, true, 3>(p, stream)
                     : launch_decode_variant<F, K, MODE, kDecodeOcc, false, 3>(p, stream);
      default:
        break;
    }
    if (!plain) return launch_decode_variant<F, K, MODE, kDecodeOcc, false>(p, stream);
    if (env_flag("ECAMD_DEC_OCC3", false))
      return launch_decode_variant<F, K, MODE, 3, true>(p, stream);
  }
  return launch_decode_variant<F, K, MODE, kDecodeOcc, kDecodePlain>(p, stream);
}

}  // namespace
}  // namespace ecamd
