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
// Addressing (GF(2^16)).  Table [c][q][v] sits at byte 512c + 128q + 8v.  For
// one input dword x (two symbols, eight nibbles) we build
//   ylo = (x << 3) & 0x78787878               nibbles 0,2,4,6 scaled by 8
//   yhi = ((x >> 1) & 0x78787878) | 0x80..80  nibbles 1,3,5,7 scaled by 8,
//                                             +128 for odd q
// and one v_perm_b32 per lookup assembles {y.byte_b, kb.byte} into the LDS
// byte offset: kb carries the table set's LDS base >> 8 (plus 1 for nibble
// positions 2-3); the per-input 512c lands in the ds_read immediate because
// the input loop is unrolled over a compile-time k.  GF(2^8) is the same with
// 128-B tables, 4-byte entries and one byte per symbol.
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
__device__ __forceinline__ Rsrc rsrc(const void* base) {
  const uint64_t a = reinterpret_cast<uint64_t>(base);
  const uint32_t lo = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(a));
  const uint32_t hi = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(a >> 32));
  return __builtin_amdgcn_make_buffer_rsrc(
      reinterpret_cast<void*>((static_cast<uint64_t>(hi) << 32) | lo), 0, -1, 0x00020000);
}
__device__ __forceinline__ uint4 buf_ld(Rsrc r, uint32_t voff, uint32_t soff) {
  const v4u v = __builtin_amdgcn_raw_buffer_load_b128(r, voff, soff, kNt);
  return make_uint4(v.x, v.y, v.z, v.w);
}
__device__ __forceinline__ void buf_st(Rsrc r, uint32_t voff, uint32_t soff, const uint4& x) {
  v4u v;
  v.x = x.x;
  v.y = x.y;
  v.z = x.z;
  v.w = x.w;
  __builtin_amdgcn_raw_buffer_store_b128(v, r, voff, soff, kNt);
}

// a ^ b ^ c in one VALU op (gfx950 v_bitop3_b32, truth table 0x96)
__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
  return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}

// ---------------- GF(2^16): liberasurecode_rs_vand ----------------

constexpr uint32_t kSel16[4] = {0x0C0C0400u, 0x0C0C0501u, 0x0C0C0402u, 0x0C0C0503u};

// NW = 2: u64 entries (up to 4 rows); NW = 1: rows <= 2, read the low dword
// only (ds_read_b32; same table layout).
template <int NW>
struct Gf16 {
  static constexpr uint32_t kW = 16;
  static constexpr uint32_t kTableBytes = 512;
  struct Acc {
    uint2 s[8];  // s[2d] / s[2d+1]: rows 0-3 of the low / high symbol of input dword d
  };
  static __device__ __forceinline__ uint32_t kb(uint32_t base) {
    return (base >> 8) * 0x0101u + 0x0100u;
  }
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
  static __device__ __forceinline__ void mac_dword(uint32_t kb, uint32_t tab, uint32_t x,
                                                   uint2& s_lo, uint2& s_hi) {
    const uint32_t ylo = (x << 3) & 0x78787878u;
    const uint32_t yhi = ((x >> 1) & 0x78787878u) | 0x80808080u;
    const uint32_t a0 = __builtin_amdgcn_perm(kb, ylo, kSel16[0]);
    const uint32_t a1 = __builtin_amdgcn_perm(kb, yhi, kSel16[0]);
    const uint32_t a2 = __builtin_amdgcn_perm(kb, ylo, kSel16[1]);
    const uint32_t a3 = __builtin_amdgcn_perm(kb, yhi, kSel16[1]);
    const uint32_t a4 = __builtin_amdgcn_perm(kb, ylo, kSel16[2]);
    const uint32_t a5 = __builtin_amdgcn_perm(kb, yhi, kSel16[2]);
    const uint32_t a6 = __builtin_amdgcn_perm(kb, ylo, kSel16[3]);
    const uint32_t a7 = __builtin_amdgcn_perm(kb, yhi, kSel16[3]);
    if constexpr (NW == 2) {
      const uint2 e0 = lds_u64(a0, tab), e1 = lds_u64(a1, tab), e2 = lds_u64(a2, tab),
                  e3 = lds_u64(a3, tab);
      const uint2 e4 = lds_u64(a4, tab), e5 = lds_u64(a5, tab), e6 = lds_u64(a6, tab),
                  e7 = lds_u64(a7, tab);
      s_lo.x = xor3(xor3(s_lo.x, e0.x, e1.x), e2.x, e3.x);
      s_lo.y = xor3(xor3(s_lo.y, e0.y, e1.y), e2.y, e3.y);
      s_hi.x = xor3(xor3(s_hi.x, e4.x, e5.x), e6.x, e7.x);
      s_hi.y = xor3(xor3(s_hi.y, e4.y, e5.y), e6.y, e7.y);
    } else {
      s_lo.x = xor3(xor3(s_lo.x, lds_u32(a0, tab), lds_u32(a1, tab)), lds_u32(a2, tab),
                    lds_u32(a3, tab));
      s_hi.x = xor3(xor3(s_hi.x, lds_u32(a4, tab), lds_u32(a5, tab)), lds_u32(a6, tab),
                    lds_u32(a7, tab));
    }
  }
  // The scheduling barriers stop hipcc from hoisting every LDS lookup of the
  // unrolled input loop ahead of the XORs that consume them (2 VGPRs each).
  static __device__ __forceinline__ void mac(uint32_t kb, uint32_t tab, const uint4& x, Acc& a) {
    mac_dword(kb, tab, x.x, a.s[0], a.s[1]);
    __builtin_amdgcn_sched_barrier(0);
    mac_dword(kb, tab, x.y, a.s[2], a.s[3]);
    __builtin_amdgcn_sched_barrier(0);
    mac_dword(kb, tab, x.z, a.s[4], a.s[5]);
    __builtin_amdgcn_sched_barrier(0);
    mac_dword(kb, tab, x.w, a.s[6], a.s[7]);
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

// One wave writes `count` 80-byte headers (fragment f at frag0 + f*stride).
__device__ __forceinline__ void copy_headers(uint8_t* frag0, uint64_t stride, const uint8_t* hdr,
                                             uint32_t count) {
  for (uint32_t i = lane_id(); i < count * 5; i += kLanes) {
    const uint32_t f = i / 5, part = i - f * 5;
    reinterpret_cast<uint4*>(frag0 + f * stride)[part] =
        reinterpret_cast<const uint4*>(hdr + f * kHeaderBytes)[part];
  }
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
// Chunk = 1 KiB of payload positions of one object (64 lanes x 16 B): one
// wave-instruction per input and per output.  Chunks [0, chunks) of every
// fragment are "interior": every lane reads 16 in-bounds bytes from every
// input and writes 16 bytes to every output, so they run with no bounds
// checks.  The flattened interior space (object-major) is cut into one
// contiguous range per wave, balanced to +-1 chunk, and each wave walks its
// range in order.  So consecutive chunks of a fragment are read (encode: the
// unaligned object slices) and written (decode: the unaligned object slices)
// by ONE wave back to back: the 128-B lines two chunks share are fetched once
// and written whole, and no other CU ever touches them.  Chunks [chunks,
// chunks + edge_chunks) -- at most two per object: the payload tail and the
// chunk reaching the zero padding / the end of the object -- are "edge" items
// with per-lane bounds, dealt to the waves from the other end of the grid.
//
// XCD placement (speed only): workgroups are dealt round-robin over the 8
// XCDs (MI355X_MICROARCH.md), so with xcd_split the range index is made
// XCD-major -- the waves of one XCD own one contiguous eighth of the space,
// and the few lines shared at range boundaries stay inside one L2.

__device__ __forceinline__ uint32_t global_wave(uint32_t xcd_split) {
  uint32_t b = blockIdx.x;
  if (xcd_split) b = (b & 7u) * (gridDim.x >> 3) + (b >> 3);
  return b * kWavesPerBlock + wave_in_block();
}

// Chunk schedule of one wave over the flattened interior space [0, total).
// run == 0: one contiguous range per wave.  run == R > 0: runs of R chunks
// dealt round-robin to the waves (run r to wave r mod W), so at any moment
// the waves of the grid work on one compact region of memory (DRAM row
// locality) while each wave still walks R chunks in order.
struct Sched {
  uint32_t total, run, waves;
  uint32_t begin, end;  // current run [begin, end)
  __device__ __forceinline__ bool valid() const { return begin < end; }
  // the run after the current one (begin >= end when there is none)
  __device__ __forceinline__ void advance() {
    if (run == 0) {
      begin = end;
      return;
    }
    const uint64_t nb = static_cast<uint64_t>(begin - begin % run) + static_cast<uint64_t>(waves) * run;
    begin = nb < total ? static_cast<uint32_t>(nb) : total;
    end = min(total, begin + run);
  }
};
__device__ __forceinline__ Sched make_sched(uint32_t total, uint32_t run, uint32_t g) {
  const uint32_t waves = gridDim.x * kWavesPerBlock;
  Sched S{total, run, waves, 0, 0};
  if (run == 0) {
    S.begin = static_cast<uint32_t>(static_cast<uint64_t>(total) * g / waves);
    S.end = static_cast<uint32_t>(static_cast<uint64_t>(total) * (g + 1) / waves);
  } else {
    const uint64_t b = static_cast<uint64_t>(g) * run;
    S.begin = b < total ? static_cast<uint32_t>(b) : total;
    S.end = min(total, S.begin + run);
  }
  return S;
}
// Flattened index of the chunk after i in the wave's schedule (i itself when
// i is the wave's last chunk); advances S across runs.
__device__ __forceinline__ uint32_t sched_next(Sched& S, uint32_t i, bool& last) {
  if (i + 1 < S.end) {
    last = false;
    return i + 1;
  }
  Sched n = S;
  n.advance();
  last = !n.valid();
  return last ? i : n.begin;
}

__device__ __forceinline__ void next_chunk(uint32_t chunks, uint32_t& o, uint32_t& c) {
  if (++c == chunks) {
    c = 0;
    ++o;
  }
}

// ---------------- encode ----------------

template <int K>
__device__ __forceinline__ void encode_load(const EncodeParams& p, uint32_t o, uint32_t c,
                                            uint4 (&x)[K]) {
  const Rsrc r = rsrc(p.objs + static_cast<uint64_t>(o) * p.obj_stride);
#pragma unroll
  for (int j = 0; j < K; ++j) x[j] = buf_ld(r, lane_id() * 16, j * p.bs + c * kChunkBytes);
}

// One interior chunk with its inputs in `cur`; first issues the loads of the
// wave's next chunk (on, cn) into `nxt` so they are in flight during the
// table lookups.  The last chunk of a range "prefetches" itself again (an L2
// hit): every memory operation in the loop body is unconditional, so hipcc's
// s_waitcnt before cur[j] waits only for cur's own loads (a branch around a
// load or store makes it fall back to the shortest path's count, measured in
// round 1 as waiting for the prefetch too).
template <class F, int K, int NR>
__device__ __forceinline__ void encode_item(const EncodeParams& p, uint32_t o, uint32_t c,
                                            uint32_t on, uint32_t cn, uint4 (&cur)[K],
                                            uint4 (&nxt)[K]) {
  encode_load<K>(p, on, cn, nxt);
  typename F::Acc s;
  F::zero(s);
#pragma unroll
  for (int j = 0; j < K; ++j) F::mac(F::kb(0), j * F::kTableBytes, cur[j], s);
  F::pin(s);
  const Rsrc par = rsrc(p.parity + static_cast<uint64_t>(o) * p.stripe_stride);
  const uint32_t soff = p.row0 * p.frag_stride + kHeaderBytes + c * kChunkBytes;
#pragma unroll
  for (int q = 0; q < NR; ++q) buf_st(par, lane_id() * 16, soff + q * p.frag_stride, F::row(s, q));
}

// Edge chunk: payload tail (t + 16 > bs) and chunks reaching the zero padding
// past obj_len (liberasurecode's prepare_fragments_for_encode zero-fills).
template <class F, int K, int NR>
__device__ __forceinline__ void encode_edge_item(const EncodeParams& p, uint32_t e) {
  const uint32_t o = e / p.edge_chunks;
  const uint32_t c = p.chunks + (e - o * p.edge_chunks);
  const uint32_t t = c * kChunkBytes + lane_id() * 16;
  if (t >= p.bs) return;
  const uint8_t* obj = p.objs + static_cast<uint64_t>(o) * p.obj_stride;
  const int64_t rem = static_cast<int64_t>(p.bs) - t;
  uint4 x[K];
#pragma unroll
  for (int j = 0; j < K; ++j) x[j] = load_clamped(obj, static_cast<uint64_t>(j) * p.bs + t, p.obj_len);
  typename F::Acc s;
  F::zero(s);
#pragma unroll
  for (int j = 0; j < K; ++j) F::mac(F::kb(0), j * F::kTableBytes, x[j], s);
  F::pin(s);
  uint8_t* par = p.parity + static_cast<uint64_t>(o) * p.stripe_stride + p.row0 * p.frag_stride +
                 kHeaderBytes + t;
#pragma unroll
  for (int q = 0; q < NR; ++q) store_partial(par + q * p.frag_stride, F::row(s, q), rem);
}

template <class F, int K, int NR>
__global__ void __launch_bounds__(kThreadsPerBlock) encode_kernel(EncodeParams p) {
  load_tables(p.tables, K * F::kTableBytes, 0);
  const uint32_t g = global_wave(p.xcd_split);
  const uint32_t G = gridDim.x * kWavesPerBlock;
  if (p.headers != nullptr && p.row0 == 0)
    for (uint32_t o = g; o < p.n_obj; o += G) {
      const uint64_t base = static_cast<uint64_t>(o) * p.stripe_stride;
      copy_headers(p.parity + base, p.frag_stride, p.headers + K * kHeaderBytes, p.m);
      if (p.data != nullptr) copy_headers(p.data + base, p.frag_stride, p.headers, K);
    }
  __syncthreads();
  Sched S = make_sched(p.n_obj * p.chunks, p.run_chunks, g);
  if (S.valid()) {
    uint4 xa[K], xb[K];
    uint32_t i = S.begin;
    encode_load<K>(p, i / p.chunks, i % p.chunks, xa);
    // two chunks per trip so cur / nxt stay compile-time register arrays
    while (true) {
      bool last;
      uint32_t ni = sched_next(S, i, last);
      encode_item<F, K, NR>(p, i / p.chunks, i % p.chunks, ni / p.chunks, ni % p.chunks, xa, xb);
      if (last) break;
      if (ni >= S.end) S.advance();
      i = ni;
      ni = sched_next(S, i, last);
      encode_item<F, K, NR>(p, i / p.chunks, i % p.chunks, ni / p.chunks, ni % p.chunks, xb, xa);
      if (last) break;
      if (ni >= S.end) S.advance();
      i = ni;
    }
  }
  const uint32_t n_edge = p.n_obj * p.edge_chunks;
  for (uint32_t e = G - 1 - g; e < n_edge; e += G) encode_edge_item<F, K, NR>(p, e);
}

// Data fragments (optional output of encode): the k padded object slices
// copied into their fragment payloads, one wave per (object, fragment, chunk).
__global__ void __launch_bounds__(kThreadsPerBlock) copy_data_kernel(EncodeParams p) {
  const uint32_t per_frag = p.chunks + p.edge_chunks;
  const uint32_t per_obj = p.k * per_frag;
  const uint32_t items = p.n_obj * per_obj;
  const uint32_t G = gridDim.x * kWavesPerBlock;
  for (uint32_t w = blockIdx.x * kWavesPerBlock + wave_in_block(); w < items; w += G) {
    const uint32_t o = w / per_obj, rest = w - o * per_obj;
    const uint32_t j = rest / per_frag, c = rest - j * per_frag;
    const uint32_t t = c * kChunkBytes + lane_id() * 16;
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
// pattern's decode rows).  Every wave owns one LDS slot and loads a set into
// it when its run moves to an object with a different pattern -- no
// workgroup barrier, since a wave's LDS operations execute in order.
//
// Realigned object stores.  Decode writes data slice j of an object at
// j*bs + t, and bs is rarely a multiple of 16 (419,432 = 8 mod 16 at 4 MiB,
// k = 10), so a plain 16-B lane store would straddle two 16-B units (the
// memory pipeline splits it in two, and the lines at both ends of every wave
// access are written as partial lines).  The shift s = (j*bs) mod 16 is
// uniform over the slice, so each lane instead stores the aligned unit that
// starts s bytes below its own address: the last s bytes of lane L-1's data
// (DPP wave_shr:1) and its own first 16 - s bytes.  Lane 0 takes its s bytes
// from lane 63 of the wave's previous chunk of the same slice, kept in SGPRs
// (`carry`, v_readlane) -- so along a run every store is one aligned
// dwordx4, and only the first chunk's lane 0 (head) and the run's last s
// bytes (tail) are written piecewise.

// Carries live in four VGPRs, one per dword: lane i of cw[w] holds dword w of
// slot i's carry (slot = the store's position in the item: input / row).
struct Carry {
  uint32_t w[4];
};
// v with lane LANE replaced by the uniform value x (v_writelane_b32; hipcc
// has no builtin for it).  The lane select is an inline constant: with an
// SGPR it would be the instruction's second constant-bus read.
template <int LANE>
__device__ __forceinline__ uint32_t writelane(uint32_t v, uint32_t x) {
  asm("v_writelane_b32 %0, %1, %2" : "+v"(v) : "s"(x), "i"(LANE));
  return v;
}

// f(std::integral_constant<int, I>) for I = 0 .. N-1, each I a compile-time
// constant (the carry slot of a store must be one).
template <int I, int N, class Fn>
__device__ __forceinline__ void static_for(Fn&& f) {
  if constexpr (I < N) {
    f(std::integral_constant<int, I>{});
    static_for<I + 1, N>(f);
  }
}
__device__ __forceinline__ uint32_t shr1(uint32_t v, uint32_t old) {
  return static_cast<uint32_t>(__builtin_amdgcn_update_dpp(
      static_cast<int>(old), static_cast<int>(v), 0x138 /* wave_shr:1 */, 0xF, 0xF, false));
}

// Store a lane's 16 B `v` for `dst` (dst mod 16 == s, uniform) of one chunk
// of a run: the unit at dst - s = last s bytes of lane L-1's v (lane 0: the
// carried lane 63 of the previous chunk) + first 16 - s bytes of its own.
// Only the dwords of the previous lane that the unit uses are moved (dword
// offset d = (16 - s) / 4).  FIRST: the run's first chunk (no carry yet:
// lane 0 writes only its own bytes).  Every path issues exactly one vector
// store instruction, so the s_waitcnt counts hipcc derives stay exact.
// (The destination is out + soff + 16*lane; outp is `out` as a pointer.)
template <bool FIRST, int SLOT>
__device__ __forceinline__ void st_slice(Rsrc out, uint8_t* outp, uint32_t soff, const uint4& v,
                                         uint32_t s, Carry& cw) {
  if (s == 0) {
    buf_st(out, lane_id() * 16, soff, v);
    return;
  }
  const uint32_t st = 16u - s, r = st & 3u;
  uint4 u;
  const uint32_t vv[4] = {v.x, v.y, v.z, v.w};
  // pv_i = dword i of lane L-1's v (lane 0: carry); update the carry with
  // lane 63's dword i for the next chunk
#define ECAMD_PV(i)                                                                 \
  const uint32_t pv##i = shr1(vv[i], __builtin_amdgcn_readlane(cw.w[i], SLOT));     \
  cw.w[i] = writelane<SLOT>(cw.w[i], __builtin_amdgcn_readlane(vv[i], 63));
  switch (st >> 2) {
    case 0: {
      ECAMD_PV(0) ECAMD_PV(1) ECAMD_PV(2) ECAMD_PV(3)
      u = make_uint4(__builtin_amdgcn_alignbyte(pv1, pv0, r), __builtin_amdgcn_alignbyte(pv2, pv1, r),
                     __builtin_amdgcn_alignbyte(pv3, pv2, r), __builtin_amdgcn_alignbyte(v.x, pv3, r));
      break;
    }
    case 1: {
      ECAMD_PV(1) ECAMD_PV(2) ECAMD_PV(3)
      u = make_uint4(__builtin_amdgcn_alignbyte(pv2, pv1, r), __builtin_amdgcn_alignbyte(pv3, pv2, r),
                     __builtin_amdgcn_alignbyte(v.x, pv3, r), __builtin_amdgcn_alignbyte(v.y, v.x, r));
      break;
    }
    case 2: {
      ECAMD_PV(2) ECAMD_PV(3)
      u = make_uint4(__builtin_amdgcn_alignbyte(pv3, pv2, r), __builtin_amdgcn_alignbyte(v.x, pv3, r),
                     __builtin_amdgcn_alignbyte(v.y, v.x, r), __builtin_amdgcn_alignbyte(v.z, v.y, r));
      break;
    }
    default: {
      ECAMD_PV(3)
      u = make_uint4(__builtin_amdgcn_alignbyte(v.x, pv3, r), __builtin_amdgcn_alignbyte(v.y, v.x, r),
                     __builtin_amdgcn_alignbyte(v.z, v.y, r), __builtin_amdgcn_alignbyte(v.w, v.z, r));
      break;
    }
  }
#undef ECAMD_PV
  if (FIRST && lane_id() == 0)
    put_bytes(outp + soff, v, 0, 16 - s);
  else
    buf_st(out, lane_id() * 16, soff - s, u);
}

// After a run: bytes [end - s, end) of the slice are the last s bytes of the
// final chunk's lane 63, i.e. dwords of the carry.
__device__ __forceinline__ void st_slice_tail(uint8_t* end, uint32_t s, const Carry& cw,
                                              int slot) {
  if (s == 0) return;
  const uint4 c = make_uint4(__builtin_amdgcn_readlane(cw.w[0], slot),
                             __builtin_amdgcn_readlane(cw.w[1], slot),
                             __builtin_amdgcn_readlane(cw.w[2], slot),
                             __builtin_amdgcn_readlane(cw.w[3], slot));
  if (lane_id() == 0) put_bytes(end - s, c, 16 - s, s);
}

// Make the table set current in this wave's LDS slot; returns its kb.
template <class F, int K>
__device__ __forceinline__ uint32_t wave_tables(const DecodeParams& p, uint32_t table,
                                                uint32_t& cur) {
  constexpr uint32_t kSlot = table_slot_bytes(K, F::kW);
  const uint32_t base = wave_in_block() * kSlot;
  if (table != cur) {
    const v4u* src =
        reinterpret_cast<const v4u*>(p.tables + static_cast<uint64_t>(table) * (K * F::kTableBytes / 4));
    auto* dst = lds_v4(base);
    for (uint32_t i = lane_id(); i < K * F::kTableBytes / 16; i += kLanes) dst[i] = src[i];
    cur = table;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  }
  return F::kb(base);
}

// Fragment group position of input c.
__device__ __forceinline__ uint32_t in_pos(const DecodeParams& p, const ObjDesc& d, int c) {
  return p.compact ? static_cast<uint32_t>(c) : d.in_idx[c];
}

template <int K>
__device__ __forceinline__ void decode_load(const DecodeParams& p, const ObjDesc& d, Rsrc in,
                                            uint32_t c, uint4 (&x)[K]) {
#pragma unroll
  for (int j = 0; j < K; ++j)
    x[j] = buf_ld(in, lane_id() * 16, in_pos(p, d, j) * p.frag_stride + kHeaderBytes + c * kChunkBytes);
}

enum DecodeMode : int {
  kDecode = 0,       // pass 0 and every missing row in it: all k data slices stored
  kReconstruct = 1,  // one fragment per object (aligned payload)
  kDecodeGeneric = 2 // other passes (more than 4 missing data fragments)
};

// Per-run constants, uniform over the wave.
struct RunCtx {
  Rsrc in;       // the object's fragment group
  Rsrc out;      // the object (decode) or output fragment (reconstruct)
  uint8_t* outp; // same, as a pointer (partial head / tail stores)
  uint32_t kb;
  uint32_t e;    // decode: missing data slices computed here
};

// kDecode: the k inputs are the first k available fragments in ascending
// order, so the present data fragments come first and the parity inputs --
// as many as there are missing data slices, e -- are the last e.  After the
// products, row q overwrites parity input K-e+q: cur[c] then holds data slice
// slice_of(c) for every c, and all K slices are stored unconditionally.
__device__ __forceinline__ uint32_t slice_of(const ObjDesc& d, uint32_t e, int K, int c) {
  return c < K - static_cast<int>(e) ? d.in_idx[c] : d.out_idx[c - (K - static_cast<int>(e))];
}

template <class F, int K>
__device__ __forceinline__ void place_rows(const typename F::Acc& s, uint32_t e, uint4 (&x)[K]) {
  constexpr int L = K < 4 ? K : 4;
  switch (e) {
#define ECAMD_PLACE(E)                                                    \
  case E:                                                                 \
    if constexpr (E <= L) {                                               \
      _Pragma("unroll") for (int q = 0; q < E; ++q) x[K - E + q] = F::row(s, q); \
    }                                                                     \
    break;
    ECAMD_PLACE(1) ECAMD_PLACE(2) ECAMD_PLACE(3) ECAMD_PLACE(4)
#undef ECAMD_PLACE
    default:
      break;
  }
}

template <class F, int K, int MODE, bool FIRST>
__device__ __forceinline__ void decode_item(const DecodeParams& p, const ObjDesc& d,
                                            const RunCtx& R, uint32_t c, uint32_t cn,
                                            uint4 (&cur)[K], uint4 (&nxt)[K], Carry& cw) {
  decode_load<K>(p, d, R.in, cn, nxt);
  const uint32_t t = c * kChunkBytes;  // + 16*lane in voffset
  typename F::Acc s;
  F::zero(s);
  const uint32_t n_rows = MODE == kDecode ? R.e : d.n_out;
  if (n_rows != 0) {
#pragma unroll
    for (int j = 0; j < K; ++j) F::mac(R.kb, j * F::kTableBytes, cur[j], s);
  }
  F::pin(s);
  if constexpr (MODE == kDecode) {
    place_rows<F, K>(s, R.e, cur);
    static_for<0, K>([&](auto J) {
      const uint32_t off = slice_of(d, R.e, K, J) * p.bs;
      st_slice<FIRST, J>(R.out, R.outp, off + t, cur[J], off & 15u, cw);
    });
  } else if constexpr (MODE == kReconstruct) {
    buf_st(R.out, lane_id() * 16, kHeaderBytes + t, F::row(s, 0));
  } else {
    if (d.copy_inputs) {
      static_for<0, K>([&](auto J) {
        const uint32_t idx = d.in_idx[J];
        if (idx < static_cast<uint32_t>(K)) {
          const uint32_t off = idx * p.bs;
          st_slice<FIRST, J>(R.out, R.outp, off + t, cur[J], off & 15u, cw);
        }
      });
    }
    static_for<0, kRowsPerPass>([&](auto Q) {
      if (Q < static_cast<int>(d.n_out)) {
        const uint32_t off = d.out_idx[Q] * p.bs;
        st_slice<FIRST, K + Q>(R.out, R.outp, off + t, F::row(s, Q), off & 15u, cw);
      }
    });
  }
}

// Chunks [c0, c1) of object o.
template <class F, int K, int MODE>
__device__ __forceinline__ void decode_run(const DecodeParams& p, uint32_t o, uint32_t c0,
                                           uint32_t c1, uint32_t& cur_table) {
  const ObjDesc& d = p.desc[o];
  RunCtx R;
  R.in = rsrc(p.frags + static_cast<uint64_t>(o) * p.stripe_stride);
  R.outp = p.out + static_cast<uint64_t>(o) * p.out_stride;
  R.out = rsrc(R.outp);
  R.e = d.n_out;
  R.kb = d.n_out != 0 ? wave_tables<F, K>(p, d.table, cur_table) : 0u;
  uint4 xa[K], xb[K];
  Carry cw = {{0, 0, 0, 0}};
  decode_load<K>(p, d, R.in, c0, xa);
  uint32_t c = c0;
  decode_item<F, K, MODE, true>(p, d, R, c, c + 1 < c1 ? c + 1 : c, xa, xb, cw);
  while (++c < c1) {
    decode_item<F, K, MODE, false>(p, d, R, c, c + 1 < c1 ? c + 1 : c, xb, xa, cw);
    if (++c >= c1) break;
    decode_item<F, K, MODE, false>(p, d, R, c, c + 1 < c1 ? c + 1 : c, xa, xb, cw);
  }
  if constexpr (MODE != kReconstruct) {
    uint8_t* end = R.outp + c1 * kChunkBytes;
    if constexpr (MODE == kDecode) {
#pragma unroll
      for (int j = 0; j < K; ++j) {
        const uint32_t off = slice_of(d, R.e, K, j) * p.bs;
        st_slice_tail(end + off, off & 15u, cw, j);
      }
    } else {
      if (d.copy_inputs) {
#pragma unroll
        for (int j = 0; j < K; ++j) {
          const uint32_t idx = d.in_idx[j];
          if (idx < static_cast<uint32_t>(K)) {
            const uint32_t off = idx * p.bs;
            st_slice_tail(end + off, off & 15u, cw, j);
          }
        }
      }
#pragma unroll
      for (int q = 0; q < kRowsPerPass; ++q)
        if (q < static_cast<int>(d.n_out)) {
          const uint32_t off = d.out_idx[q] * p.bs;
          st_slice_tail(end + off, off & 15u, cw, K + q);
        }
    }
  }
}

// Edge chunk of decode / reconstruct: payload tail, and (decode) outputs
// that cross the end of the object.  Byte-exact stores.
template <class F, int K>
__device__ __forceinline__ void decode_edge_item(const DecodeParams& p, uint32_t e,
                                                 uint32_t& cur_table) {
  const uint32_t o = e / p.edge_chunks;
  const uint32_t c = p.chunks + (e - o * p.edge_chunks);
  const ObjDesc& d = p.desc[o];
  const uint32_t kb = d.n_out != 0 ? wave_tables<F, K>(p, d.table, cur_table) : 0u;
  const uint32_t t = c * kChunkBytes + lane_id() * 16;
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
  if (d.n_out != 0) {
#pragma unroll
    for (int j = 0; j < K; ++j) F::mac(kb, j * F::kTableBytes, x[j], s);
  }
  F::pin(s);
  if (d.copy_inputs) {
#pragma unroll
    for (int j = 0; j < K; ++j) {
      const uint32_t idx = d.in_idx[j];
      if (idx >= K) continue;
      const int64_t n = object_bytes(idx, p.bs, t, p.obj_len);
      if (n > 0) store_partial(out + static_cast<uint64_t>(idx) * p.bs + t, x[j], n);
    }
  }
  for (uint32_t q = 0; q < d.n_out; ++q) {
    if (p.reconstruct) {
      store_partial(out + kHeaderBytes + t, F::row(s, q), static_cast<int64_t>(p.bs) - t);
    } else {
      const uint32_t idx = d.out_idx[q];
      const int64_t n = object_bytes(idx, p.bs, t, p.obj_len);
      if (n > 0) store_partial(out + static_cast<uint64_t>(idx) * p.bs + t, F::row(s, q), n);
    }
  }
}

template <class F, int K, int MODE>
__global__ void __launch_bounds__(kThreadsPerBlock) __attribute__((amdgpu_waves_per_eu(4)))
decode_kernel(DecodeParams p) {
  const uint32_t g = global_wave(p.xcd_split);
  const uint32_t G = gridDim.x * kWavesPerBlock;
  if (MODE == kReconstruct && p.headers != nullptr)
    for (uint32_t o = g; o < p.n_obj; o += G)
      copy_headers(p.out + static_cast<uint64_t>(o) * p.out_stride, 0,
                   p.headers + static_cast<uint64_t>(p.desc[o].header) * kHeaderBytes, 1);
  uint32_t cur_table = 0xFFFFFFFFu;
  for (Sched S = make_sched(p.n_obj * p.chunks, p.run_chunks, g); S.valid(); S.advance()) {
    for (uint32_t i = S.begin; i < S.end;) {  // split the run at object boundaries
      const uint32_t o = i / p.chunks, c0 = i - o * p.chunks;
      const uint32_t c1 = min(p.chunks, c0 + (S.end - i));
      decode_run<F, K, MODE>(p, o, c0, c1, cur_table);
      i += c1 - c0;
    }
  }
  const uint32_t n_edge = p.n_obj * p.edge_chunks;
  for (uint32_t e = G - 1 - g; e < n_edge; e += G) decode_edge_item<F, K>(p, e, cur_table);
}

// ---------------- launch ----------------

inline bool env_flag(const char* name, bool dflt) {
  const char* v = std::getenv(name);
  if (v == nullptr || *v == 0) return dflt;
  return v[0] != '0';
}

// Schedule tuning (read at each launch so tools/ab_bench.py can compare them
// in one process): ECAMD_RUN = chunks per run (0 = one contiguous range per
// wave).
constexpr uint32_t kDefaultRunChunks = 8;
inline uint32_t env_uint(const char* name, uint32_t dflt) {
  const char* v = std::getenv(name);
  if (v == nullptr || *v == 0) return dflt;
  return static_cast<uint32_t>(std::strtoul(v, nullptr, 10));
}

// Resident workgroups for the kernel (a multiple of 8 when >= 8, so the XCD
// split is even), capped by the work available.
inline int grid_for(const void* kernel, size_t lds_bytes, uint32_t wave_items) {
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
  // (MI355X_MICROARCH.md, Residency); stay at <= 4 per CU.
  per_cu = std::min(per_cu, 4);
  const uint32_t resident = static_cast<uint32_t>(cus * per_cu);
  const uint32_t want = std::max<uint32_t>(1, (wave_items + kWavesPerBlock - 1) / kWavesPerBlock);
  uint32_t grid = std::min(resident, want);
  if (grid >= 8) grid &= ~7u;
  return static_cast<int>(grid);
}

// Interior chunks per fragment: chunks whose 1 KiB of positions end at or
// before min(bs, room), where room = payload bytes of the last data fragment
// that lie inside the object (decode outputs / encode inputs stop there).
inline void split_chunks(uint32_t bs, uint64_t obj_len, uint32_t k, bool whole_payload,
                         uint32_t& chunks, uint32_t& edge_chunks) {
  const uint32_t total = (bs + kChunkBytes - 1) / kChunkBytes;
  int64_t room = whole_payload ? static_cast<int64_t>(bs)
                               : static_cast<int64_t>(obj_len) - static_cast<int64_t>(k - 1) * bs;
  if (room > static_cast<int64_t>(bs)) room = bs;
  if (room < 0) room = 0;
  chunks = static_cast<uint32_t>(room / kChunkBytes);
  edge_chunks = total - chunks;
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
hipError_t launch(Kern kern, Params p, size_t lds, uint32_t wave_items, hipStream_t stream) {
  if (wave_items == 0) return hipSuccess;
  const void* k = reinterpret_cast<const void*>(kern);
  if (!lds_starts_at_zero(k)) return hipErrorInvalidKernelFile;
  const int grid = grid_for(k, lds, wave_items);
  p.xcd_split = (grid >= 8 && grid % 8 == 0 && env_flag("ECAMD_XCD", true)) ? 1u : 0u;
  p.run_chunks = env_uint("ECAMD_RUN", kDefaultRunChunks);
  hipLaunchKernelGGL(kern, dim3(grid), dim3(kThreadsPerBlock), lds, stream, p);
  return hipGetLastError();
}

template <class F, int K, int NR>
hipError_t launch_encode_k(EncodeParams p, hipStream_t stream) {
  split_chunks(p.bs, p.obj_len, K, false, p.chunks, p.edge_chunks);
  const uint32_t items = std::max(p.n_obj * p.chunks,
                                  std::max(p.n_obj * p.edge_chunks, p.headers ? p.n_obj : 0u));
  hipError_t e = launch(encode_kernel<F, K, NR>, p, K * F::kTableBytes, items, stream);
  if (e != hipSuccess || p.data == nullptr || p.row0 != 0) return e;
  return launch(copy_data_kernel, p, 0, p.n_obj * K * (p.chunks + p.edge_chunks), stream);
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

template <class F, int K, int MODE>
hipError_t launch_decode_mode(DecodeParams p, hipStream_t stream) {
  split_chunks(p.bs, p.obj_len, K, p.reconstruct != 0, p.chunks, p.edge_chunks);
  const uint32_t items = std::max(p.n_obj * p.chunks,
                                  std::max(p.n_obj * p.edge_chunks, p.reconstruct ? p.n_obj : 0u));
  const size_t lds = kWavesPerBlock * table_slot_bytes(K, F::kW);
  return launch(decode_kernel<F, K, MODE>, p, lds, items, stream);
}

}  // namespace
}  // namespace ecamd
