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
// start at j*bs, which is only 2-byte (GF(2^16)) or 1-byte aligned; the loads
// rely on gfx9's unaligned-access mode for those inputs.
#pragma once

#include <algorithm>
#include <cstdlib>
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

// 16 bytes at base+off; bytes at or past `len` read as zero (encode padding).
__device__ __forceinline__ uint4 load_clamped(const uint8_t* base, uint64_t off, uint64_t len) {
  if (off + 16 <= len) return *reinterpret_cast<const uint4*>(base + off);
  uint32_t w[4] = {0, 0, 0, 0};
  for (int i = 0; i < 16; ++i)
    if (off + i < len) w[i >> 2] |= static_cast<uint32_t>(base[off + i]) << (8 * (i & 3));
  return make_uint4(w[0], w[1], w[2], w[3]);
}

// Store the first `n` (> 0) bytes of v at dst.
__device__ __forceinline__ void store_partial(uint8_t* dst, const uint4& v, int64_t n) {
  if (n >= 16) {
    *reinterpret_cast<uint4*>(dst) = v;
    return;
  }
  const uint32_t w[4] = {v.x, v.y, v.z, v.w};
  for (int64_t i = 0; i < n; ++i) dst[i] = static_cast<uint8_t>(w[i >> 2] >> (8 * (i & 3)));
}

__device__ __forceinline__ void copy_headers(uint8_t* frag0, uint64_t stride, const uint8_t* hdr,
                                             uint32_t count) {
  for (uint32_t i = threadIdx.x; i < count * 5; i += blockDim.x) {
    const uint32_t f = i / 5, part = i - f * 5;
    reinterpret_cast<uint4*>(frag0 + f * stride)[part] =
        reinterpret_cast<const uint4*>(hdr + f * kHeaderBytes)[part];
  }
}

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
// Work item = (object o, tile of 256 lane chunks = 4 KiB of payload
// positions).  Tiles [0, first_edge) of every object are "interior": all
// lanes read 16 in-bounds bytes from every input and write 16 bytes to every
// output, so they run with no bounds checks, unrolled over K and with the
// next item's loads in flight (register double buffering).  Tiles
// [first_edge, tiles) -- at most two per object: the payload tail and the
// tile reaching the zero padding / the end of the object -- are "edge" items
// with per-lane bounds; each block takes its share of them before entering
// the interior loop, all K loads of an edge item in flight at once.

__device__ __forceinline__ void tile_of(uint32_t w, uint32_t per_obj, uint32_t first,
                                        uint32_t& o, uint32_t& tile, uint32_t& t) {
  o = w / per_obj;
  tile = first + (w - o * per_obj);
  t = (tile * kThreadsPerBlock + threadIdx.x) << 4;
}

// Interior item ranges.  Blocks are dealt round-robin over the 8 XCDs (blocks
// b and b+8 share one; MI355X_MICROARCH.md), each XCD with its own L2.  With
// xcd_split the item list is cut into 8 contiguous ranges and range x is
// walked, grid-stride, by the blocks with b % 8 == x: neighbouring tiles of a
// fragment then run on one XCD at about the same time, so the 128-B lines
// they share -- the unaligned object slices that encode reads and decode
// writes -- meet in one L2 instead of being fetched twice or written back as
// two partial lines.  Placement only changes speed, never results.
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

// ---------------- encode ----------------

__device__ __forceinline__ void encode_headers(const EncodeParams& p, uint32_t o, uint32_t k) {
  if (p.headers == nullptr) return;
  if (p.row0 == 0)
    copy_headers(p.parity + static_cast<uint64_t>(o) * p.stripe_stride, p.frag_stride,
                 p.headers + k * kHeaderBytes, p.m);
  if (p.data != nullptr)
    copy_headers(p.data + static_cast<uint64_t>(o) * p.stripe_stride, p.frag_stride, p.headers,
                 k);
}

template <int K>
__device__ __forceinline__ void encode_load(const EncodeParams& p, uint32_t o, uint32_t t,
                                            uint4 (&x)[K]) {
  const uint8_t* obj = p.objs + static_cast<uint64_t>(o) * p.obj_stride + t;
#pragma unroll
  for (int j = 0; j < K; ++j) x[j] = ld_stream(obj + static_cast<uint64_t>(j) * p.bs);
}

// One interior item with its inputs in `cur`.  PREFETCH: first issue the
// loads of the block's next item (w + step) into `nxt`, so they are in flight
// while this item's table lookups run.
//
// Every memory operation in here is unconditional (NR output rows, no
// headers, no data copies) so that hipcc's s_waitcnt insertion sees one
// sequence per item: before using cur[j] it then waits only for cur's own
// loads (vmcnt = the ops issued after them), not for the prefetch.  A branch
// around any load or store in the loop body makes it fall back to the
// shortest path's count -- measured as vmcnt(9) before cur[0], i.e. waiting
// for the next item's loads too, which serialised memory and compute.
template <class F, int K, int NR, bool PREFETCH>
__device__ __forceinline__ void encode_item(const EncodeParams& p, uint32_t w, uint32_t step,
                                            uint4 (&cur)[K], uint4 (&nxt)[K]) {
  uint32_t o, tile, t;
  tile_of(w, p.first_edge, 0, o, tile, t);
  if constexpr (PREFETCH) {
    uint32_t on, tn, ttn;
    tile_of(w + step, p.first_edge, 0, on, tn, ttn);
    encode_load<K>(p, on, ttn, nxt);
  }
  typename F::Acc s;
  F::zero(s);
#pragma unroll
  for (int j = 0; j < K; ++j) F::mac(F::kb(0), j * F::kTableBytes, cur[j], s);
  F::pin(s);
  uint8_t* par = p.parity + static_cast<uint64_t>(o) * p.stripe_stride + p.row0 * p.frag_stride +
                 kHeaderBytes + t;
#pragma unroll
  for (int q = 0; q < NR; ++q) st_stream(par + q * p.frag_stride, F::row(s, q));
}

// Edge item: payload tail (t + 16 > bs) and chunks reaching the zero padding
// past obj_len (liberasurecode's prepare_fragments_for_encode zero-fills).
template <class F, int K, int NR>
__device__ __forceinline__ void encode_edge_item(const EncodeParams& p, uint32_t e) {
  uint32_t o, tile, t;
  tile_of(e, p.tiles - p.first_edge, p.first_edge, o, tile, t);
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
  if (p.headers != nullptr)
    for (uint32_t o = blockIdx.x; o < p.n_obj; o += gridDim.x) encode_headers(p, o, K);
  __syncthreads();
  const ItemRange r = item_range(p.n_obj * p.first_edge, p.xcd_split);
  uint4 xa[K], xb[K];
  uint32_t w = r.begin;
  if (w < r.end) {
    uint32_t o, tile, t;
    tile_of(w, p.first_edge, 0, o, tile, t);
    encode_load<K>(p, o, t, xa);
    // two items per trip so cur / nxt stay compile-time register arrays;
    // the last item of the range runs without a prefetch
    while (true) {
      if (w + r.step >= r.end) {
        encode_item<F, K, NR, false>(p, w, r.step, xa, xb);
        break;
      }
      encode_item<F, K, NR, true>(p, w, r.step, xa, xb);
      w += r.step;
      if (w + r.step >= r.end) {
        encode_item<F, K, NR, false>(p, w, r.step, xb, xa);
        break;
      }
      encode_item<F, K, NR, true>(p, w, r.step, xb, xa);
      w += r.step;
    }
  }
  // edge items last, on the highest-numbered blocks (those with the fewest
  // interior items)
  const uint32_t n_edge = p.n_obj * (p.tiles - p.first_edge);
  for (uint32_t e = gridDim.x - 1 - blockIdx.x; e < n_edge; e += gridDim.x)
    encode_edge_item<F, K, NR>(p, e);
}

// Data fragments (optional output of encode): the k padded object slices
// copied into their fragment payloads.  Item = (object, fragment, 4 KiB tile).
__global__ void __launch_bounds__(kThreadsPerBlock) copy_data_kernel(EncodeParams p) {
  const uint32_t per_obj = p.k * p.tiles;
  const uint32_t items = p.n_obj * per_obj;
  for (uint32_t w = blockIdx.x; w < items; w += gridDim.x) {
    const uint32_t o = w / per_obj, rest = w - o * per_obj;
    const uint32_t j = rest / p.tiles, tile = rest - j * p.tiles;
    const uint32_t t = (tile * kThreadsPerBlock + threadIdx.x) << 4;
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
// only after finishing the items that read slot s.  The interior loop fetches
// the next item's set into registers together with its payload loads, so a
// change costs a few ds_writes and one barrier, not an L2 round trip.

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

// Make d's table set current; returns its kb.  Block-uniform (barrier).
template <class F, int K>
__device__ __forceinline__ uint32_t ensure_tables(const DecodeParams& p, const ObjDesc& d,
                                                  Slots& st, const TablePre<F, K>& pre) {
  constexpr uint32_t kSlot = table_slot_bytes(K, F::kW);
  if (d.n_out != 0 && d.table != st.table) {
    st.slot ^= 1u;
    const uint32_t base = st.slot * kSlot;
    if (pre.table == d.table) {
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
      load_tables(p.tables + static_cast<uint64_t>(d.table) * (K * F::kTableBytes / 4),
                  K * F::kTableBytes, base);
    }
    __syncthreads();
    st.table = d.table;
  }
  return F::kb(st.slot * kSlot);
}

__device__ __forceinline__ void reconstruct_header(const DecodeParams& p, const ObjDesc& d,
                                                   uint8_t* out) {
  if (threadIdx.x < 5)
    reinterpret_cast<uint4*>(out)[threadIdx.x] = reinterpret_cast<const uint4*>(
        p.headers + static_cast<uint64_t>(d.header) * kHeaderBytes)[threadIdx.x];
}

// Position of input c inside the object's fragment group.
__device__ __forceinline__ uint32_t in_pos(const DecodeParams& p, const ObjDesc& d, int c) {
  return p.compact ? static_cast<uint32_t>(c) : d.in_idx[c];
}

template <int K>
__device__ __forceinline__ void decode_load(const DecodeParams& p, uint32_t o, uint32_t t,
                                            uint4 (&x)[K]) {
  const ObjDesc& d = p.desc[o];
  const uint8_t* frags = p.frags + static_cast<uint64_t>(o) * p.stripe_stride + kHeaderBytes + t;
  if (p.flags & kFlagCachedLoads) {
#pragma unroll
    for (int j = 0; j < K; ++j)
      x[j] = *reinterpret_cast<const uint4*>(frags + in_pos(p, d, j) * p.frag_stride);
  } else {
#pragma unroll
    for (int j = 0; j < K; ++j) x[j] = ld_stream(frags + in_pos(p, d, j) * p.frag_stride);
  }
}

__device__ __forceinline__ void st_out(uint8_t* dst, const uint4& v, uint32_t flags) {
  if (flags & kFlagPlainStores)
    *reinterpret_cast<uint4*>(dst) = v;
  else
    st_stream(dst, v);
}

// Realigned object stores.  Decode writes data slice j of an object at
// j*bs + t, and bs is rarely a multiple of 16 (419,432 = 8 mod 16 at 4 MiB,
// k = 10), so a plain 16-B store per lane straddles two 16-B units and the
// memory pipeline splits every one of them.  The 64 lanes of an interior
// item hold one contiguous 1 KiB run, and the misalignment S = dst mod 16 is
// the same for all of them.  Each lane takes the last S bytes of lane - 1
// (ds_bpermute) and stores the aligned 16-B unit that begins S bytes before
// its own address; lane 0 writes the head (its first 16 - S bytes) and
// lane 63 the tail (its last S bytes) with naturally aligned 8/4/2/1-B
// stores.  Neighbouring waves' head and tail share one 16-B unit, disjoint
// bytes.  Requires all 64 lanes active with consecutive 16-B addresses.

// Bytes [FROM, FROM + N) of v stored at p, where p mod 16 == AMOD: the largest
// naturally aligned piece each time.
template <int FROM, int N, int AMOD>
__device__ __forceinline__ void put_bytes(uint8_t* p, const uint4& v) {
  if constexpr (N > 0) {
    constexpr int sz = (AMOD % 8 == 0 && N >= 8)   ? 8
                       : (AMOD % 4 == 0 && N >= 4) ? 4
                       : (AMOD % 2 == 0 && N >= 2) ? 2
                                                   : 1;
    const uint64_t lo = v.x | (static_cast<uint64_t>(v.y) << 32);
    const uint64_t hi = v.z | (static_cast<uint64_t>(v.w) << 32);
    uint64_t x;
    if constexpr (FROM == 0)
      x = lo;
    else if constexpr (FROM < 8)
      x = (lo >> (8 * FROM)) | (hi << (64 - 8 * FROM));
    else if constexpr (FROM == 8)
      x = hi;
    else
      x = hi >> (8 * (FROM - 8));
    if constexpr (sz == 8)
      *reinterpret_cast<uint64_t*>(p) = x;
    else if constexpr (sz == 4)
      *reinterpret_cast<uint32_t*>(p) = static_cast<uint32_t>(x);
    else if constexpr (sz == 2)
      *reinterpret_cast<uint16_t*>(p) = static_cast<uint16_t>(x);
    else
      *p = static_cast<uint8_t>(x);
    put_bytes<FROM + sz, N - sz, (AMOD + sz) % 16>(p + sz, v);
  }
}

template <int S>
__device__ __forceinline__ void st_shifted(uint8_t* dst, const uint4& v, const uint4& prev,
                                           uint32_t lane, uint32_t flags) {
  // unit byte b = concat(prev, v)[16 - S + b]
  constexpr int st = 16 - S, d = st >> 2, r = st & 3;
  const uint32_t w[8] = {prev.x, prev.y, prev.z, prev.w, v.x, v.y, v.z, v.w};
  uint32_t c[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    if constexpr (r == 0)
      c[i] = w[d + i];
    else
      c[i] = __builtin_amdgcn_alignbyte(w[d + i + 1], w[d + i], r);
  }
  uint8_t* unit = dst - S;
  if (lane != 0)
    st_out(unit, make_uint4(c[0], c[1], c[2], c[3]), flags);
  else
    put_bytes<0, 16 - S, S>(dst, v);
  if (lane == 63) put_bytes<16 - S, S, 0>(unit + 16, v);
}

__device__ __forceinline__ void st_object(uint8_t* dst, const uint4& v, uint32_t flags) {
  const uint32_t s = __builtin_amdgcn_readfirstlane(
      static_cast<uint32_t>(reinterpret_cast<uintptr_t>(dst)) & 15u);
  if (s == 0 || (flags & kFlagNoRealign)) {
    st_out(dst, v, flags);
    return;
  }
  const uint4 prev = make_uint4(static_cast<uint32_t>(__shfl_up(static_cast<int>(v.x), 1)),
                                static_cast<uint32_t>(__shfl_up(static_cast<int>(v.y), 1)),
                                static_cast<uint32_t>(__shfl_up(static_cast<int>(v.z), 1)),
                                static_cast<uint32_t>(__shfl_up(static_cast<int>(v.w), 1)));
  const uint32_t lane = threadIdx.x & 63u;
  switch (s) {
#define ECAMD_SHIFT_CASE(S) \
  case S:                   \
    st_shifted<S>(dst, v, prev, lane, flags); \
    break;
    ECAMD_SHIFT_CASE(1) ECAMD_SHIFT_CASE(2) ECAMD_SHIFT_CASE(3) ECAMD_SHIFT_CASE(4)
    ECAMD_SHIFT_CASE(5) ECAMD_SHIFT_CASE(6) ECAMD_SHIFT_CASE(7) ECAMD_SHIFT_CASE(8)
    ECAMD_SHIFT_CASE(9) ECAMD_SHIFT_CASE(10) ECAMD_SHIFT_CASE(11) ECAMD_SHIFT_CASE(12)
    ECAMD_SHIFT_CASE(13) ECAMD_SHIFT_CASE(14) ECAMD_SHIFT_CASE(15)
#undef ECAMD_SHIFT_CASE
    default:
      break;
  }
}

// One interior decode / reconstruct item with inputs in `cur`; prefetches the
// block's next item (payloads into `nxt`, its table set into `pre`).
template <class F, int K>
__device__ __forceinline__ void decode_item(const DecodeParams& p, uint32_t w, const ItemRange& r,
                                            Slots& st, TablePre<F, K>& pre, uint4 (&cur)[K],
                                            uint4 (&nxt)[K]) {
  const uint32_t bs = p.bs;
  uint32_t o, tile, t;
  tile_of(w, p.first_edge, 0, o, tile, t);
  const bool more = w + r.step < r.end;
  uint32_t on = 0;
  if (more) {
    uint32_t tn, ttn;
    tile_of(w + r.step, p.first_edge, 0, on, tn, ttn);
    decode_load<K>(p, on, ttn, nxt);
  }
  const ObjDesc& d = p.desc[o];
  const uint32_t kb = ensure_tables<F, K>(p, d, st, pre);
  if (more) {
    const ObjDesc& dn = p.desc[on];
    if (dn.n_out != 0 && dn.table != st.table && dn.table != pre.table)
      table_prefetch<F, K>(p, dn.table, pre);
  }
  uint8_t* out = p.out + static_cast<uint64_t>(o) * p.out_stride;
  if (p.reconstruct && tile == 0) reconstruct_header(p, d, out);
  const uint32_t n_out = d.n_out;

  typename F::Acc s;
  F::zero(s);
  if (n_out != 0) {
#pragma unroll
    for (int j = 0; j < K; ++j) F::mac(kb, j * F::kTableBytes, cur[j], s);
  }
  F::pin(s);

#pragma unroll
  for (int q = 0; q < kRowsPerPass; ++q) {
    if (q >= static_cast<int>(n_out)) break;
    uint8_t* dst = p.reconstruct ? out + kHeaderBytes + t
                                 : out + static_cast<uint64_t>(d.out_idx[q]) * bs + t;
    st_object(dst, F::row(s, q), p.flags);
  }
  if (d.copy_inputs) {
#pragma unroll
    for (int j = 0; j < K; ++j) {
      const uint32_t idx = d.in_idx[j];
      if (idx < K) st_object(out + static_cast<uint64_t>(idx) * bs + t, cur[j], p.flags);
    }
  }
}

// Edge item of decode / reconstruct: payload tail, and (decode) outputs that
// cross the end of the object.
template <class F, int K>
__device__ __forceinline__ void decode_edge_item(const DecodeParams& p, uint32_t e, Slots& st,
                                                 const TablePre<F, K>& pre) {
  uint32_t o, tile, t;
  tile_of(e, p.tiles - p.first_edge, p.first_edge, o, tile, t);
  const ObjDesc& d = p.desc[o];
  const uint32_t kb = ensure_tables<F, K>(p, d, st, pre);
  uint8_t* out = p.out + static_cast<uint64_t>(o) * p.out_stride;
  if (p.reconstruct && tile == 0) reconstruct_header(p, d, out);
  if (t >= p.bs) return;
  // t < bs and 16 | t, so t + 16 <= round16(bs) <= frag_stride - 80: in bounds
  const uint8_t* frags = p.frags + static_cast<uint64_t>(o) * p.stripe_stride + kHeaderBytes + t;
  uint4 x[K];
#pragma unroll
  for (int j = 0; j < K; ++j)
    x[j] = *reinterpret_cast<const uint4*>(frags + in_pos(p, d, j) * p.frag_stride);
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

template <class F, int K>
__global__ void __launch_bounds__(kThreadsPerBlock) decode_kernel(DecodeParams p) {
  const ItemRange r = item_range(p.n_obj * p.first_edge, p.xcd_split);
  Slots st{0xFFFFFFFFu, 1u};
  TablePre<F, K> pre;
  pre.table = 0xFFFFFFFFu;
  uint4 xa[K], xb[K];
  uint32_t w = r.begin;
  if (w < r.end) {
    uint32_t o, tile, t;
    tile_of(w, p.first_edge, 0, o, tile, t);
    decode_load<K>(p, o, t, xa);
    const ObjDesc& d0 = p.desc[o];
    if (d0.n_out != 0) table_prefetch<F, K>(p, d0.table, pre);
  }
  const uint32_t n_edge = p.n_obj * (p.tiles - p.first_edge);
  for (uint32_t e = blockIdx.x; e < n_edge; e += gridDim.x) decode_edge_item<F, K>(p, e, st, pre);
  while (w < r.end) {
    decode_item<F, K>(p, w, r, st, pre, xa, xb);
    w += r.step;
    if (w >= r.end) break;
    decode_item<F, K>(p, w, r, st, pre, xb, xa);
    w += r.step;
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

// Interior tiles per object: tiles whose 4 KiB of positions end at or before
// min(bs, room), where room = payload bytes of the last data fragment that
// lie inside the object (decode outputs / encode inputs stop there).
inline void split_tiles(uint32_t bs, uint64_t obj_len, uint32_t k, bool whole_payload,
                        uint32_t& tiles, uint32_t& first_edge) {
  tiles = tiles_per_fragment(bs);
  int64_t room = whole_payload ? static_cast<int64_t>(bs)
                               : static_cast<int64_t>(obj_len) - static_cast<int64_t>(k - 1) * bs;
  if (room > static_cast<int64_t>(bs)) room = bs;
  if (room < 0) room = 0;
  first_edge = static_cast<uint32_t>(room / (kThreadsPerBlock * 16));
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

template <class F, int K, int NR>
hipError_t launch_encode_k(EncodeParams p, hipStream_t stream) {
  split_tiles(p.bs, p.obj_len, K, false, p.tiles, p.first_edge);
  const uint32_t interior = p.n_obj * p.first_edge;
  const uint32_t edge = p.n_obj * (p.tiles - p.first_edge);
  hipError_t e = launch(encode_kernel<F, K, NR>, p, K * F::kTableBytes,
                        std::max(std::max(interior, edge), p.headers ? p.n_obj : 0u), stream);
  if (e != hipSuccess || p.data == nullptr || p.row0 != 0) return e;
  return launch(copy_data_kernel, p, 0, p.n_obj * K * p.tiles, stream);
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

template <class F, int K>
hipError_t launch_decode_k(DecodeParams p, hipStream_t stream) {
  split_tiles(p.bs, p.obj_len, K, p.reconstruct != 0, p.tiles, p.first_edge);
  p.flags = (env_flag("ECAMD_DEC_PLAIN_STORES", false) ? kFlagPlainStores : 0u) |
            (env_flag("ECAMD_DEC_CACHED_LOADS", false) ? kFlagCachedLoads : 0u) |
            (env_flag("ECAMD_DEC_REALIGN", false) ? 0u : kFlagNoRealign);
  const uint32_t interior = p.n_obj * p.first_edge;
  const uint32_t edge = p.n_obj * (p.tiles - p.first_edge);
  return launch(decode_kernel<F, K>, p, 2 * table_slot_bytes(K, F::kW), std::max(interior, edge),
                stream);
}

#define ECAMD_K_CASES(X) \
  X(1) X(2) X(3) X(4) X(5) X(6) X(7) X(8) X(9) X(10) X(11) X(12) X(13) X(14) X(15) X(16) \
  X(17) X(18) X(19) X(20) X(21) X(22) X(23) X(24) X(25) X(26) X(27) X(28) X(29) X(30) X(31)

}  // namespace
}  // namespace ecamd
