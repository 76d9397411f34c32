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
// reads those slices with gfx9's unaligned loads and decode writes them with
// unaligned stores (see "Object stores").
#pragma once

#include <algorithm>
#include <cstdlib>
#include <cstddef>
#include <type_traits>
#include <atomic>
#include <map>
#include <mutex>
#include <tuple>
#include <utility>
#include <unordered_map>

#include "crc32.hpp"
#include "crc_device.hpp"
#include "ec_crc.hpp"
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
__device__ __forceinline__ uint32_t to_sgpr(uint32_t v);
__device__ __forceinline__ Rsrc rsrc(const void* base, int records = -1) {
  const uint64_t a = reinterpret_cast<uint64_t>(base);
  const uint32_t lo = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(a));
  const uint32_t hi = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(a >> 32));
  const int n = static_cast<int>(to_sgpr(static_cast<uint32_t>(records)));
  return __builtin_amdgcn_make_buffer_rsrc(
      reinterpret_cast<void*>((static_cast<uint64_t>(hi) << 32) | lo), 0, n, 0x00020000);
}
// CACHED: default cache policy instead of nontemporal.
template <bool CACHED = false>
__device__ __forceinline__ uint4 buf_ld(Rsrc r, uint32_t voff, uint32_t soff) {
  const v4u v = __builtin_amdgcn_raw_buffer_load_b128(r, voff, soff, CACHED ? 0 : kNt);
  return make_uint4(v.x, v.y, v.z, v.w);
}
// (Stores keep the nt policy.  Measured round 2 in the bench's alternating
// encode/decode step, k = 10, 256 x 4 MiB, profiles/r02y_store_policy.txt:
// nt 2,708 GiB/s; default policy 2,556; sc1 2,523; nt sc1 2,587.)
// One wait state after a 16-B buffer store.  Measured on MI355X (round 2):
// a `buffer_store_dwordx4 v[30:33], v52, s[24:27], s31 offen` directly
// followed by a VALU write of v30 stored a wrong first dword.  hipcc's hazard
// recognizer only guards stores of > 8 bytes whose soffset is NOT an SGPR, so
// every store here gets its own wait state (the sched barriers keep the
// s_nop directly behind the store); tools/store_hazard.py checks the
// generated code.
__device__ __forceinline__ void st_fence() {
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_nop 0");
  __builtin_amdgcn_sched_barrier(0);
}

template <bool CACHED = false>
__device__ __forceinline__ void buf_st(Rsrc r, uint32_t voff, uint32_t soff, const uint4& x) {
  v4u v;
  v.x = x.x;
  v.y = x.y;
  v.z = x.z;
  v.w = x.w;
  __builtin_amdgcn_raw_buffer_store_b128(v, r, voff, soff, CACHED ? 0 : kNt);
  st_fence();
}

// Between the lookup groups of one input: keeps hipcc from hoisting every
// LDS lookup of the unrolled input loop ahead of the XORs that consume them
// (2 VGPRs each).  The scheduling barrier alone holds only in the machine
// scheduler: for small k (2..6) the IR passes had moved all 128 lookups of an
// item to its top and sunk the XORs to the stores (256 VGPRs unconstrained,
// up to 1.4 KB per lane of spills at the 64-VGPR budget).  The empty asm with
// a memory clobber keeps the lookups in place at the IR level, and each
// accumulator group is pinned (empty asm on it) right after its XORs so they
// cannot sink; neither emits an instruction.
__device__ __forceinline__ void lookup_fence() {
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("" ::: "memory");
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
  static constexpr int kRows = NW == 2 ? 4 : 2;  // output rows one table entry carries
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
      asm volatile("" : "+v"(s_lo.x), "+v"(s_lo.y), "+v"(s_hi.x), "+v"(s_hi.y));
    } else {
      // Rows <= 2 use the low dword of each entry, but read the whole entry:
      // the entries of a nibble position are 16 B apart, so ds_read_b32
      // (banks (a/4) mod 32) puts v and v + 8 on one bank -- two-way
      // conflicts on every lookup -- where ds_read_b64 (mod 64) is
      // conflict-free at the same two cycles.  The high dwords feed the pin
      // below only, so the loads are not narrowed (round 5: reconstruct, the
      // m <= 2 decode and encode).
      const uint2 e0 = lds_u64(a[0], tab + qoff(0)), e1 = lds_u64(a[1], tab + qoff(1)),
                  e2 = lds_u64(a[2], tab + qoff(2)), e3 = lds_u64(a[3], tab + qoff(3));
      const uint2 e4 = lds_u64(a[4], tab + qoff(0)), e5 = lds_u64(a[5], tab + qoff(1)),
                  e6 = lds_u64(a[6], tab + qoff(2)), e7 = lds_u64(a[7], tab + qoff(3));
      s_lo.x = xor3(xor3(s_lo.x, e0.x, e1.x), e2.x, e3.x);
      s_hi.x = xor3(xor3(s_hi.x, e4.x, e5.x), e6.x, e7.x);
      asm volatile("" : "+v"(s_lo.x), "+v"(s_hi.x)
                   : "v"(e0.y), "v"(e1.y), "v"(e2.y), "v"(e3.y), "v"(e4.y), "v"(e5.y), "v"(e6.y),
                     "v"(e7.y));
    }
  }
  // One symbol (h = 0: low half-word) of x at a time: half the lookup
  // temporaries of mac_dword live at once (register-lean kernels).
  template <bool Z>
  static __device__ __forceinline__ void mac_dword_split(uint32_t kb, uint32_t tab, uint32_t x,
                                                         uint2& s_lo, uint2& s_hi) {
    uint32_t a[8];
    addrs<Z>(kb, x, a);
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      uint2& s = h ? s_hi : s_lo;
      if constexpr (NW == 2) {
        const uint2 e0 = lds_u64(a[4 * h], tab + qoff(0)), e1 = lds_u64(a[4 * h + 1], tab + qoff(1)),
                    e2 = lds_u64(a[4 * h + 2], tab + qoff(2)), e3 = lds_u64(a[4 * h + 3], tab + qoff(3));
        s.x = xor3(xor3(s.x, e0.x, e1.x), e2.x, e3.x);
        s.y = xor3(xor3(s.y, e0.y, e1.y), e2.y, e3.y);
        asm volatile("" : "+v"(s.x), "+v"(s.y));
      } else {  // whole entries, as mac_dword
        const uint2 e0 = lds_u64(a[4 * h], tab + qoff(0)), e1 = lds_u64(a[4 * h + 1], tab + qoff(1)),
                    e2 = lds_u64(a[4 * h + 2], tab + qoff(2)), e3 = lds_u64(a[4 * h + 3], tab + qoff(3));
        s.x = xor3(xor3(s.x, e0.x, e1.x), e2.x, e3.x);
        asm volatile("" : "+v"(s.x) : "v"(e0.y), "v"(e1.y), "v"(e2.y), "v"(e3.y));
      }
      lookup_fence();
    }
  }
  // The scheduling barriers stop hipcc from hoisting every LDS lookup of the
  // unrolled input loop ahead of the XORs that consume them (2 VGPRs each).
  template <bool Z = false, bool SPLIT = false>
  static __device__ __forceinline__ void mac(uint32_t kb, uint32_t tab, const uint4& x, Acc& a) {
    if constexpr (SPLIT) {
      mac_dword_split<Z>(kb, tab, x.x, a.s[0], a.s[1]);
      mac_dword_split<Z>(kb, tab, x.y, a.s[2], a.s[3]);
      mac_dword_split<Z>(kb, tab, x.z, a.s[4], a.s[5]);
      mac_dword_split<Z>(kb, tab, x.w, a.s[6], a.s[7]);
      return;
    }
    mac_dword<Z>(kb, tab, x.x, a.s[0], a.s[1]);
    lookup_fence();
    mac_dword<Z>(kb, tab, x.y, a.s[2], a.s[3]);
    lookup_fence();
    mac_dword<Z>(kb, tab, x.z, a.s[4], a.s[5]);
    lookup_fence();
    mac_dword<Z>(kb, tab, x.w, a.s[6], a.s[7]);
    lookup_fence();
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

// Eight output rows per lookup (encode with 4 < m <= 8 in one pass: the
// object is read once instead of once per four rows).  Entry (c, q, v) is a
// u128 holding the products of rows 0..7 (gf16.hpp build_nibble_tables_x8),
// at byte 1024c + 256q + 16v: one ds_read_b128 per nibble.  A 16-entry table
// spans all 64 banks in 16-B entries, so any 16 lanes of a ds_read_b128 lane
// group read it conflict-free.  Tables at LDS 0 only (encode).
__device__ __forceinline__ v4u lds_u128(uint32_t a, uint32_t tab) {
  return *reinterpret_cast<const __attribute__((address_space(3))) v4u*>(
      reinterpret_cast<const lds_char*>(static_cast<uintptr_t>(a)) + tab);
}
struct Gf16x8 {
  static constexpr uint32_t kW = 16;
  static constexpr int kRows = 8;
  static constexpr uint32_t kTableBytes = 1024;
  struct Acc {
    v4u s[8];  // s[2d] / s[2d+1]: rows 0-7 of the low / high symbol of input dword d
  };
  static __device__ __forceinline__ uint32_t kb(uint32_t base) { return base >> 8; }
  static __device__ __forceinline__ void zero(Acc& a) {
#pragma unroll
    for (int i = 0; i < 8; ++i) a.s[i] = v4u{0u, 0u, 0u, 0u};
  }
  static __device__ __forceinline__ void pin(Acc& a) {
#pragma unroll
    for (int i = 0; i < 8; ++i)
      asm volatile("" : "+v"(a.s[i].x), "+v"(a.s[i].y), "+v"(a.s[i].z), "+v"(a.s[i].w));
  }
  static constexpr uint32_t qoff(int q) { return 256u * q; }
  static __device__ __forceinline__ void mac_dword(uint32_t tab, uint32_t x, v4u& s_lo, v4u& s_hi) {
    uint32_t a[8];
    Gf16<2>::addrs<true>(0, x, a);
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      v4u& s = h ? s_hi : s_lo;
      const v4u e0 = lds_u128(a[4 * h], tab + qoff(0)), e1 = lds_u128(a[4 * h + 1], tab + qoff(1)),
                e2 = lds_u128(a[4 * h + 2], tab + qoff(2)), e3 = lds_u128(a[4 * h + 3], tab + qoff(3));
      s.x = xor3(xor3(s.x, e0.x, e1.x), e2.x, e3.x);
      s.y = xor3(xor3(s.y, e0.y, e1.y), e2.y, e3.y);
      s.z = xor3(xor3(s.z, e0.z, e1.z), e2.z, e3.z);
      s.w = xor3(xor3(s.w, e0.w, e1.w), e2.w, e3.w);
      asm volatile("" : "+v"(s.x), "+v"(s.y), "+v"(s.z), "+v"(s.w));
      lookup_fence();
    }
  }
  template <bool Z = true, bool SPLIT = false>
  static __device__ __forceinline__ void mac(uint32_t, uint32_t tab, const uint4& x, Acc& a) {
    static_assert(Z, "eight-row tables live at LDS 0");
    mac_dword(tab, x.x, a.s[0], a.s[1]);
    mac_dword(tab, x.y, a.s[2], a.s[3]);
    mac_dword(tab, x.z, a.s[4], a.s[5]);
    mac_dword(tab, x.w, a.s[6], a.s[7]);
  }
  static __device__ __forceinline__ uint32_t pack(const v4u& lo, const v4u& hi, int r) {
    const uint32_t a = r < 2 ? lo.x : r < 4 ? lo.y : r < 6 ? lo.z : lo.w;
    const uint32_t b = r < 2 ? hi.x : r < 4 ? hi.y : r < 6 ? hi.z : hi.w;
    return __builtin_amdgcn_perm(b, a, (r & 1) ? 0x07060302u : 0x05040100u);
  }
  static __device__ __forceinline__ uint4 row(const Acc& a, int r) {
    return make_uint4(pack(a.s[0], a.s[1], r), pack(a.s[2], a.s[3], r), pack(a.s[4], a.s[5], r),
                      pack(a.s[6], a.s[7], r));
  }
};

// ---------------- GF(2^8): ISA-L layout ----------------

struct Gf8 {
  static constexpr uint32_t kW = 8;
  static constexpr int kRows = 4;
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
    asm volatile("" : "+v"(a[0]), "+v"(a[1]), "+v"(a[2]), "+v"(a[3]));
  }
  template <bool Z = false, bool SPLIT = false>
  static __device__ __forceinline__ void mac(uint32_t kb, uint32_t tab, const uint4& x, Acc& a) {
    mac_dword(kb, tab, x.x, a.a + 0);
    lookup_fence();
    mac_dword(kb, tab, x.y, a.a + 4);
    lookup_fence();
    mac_dword(kb, tab, x.z, a.a + 8);
    lookup_fence();
    mac_dword(kb, tab, x.w, a.a + 12);
    lookup_fence();
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

// A wave-uniform value computed by VALU code (a 32-bit division by a runtime
// divisor has no scalar form) moved into an SGPR.  hipcc drops a plain
// readfirstlane of a value it already knows to be uniform, then keeps the
// value in a VGPR, and every buffer access whose descriptor or soffset
// derives from it is wrapped in a waterfall loop (round 3: 10 per item in the
// decode stream, found in the generated code).  The empty asm hides the
// uniformity, so the readfirstlane stays.
__device__ __forceinline__ uint32_t to_sgpr(uint32_t v) {
  asm("" : "+v"(v));
  return __builtin_amdgcn_readfirstlane(v);
}

// 16 bytes at base+off; bytes at or past `len` read as zero (encode padding).
// Two 16-B loads at 16-B-aligned offsets inside [0, round16(len)) -- the
// object's buffer spans at least that (obj_stride is a multiple of 16 and
// >= len) -- funnel-shifted into place: no byte loads, 8 VGPRs per input,
// whatever the alignment of off.
__device__ __forceinline__ uint4 load_clamped(const uint8_t* base, uint64_t off, uint64_t len) {
  // len > 0 (no edge item runs for an empty object); branch-free: units past
  // the last one holding object bytes are read from that one and masked off
  const uint64_t last = (len - 1) & ~uint64_t(15);
  const uint64_t a = off & ~uint64_t(15);
  const uint64_t a0 = a < last ? a : last;
  const uint64_t a1 = a0 + 16 <= last ? a0 + 16 : a0;
  const uint4 u = *reinterpret_cast<const uint4*>(base + a0);
  const uint4 v = *reinterpret_cast<const uint4*>(base + a1);
  const uint32_t s = static_cast<uint32_t>(off & 15);
  uint32_t w[8] = {u.x, u.y, u.z, u.w, v.x, v.y, v.z, v.w};
  if (s & 8) {
#pragma unroll
    for (int i = 0; i < 6; ++i) w[i] = w[i + 2];
  }
  if (s & 4) {
#pragma unroll
    for (int i = 0; i < 5; ++i) w[i] = w[i + 1];
  }
  uint32_t r[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) r[i] = __builtin_amdgcn_alignbyte(w[i + 1], w[i], s & 3);
  const int64_t n = static_cast<int64_t>(len) - static_cast<int64_t>(off);
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int64_t valid = n - 4 * i;
    r[i] &= valid >= 4 ? 0xFFFFFFFFu : (valid <= 0 ? 0u : (1u << (8 * valid)) - 1u);
  }
  return make_uint4(r[0], r[1], r[2], r[3]);
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

// The first n (> 0) bytes of v, the rest of the 16-B unit zeroed: a
// fragment payload's last unit, whose bytes past the payload are slot
// padding (frag_stride >= 80 + round16(bs)), is then stored whole.
__device__ __forceinline__ uint4 zero_tail(const uint4& v, int64_t n) {
  uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int64_t valid = n - 4 * i;
    w[i] &= valid >= 4 ? 0xFFFFFFFFu : (valid <= 0 ? 0u : (1u << (8 * valid)) - 1u);
  }
  return make_uint4(w[0], w[1], w[2], w[3]);
}

// Whole block copies `bytes` of tables from global memory to LDS byte `dst`.
// (threads: how many of the block's first threads take part -- the edge
// items of the 1024-thread loader / consumer kernels run on 256)
__device__ __forceinline__ void load_tables(const uint32_t* src, uint32_t bytes, uint32_t dst,
                                            uint32_t threads = 0) {
  auto* d = lds_v4(dst);
  const v4u* s = reinterpret_cast<const v4u*>(src);
  const uint32_t step = threads ? threads : blockDim.x;
  for (uint32_t i = threadIdx.x; i < bytes / 16; i += step) d[i] = s[i];
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
// Work item = (object o, tile): the block's 4 waves each take one 1 KiB chunk
// (64 lanes x 16 B) of consecutive payload positions of object o; tile =
// 4 KiB.  Tiles [0, tiles) of every object are "interior": every lane reads
// 16 in-bounds bytes from every input and writes one 16-byte unit to every
// output, so they run unconditionally, unrolled over K, as a stream (see
// "streaming").  The rest of each payload -- the tails of decode's object
// slices, the payload tail, the zero padding -- are "edge" items (4 KiB
// each, per-lane byte bounds) in a launch of their own.
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
// Interior block b of G: the launch's first edge_blocks blocks (a multiple of
// 8, so b keeps its XCD) run only edge items (see encode_kernel).
struct IBlock {
  uint32_t b, g;
};
__device__ __forceinline__ IBlock interior_block(uint32_t edge_blocks) {
  return {blockIdx.x - edge_blocks, gridDim.x - edge_blocks};
}
__device__ __forceinline__ ItemRange item_range(uint32_t items, uint32_t xcd_split, IBlock ib) {
  if (!xcd_split) return {ib.b, items, ib.g};
  const uint32_t x = ib.b & 7u;
  const uint32_t lo = static_cast<uint32_t>(static_cast<uint64_t>(items) * x / 8);
  const uint32_t hi = static_cast<uint32_t>(static_cast<uint64_t>(items) * (x + 1) / 8);
  return {lo + (ib.b >> 3), hi, ib.g >> 3};
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

// ---------------- streaming ----------------
//
// Every interior loop streams its inputs: a wave keeps NB input chunks
// (16 B per lane each) in flight continuously.  The products of input j are
// taken as soon as its chunk has arrived, and its registers are immediately
// refilled with input j + NB -- past the item's last input the stream moves
// on to the block's next item (through a zero-record descriptor after the
// last item: no traffic).  A wave therefore needs NB x 16 B of input
// registers instead of a whole item double-buffered (2K x 16 B), so 6-8 waves
// per SIMD fit, and memory and the table lookups overlap across them.  NB
// divides K so every item uses the registers in the same order (the loop body
// is one item, unrolled over K, with exact s_waitcnt counts: no memory
// instruction sits behind a branch).
//
// Measured (round 2, tools/ab_bench.py, k = 10, m = 4, 256 x 4 MiB, same
// process): encode 284.4 -> 274.3 us, decode 453.3 -> 436.6 us against the
// previous register double-buffered kernels (4 waves per SIMD, spills in the
// decode loop).
template <int K>
__host__ __device__ constexpr int stream_bufs() {
  for (int d = 6; d >= 2; --d)
    if (K % d == 0) return d;
  return K < 4 ? K : 4;  // prime K > 3: 4 buffers, the item padded (stream_slots)
}
// Slots per item: K rounded up to a multiple of NB.  Slots past K load and
// compute nothing (compile-time), so every item still issues the same memory
// instructions in the same order.  (Round 1-2 used NB = K for prime K: 7, 11,
// 13, ... -- up to 31 inputs in registers, and the kernels spilled.)
template <int K, int NB>
__host__ __device__ constexpr int stream_slots() {
  return (K + NB - 1) / NB * NB;
}

// Waves per SIMD the streaming kernels are built for (register budget) and
// launched at (blocks per CU; each block has one wave per SIMD).  Both run
// fewer blocks than their budget allows: fewer waves streaming at once keep
// the HBM side more efficient (tools/membench.hip: the encode pattern's best
// rows are at 1-2 blocks per CU), while 2 still hide the lookups.
//   decode 2 per CU (same process, profiles/r02q_ab_per_cu.txt,
//     r02r_ab_per_cu.txt: 405.8 us at 2, 411.8 at 3, 424.1 at 4, 424.5 at 5);
//   encode 2 per CU once the edge items run in blocks of their own
//     (launch_edges_apart; round 3, profiles/r03g_ab_alt.txt: 283.2 us at 2
//     vs 305.8 at 8; at 2 with the edges in front of interior blocks
//     301.7).  2 is also the best of 2/3/4/8 for k = 2, 4, 6, 7, 8, 12, for
//     k = 4 m = 2 and for the GF(2^8) codes (profiles/r03h_ab_per_cu_by_k.txt), and
//     for the fused-CRC encode (339.7 vs 362.6 us at 8).
// (Measured round 3 and not kept: all 32 lookups of an input -- and of a CRC
// row -- issued before their XORs, one LDS round trip per input instead of
// four, at a 2-wave budget: encode 297.7 vs 284.6 us, fused-CRC encode 350.8
// vs 353.6; profiles/r03s_ab_*.txt.  The lookup latency is not what the
// 2-per-CU launch waits on.)
constexpr int kEncodeOcc = 8, kEncodePerCu = 2;
// Eight-row (m = 5..8) parity encode, stream kernel: blocks per CU.  Round 5,
// k=10 m=5 256 x 4 MiB, alternating, one box (profiles/r05s_km_sweep.txt):
// 321.2 us at 3 against 348.3 at 2 (545.7 at 1).
constexpr int kEncode8PerCu = 3;
// The fused-CRC encode's register budget: 7 waves per SIMD (72 VGPRs, no
// scratch at k = 10, m = 4) once its item range stopped feeding waterfall
// loops (encode_crc_interior); 6 with six inputs in flight (k = 18, 24,
// 30: 72 VGPRs spilled 8-36 B); the full-stripe form (data fragments stored
// too) keeps 5.
constexpr int kEncodeCrcOcc = 7, kEncodeCrcDataOcc = 5;
// (Round 3 also measured the fused-CRC encode walking runs of R interior
// tiles dealt grid-stride, XCD-major -- a compact footprint like the plain
// encode's -- with a block join per run: 371.3 us at R = 8, 418.4 at 4,
// 387.7 at 16, against 342.7 for one contiguous range per block
// (profiles/r03l_ab_crc.txt).  The per-run joins cost more than the order
// gains; not kept.)
// Full-stripe encode (data fragments stored too): no register cap.  Capped
// at 64 VGPRs the edge items' extra stores spilled (44 B per lane of
// scratch), and hipcc still spilled 12 B at a 72 cap; uncapped it takes 70
// (k = 10: 7 waves per SIMD), and the launcher sizes the grid from the
// kernel's actual register count (resident_per_cu).
constexpr int kEncodeDataOcc = 1;
constexpr int kDecodeOcc = 4, kDecodePerCu = 2;
// Reconstruct (k reads, one row written): 2 per CU since its edge items run
// in blocks of their own (round 3, config 3: GF(2^8) k = 12, 128 x 16 MiB,
// bench.py --second reconstruct: 448.0 us at 2, 451.7 at 3, 477.4 at 4,
// 476.9 at 6; profiles/r03t_config3_rec*.json).  Round 2, with the edges in
// front of interior blocks, measured 0.586 ms at 2 vs 0.500 at 4.
constexpr int kReconstructPerCu = 2;
// Decode walks its items without the XCD-major split (grid-stride over the
// whole list): measured round 2, same process, three boxes: 437.0 vs 446.1,
// 438.8 vs 445.6, 436.5 vs 444.3 us.  Encode is indifferent (+-0.3 us) and
// keeps the split.
constexpr bool kDecodeXcd = false;

// ---------------- encode ----------------

// Interior item w: 4 KiB of payload positions starting at t0 = tile*4096;
// this wave's chunk at t0 + 1024*wave, the lane at + 16*lane (voffset).
constexpr uint32_t kTile = kWavesPerBlock * kChunkBytes;
// CH chunks per wave: the item spans CH * 4 KiB, the wave CH KiB of it.
template <int CH = 1>
__device__ __forceinline__ void enc_item_pos(const EncodeParams& p, uint32_t w, uint32_t& o,
                                             uint32_t& x) {
  o = to_sgpr(w / p.tiles);
  x = (w - o * p.tiles) * (kTile * CH) + wave_in_block() * (kChunkBytes * CH);
}

// Store descriptors of object o's parity and data fragments, clipped to
// those fragments' bytes (m or k fragment strides; below 4 GiB by
// layout_fits), so the range check drops any store that would leave them
// (round 6; until then they held 4 GiB - 1 records).
__device__ __forceinline__ Rsrc rsrc_parity(const EncodeParams& p, uint32_t o) {
  return rsrc(p.parity + static_cast<uint64_t>(o) * p.stripe_stride,
              static_cast<int>(p.m * static_cast<uint32_t>(p.frag_stride)));
}
// A 1 KiB chunk at offset c is inside [lo, hi) of an in-place single
// object (EncodeParams / DecodeParams::direct; wave-uniform).
__device__ __forceinline__ bool in_window(const void* direct, uint32_t lo, uint32_t hi, uint32_t c) {
  return direct != nullptr && c >= lo && c + kChunkBytes <= hi;
}
__device__ __forceinline__ Rsrc rsrc_data(const EncodeParams& p, uint32_t o) {
  return rsrc(p.data + static_cast<uint64_t>(o) * p.stripe_stride,
              static_cast<int>(p.k * static_cast<uint32_t>(p.frag_stride)));
}

// The stream kernels skip a dropped row's store outright (a uniform branch:
// round 5, the eight-row pass at m = 5 issued three stores per chunk into a
// zero-record descriptor); the loader / consumer kernel keeps the dropped
// stores, whose count its vmcnt waits assume.
__device__ __forceinline__ bool row_live(const EncodeParams& p, int q) {
  return q == 0 || static_cast<uint32_t>(q) < p.nrows;
}

// Parity row q's store descriptor.  A pass computes NR rows (2, 4 or 8: the
// kernels are instantiated for those only) and the pass may hold fewer
// (p.nrows: m = 1, 3, 5..7); the rows past p.nrows come from zero
// coefficients and their stores go through a zero-record descriptor and are
// dropped, so every item still issues the same instructions.
template <int NR>
__device__ __forceinline__ Rsrc parity_row(const EncodeParams& p, uint32_t o, int q, Rsrc par) {
  if (q == 0 || static_cast<uint32_t>(q) < p.nrows) return par;  // every pass has a first row
  return rsrc(p.parity, 0);
}

// Inputs an edge item holds in registers at once (edge items run inside the
// streaming kernels, ahead of their interior items).
constexpr int kEdgeGroup = 1;

// Edge item: payload tail and chunks reaching the zero padding past obj_len
// (liberasurecode's prepare_fragments_for_encode zero-fills).  DATA: the
// padded input chunks are also the data fragments' payload bytes.
template <class F, int K, int NR, bool DATA>
__device__ __forceinline__ void encode_edge_item(const EncodeParams& p, uint32_t e) {
  const uint32_t o = e / p.edge_tiles;
  const uint32_t t = (p.tiles * p.tile_ch + (e - o * p.edge_tiles)) * kTile + threadIdx.x * 16;
  if (t >= p.bs) return;
  const uint8_t* obj = p.objs + static_cast<uint64_t>(o) * p.obj_stride;
  const int64_t rem = static_cast<int64_t>(p.bs) - t;
  // kEdgeGroup inputs in registers at a time, the groups fenced off from
  // each other: this runs inside the streaming kernel (encode_edges), whose
  // register budget it must not raise
  typename F::Acc s;
  F::zero(s);
  Rsrc dat;
  if constexpr (DATA) dat = rsrc_data(p, o);
#pragma unroll
  for (int j0 = 0; j0 < K; j0 += kEdgeGroup) {
    constexpr int G = kEdgeGroup;
    uint4 x[G];
#pragma unroll
    for (int j = 0; j < G; ++j)
      if (j0 + j < K) x[j] = load_clamped(obj, static_cast<uint64_t>(j0 + j) * p.bs + t, p.obj_len);
#pragma unroll
    for (int j = 0; j < G; ++j)
      if (j0 + j < K) F::template mac<true>(F::kb(0), (j0 + j) * F::kTableBytes, x[j], s);
    if constexpr (DATA) {
      // one 16-B store per input through the object's data descriptor (an
      // address pair per input, or the byte loop of store_partial, made
      // hipcc spill the streaming kernel)
#pragma unroll
      for (int j = 0; j < G; ++j)
        if (j0 + j < K)
          buf_st(dat, t, (j0 + j) * p.frag_stride + kHeaderBytes, zero_tail(x[j], rem));
    }
    __builtin_amdgcn_sched_barrier(0);
  }
  F::pin(s);
  // the payload's last unit is stored whole with its bytes past bs zeroed
  // (slot padding): no byte loop (store_partial's, inlined here, put up to
  // 1.4 KB per lane of scratch in the small-k kernels)
  const Rsrc par = rsrc_parity(p, o);
#pragma unroll
  for (int q = 0; q < NR; ++q)
    if (row_live(p, q))
      buf_st(par, t, (p.row0 + q) * p.frag_stride + kHeaderBytes, zero_tail(F::row(s, q), rem));
}

// ---------------- inline CRC-32 of the chunks a launch writes ----------------
//
// inline_crc32 (liberasurecode's set_checksum, upstream erasurecode_helpers.c;
// pyeclib core.py:59-63 -> pyeclib_c.c:248): every wave takes the raw CRC of
// each 1 KiB fragment chunk it writes while the chunk is in its registers
// (crc_device.hpp chunk_crc: per lane raw16 and its lane map, 40 nibble
// lookups per 16 B, then an XOR across the wave) and one lane stores it; the
// finishing pass (ec_crc.hip) shifts the chunks' CRCs into place and reads
// back only the edge items' bytes.  The partials are independent of the
// order items are dealt in, so the CRC kernels walk the items exactly as the
// plain ones do.  (Rounds 2-4 kept a Horner accumulator per thread instead,
// which needs each block to walk a contiguous item range, and joined the
// threads at every run end behind block barriers: 1.21-1.26x the plain
// encode, 10 % of it the order; profiles/r04n_ab_contig.txt.)  The lane
// tables (CrcLaneTables, 34 KiB) sit in LDS after the GF tables.
constexpr uint32_t kCrcLaneBytes = kCrcLdsBytes;
template <class F, int K>
__host__ __device__ constexpr uint32_t crc_lds_base() {
  return (K * F::kTableBytes + 255u) & ~255u;
}
// 1 KiB chunks of every payload covered by a launch's interior items.
__host__ __device__ constexpr uint32_t crc_chunks(uint32_t tiles, uint32_t tile_ch) {
  return tiles * tile_ch * (kTile / kChunkBytes);
}
// A wave-uniform raw CRC stored by one lane (a vector store).
__device__ __forceinline__ void crc_store(uint32_t* dst, uint32_t v) {
  if (lane_id() == 0) *dst = v;
}

// Interior encode: object slices streamed in (default cache policy --
// neighbouring slices share 128-B lines, which L2 then serves twice), parity
// chunks stored nontemporal and line-aligned.  DATA (full-stripe encode,
// liberasurecode_encode's k data + m parity fragments, pyeclib_c.c:544-560):
// each input chunk, already in registers for its products, is also stored to
// its data fragment's line-aligned payload before the registers are refilled
// -- one pass over the object instead of a separate copy.  NOCOMP:
// memory-only probe (inputs XORed, no lookups; wrong parity) for the
// benchmark shape.  CRC: inline_crc32 partials of the parity chunks (and of
// the data chunks, DATA), CH = 1.
//
// CH (A/B, k = 10): an item spans CH * 4 KiB of payload positions and each
// wave takes CH KiB contiguous of every slice; the stream runs chunk-major
// (the K inputs of chunk 0, its parity stores, then chunk 1 ...), so the
// registers stay those of CH = 1.  NTL: nontemporal input loads.
//
// Prologue (HEAD).  The first NB loads are issued as the refills of a
// previous item's last NB slots would be, with that item's stores -- data
// fragment stores, then the NR parity stores -- through a zero-record
// descriptor (no memory access).  hipcc computes one s_waitcnt per
// instruction for every path into the loop head: with the stores missing on
// the entry path, the wait for input 0 was vmcnt(4) there, and the steady
// state (where the 4 parity stores are the youngest operations) inherited
// it, so every wave drained all NB of its in-flight loads at every item
// boundary (round 4, found in the generated code).  With the entry path
// shaped like the back edge the wait is vmcnt(NB - 1 + NR (+ data stores)),
// and loads stay in flight across items.  Measured (tools/ab_bench.py, same
// process, profiles/r04e_ab.txt): encode 297.4 us with it against 285.7
// without -- the deeper stream costs more at the HBM than the drain did --
// so the encode keeps HEAD = false; decode (decode_interior) keeps its own.
template <class F, int K, int NR, bool NOCOMP = false, bool DATA = false, int CH = 1,
          bool NTL = false, int NBX = 0, bool HEAD = false, bool CRC = false>
__device__ __forceinline__ void encode_interior(const EncodeParams& p) {
  constexpr int NB = NBX ? NBX : stream_bufs<K>();  // NBX: A/B (divides K)
  static_assert(!CRC || CH == 1, "CRC partials per 1 KiB chunk");
  const uint32_t chunks = crc_chunks(p.tiles, p.tile_ch);
  const uint32_t lane4 = lane_id() * 4;
  const ItemRange r = item_range(p.n_obj * p.tiles, p.xcd_split, interior_block(p.edge_blocks));
  uint32_t w = r.begin;
  if (w >= r.end) return;
  uint32_t o, x;
  enc_item_pos<CH>(p, w, o, x);
  Rsrc cur = rsrc(p.objs + static_cast<uint64_t>(o) * p.obj_stride);
  const uint32_t lane16 = lane_id() * 16;
  constexpr int KP = stream_slots<K, NB>();
  constexpr int SL = KP * CH;  // stream slots per item: slot i = chunk i / KP, input i % KP
  uint4 buf[NB];
  const Rsrc none = rsrc(p.parity, 0);
  const uint4 zero4 = make_uint4(0, 0, 0, 0);
  // in-place single object (EncodeParams::direct): a wave-uniform choice of
  // descriptor per chunk, no extra instruction on the vector side
  const Rsrc dir = rsrc(p.direct);
  auto src = [&](Rsrc r, bool live, uint32_t soff) {
    return live && in_window(p.direct, p.direct_lo, p.direct_hi, soff) ? dir : r;
  };
#pragma unroll
  for (int j = 0; j < NB; ++j) {
    if constexpr (HEAD && DATA)
      if ((SL - NB + j) % KP < K) buf_st(none, lane16, 0, zero4);
    if (j < K) buf[j] = buf_ld<!NTL>(src(cur, true, j * p.bs + x), lane16, j * p.bs + x);
  }
  if constexpr (HEAD)
#pragma unroll
    for (int q = 0; q < NR; ++q) buf_st(none, lane16, 0, zero4);
  // one item per trip: hipcc would otherwise unroll the item loop for small k
  // (k = 2..6: 256 VGPRs unconstrained, up to 1.4 KB per lane of spills at 64)
#pragma clang loop unroll(disable)
  while (true) {
    // the next item, or this one again through a zero-record descriptor
    const uint32_t wn = w + r.step < r.end ? w + r.step : w;
    uint32_t on, xn;
    enc_item_pos<CH>(p, wn, on, xn);
    const Rsrc nxt = rsrc(p.objs + static_cast<uint64_t>(on) * p.obj_stride, wn == w ? 0 : -1);
    Rsrc dat;
    if constexpr (DATA) dat = rsrc_data(p, o);
    const Rsrc par = rsrc_parity(p, o);
    typename F::Acc s;
    F::zero(s);
#pragma unroll
    for (int i = 0; i < SL; ++i) {
      const int j = i % KP, c = i / KP;
      if (j < K) {
        if constexpr (NOCOMP) {
          uint32_t* a = reinterpret_cast<uint32_t*>(&s);
          a[0] ^= buf[i % NB].x;
          a[2] ^= buf[i % NB].y;
          a[4] ^= buf[i % NB].z;
          a[6] ^= buf[i % NB].w;
        } else {
          F::template mac<true>(F::kb(0), j * F::kTableBytes, buf[i % NB], s);
        }
        if constexpr (DATA) {
          buf_st(dat, lane16, j * p.frag_stride + kHeaderBytes + x + kChunkBytes * c, buf[i % NB]);
          if constexpr (CRC)
            crc_store(p.crc_part_data + (static_cast<uint64_t>(o) * chunks + x / kChunkBytes) * K + j,
                      crcdev::chunk_crc(buf[i % NB], crc_lds_base<F, K>(), lane4));
        }
      }
      const int in = i + NB;  // slot refilled into this buffer
      if (in < SL) {
        const uint32_t so = (in % KP) * p.bs + x + kChunkBytes * (in / KP);
        if (in % KP < K) buf[i % NB] = buf_ld<!NTL>(src(cur, true, so), lane16, so);
      } else if ((in - SL) % KP < K) {
        const uint32_t so = ((in - SL) % KP) * p.bs + xn + kChunkBytes * ((in - SL) / KP);
        buf[i % NB] = buf_ld<!NTL>(src(nxt, wn != w, so), lane16, so);
      }
      if (j == KP - 1) {  // chunk c complete: its parity rows
        F::pin(s);
        const uint32_t soff = p.row0 * p.frag_stride + kHeaderBytes + x + kChunkBytes * c;
#pragma unroll
        for (int q = 0; q < NR; ++q)
          if (row_live(p, q)) {
            // in place (EncodeParams::dpar): a wave-uniform choice of
            // descriptor and offset, one store either way
            const uint32_t xc = x + kChunkBytes * c;
            const bool dq = q < 8 && in_window(p.dpar[q & 7], p.dpar_lo[q & 7], p.dpar_hi[q & 7], xc);
            buf_st(dq ? rsrc(p.dpar[q & 7]) : par, lane16, dq ? xc : soff + q * p.frag_stride,
                   F::row(s, q));
          }
        if constexpr (CRC) {
          uint32_t* part = p.crc_part + (static_cast<uint64_t>(o) * chunks + x / kChunkBytes) * p.m + p.row0;
#pragma unroll
          for (int q = 0; q < NR; ++q)
            if (static_cast<uint32_t>(q) < p.nrows)
              crc_store(part + q, crcdev::chunk_crc(F::row(s, q), crc_lds_base<F, K>(), lane4));
        }
        if (c + 1 < CH) F::zero(s);
      }
    }
    if (wn == w) break;
    w = wn;
    o = on;
    x = xn;
    cur = nxt;
  }
}

// Headers and edge items of an encode, block b taking objects / items
// b, b + G, ... (b counted from `first`, G = `step` blocks).  Tables are at LDS 0.
template <class F, int K, int NR, bool DATA>
__device__ __forceinline__ void encode_edges(const EncodeParams& p, uint32_t first, uint32_t step) {
  if (p.headers != nullptr && p.row0 == 0)
    for (uint32_t o = first; o < p.n_obj; o += step) {
      const uint64_t base = static_cast<uint64_t>(o) * p.stripe_stride;
      block_headers(p.parity + base, p.frag_stride, p.headers + K * kHeaderBytes, p.m);
      if (p.data != nullptr) block_headers(p.data + base, p.frag_stride, p.headers, K);
    }
  for (uint32_t e = first; e < p.n_obj * p.edge_tiles; e += step)
    encode_edge_item<F, K, NR, DATA>(p, e);
}

// One launch per encode: the headers and edge items, in the blocks counted
// from the END of the grid -- which hold one interior item fewer whenever the
// items do not divide evenly, so the edge latency is absorbed -- then the
// interior stream.  Measured round 2 (rocprof timeline,
// profiles/r02l_timeline.txt): with the edges in a launch of their own on a
// side stream, the fork / join left the GPU idle 25-32 us between
// consecutive interior kernels.
// Register budget (waves per SIMD) of an encode instantiation.  GF(2^8)
// with k >= 18 (six inputs in flight, 4-byte table entries) spilled 12 B per
// lane at 64 VGPRs and gets 72.
template <class F, int K, bool DATA, int NBX, bool CRC = false>
__host__ __device__ constexpr int encode_occ() {
  if (F::kRows > kRowsPerPass) return 4;  // eight-row accumulators: 32 VGPRs
  if (CRC) return DATA ? kEncodeCrcDataOcc : (stream_bufs<K>() >= 6 ? 6 : kEncodeCrcOcc);
  if (DATA) return kEncodeDataOcc;
  if (NBX > 6) return 4;
  if (F::kW == 8 && K >= 18) return 7;
  return kEncodeOcc;
}

template <class F, int K, int NR, bool NOCOMP = false, bool DATA = false, int CH = 1,
          bool NTL = false, int NBX = 0, bool HEAD = false, bool CRC = false>
__global__ void __launch_bounds__(kThreadsPerBlock)
    __attribute__((amdgpu_waves_per_eu(encode_occ<F, K, DATA, NBX, CRC>(), 8)))
    encode_kernel(EncodeParams p) {
  load_tables(p.tables, K * F::kTableBytes, 0);
  if constexpr (CRC)
    load_tables(static_cast<const uint32_t*>(p.crc_lanes), kCrcLaneBytes, crc_lds_base<F, K>());
  __syncthreads();
  if (p.fused_edges) {
    if (p.edge_blocks == 0) {
      encode_edges<F, K, NR, DATA>(p, gridDim.x - 1 - blockIdx.x, gridDim.x);
    } else if (blockIdx.x < p.edge_blocks) {
      encode_edges<F, K, NR, DATA>(p, blockIdx.x, p.edge_blocks);
      return;
    }
  }
  encode_interior<F, K, NR, NOCOMP, DATA, CH, NTL, NBX, HEAD, CRC>(p);
}

// Headers and edge items of an encode in a launch of their own (the
// side-stream variant, ECAMD_EDGE_SIDE=1, kept for A/B runs).
template <class F, int K, int NR>
__global__ void __launch_bounds__(kThreadsPerBlock) encode_edge_kernel(EncodeParams p) {
  load_tables(p.tables, K * F::kTableBytes, 0);
  __syncthreads();
  encode_edges<F, K, NR, false>(p, blockIdx.x, gridDim.x);
}

// ---------------- encode with a loader / consumer split (LDS-DMA ring) ----------------
//
// One 512-thread block (8 waves, two per SIMD) per CU.  An item is 8 KiB of
// payload positions; a ring slot holds one input of one item (8 KiB).  Waves
// 0-3 (one per SIMD) are the loaders: they move every input chunk from HBM
// straight into the LDS ring with buffer_load_dwordx4 ... lds (1 KiB per
// wave-instruction, no VGPRs held), R - 1 slots ahead.  All 8 waves consume:
// each reads its 1 KiB of the slot from LDS (ds_read_b128), takes the nibble
// lookups and, after the item's last input, stores its parity rows.  So HBM
// sees 4 issuing waves per CU keeping (R - 1) x 8 KiB in flight, while the
// lookups still have 2 waves per SIMD to hide behind.
//
// Ordering (MI355X_MICROARCH.md, LDS-DMA): slot t is read only after its
// loaders' s_waitcnt vmcnt (their DMAs of slot t retired) and a barrier all
// waves pass; the DMA of slot t + R - 1 overwrites ring[(t - 1) % R], issued
// only after that same barrier, which every wave reaches after reading slot
// t - 1.  The DMAs are inline asm (hipcc does not see them, so it neither
// drains them before LDS reads nor counts them); the waits are explicit.
// Edge items and headers run in blocks of their own, 256 threads of them.
// inline_crc32 (p.crc_lanes set, a runtime switch: the kernel's register
// budget has room): the lane tables follow the GF tables in LDS, the ring
// after them, and every consumer wave stores its parity chunks' (and, with
// DATA, its data chunks') raw CRCs.
constexpr uint32_t kDmaSlot = 8192;  // bytes of a ring slot per KiB of SW (8 waves x 1 KiB)
constexpr uint32_t kDmaThreads = 512;

typedef unsigned int v4u_s __attribute__((ext_vector_type(4)));
// Buffer descriptor in SGPRs as the 4 dwords of the V# (gfx9: base, stride 0,
// num_records, dword3 as __builtin_amdgcn_make_buffer_rsrc builds it).
__device__ __forceinline__ v4u_s rsrc4(const void* base, uint32_t records) {
  const uint64_t a = reinterpret_cast<uint64_t>(base);
  v4u_s r;
  r.x = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(a));
  r.y = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(a >> 32)) & 0xFFFFu;
  r.z = to_sgpr(records);
  r.w = 0x00020000u;
  return r;
}
// 16 B per lane from buffer r at voff + soff into LDS at lds + 16 * lane.
template <bool NT>
__device__ __forceinline__ void dma16(v4u_s r, uint32_t voff, uint32_t soff, uint32_t lds) {
  uint32_t keep;
  if constexpr (NT)
    asm volatile(
        "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\t"
        "buffer_load_dwordx4 %1, %2, %4 offen nt lds\n\ts_mov_b32 m0, %0"
        : "=&s"(keep) : "v"(voff), "s"(r), "s"(lds), "s"(soff) : "memory");
  else
    asm volatile(
        "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\t"
        "buffer_load_dwordx4 %1, %2, %4 offen lds\n\ts_mov_b32 m0, %0"
        : "=&s"(keep) : "v"(voff), "s"(r), "s"(lds), "s"(soff) : "memory");
}
template <int N>
__device__ __forceinline__ void wait_vm() {
  static_assert(N >= 0 && N <= 63, "vmcnt range");
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}
__device__ __forceinline__ void ring_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");  // no LDS read of the slot moves above the barrier
}

template <class F, int K>
__host__ __device__ constexpr uint32_t dma_ring_base() {
  return (K * F::kTableBytes + 255u) & ~255u;
}
// SW: KiB of each slot a consumer wave takes (slot = 8 * SW KiB, item = one
// slot's positions across the k inputs); L: loader waves.
template <class F, int K, int R, int SW, int W = 8>
__host__ __device__ constexpr uint32_t dma_lds_bytes(bool crc = false) {
  return dma_ring_base<F, K>() + (crc ? kCrcLaneBytes : 0u) + R * 1024 * W * SW;
}

// W: waves per block (8 = 2 per SIMD, 16 = 4 per SIMD).  DATA: the consumers
// also store each slot they read from LDS into its data fragment.
// CONTIG (A/B): each block streams a contiguous range of items (the fused-CRC
// kernel's order) instead of the XCD-split grid stride.  RUNS (A/B): runs of
// RUNS consecutive items dealt to the blocks grid-stride.
// COMB (A/B): groups of COMB consecutive blocks share an object, block r of a
// group taking its tiles r, r + COMB, ... (the order a Horner CRC with a
// COMB-item stride could use); G / COMB objects in flight.
// CV (A/B, inline CRC): 0 = the parity chunks' CRC steps deferred over the
// next item's slots (the product), 1 = taken at the item's end, 2 = at the
// item's end with unfenced raw16 lookups (crcdev::raw16_free), 4 = deferred
// like 0, on the matrix cores (crcdev::mfma_*: 8 v_mfma_i32_32x32x32_i8 and 4
// lookups per row chunk instead of 40 lookups).
template <class F, int K, int NR, int R, bool NT, int L = 4, int SW = 1, int W = 8,
          bool DATA = false, bool NOCOMP = false, bool CONTIG = false, int RUNS = 0, int COMB = 0,
          int CV = 6>
__global__ void __launch_bounds__(W * 64) encode_dma_kernel(EncodeParams p) {
  static_assert(R >= 2 && R <= K + 1, "ring of 2 .. K + 1 slots");
  static_assert(L == 2 || L == 4 || L == 8 || L == 16, "loader waves");
  constexpr uint32_t kSlot = 1024u * W * SW;       // bytes of one ring slot
  constexpr int kPerLoader = kSlot / 1024 / L;    // DMA wave-instructions per loader and slot
  const uint32_t wave = wave_in_block();
  if (blockIdx.x < p.edge_blocks) {  // edge items and headers: 256 threads
    if (threadIdx.x >= kThreadsPerBlock) return;
    for (uint32_t i = threadIdx.x; i < K * F::kTableBytes / 16; i += kThreadsPerBlock)
      lds_v4(0)[i] = reinterpret_cast<const v4u*>(p.tables)[i];
    __syncthreads();
    encode_edges<F, K, NR, DATA>(p, blockIdx.x, p.edge_blocks);
    return;
  }
  const bool crc = p.crc_lanes != nullptr;
  for (uint32_t i = threadIdx.x; i < K * F::kTableBytes / 16; i += W * 64)
    lds_v4(0)[i] = reinterpret_cast<const v4u*>(p.tables)[i];
  if (crc)
    load_tables(static_cast<const uint32_t*>(p.crc_lanes), kCrcLaneBytes, dma_ring_base<F, K>(), W * 64);
  __syncthreads();
  ItemRange rg = item_range(p.n_obj * p.tiles, p.xcd_split, interior_block(p.edge_blocks));
  if constexpr (CONTIG) {
    const uint64_t nall = static_cast<uint64_t>(p.n_obj) * p.tiles;
    const IBlock ib = interior_block(p.edge_blocks);
    rg = {static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(static_cast<uint32_t>(nall * ib.b / ib.g))),
          static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(static_cast<uint32_t>(nall * (ib.b + 1) / ib.g))),
          1u};
  }
  uint32_t n_items = 0;
  const IBlock ibk = interior_block(p.edge_blocks);
  const uint32_t nall = p.n_obj * p.tiles;
  const uint32_t runs_total = RUNS ? (nall + RUNS - 1) / RUNS : 0;
  const uint32_t groups = COMB ? ibk.g / COMB : 1, r0 = COMB ? ibk.b % COMB : 0;
  const uint32_t per_obj = COMB ? (p.tiles > r0 ? (p.tiles - r0 + COMB - 1) / COMB : 0) : 0;
  if constexpr (COMB > 0) {
    const uint32_t g0 = ibk.b / COMB;
    if (per_obj == 0 || g0 >= p.n_obj || ibk.b >= groups * COMB) return;  // block-uniform
    n_items = to_sgpr((p.n_obj - g0 + groups - 1) / groups * per_obj);
  } else if constexpr (RUNS > 0) {
    if (ibk.b >= runs_total) return;  // block-uniform
    n_items = (runs_total - ibk.b + ibk.g - 1) / ibk.g * RUNS;
    if ((runs_total - 1 - ibk.b) % ibk.g == 0) n_items -= runs_total * RUNS - nall;
    n_items = to_sgpr(n_items);
  } else {
    if (rg.begin >= rg.end) return;  // block-uniform
    n_items = to_sgpr((rg.end - rg.begin + rg.step - 1) / rg.step);
  }
  const bool loader = wave < static_cast<uint32_t>(L);
  const uint32_t lane16 = lane_id() * 16, lane4 = lane_id() * 4;
  const uint32_t kRing = to_sgpr(dma_ring_base<F, K>() + (crc ? kCrcLaneBytes : 0u));
  const uint32_t chunks = crc_chunks(p.tiles, p.tile_ch);
  // item i of this block: object and first payload position
  auto item_at = [&](uint32_t i, uint32_t& o, uint32_t& x0) {
    if constexpr (COMB > 0) {
      const uint32_t q = i / per_obj, sidx = i - q * per_obj;
      o = to_sgpr(ibk.b / COMB + q * groups);
      x0 = (r0 + sidx * COMB) * kSlot;
      return;
    }
    const uint32_t w = RUNS ? (ibk.b + ibk.g * (i / (RUNS ? RUNS : 1))) * RUNS + i % (RUNS ? RUNS : 1)
                            : rg.begin + i * rg.step;
    o = to_sgpr(w / p.tiles);
    x0 = (w - o * p.tiles) * kSlot;
  };
  // loaders: the DMAs of slot (item i, input j) into ring slot `ri`
  auto issue = [&](uint32_t i, int j, uint32_t ri) {
    if (!loader) return;
    uint32_t o, x0;
    const bool valid = i < n_items;
    item_at(valid ? i : 0, o, x0);
    const v4u_s src = rsrc4(p.objs + static_cast<uint64_t>(o) * p.obj_stride, valid ? ~0u : 0u);
    const uint32_t part = wave * (kSlot / L);
    const uint32_t lds = kRing + ri * kSlot + part;
    const uint32_t soff = to_sgpr(j * p.bs + x0 + part);
#pragma unroll
    for (int c = 0; c < kPerLoader; ++c) dma16<NT>(src, lane16, soff + 1024 * c, lds + 1024 * c);
  };
  // prologue: slots 0 .. R-2
#pragma unroll
  for (int t = 0; t < R - 1; ++t) issue(t / K, t % K, t);
  uint32_t ring = 0;  // ring slot of the current slot t
  typename F::Acc s[SW];
#pragma unroll
  for (int c = 0; c < SW; ++c) F::zero(s[c]);
  // inline_crc32 (SW = 1): an item's parity chunk CRCs are taken during the
  // NEXT item's K slots, kCrcSteps / K steps of 8 lookups per slot (row q:
  // its raw16 by dword, then its lane map, the wave XOR and the store), so
  // no wave carries a burst of lookups into a ring barrier -- taken all at
  // the item's end they held the ring for ~3.8 K LDS cycles per CU and item
  // (the CRC encode ran 1.28x the plain one; profiles/r05b_*).
  // CV 4: 9 steps per row -- its 8 bit planes on the matrix cores into one
  // accumulator (rows one after another), then the 4 lookups and the store.
  // CV 6 (the product): as 4, each row's lookups kept per lane and one wave
  // XOR for all the rows at the end (crcdev::wave_xor4; a last step).
  constexpr bool kMf = CV == 4 || CV == 6;
  constexpr bool kMf4 = CV == 6;
  constexpr int kPerRow = kMf ? 9 : 5;
  constexpr int kCrcSteps = kPerRow * NR + (kMf4 ? 1 : 0);
  static_assert(!kMf4 || NR <= 4, "one joint wave XOR");
  uint32_t cfin[kMf4 ? 4 : 1] = {};
  uint4 crow[NR];
  uint32_t cacc[NR];
  uint32_t* cpart = p.crc_part;
  bool cpend = false;
  crcdev::mfma_v4i mb[kMf ? 8 : 1];
  crcdev::mfma_v16i macc = {};
  if constexpr (kMf) {
    if (crc) crcdev::mfma_load_b(p.crc_lanes, lane_id(), mb);
  }
  // full stripe: the data chunks' CRCs (input c of an item, its payload
  // xprev, CRCs stored at base[c]): 8 planes into an accumulator of their
  // own, the lookups kept per lane, one wave XOR per 4 inputs (lanes 0..3
  // store the CRCs)
  uint32_t dfin[kMf4 && DATA ? 4 : 1] = {};
  uint4 xprev = {};
  uint32_t* dprev = nullptr;
  bool dpend = false;
  auto data_crc = [&](int c, uint32_t* base) {
    if constexpr (kMf4 && DATA) {
      crcdev::mfma_v16i dacc = {};
#pragma unroll
      for (int d = 0; d < 8; ++d) dacc = crcdev::mfma_plane(xprev, d, mb[d], d == 0 ? crcdev::mfma_v16i{} : dacc);
      dfin[c % 4] = crcdev::mfma_lanes(dacc, dma_ring_base<F, K>() + offsetof(CrcLaneTables, mst), lane4);
      if (c % 4 == 3 || c == K - 1) {
        const int n = c % 4 + 1;
        const uint32_t t = crcdev::wave_xor4(dfin[0], n > 1 ? dfin[1] : 0u, n > 2 ? dfin[2] : 0u,
                                             n > 3 ? dfin[3] : 0u, lane_id());
        if (lane_id() < static_cast<uint32_t>(n)) base[c + 1 - n + lane_id()] = t;
      }
    }
  };
  auto crc_step = [&](int u) {
    if constexpr (kMf4) {
      if (u == kPerRow * NR) {
        const uint32_t t = crcdev::wave_xor4(cfin[0], cfin[1], cfin[2], cfin[3], lane_id());
        if (lane_id() < p.nrows && lane_id() < static_cast<uint32_t>(NR)) cpart[lane_id()] = t;
        return;
      }
      const int q = u / kPerRow, d = u % kPerRow;
      if (d < 8)
        macc = crcdev::mfma_plane(crow[q], d, mb[d], d == 0 ? crcdev::mfma_v16i{} : macc);
      else
        cfin[q] = crcdev::mfma_lanes(macc, dma_ring_base<F, K>() + offsetof(CrcLaneTables, mst), lane4);
      return;
    }
    if constexpr (kMf) {
      const int q = u / kPerRow, d = u % kPerRow;
      if (d < 8) {
        macc = crcdev::mfma_plane(crow[q], d, mb[d], d == 0 ? crcdev::mfma_v16i{} : macc);
      } else if (static_cast<uint32_t>(q) < p.nrows) {
        crc_store(cpart + q, crcdev::mfma_finish(macc, dma_ring_base<F, K>() + offsetof(CrcLaneTables, mst), lane4));
      }
      return;
    }
    const int q = u / kPerRow, d = u % kPerRow;
    if (d < 4) {
      const uint32_t w = d == 0 ? crow[q].x : d == 1 ? crow[q].y : d == 2 ? crow[q].z : crow[q].w;
      cacc[q] ^= crcdev::raw_dword(w, d, dma_ring_base<F, K>());
    } else if (static_cast<uint32_t>(q) < p.nrows) {
      crc_store(cpart + q, crcdev::wave_xor(crcdev::lane_map(
                               cacc[q], dma_ring_base<F, K>() + offsetof(CrcLaneTables, lane), lane4)));
    }
  };
#pragma clang loop unroll(disable)
  for (uint32_t i = 0; i < n_items; ++i) {
    uint32_t o, x0;
    item_at(i, o, x0);
    const Rsrc par = rsrc_parity(p, o);
    Rsrc dat;
    if constexpr (DATA) dat = rsrc_data(p, o);
#pragma unroll
    for (int j = 0; j < K; ++j) {
      // (vmcnt counts the data-fragment stores too: the wait is then
      // conservative, never short -- loads retire in order)
      if (loader) wait_vm<kPerLoader * (R - 2)>();  // this wave's DMAs of slot t retired
      ring_barrier();                                // ... everyone's; ring[t-1] read by all
      // slot t + R - 1 = (item i + (j + R - 1) / K, input (j + R - 1) % K)
      const uint32_t rn = ring == 0 ? R - 1 : ring - 1;
      issue(i + (j + R - 1) / K, (j + R - 1) % K, rn);
#pragma unroll
      for (int c = 0; c < SW; ++c) {
        const v4u xin = *lds_v4(kRing + ring * kSlot + (wave * SW + c) * 1024 + lane16);
        const uint4 x = make_uint4(xin.x, xin.y, xin.z, xin.w);
        if constexpr (NOCOMP) {  // memory-only probe (A/B builds): WRONG parity
          uint32_t* a = reinterpret_cast<uint32_t*>(&s[c]);
          a[0] ^= x.x;
        } else {
          F::template mac<true>(F::kb(0), j * F::kTableBytes, x, s[c]);
        }
        if constexpr (DATA) {
          buf_st(dat, lane16, j * p.frag_stride + kHeaderBytes + x0 + (wave * SW + c) * 1024, x);
          uint32_t* dpart = p.crc_part_data + (static_cast<uint64_t>(o) * chunks + x0 / 1024 + wave * SW + c) * K;
          if constexpr (kMf4 && SW == 1) {
            // the data chunk's CRC on the matrix cores too, one slot later
            // (data_crc: input j - 1 now, the item's last input in the next
            // item's first slot), so its MFMA chain does not wait on this
            // slot's LDS read
            if (crc) {
              if (j > 0) data_crc(j - 1, dpart);
              else if (dpend) data_crc(K - 1, dprev);
              xprev = x;
              if (j == K - 1) {
                dprev = dpart;
                dpend = true;
              }
            }
          } else if (crc) {
            crc_store(dpart + j, crcdev::chunk_crc(x, dma_ring_base<F, K>(), lane4));
          }
        }
      }
      if constexpr (SW == 1 && (CV == 0 || CV == 4 || CV == 6)) {
        if (cpend) {  // the previous item's CRC steps [kCrcSteps j / K, kCrcSteps (j + 1) / K)
#pragma unroll
          for (int u = j * kCrcSteps / K; u < (j + 1) * kCrcSteps / K; ++u) crc_step(u);
        }
      }
      ring = ring + 1 == R ? 0 : ring + 1;
    }
#pragma unroll
    for (int c = 0; c < SW; ++c) {
      F::pin(s[c]);
      const uint32_t soff = p.row0 * p.frag_stride + kHeaderBytes + x0 + (wave * SW + c) * 1024;
#pragma unroll
      for (int q = 0; q < NR; ++q)
        buf_st(parity_row<NR>(p, o, q, par), lane16, soff + q * p.frag_stride, F::row(s[c], q));
      if (crc) {
        uint32_t* part = p.crc_part + (static_cast<uint64_t>(o) * chunks + x0 / 1024 + wave * SW + c) * p.m + p.row0;
        if constexpr (SW == 1 && (CV == 0 || CV == 4 || CV == 6)) {  // taken during the next item (or after the last)
#pragma unroll
          for (int q = 0; q < NR; ++q) {
            crow[q] = F::row(s[c], q);
            cacc[q] = 0;
          }
          cpart = part;
          cpend = true;
        } else {
#pragma unroll
          for (int q = 0; q < NR; ++q)
            if (static_cast<uint32_t>(q) < p.nrows)
              crc_store(part + q, crcdev::chunk_crc<CV == 2>(F::row(s[c], q), dma_ring_base<F, K>(), lane4));
        }
      }
      F::zero(s[c]);
    }
  }
  if constexpr (kMf4 && DATA && SW == 1) {
    if (crc && dpend) data_crc(K - 1, dprev);  // the block's last data chunk
  }
  if constexpr (SW == 1 && (CV == 0 || CV == 4 || CV == 6)) {
    if (cpend) {  // the block's last item
#pragma unroll
      for (int u = 0; u < kCrcSteps; ++u) crc_step(u);
    }
  }
  if (loader) wait_vm<0>();  // no DMA may land in LDS after the block ends
}

// Data fragments (optional output of encode): the k padded object slices
// copied into their fragment payloads.  Item = (object, fragment, 4 KiB).
__global__ void __launch_bounds__(kThreadsPerBlock) __attribute__((unused))
    copy_data_kernel(EncodeParams p) {
  const uint32_t per_frag = (p.bs + kTile - 1) / kTile;
  const uint32_t per_obj = p.k * per_frag;
  const uint32_t items = p.n_obj * per_obj;
  for (uint32_t w = blockIdx.x; w < items; w += gridDim.x) {
    const uint32_t o = w / per_obj, rest = w - o * per_obj;
    const uint32_t j = rest / per_frag, c = rest - j * per_frag;
    const uint32_t t = c * kTile + threadIdx.x * 16;
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
// Object stores.  Decode writes data slice j of an object at j*bs + t, and
// bs is rarely a multiple of 16 (419,432 = 8 mod 16 at 4 MiB, k = 10), so
// lane stores straddle 16-B units.  Realigning them was measured four ways
// and each lost to the plain stores (round 1-2, profiles/): an overlap lane
// per chunk (1008-B chunks: +12 % HBM traffic), LDS-staged whole tiles (438
// vs 444 us, and 3 waves per SIMD), DPP-shifted units with half-unit stores
// at the chunk ends (440.8 vs 436.6 us with the streaming kernel), and
// copies of misaligned present slices from a second load shifted by the
// misalignment, so every copy store is a whole aligned unit (432.2 vs 417.8
// us with the fused-edge kernel, profiles/r02o_ab_shift.txt: the extra load
// per input and the 102-VGPR budget cost more than the alignment gains).

struct Slots {
  uint32_t table;  // set in the current slot (0xFFFFFFFF = none)
  uint32_t slot;   // 0 / 1
};

template <class F, int K>
struct TablePre {
  static constexpr int kChunks = K * F::kTableBytes / 16;
  static constexpr int kPer = (kChunks + kThreadsPerBlock - 1) / kThreadsPerBlock;
  uint4 v[kPer];
  uint32_t table;  // set held in v (0xFFFFFFFF = none)
};

// Prefetch a table set into registers: always issued (exact wait counts),
// through a zero-record descriptor -- zeros, no traffic -- when not needed;
// lanes past the set's end are dropped by the range check.
template <class F, int K>
__device__ __forceinline__ void table_prefetch(const DecodeParams& p, uint32_t table, bool need,
                                               TablePre<F, K>& pre) {
  constexpr uint32_t kBytes = K * F::kTableBytes;
  const Rsrc t = rsrc(p.tables + static_cast<uint64_t>(table) * (kBytes / 4), need ? kBytes : 0);
#pragma unroll
  for (int i = 0; i < TablePre<F, K>::kPer; ++i)
    pre.v[i] = buf_ld<true>(t, (threadIdx.x + i * kThreadsPerBlock) * 16, 0);
  pre.table = need ? table : 0xFFFFFFFFu;
}

// Make d's table set current; returns its kb.  Block-uniform (barrier).
template <class F, int K, class D>
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
                  K * F::kTableBytes, base, kThreadsPerBlock);
    }
    __syncthreads();
    st.table = d.table();
  }
  return F::kb(st.slot * kSlot);
}

enum DecodeMode : int {
  kDecode = 0,        // one pass holds every missing row
  kReconstruct = 1,   // one fragment per object (aligned payload)
  kDecodeGeneric = 2  // more than 4 missing data fragments (several passes)
};

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
// S (default): through the constant address space, so hipcc issues scalar
// loads (s_load_dwordx8 + x4, counted by lgkmcnt) -- the descriptors are
// written by the host before the launch and never by a kernel.  As vector
// loads (S = false, the form up to round 3) they were counted by vmcnt
// behind the item's in-flight payload loads and stores, and the wait for
// them at every item boundary (vmcnt(0): the descriptor is the youngest
// load) drained the whole stream (round 4, found in the generated code).
typedef const __attribute__((address_space(4))) uint32_t const_u32;
template <bool S = true>
__device__ __forceinline__ DescU load_desc(const DecodeParams& p, uint32_t o) {
  DescU u;
  if constexpr (S) {
    const const_u32* src =
        reinterpret_cast<const const_u32*>(reinterpret_cast<uintptr_t>(p.desc + o));
#pragma unroll
    for (uint32_t i = 0; i < sizeof(ObjDesc) / 4; ++i) u.w[i] = src[i];
  } else {
    const uint32_t* src = reinterpret_cast<const uint32_t*>(p.desc + o);
#pragma unroll
    for (uint32_t i = 0; i < sizeof(ObjDesc) / 4; ++i)
      u.w[i] = __builtin_amdgcn_readfirstlane(src[i]);
  }
  return u;
}

// Debug builds (`make -C pyeclib_amd/csrc checks`, -DECAMD_DEVICE_CHECKS):
// every descriptor is checked before a store that depends on it, and the
// edge items' flat stores against their slice; a violation prints what it
// found (lane 0) and traps, so the launch fails with an error instead of
// writing where a bad index points.  The product build compiles none of it.
#ifdef ECAMD_DEVICE_CHECKS
#define ECAMD_DEVICE_ASSERT(cond, ...)               \
  do {                                               \
    if (!(cond)) {                                   \
      if (lane_id() == 0) printf(__VA_ARGS__);       \
      __builtin_trap();                              \
    }                                                \
  } while (0)
#else
#define ECAMD_DEVICE_ASSERT(cond, ...) \
  do {                                 \
  } while (0)
#endif

// Object o's descriptor: inputs are fragment indices < k + m; rows per pass
// at most 8; decode rows rebuild data indices < k, a reconstruct row any
// fragment index.
template <int K, int MODE>
__device__ __forceinline__ void check_desc(const DecodeParams& p, const DescU& d, uint32_t o) {
#ifdef ECAMD_DEVICE_CHECKS
  const uint32_t n = p.k + p.m;
  ECAMD_DEVICE_ASSERT(o < p.n_obj && p.k == static_cast<uint32_t>(K),
                      "ecamd check: object %u of %u, k %u (kernel K %d)\n", o, p.n_obj, p.k, K);
#pragma unroll
  for (int c = 0; c < K; ++c)
    ECAMD_DEVICE_ASSERT(d.in_idx(c) < n, "ecamd check: object %u input %d index %u >= %u\n", o, c,
                        d.in_idx(c), n);
  ECAMD_DEVICE_ASSERT(d.n_out() <= 4u, "ecamd check: object %u rows %u\n", o, d.n_out());
  const uint32_t lim = MODE == kReconstruct ? n : static_cast<uint32_t>(K);
#pragma unroll
  for (uint32_t q = 0; q < 4; ++q)
    ECAMD_DEVICE_ASSERT(q >= d.n_out() || d.out_idx(q) < lim,
                        "ecamd check: object %u row %u index %u >= %u\n", o, q, d.out_idx(q), lim);
#else
  (void)p;
  (void)d;
  (void)o;
#endif
}

// Fragment group position of input c.
__device__ __forceinline__ uint32_t in_pos(const DecodeParams& p, const DescU& d, int c) {
  return p.compact ? static_cast<uint32_t>(c) : d.in_idx(c);
}

// Input c's 16 B per lane at payload position x (+ 16 * lane): from the
// object's stripe, or -- an in-place single object (DecodeParams::din) --
// from the caller's fragment when the wave's chunk is inside its window
// (a wave-uniform choice of descriptor and offset, one load either way).
// live: r is a real descriptor (not the zero-record one past the last item).
// Only for k <= kDinMax: with more inputs the per-input pointers pushed the
// prime-k kernels past the SGPRs (k = 17 spilled 68 B per lane).
template <int K>
__device__ __forceinline__ uint4 dec_ld(const DecodeParams& p, Rsrc r, bool live, const DescU& d, int c,
                                        uint32_t x, uint32_t lane16) {
  const bool dq = K <= kDinMax && live && in_window(p.din[c & 31], p.din_lo[c & 31], p.din_hi[c & 31], x);
  return buf_ld(dq ? rsrc(p.din[c]) : r, lane16,
                dq ? x : in_pos(p, d, c) * p.frag_stride + kHeaderBytes + x);
}

__device__ __forceinline__ void dec_item_pos(const DecodeParams& p, uint32_t w, uint32_t& o,
                                             uint32_t& x) {
  o = to_sgpr(w / p.tiles);
  x = (w - o * p.tiles) * kTile + wave_in_block() * kChunkBytes;
}

// Output descriptor of one object (decode: its obj_len bytes) or one
// fragment (reconstruct: 80 + bs bytes), so the hardware range check clips
// any store that would leave the destination (round 6; until then every
// output descriptor held 2 GiB - 1 records).  Every extent is below 2 GiB
// (layout_fits), so a store sent to voffset kDrop (2 GiB) with soffset 0 is
// always discarded: drop_st never adds a per-input soffset to kDrop, whose
// sum could wrap past 2^32 back into the destination.
constexpr uint32_t kDrop = 0x80000000u;
template <int MODE>
__device__ __forceinline__ uint32_t out_extent(const DecodeParams& p) {
  return MODE == kReconstruct ? kHeaderBytes + p.bs : static_cast<uint32_t>(p.obj_len);
}
__device__ __forceinline__ Rsrc rsrc_out(const void* base, uint32_t records) {
  const uint64_t a = reinterpret_cast<uint64_t>(base);
  const uint32_t lo = to_sgpr(static_cast<uint32_t>(a));
  const uint32_t hi = to_sgpr(static_cast<uint32_t>(a >> 32));
  return __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void*>((static_cast<uint64_t>(hi) << 32) | lo),
                                           0, static_cast<int>(to_sgpr(records)), 0x00020000);
}
// A store that applies only when `live` (wave-uniform): otherwise it goes to
// kDrop with soffset 0 and the range check discards it.
__device__ __forceinline__ void drop_st(Rsrc r, bool live, uint32_t lane16, uint32_t soff, const uint4& v) {
  buf_st(r, live ? lane16 : kDrop, live ? soff : 0u, v);
}

// Interior decode / reconstruct, streaming the first k available fragments.
//   decode (and each pass of a multi-pass decode): a present data input --
//   descriptor copy_inputs set and input index < k -- is stored to its object
//   slice as soon as its products are taken (before its registers are
//   refilled); the n_out rebuilt rows after the last input.
//   reconstruct: row 0 into the fragment payload.
// Stores that do not apply (parity inputs, rows past n_out) go to voffset
// kDrop and are discarded by the range check, so every item issues the same
// memory instructions.  NOCOMP: memory-only probe (no lookups; wrong rows).
template <class F, int K, int MODE, bool NOCOMP = false, int NBX = 0, bool SDESC = true,
          bool CRCFREE = false>
__device__ __forceinline__ void decode_interior(const DecodeParams& p, Slots& st,
                                                TablePre<F, K>& pre) {
  constexpr int NB = NBX ? NBX : stream_bufs<K>();  // NBX: A/B (divides K)
  const ItemRange r = item_range(p.n_obj * p.tiles, p.xcd_split, interior_block(p.edge_blocks));
  uint32_t w = r.begin;
  if (w >= r.end) return;  // block-uniform: no wave of this block reaches a barrier
  const uint32_t lane16 = lane_id() * 16;
  uint32_t o, x;
  dec_item_pos(p, w, o, x);
  DescU d = load_desc<SDESC>(p, o);
  constexpr int KP = stream_slots<K, NB>();
  uint4 buf[NB];
  if constexpr (SDESC) {
    // Prologue shaped like the back edge (see encode_interior, HEAD): the
    // table prefetch first, then the item's vector-memory sequence -- a
    // (zero-record, no access) store for each data store and each refill of
    // the current item, the real loads where the refills fetch the next
    // item's first NB inputs, the row stores.  The table switch at the loop
    // head then waits only for the prefetch; with the prefetch last on the
    // entry path it waited vmcnt(0/1) there, and so in the steady state too,
    // draining the stream at every table change -- every item in the bench
    // (round 4, found in the generated code).
    table_prefetch<F, K>(p, d.table(), d.n_out() != 0, pre);
    const Rsrc first = rsrc(p.frags + static_cast<uint64_t>(o) * p.stripe_stride);
    const Rsrc none = rsrc(p.frags, 0);
    const uint4 zero4 = make_uint4(0, 0, 0, 0);
#pragma unroll
    for (int j = 0; j < KP; ++j) {
      if (MODE != kReconstruct && j < K) buf_st(none, lane16, 0, zero4);
      if (j + NB < KP) {
        if (j + NB < K) buf_st(none, lane16, 0, zero4);
      } else if (j + NB - KP < K) {
        buf[j % NB] = dec_ld<K>(p, first, true, d, j + NB - KP, x, lane16);
      }
    }
#pragma unroll
    for (int q = 0; q < (MODE == kReconstruct ? 1 : F::kRows); ++q) buf_st(none, lane16, 0, zero4);
  } else {  // the round-3 prologue (A/B builds)
    const Rsrc first = rsrc(p.frags + static_cast<uint64_t>(o) * p.stripe_stride);
#pragma unroll
    for (int j = 0; j < NB; ++j)
      if (j < K) buf[j] = buf_ld(first, lane16, in_pos(p, d, j) * p.frag_stride + kHeaderBytes + x);
    table_prefetch<F, K>(p, d.table(), d.n_out() != 0, pre);
  }
  // one item per trip: hipcc would otherwise unroll the item loop for small k
  // (k = 2..6: 256 VGPRs unconstrained, up to 1.4 KB per lane of spills at 64)
#pragma clang loop unroll(disable)
  while (true) {
    const uint32_t wn = w + r.step < r.end ? w + r.step : w;
    uint32_t on, xn;
    dec_item_pos(p, wn, on, xn);
    const DescU dn = load_desc<SDESC>(p, on);
    // rebuilt from the object index each trip rather than carried over from
    // the last trip's `nxt`: the loop-carried 128-bit descriptor was kept in
    // VGPRs, and every input load went through a waterfall loop (10 per item
    // at k = 10 until round 3)
    const Rsrc cur = rsrc(p.frags + static_cast<uint64_t>(o) * p.stripe_stride);
    const Rsrc nxt = rsrc(p.frags + static_cast<uint64_t>(on) * p.stripe_stride, wn == w ? 0 : -1);
    const uint32_t kb = ensure_tables<F, K>(p, d, st, pre);
    table_prefetch<F, K>(p, dn.table(), wn != w && dn.n_out() != 0 && dn.table() != st.table,
                         pre);
    const Rsrc out = rsrc_out(p.out + static_cast<uint64_t>(o) * p.out_stride, out_extent<MODE>(p));
    // in-place single object (DecodeParams::direct): rebuilt rows' chunks
    const Rsrc dir = rsrc_out(p.direct, out_extent<MODE>(p));
    const bool copy = MODE != kReconstruct && d.copy_inputs() != 0;
    check_desc<K, MODE>(p, d, o);
    typename F::Acc s;
    F::zero(s);
#pragma unroll
    for (int j = 0; j < KP; ++j) {
      if (j < K) {
        if constexpr (NOCOMP) {
          uint32_t* a = reinterpret_cast<uint32_t*>(&s);
          a[0] ^= buf[j % NB].x;
        } else {
          F::mac(kb, j * F::kTableBytes, buf[j % NB], s);
        }
        if constexpr (MODE != kReconstruct)
          drop_st(out, copy && d.in_idx(j) < static_cast<uint32_t>(K), lane16, d.in_idx(j) * p.bs + x,
                  buf[j % NB]);
      }
      if (j + NB < KP) {
        if (j + NB < K) buf[j % NB] = dec_ld<K>(p, cur, true, d, j + NB, x, lane16);
      } else if (j + NB - KP < K) {
        buf[j % NB] = dec_ld<K>(p, nxt, wn != w, dn, j + NB - KP, xn, lane16);
      }
    }
    F::pin(s);
    if constexpr (MODE == kReconstruct) {
      buf_st(out, lane16, kHeaderBytes + x, F::row(s, 0));
      if (p.crc_part != nullptr)  // inline_crc32: the chunk's raw CRC (launch_decode_mode)
        crc_store(p.crc_part + static_cast<uint64_t>(o) * crc_chunks(p.tiles, p.tile_ch) + x / kChunkBytes,
                  crcdev::chunk_crc<CRCFREE>(F::row(s, 0), 2 * table_slot_bytes(K, F::kW), lane_id() * 4));
    } else {
      const uint32_t e = d.n_out();
#pragma unroll
      for (int q = 0; q < F::kRows; ++q) {
        const uint32_t so = d.out_idx(q) * p.bs + x;
        drop_st(in_window(p.direct, p.direct_lo, p.direct_hi, so) ? dir : out, q < static_cast<int>(e),
                lane16, so, F::row(s, q));
      }
    }
    if (wn == w) break;
    w = wn;
    o = on;
    x = xn;
    d = dn;
  }
}

// Edge item: 4 KiB of positions from the end of the interior tiles (+ 16 per
// thread), byte-exact stores clipped to each output's window: an object
// slice's bytes inside the object (decode), or the payload (reconstruct).
template <class F, int K, int MODE>
__device__ __forceinline__ void decode_edge_item(const DecodeParams& p, uint32_t e, Slots& st,
                                                 const TablePre<F, K>& pre) {
  const uint32_t o = e / p.edge_tiles;
  const uint32_t tail0 = p.tiles * p.tile_ch * kTile;
  const DescU d = load_desc(p, o);
  check_desc<K, MODE>(p, d, o);
  const uint32_t kb = ensure_tables<F, K>(p, d, st, pre);
  const uint32_t t = tail0 + (e - o * p.edge_tiles) * kTile + threadIdx.x * 16;
  if (t >= p.bs) return;
  // (the flat stores below stay inside the object: each is clipped to
  // [tail0, object_bytes) of its slice, whose index check_desc has checked)
  uint8_t* out = p.out + static_cast<uint64_t>(o) * p.out_stride;
  // t < bs and 16 | t, so t + 16 <= round16(bs) <= frag_stride - 80: in bounds
  const uint8_t* in = p.frags + static_cast<uint64_t>(o) * p.stripe_stride + kHeaderBytes + t;
  // kEdgeGroup inputs in registers at a time (this runs inside the streaming
  // kernel, decode_edges: see encode_edge_item)
  typename F::Acc s;
  F::zero(s);
#pragma unroll
  for (int j0 = 0; j0 < K; j0 += kEdgeGroup) {
    constexpr int G = kEdgeGroup;
    uint4 x[G];
#pragma unroll
    for (int j = 0; j < G; ++j)
      if (j0 + j < K) x[j] = *reinterpret_cast<const uint4*>(in + in_pos(p, d, j0 + j) * p.frag_stride);
    if (d.n_out() != 0) {
#pragma unroll
      for (int j = 0; j < G; ++j)
        if (j0 + j < K) F::mac(kb, (j0 + j) * F::kTableBytes, x[j], s);
    }
    if (MODE != kReconstruct && d.copy_inputs()) {
#pragma unroll
      for (int j = 0; j < G; ++j) {
        if (j0 + j >= K) continue;
        const uint32_t idx = d.in_idx(j0 + j);
        if (idx >= K) continue;
        store_window(out + static_cast<uint64_t>(idx) * p.bs, t, x[j], tail0,
                     object_bytes(idx, p.bs, 0, p.obj_len));
      }
    }
    __builtin_amdgcn_sched_barrier(0);
  }
  F::pin(s);
  if (MODE == kReconstruct) {
    if (d.n_out() != 0) store_window(out + kHeaderBytes, t, F::row(s, 0), tail0, p.bs);
    return;
  }
  for (uint32_t q = 0; q < d.n_out(); ++q) {
    const uint32_t idx = d.out_idx(q);
    store_window(out + static_cast<uint64_t>(idx) * p.bs, t, F::row(s, q), tail0,
                 object_bytes(idx, p.bs, 0, p.obj_len));
  }
}

// Reconstruct headers and the edge items of a decode / reconstruct, block b
// taking objects / items b, b + G, ... (b counted from `first`, G = `step`).
// Block-uniform (ensure_tables has a barrier).
template <class F, int K, int MODE>
__device__ __forceinline__ void decode_edges(const DecodeParams& p, uint32_t first, uint32_t step,
                                             Slots& st, TablePre<F, K>& pre) {
  if (MODE == kReconstruct && p.headers != nullptr)
    for (uint32_t o = first; o < p.n_obj; o += step)
      block_headers(p.out + static_cast<uint64_t>(o) * p.out_stride, 0,
                    p.headers + static_cast<uint64_t>(load_desc(p, o).header()) * kHeaderBytes, 1);
  pre.table = 0xFFFFFFFFu;
  for (uint32_t e = first; e < p.n_obj * p.edge_tiles; e += step)
    decode_edge_item<F, K, MODE>(p, e, st, pre);
}

// One launch per decode / reconstruct pass: the edge items in the blocks
// counted from the end of the grid (see encode_kernel), then the interior
// stream.  The interior's first table change goes into the LDS slot the edge
// items did not use, behind a barrier, as between any two items.
// CRCFREE (A/B): reconstruct's chunk CRC with unfenced raw16 lookups.
template <class F, int K, int MODE, bool NOCOMP = false, int NBX = 0, bool SDESC = true,
          bool CRCFREE = false>
__global__ void __launch_bounds__(kThreadsPerBlock)
    __attribute__((amdgpu_waves_per_eu(NBX > 6 ? 4 : kDecodeOcc, 8))) decode_kernel(DecodeParams p) {
  Slots st{0xFFFFFFFFu, 1u};
  TablePre<F, K> pre;
  if constexpr (MODE == kReconstruct) {
    if (p.crc_lanes != nullptr) {  // block-uniform: the lane tables after the two table slots
      load_tables(static_cast<const uint32_t*>(p.crc_lanes), kCrcLaneBytes, 2 * table_slot_bytes(K, F::kW));
      __syncthreads();
    }
  }
  if (p.fused_edges) {
    if (p.edge_blocks == 0) {
      decode_edges<F, K, MODE>(p, gridDim.x - 1 - blockIdx.x, gridDim.x, st, pre);
    } else if (blockIdx.x < p.edge_blocks) {
      decode_edges<F, K, MODE>(p, blockIdx.x, p.edge_blocks, st, pre);
      return;
    }
  }
  decode_interior<F, K, MODE, NOCOMP, NBX, SDESC, CRCFREE>(p, st, pre);
}

// The edge work in a launch of its own (side-stream variant, ECAMD_EDGE_SIDE=1).
template <class F, int K, int MODE>
__global__ void __launch_bounds__(kThreadsPerBlock) decode_edge_kernel(DecodeParams p) {
  Slots st{0xFFFFFFFFu, 1u};
  TablePre<F, K> pre;
  decode_edges<F, K, MODE>(p, blockIdx.x, gridDim.x, st, pre);
}

// ---------------- decode, loader / consumer split ----------------
//
// decode_dma_kernel: the decode pass (MODE kDecode) and reconstruct (MODE
// kReconstruct: row 0 into the fragment payload, no input copies) in the
// shape of encode_dma_kernel.  An item is W KiB of payload positions of one object;
// the L loader waves DMA input j of it -- the payload of fragment
// d.in_idx(j) -- into an R-slot LDS ring, and every wave takes the products
// of its 1 KiB from LDS, stores a present data input to its object slice at
// once (kDrop otherwise, as decode_interior) and the rebuilt rows at the
// item's end.  Table sets live in two LDS slots: the consumer waves (waves
// >= L, so the loaders' vmcnt carries only DMAs and stores) fetch the set of
// item i + 1 into registers during item i - 1 and write it to the free slot
// right after item i's first barrier; the ring's next barrier publishes it.
// vmcnt: a loader issues, per slot, kPerLoader DMAs then one store (the
// prologue adds a zero-record store per slot to keep that shape), so slot t
// has landed when at most 1 + (R - 2) * (kPerLoader + 1) of its operations
// are younger -- the rows' stores at an item's end only make it conservative.
template <class F, int K>
struct TableRegs {
  static constexpr int kChunks = K * F::kTableBytes / 16;
  uint4 v[(kChunks + 255) / 256];  // enough for >= 256 fetching threads
};

// PROBE (A/B builds, WRONG objects): 1 = XORs instead of the lookups
// (memory-only), 2 = object stores moved down to 16-B alignment.
template <class F, int K, int R, bool NT, int L = 4, int W = 16, int PROBE = 0, int MODE = kDecode>
__global__ void __launch_bounds__(W * 64) decode_dma_kernel(DecodeParams p) {
  static_assert(MODE == kDecode || MODE == kReconstruct, "decode pass or reconstruct");
  constexpr int S = MODE == kReconstruct ? 0 : 1;  // stores per slot (decode: the input copy)
  static_assert(R >= 2 && R <= K + 1, "ring of 2 .. K + 1 slots");
  static_assert(L == 2 || L == 4 || L == 8, "loader waves");
  static_assert((W - L) * 64 >= 256, "at least 256 table-fetching threads");
  constexpr uint32_t kSlot = 1024u * W;
  constexpr int kPerLoader = W / L;
  constexpr uint32_t kTab = table_slot_bytes(K, F::kW);
  constexpr uint32_t kRing = 2 * kTab;
  constexpr int kChunks = TableRegs<F, K>::kChunks;
  constexpr int kFetchers = (W - L) * 64;
  constexpr int kPerFetcher = (kChunks + kFetchers - 1) / kFetchers;
  static_assert(kPerFetcher <= static_cast<int>(sizeof(TableRegs<F, K>::v) / 16), "table registers");
  const uint32_t wave = wave_in_block();
  if (blockIdx.x < p.edge_blocks) {  // edge items: 256 threads, the stream kernel's code
    if (threadIdx.x >= kThreadsPerBlock) return;
    Slots st{0xFFFFFFFFu, 1u};
    TablePre<F, K> pre;
    decode_edges<F, K, MODE>(p, blockIdx.x, p.edge_blocks, st, pre);
    return;
  }
  const ItemRange rg = item_range(p.n_obj * p.tiles, p.xcd_split, interior_block(p.edge_blocks));
  if (rg.begin >= rg.end) return;  // block-uniform
  const uint32_t n_items = to_sgpr((rg.end - rg.begin + rg.step - 1) / rg.step);
  const bool loader = wave < static_cast<uint32_t>(L);
  const uint32_t lane16 = lane_id() * 16;
  const uint32_t fetcher = threadIdx.x - L * 64;  // < kFetchers for the consumer waves
  auto item_at = [&](uint32_t i, uint32_t& o, uint32_t& x0) {
    const uint32_t w = rg.begin + (i < n_items ? i : 0) * rg.step;
    o = to_sgpr(w / p.tiles);
    x0 = (w - o * p.tiles) * kSlot;
  };
  auto desc_at = [&](uint32_t i) {
    uint32_t o, x0;
    item_at(i, o, x0);
    return load_desc(p, o);
  };
  // loaders: the DMAs of slot (item i with descriptor d, input j) into ring slot ri
  auto issue = [&](uint32_t i, const DescU& d, int j, uint32_t ri) {
    if (!loader) return;
    uint32_t o, x0;
    item_at(i, o, x0);
    const v4u_s src = rsrc4(p.frags + static_cast<uint64_t>(o) * p.stripe_stride,
                            i < n_items ? ~0u : 0u);
    const uint32_t part = wave * (kSlot / L);
    const uint32_t lds = kRing + ri * kSlot + part;
    const uint32_t soff = to_sgpr(in_pos(p, d, j) * p.frag_stride + kHeaderBytes + x0 + part);
#pragma unroll
    for (int c = 0; c < kPerLoader; ++c) dma16<NT>(src, lane16, soff + 1024 * c, lds + 1024 * c);
  };
  // consumers: table set `table` into registers (zero-record when not needed)
  TableRegs<F, K> tr;
  auto fetch = [&](uint32_t table, bool need) {
    if (loader) return;
    const Rsrc t = rsrc(p.tables + static_cast<uint64_t>(table) * (K * F::kTableBytes / 4),
                        need ? K * F::kTableBytes : 0);
#pragma unroll
    for (int c = 0; c < kPerFetcher; ++c) tr.v[c] = buf_ld<true>(t, (fetcher + c * kFetchers) * 16, 0);
  };
  auto publish = [&](uint32_t slot) {  // tr into table slot `slot` (visible after a barrier)
    if (loader) return;
    auto* dst = lds_v4(slot * kTab);
#pragma unroll
    for (int c = 0; c < kPerFetcher; ++c) {
      const uint32_t i = fetcher + c * kFetchers;
      if (i < static_cast<uint32_t>(kChunks)) {
        v4u v;
        v.x = tr.v[c].x;
        v.y = tr.v[c].y;
        v.z = tr.v[c].z;
        v.w = tr.v[c].w;
        dst[i] = v;
      }
    }
  };
  DescU d = desc_at(0);
  DescU dn = desc_at(1);
  // item 0's set into slot 0 directly; item 1's into registers
  uint32_t slot = 0, table = d.table();
  load_tables(p.tables + static_cast<uint64_t>(table) * (K * F::kTableBytes / 4), K * F::kTableBytes, 0);
  fetch(dn.table(), 1 < n_items && dn.n_out() != 0 && dn.table() != table);
  __syncthreads();
  // prologue: slots 0 .. R-2, each followed by a (zero-record) store as in the loop
  const Rsrc none = rsrc(p.frags, 0);
#pragma unroll
  for (int t = 0; t < R - 1; ++t) {
    issue(t / K, t / K == 0 ? d : dn, t % K, t);
    if (S && loader) buf_st(none, lane16, 0, make_uint4(0, 0, 0, 0));
  }
  uint32_t ring = 0;
#pragma clang loop unroll(disable)
  for (uint32_t i = 0; i < n_items; ++i) {
    uint32_t o, x0;
    item_at(i, o, x0);
    const Rsrc out = rsrc_out(p.out + static_cast<uint64_t>(o) * p.out_stride, out_extent<MODE>(p));
    const bool copy = MODE != kReconstruct && d.copy_inputs() != 0;
    check_desc<K, MODE>(p, d, o);
    // the slot of item i + 1's set (the one item i - 1 used, or this one again)
    const bool swap = i + 1 < n_items && dn.n_out() != 0 && dn.table() != table;
    const uint32_t kb = F::kb(slot * kTab);
    const DescU d2 = desc_at(i + 2);
    typename F::Acc s;
    F::zero(s);
#pragma unroll
    for (int j = 0; j < K; ++j) {
      if (loader) wait_vm<S + (R - 2) * (kPerLoader + S)>();
      ring_barrier();
      if (j == 0) {
        // item i + 1's set into the free slot; item i + 2's into registers
        // when item i + 1's swap will leave a different set in LDS
        if (swap) publish(slot ^ 1u);
        const uint32_t after = swap ? dn.table() : table;
        fetch(d2.table(), i + 2 < n_items && d2.n_out() != 0 && d2.table() != after);
      }
      const uint32_t rn = ring == 0 ? R - 1 : ring - 1;
      if (j + R - 1 < K)
        issue(i, d, j + R - 1, rn);
      else
        issue(i + 1, dn, j + R - 1 - K, rn);
      const v4u xin = *lds_v4(kRing + ring * kSlot + wave * 1024 + lane16);
      const uint4 xv = make_uint4(xin.x, xin.y, xin.z, xin.w);
      if constexpr (PROBE == 1) {
        uint32_t* a = reinterpret_cast<uint32_t*>(&s);
        a[0] ^= xv.x;
      } else {
        F::mac(kb, j * F::kTableBytes, xv, s);
      }
      if constexpr (MODE != kReconstruct) {
        const uint32_t slice = PROBE == 2 ? (d.in_idx(j) * p.bs) & ~15u : d.in_idx(j) * p.bs;
        drop_st(out, copy && d.in_idx(j) < static_cast<uint32_t>(K), lane16, slice + x0 + wave * 1024, xv);
      }
      ring = ring + 1 == R ? 0 : ring + 1;
    }
    F::pin(s);
    if constexpr (MODE == kReconstruct) {
      buf_st(out, lane16, kHeaderBytes + x0 + wave * 1024, F::row(s, 0));
    } else {
      const uint32_t e = d.n_out();
#pragma unroll
      for (int q = 0; q < F::kRows; ++q) {
        const uint32_t slice = PROBE == 2 ? (d.out_idx(q) * p.bs) & ~15u : d.out_idx(q) * p.bs;
        drop_st(out, q < static_cast<int>(e), lane16, slice + x0 + wave * 1024, F::row(s, q));
      }
    }
    if (swap) {
      slot ^= 1u;
      table = dn.table();
    }
    d = dn;
    dn = d2;
  }
  if (loader) wait_vm<0>();  // no DMA may land in LDS after the block ends
}

// ---------------- launch ----------------


// Blocks per CU that are resident at once: the occupancy API's answer capped
// by the register file (512 VGPRs per lane per SIMD, one wave per SIMD per
// block) -- the API can report one block per CU more than fits
// (MI355X_MICROARCH.md, Residency), and a grid-stride kernel must not queue
// blocks behind the resident ones -- and by `max_per_cu`.
inline int resident_per_cu(const void* kernel, size_t lds_bytes, int max_per_cu) {
  // the hardware limit of a (device, kernel, LDS size) triple, asked once: the
  // two runtime queries cost host time on every launch of a small call
  static std::mutex mu;
  static std::map<std::tuple<int, const void*, size_t>, int> limit;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) dev = -1;
  const auto key = std::make_tuple(dev, kernel, lds_bytes);
  int hw = 0;
  {
    std::lock_guard<std::mutex> lk(mu);
    auto it = limit.find(key);
    if (it != limit.end()) hw = it->second;
  }
  if (hw == 0) {
    hw = 64;
    int b = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&b, kernel, kThreadsPerBlock, lds_bytes) ==
            hipSuccess &&
        b > 0)
      hw = std::min(hw, b);
    hipFuncAttributes attr{};
    if (hipFuncGetAttributes(&attr, kernel) == hipSuccess && attr.numRegs > 0)
      hw = std::min(hw, 512 / ((attr.numRegs + 7) / 8 * 8));
    std::lock_guard<std::mutex> lk(mu);
    limit[key] = hw;
  }
  return std::max(std::min(max_per_cu, hw), 1);
}

// Compute units of the current device (asked once per device).
inline int device_cus() {
  static std::atomic<int> cache[64];
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 256;
  int cus = cache[dev].load(std::memory_order_relaxed);
  if (cus == 0) {
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
        cus <= 0)
      cus = 256;
    cache[dev].store(cus, std::memory_order_relaxed);
  }
  return cus;
}

inline int grid_for(const void* kernel, size_t lds_bytes, uint32_t items, int max_per_cu) {
  const uint32_t resident =
      static_cast<uint32_t>(device_cus() * resident_per_cu(kernel, lds_bytes, max_per_cu));
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

// XCD-major work split (item_range) for a grid of `grid` blocks.
inline uint32_t xcd_split_for(int grid, bool xcd) {
  return (grid >= 8 && grid % 8 == 0 && ab_knob("ECAMD_XCD", xcd)) ? 1u : 0u;
}

template <typename Kern, typename Params>
hipError_t launch(Kern kern, Params p, size_t lds, uint32_t items, hipStream_t stream,
                  int max_per_cu = 4, bool xcd = true, int* grid_out = nullptr) {
  if (items == 0) return hipSuccess;
  const void* k = reinterpret_cast<const void*>(kern);
  if (!lds_starts_at_zero(k)) return hipErrorInvalidKernelFile;
  const int grid = grid_for(k, lds, items, max_per_cu);
  p.xcd_split = xcd_split_for(grid, xcd);
  if (grid_out) *grid_out = grid;

  hipLaunchKernelGGL(kern, dim3(grid), dim3(kThreadsPerBlock), lds, stream, p);
  return hipGetLastError();
}

// A launch whose edge items run in blocks of their own: blocks [0, E) take
// the edge items (E = their count rounded up to 8, at most one per CU) and
// return; blocks [E, E + G) stream the interior items exactly as a launch of
// G blocks would.  All E + G blocks must be resident at once -- otherwise
// interior blocks would queue behind the edge blocks -- else (or with the
// caller's no_edge_blocks) every block runs its share of the edge items first.
// Why: an edge item is a chain of K dependent loads (one input in registers
// at a time), ~12 us; with the edges at the front of some interior blocks,
// those blocks finish that much after the rest (measured round 3 at 2 blocks
// per CU, 256 x 4 MiB k = 10: encode 297.7 us fused, 291.0 with the edges
// in a launch of their own before it, 284.7 for the interior alone).
template <typename Kern, typename Params>
hipError_t launch_edges_apart(Kern kern, Params p, size_t lds, uint32_t interior_items,
                              uint32_t edge_items, hipStream_t stream, int max_per_cu, bool xcd,
                              int* grid_out = nullptr) {
  p.edge_blocks = 0;
  const void* k = reinterpret_cast<const void*>(kern);
  const int cus = device_cus();
  const uint32_t e = (std::min<uint32_t>(edge_items, static_cast<uint32_t>(cus)) + 7u) & ~7u;
  if (p.no_edge_blocks || edge_items == 0 || interior_items == 0 || !lds_starts_at_zero(k))
    return launch(kern, p, lds, std::max(interior_items, edge_items), stream, max_per_cu, xcd,
                  grid_out);
  const int grid = grid_for(k, lds, interior_items, max_per_cu);
  const int resident = cus * resident_per_cu(k, lds, 64);
  if (grid + static_cast<int>(e) > resident)
    return launch(kern, p, lds, std::max(interior_items, edge_items), stream, max_per_cu, xcd,
                  grid_out);
  p.edge_blocks = e;
  p.xcd_split = xcd_split_for(grid, xcd);
  if (grid_out) *grid_out = grid;
  hipLaunchKernelGGL(kern, dim3(grid + static_cast<int>(e)), dim3(kThreadsPerBlock), lds, stream, p);
  return hipGetLastError();
}

// A/B builds only (ECAMD_EDGE_SIDE): the round-2 launch forms with the edge
// items in a launch of their own, forked onto a side stream and joined back
// with events (=1) or launched first on the same stream (=2).  Measured round
// 2 (rocprof timeline, profiles/r02l_timeline.txt): the fork / join left the
// GPU idle 25-32 us between consecutive interior kernels, hence the fused
// launch of the product.
struct SideStream {
  hipStream_t s = nullptr;
  hipEvent_t fork = nullptr, join = nullptr;
};

template <class Main, class Side>
hipError_t fork_join(hipStream_t stream, Main main, Side side) {
  static std::mutex mu;
  static SideStream per_dev[64];
  std::lock_guard<std::mutex> lk(mu);
  int dev = 0;
  SideStream* sd = nullptr;
  if (ab_knob("ECAMD_EDGE_SIDE", 0) == 2) {
    const hipError_t e = side(stream);
    return e != hipSuccess ? e : main(stream);
  }
  if (hipGetDevice(&dev) == hipSuccess && dev >= 0 && dev < 64) {
    sd = &per_dev[dev];
    if (sd->s == nullptr &&
        (hipStreamCreateWithFlags(&sd->s, hipStreamNonBlocking) != hipSuccess ||
         hipEventCreateWithFlags(&sd->fork, hipEventDisableTiming) != hipSuccess ||
         hipEventCreateWithFlags(&sd->join, hipEventDisableTiming) != hipSuccess)) {
      (void)hipGetLastError();
      sd->s = nullptr;
      sd = nullptr;
    }
  }
  if (sd == nullptr) {  // no side stream: one after the other
    const hipError_t e = side(stream);
    return e != hipSuccess ? e : main(stream);
  }
  hipError_t e = hipEventRecord(sd->fork, stream);
  if (e == hipSuccess) e = hipStreamWaitEvent(sd->s, sd->fork, 0);
  if (e != hipSuccess) return e;
  const hipError_t em = main(stream);
  const hipError_t es = side(sd->s);
  e = hipEventRecord(sd->join, sd->s);
  if (e == hipSuccess) e = hipStreamWaitEvent(stream, sd->join, 0);
  return em != hipSuccess ? em : (es != hipSuccess ? es : e);
}

// Bytes of the last data fragment that lie inside the object (encode inputs
// and decode outputs stop there; <= bs).
inline int64_t last_room(uint32_t bs, uint64_t obj_len, uint32_t k) {
  int64_t room = static_cast<int64_t>(obj_len) - static_cast<int64_t>(k - 1) * bs;
  if (room > static_cast<int64_t>(bs)) room = bs;
  return room < 0 ? 0 : room;
}

// Interior items of `ch` * 4 KiB: the tiles and the 4-KiB edge tiles past them.
inline void set_tiles(EncodeParams& p, int64_t room, uint32_t ch) {
  p.tile_ch = ch;
  p.tiles = static_cast<uint32_t>(room / (kTile * ch));
  p.edge_tiles = (p.bs + kTile - 1) / kTile - p.tiles * ch;
}

// inline_crc32: the finishing pass (ec_crc.hip) over `count` fragments of
// every object whose chunk partials a launch has just stored.
inline hipError_t crc_finish(uint8_t* frags, uint64_t frag_stride, uint64_t stripe_stride,
                             const uint32_t* part, uint32_t part_rows, uint32_t part_row0,
                             const void* lanes, const void* tables, uint32_t n_obj, uint32_t count,
                             uint32_t bs, uint32_t chunks, hipStream_t stream) {
  CrcFinishParams fp{};
  fp.frags = frags;
  fp.frag_stride = frag_stride;
  fp.stripe_stride = stripe_stride;
  fp.part = part;
  fp.part_rows = part_rows;
  fp.part_row0 = part_row0;
  fp.lanes = lanes;
  fp.tables = tables;
  fp.n_obj = n_obj;
  fp.count = count;
  fp.bs = bs;
  fp.chunks = chunks;
  return launch_crc_finish(fp, stream);
}

// The parity rows' (and, with the full stripe, the data fragments') headers
// of an inline_crc32 encode launch whose interior covered `chunks` KiB.
template <int K>
hipError_t encode_crc_finish(const EncodeParams& p, bool data, uint32_t chunks, hipStream_t stream) {
  hipError_t e = crc_finish(p.parity + static_cast<uint64_t>(p.row0) * p.frag_stride, p.frag_stride,
                            p.stripe_stride, p.crc_part, p.m, p.row0, p.crc_lanes,
                            p.crc_finish_tables, p.n_obj, p.nrows, p.bs, chunks, stream);
  if (e != hipSuccess || !data) return e;
  return crc_finish(p.data, p.frag_stride, p.stripe_stride, p.crc_part_data, K, 0, p.crc_lanes,
                    p.crc_finish_tables, p.n_obj, K, p.bs, chunks, stream);
}

// The loader / consumer encode (encode_dma_kernel): one W * 64-thread block
// per CU (a multiple of 8, so blocks keep their XCD) after E edge blocks.
// Measured round 4 (tools/ab_bench.py, same process, k = 10, m = 4,
// 256 x 4 MiB, profiles/r04e_ab.txt): R = 3, W = 16 (four consumer waves per
// SIMD, 16 KiB slots), L = 4 loaders 271.5 us against 285.7 for the stream
// kernel; R = 3 SW = 2 276.4, R = 5 280.6, R = 4 W = 16 274.6, L = 8 273.4.
// Then (profiles/r04j_ab.txt): W = 12 (three waves per SIMD, 12 KiB slots)
// 267.9 against 270.4 at W = 16; L = 2 269.0; R = 4 W = 12 274.5; cached
// (not nontemporal) DMA loads 270.3.  The default path takes W = 12 for
// k >= kDmaMinK when the batch has a 16 KiB item for every CU (smaller
// batches keep the stream kernel's 4 KiB items).
template <class F, int K, int NR, int R, bool NT, int L = 4, int SW = 1, int W = 8,
          bool DATA = false, bool NOCOMP = false, bool CONTIG = false, int RUNS = 0, int COMB = 0,
          int CV = 6>
hipError_t launch_encode_dma(EncodeParams p, hipStream_t stream, uint32_t* chunks = nullptr,
                             bool xcd = true) {
  set_tiles(p, last_room(p.bs, p.obj_len, K), 1024u * W * SW / kTile);
  if (chunks) *chunks = crc_chunks(p.tiles, p.tile_ch);
  const auto kern = encode_dma_kernel<F, K, NR, R, NT, L, SW, W, DATA, NOCOMP, CONTIG, RUNS, COMB, CV>;
  const size_t lds = dma_lds_bytes<F, K, R, SW, W>(p.crc_lanes != nullptr);
  if (!lds_starts_at_zero(reinterpret_cast<const void*>(kern))) return hipErrorInvalidKernelFile;
  const int cus = device_cus();
  const uint32_t items = p.n_obj * p.tiles;
  const uint32_t edge_items = std::max(p.n_obj * p.edge_tiles, p.headers ? p.n_obj : 0u);
  const uint32_t e = (std::min<uint32_t>(edge_items, static_cast<uint32_t>(cus)) + 7u) & ~7u;
  uint32_t g = std::min<uint32_t>(static_cast<uint32_t>(cus) & ~7u, std::max(items, 1u));
  if (g >= 8) g &= ~7u;
  p.edge_blocks = edge_items ? e : 0;
  p.fused_edges = 1;
  p.xcd_split = xcd_split_for(static_cast<int>(g), xcd);
  hipLaunchKernelGGL(kern, dim3(g + p.edge_blocks), dim3(W * 64), lds, stream, p);
  return hipGetLastError();
}

// A/B builds: the alternative encode launches of past measurements (the
// switches are documented where each one was measured: DESIGN.md §4).
// Returns hipErrorNotSupported when no switch applies to this launch.
template <class F, int K, int NR>
hipError_t launch_encode_ab(EncodeParams p, hipStream_t stream, bool data, uint32_t edge_items) {
  constexpr size_t lds = K * F::kTableBytes;
  const int per_cu = ab_knob("ECAMD_ENC_PER_CU", kEncodePerCu);
  if (p.crc_lanes != nullptr) return hipErrorNotSupported;  // no A/B forms of the CRC encode
  if (ab_knob("ECAMD_EDGE_SIDE", 0)) {
    p.fused_edges = 0;
    hipError_t e = fork_join(
        stream,
        [&](hipStream_t s) { return launch(encode_kernel<F, K, NR>, p, lds, p.n_obj * p.tiles, s, per_cu); },
        [&](hipStream_t s) {
          return launch(encode_edge_kernel<F, K, NR>, p, lds,
                        std::max(p.n_obj * p.edge_tiles, p.headers ? p.n_obj : 0u), s);
        });
    if (e != hipSuccess || !data) return e;
    return launch(copy_data_kernel, p, 0, p.n_obj * K * ((p.bs + kTile - 1) / kTile), stream);
  }
  p.fused_edges = 1;
  const uint32_t items = p.n_obj * p.tiles;
  if (data && ab_knob("ECAMD_DATA_COPY", 0)) {
    const hipError_t e = launch_edges_apart(encode_kernel<F, K, NR>, p, lds, items, edge_items,
                                            stream, per_cu, true);
    if (e != hipSuccess) return e;
    return launch(copy_data_kernel, p, 0, p.n_obj * K * ((p.bs + kTile - 1) / kTile), stream);
  }
  if constexpr (K == 10 && NR == 4) {
    const bool ntl = ab_knob("ECAMD_ENC_NTL", 0);
    if (!data) {
      // loader / consumer split: ring slots R, loader waves L, KiB per consumer wave SW
      const int ring = ab_knob("ECAMD_ENC_DMA", 0);
      const int lw = ab_knob("ECAMD_ENC_DMA_L", 4), sw = ab_knob("ECAMD_ENC_DMA_SW", 1);
      const int nw = ab_knob("ECAMD_ENC_DMA_W", 8);
      if (ring == 5 && lw == 4 && sw == 1 && nw == 8) return launch_encode_dma<F, K, NR, 5, true>(p, stream);
      if (ring == 3 && lw == 4 && sw == 2 && nw == 8) return launch_encode_dma<F, K, NR, 3, true, 4, 2>(p, stream);
      if (ring == 3 && lw == 8 && sw == 2 && nw == 8) return launch_encode_dma<F, K, NR, 3, true, 8, 2>(p, stream);
      if (ring == 2 && lw == 4 && sw == 4 && nw == 8) return launch_encode_dma<F, K, NR, 2, true, 4, 4>(p, stream);
      if (ring == 3 && lw == 4 && sw == 4 && nw == 8) return launch_encode_dma<F, K, NR, 3, true, 4, 4>(p, stream);
      if (ring == 3 && lw == 4 && sw == 1 && nw == 16) return launch_encode_dma<F, K, NR, 3, true, 4, 1, 16>(p, stream);
      if (ring == 3 && lw == 8 && sw == 1 && nw == 16) return launch_encode_dma<F, K, NR, 3, true, 8, 1, 16>(p, stream);
      if (ring == 4 && lw == 4 && sw == 1 && nw == 16) return launch_encode_dma<F, K, NR, 4, true, 4, 1, 16>(p, stream);
      if (ring == 3 && lw == 4 && sw == 2 && nw == 16) return launch_encode_dma<F, K, NR, 3, true, 4, 2, 16>(p, stream);
      if (ring == 3 && lw == 2 && sw == 1 && nw == 16) return launch_encode_dma<F, K, NR, 3, true, 2, 1, 16>(p, stream);
      if (ring == 3 && lw == 4 && sw == 1 && nw == 12) return launch_encode_dma<F, K, NR, 3, true, 4, 1, 12>(p, stream);
      if (ring == 4 && lw == 4 && sw == 1 && nw == 12) return launch_encode_dma<F, K, NR, 4, true, 4, 1, 12>(p, stream);
      if (ring == 4 && lw == 4 && sw == 1 && nw == 8) return launch_encode_dma<F, K, NR, 4, true, 4, 1, 8>(p, stream);
      if (ring == 5 && lw == 4 && sw == 1 && nw == 12) return launch_encode_dma<F, K, NR, 5, true, 4, 1, 12>(p, stream);
      if (ring == -3 && lw == 4 && sw == 1 && nw == 16) return launch_encode_dma<F, K, NR, 3, false, 4, 1, 16>(p, stream);
      if (ab_knob("ECAMD_ENC_DMA_NOCOMP", 0))
        return launch_encode_dma<F, K, NR, 3, true, 4, 1, 12, false, true>(p, stream);
      if (ab_knob("ECAMD_ENC_DMA_CONTIG", 0) == 12)
        return launch_encode_dma<F, K, NR, 3, true, 4, 1, 12, false, false, true>(p, stream);
      if (ab_knob("ECAMD_ENC_DMA_CONTIG", 0) == 16)
        return launch_encode_dma<F, K, NR, 3, true, 4, 1, 16, false, false, true>(p, stream);
      const int runs = ab_knob("ECAMD_ENC_DMA_RUNS", 0);
      if (runs == 2) return launch_encode_dma<F, K, NR, 3, true, 4, 1, 16, false, false, false, 2>(p, stream);
      if (runs == 4) return launch_encode_dma<F, K, NR, 3, true, 4, 1, 16, false, false, false, 4>(p, stream);
      if (runs == 8) return launch_encode_dma<F, K, NR, 3, true, 4, 1, 16, false, false, false, 8>(p, stream);
      const int comb = ab_knob("ECAMD_ENC_DMA_COMB", 0);
      if (comb == 4) return launch_encode_dma<F, K, NR, 3, true, 4, 1, 16, false, false, false, 0, 4>(p, stream);
      if (comb == 5) return launch_encode_dma<F, K, NR, 3, true, 4, 1, 16, false, false, false, 0, 5>(p, stream);
      if (comb == 8) return launch_encode_dma<F, K, NR, 3, true, 4, 1, 16, false, false, false, 0, 8>(p, stream);
      if (comb == 16) return launch_encode_dma<F, K, NR, 3, true, 4, 1, 16, false, false, false, 0, 16>(p, stream);
    }
    if (ab_knob("ECAMD_ENC_NOCOMP", 0))  // memory-only probe: WRONG parity
      return ntl ? launch_edges_apart(encode_kernel<F, K, NR, true, false, 1, true>, p, lds, items,
                                      edge_items, stream, per_cu, true)
                 : launch_edges_apart(encode_kernel<F, K, NR, true>, p, lds, items, edge_items,
                                      stream, per_cu, true);
    if (!data && ab_knob("ECAMD_ENC_R3", 0))  // the round-3 prologue (item-boundary drain)
      return launch_edges_apart(encode_kernel<F, K, NR, false, false, 1, false, 0, false>, p, lds,
                                items, edge_items, stream, per_cu, true);
  }
  if (per_cu != kEncodePerCu)
    return data ? launch_edges_apart(encode_kernel<F, K, NR, false, true>, p, lds, items,
                                     edge_items, stream, per_cu, true)
                : launch_edges_apart(encode_kernel<F, K, NR>, p, lds, items, edge_items, stream,
                                     per_cu, true);
  return hipErrorNotSupported;
}

// Encode: one launch -- interior stream + edge items + headers, and the data
// fragments when asked (stored from the input registers); with inline_crc32
// the same launch stores its chunks' CRC partials, and the finishing pass
// follows.
template <class F, int K, int NR>
hipError_t launch_encode_k(EncodeParams p, hipStream_t stream) {
  const int64_t room = last_room(p.bs, p.obj_len, K);
  set_tiles(p, room, 1);
  constexpr size_t lds = K * F::kTableBytes;
  // data fragments are written by the first pass (rows 0..3) only
  const bool data = p.data != nullptr && p.row0 == 0;
  // interior and edge work items (edge items include the headers' objects)
  const uint32_t edge_items = std::max(p.n_obj * p.edge_tiles, p.headers ? p.n_obj : 0u);
  if constexpr (kAB && F::kRows <= kRowsPerPass) {
    const hipError_t e = launch_encode_ab<F, K, NR>(p, stream, data, edge_items);
    if (e != hipErrorNotSupported) return e;
  }
  if constexpr (kAB && F::kRows > kRowsPerPass) {  // eight-row encode: blocks per CU
    const int per_cu = ab_knob("ECAMD_ENC_PER_CU", kEncode8PerCu);
    if (per_cu != kEncode8PerCu && !data && p.crc_lanes == nullptr) {
      p.fused_edges = 1;
      return launch_edges_apart(encode_kernel<F, K, NR>, p, lds, p.n_obj * p.tiles, edge_items,
                                stream, per_cu, true);
    }
  }
  // Which kernel.  For k >= kDmaMinK the loader / consumer encode takes
  // every launch with the full stripe or the inline CRC, whatever the batch
  // size -- the stream kernel exists in those forms only for k < kDmaMinK
  // (round 5: the library held every (field, k, rows, data, CRC) stream
  // form, 149 MB; those forms only matter for throughput on large batches,
  // where the loader / consumer kernel is the faster one anyway) -- and the
  // plain parity encode of a batch with a 16 KiB item per CU.  Its input
  // offsets j * bs + x are 32-bit.
  const bool crc = p.crc_lanes != nullptr;
  uint32_t chunks = 0;
  hipError_t e = hipErrorInvalidValue;
  bool done = false;
  if constexpr (kAB && K == 10 && NR == 4) {
    // A/B: the inline CRC's forms (CV, see encode_dma_kernel) and a 4-slot ring
    // (ECAMD_CRC_V=10: the round-5 lookup form, CV 0; ECAMD_ENC_CV0=1: the
    // plain and full-stripe encodes built with CV 0, i.e. without the
    // matrix-core CRC's registers)
    const int cv = ab_knob("ECAMD_CRC_V", 0), cr = ab_knob("ECAMD_CRC_R", 3);
    if (!crc && ab_knob("ECAMD_ENC_CV0", 0))
      return data ? launch_encode_dma<F, K, NR, 4, true, 4, 1, 8, true, false, false, 0, 0, 0>(p, stream, &chunks, false)
                  : launch_encode_dma<F, K, NR, 3, true, 4, 1, 12, false, false, false, 0, 0, 0>(p, stream, &chunks);
    if (crc && data && cv == 10) {  // the full stripe's CRCs by lookups (CV 0)
      e = launch_encode_dma<F, K, NR, 4, true, 4, 1, 8, true, false, false, 0, 0, 0>(p, stream, &chunks, false);
      if (e != hipSuccess) return e;
      return encode_crc_finish<K>(p, data, chunks, stream);
    }
    if (crc && !data && (cv != 0 || cr != 3)) {
      if (cv == 10 && cr == 3) e = launch_encode_dma<F, K, NR, 3, true, 4, 1, 12, false, false, false, 0, 0, 0>(p, stream, &chunks);
      else if (cv == 1 && cr == 3) e = launch_encode_dma<F, K, NR, 3, true, 4, 1, 12, false, false, false, 0, 0, 1>(p, stream, &chunks);
      else if (cv == 2 && cr == 3) e = launch_encode_dma<F, K, NR, 3, true, 4, 1, 12, false, false, false, 0, 0, 2>(p, stream, &chunks);
      else if (cv == 10 && cr == 4) e = launch_encode_dma<F, K, NR, 4, true, 4, 1, 12, false, false, false, 0, 0, 0>(p, stream, &chunks);
      else if (cv == 1 && cr == 4) e = launch_encode_dma<F, K, NR, 4, true, 4, 1, 12, false, false, false, 0, 0, 1>(p, stream, &chunks);
      else if (cv == 4 && cr == 3) e = launch_encode_dma<F, K, NR, 3, true, 4, 1, 12, false, false, false, 0, 0, 4>(p, stream, &chunks);
      else if (cv == 4 && cr == 4) e = launch_encode_dma<F, K, NR, 4, true, 4, 1, 12, false, false, false, 0, 0, 4>(p, stream, &chunks);
      else return hipErrorInvalidValue;
      if (e != hipSuccess) return e;
      return encode_crc_finish<K>(p, data, chunks, stream);
    }
  }
  if constexpr (F::kRows <= kRowsPerPass && K >= kDmaMinK) {
    // Two-row passes (m <= 2) too, since round 6: k=10 m=2 256 x 4 MiB, one
    // box (profiles/r06h_ab_m2.txt), 236.5 us against 249.4 for the stream
    // kernel, both with 0 LDS bank conflicts (r06h_sq_table_m2.txt).  Round 5
    // had measured 309.5 against 250.7 and kept m <= 2 on the stream kernel:
    // that was before the two-row lookups read whole 8-B entries (section
    // 4.7 of DESIGN.md), a two-way bank conflict on every lookup.
    // (A/B: ECAMD_ENC_STREAM2=1 keeps the two-row passes on the stream
    // kernel, the round-5 form; ECAMD_ENC_DATA_W / _R: the full stripe's
    // block width and ring depth)
    if (crc || data ||
        ((NR > 2 || !ab_knob("ECAMD_ENC_STREAM2", 0)) &&
         dma_batch(K, p.bs, p.obj_len, p.n_obj, device_cus(), p.direct) && !ab_knob("ECAMD_ENC_STREAM", 0))) {
      if (static_cast<uint64_t>(K) * p.bs + 65536u > 0xFFFFFFFFull) return hipErrorInvalidValue;
      if constexpr (kAB && K == 10 && NR == 4) {
        const int dw = ab_knob("ECAMD_ENC_DATA_W", 8), dr = ab_knob("ECAMD_ENC_DATA_R", 4);
        if (data && (dw != 8 || dr != 4)) {
          if (dw == 16 && dr == 3) e = launch_encode_dma<F, K, NR, 3, true, 4, 1, 16, true>(p, stream, &chunks);
          else if (dw == 12 && dr == 4) e = launch_encode_dma<F, K, NR, 4, true, 4, 1, 12, true>(p, stream, &chunks);
          else if (dw == 12 && dr == 3) e = launch_encode_dma<F, K, NR, 3, true, 4, 1, 12, true>(p, stream, &chunks);
          else if (dw == 8 && dr == 3) e = launch_encode_dma<F, K, NR, 3, true, 4, 1, 8, true>(p, stream, &chunks);
          else if (dw == 8 && dr == 5) e = launch_encode_dma<F, K, NR, 5, true, 4, 1, 8, true>(p, stream, &chunks);
          else return hipErrorInvalidValue;
          if (e != hipSuccess || !crc) return e;
          return encode_crc_finish<K>(p, data, chunks, stream);
        }
      }
      // The full stripe (data fragments stored from the ring too) at W = 8,
      // R = 4: round 6, tools/ab_bench.py --full-stripe, one box
      // (profiles/r06h_ab_full.txt): 455.4 us against 469.7 at W = 12, R = 3
      // (465.4 at 12 / 4, 468.4 at 16 / 3, 528.4 at 8 / 3); the same order
      // in membench's pattern (452.0 vs 465.6); and walking the items
      // grid-stride without the XCD split, 448.5 against 457.3 (r06j).  The
      // plain parity encode stays at W = 12, R = 3, XCD split: at W = 8 its
      // two waves per SIMD cannot hide the lookups (308.0 us against 271.3
      // at R = 4, 284.8 at R = 5; r06i_ab_alt.txt).  The full stripe with
      // the inline CRC (every chunk's CRC on the matrix cores: 14 per item
      // and wave) runs at W = 12, R = 3 like the parity encode: 587.5 us
      // against 641.0 at W = 8, R = 4 (637.0 at 16 / 3; r06z_ab_full_crc.txt).
      // (Four-row GF(2^16) passes only -- m = 3, 4 and the first pass of
      // larger m: the library's size.)
      if constexpr (std::is_same_v<F, Gf16<2>> && NR == 4) {
        if (data && crc) {
          e = launch_encode_dma<F, K, NR, 3, true, 4, 1, 12, true>(p, stream, &chunks);
          return e != hipSuccess ? e : encode_crc_finish<K>(p, data, chunks, stream);
        }
      }
      e = data ? launch_encode_dma<F, K, NR, 4, true, 4, 1, 8, true>(p, stream, &chunks, false)
               : launch_encode_dma<F, K, NR, 3, true, 4, 1, 12>(p, stream, &chunks);
      done = true;
    }
  }
  if (!done) {
    p.fused_edges = 1;
    const uint32_t items = p.n_obj * p.tiles;
    chunks = crc_chunks(p.tiles, p.tile_ch);
    if constexpr (F::kRows > kRowsPerPass) {
      if (crc) return hipErrorInvalidValue;  // the inline CRC runs in four-row passes
      e = data ? launch_edges_apart(encode_kernel<F, K, NR, false, true>, p, lds, items, edge_items,
                                    stream, kEncodePerCu, true)
               : launch_edges_apart(encode_kernel<F, K, NR>, p, lds, items, edge_items, stream,
                                    kEncode8PerCu, true);
    } else if constexpr (K < kDmaMinK) {
      const size_t crc_lds = crc_lds_base<F, K>() + kCrcLaneBytes;
      if (crc)
        e = data ? launch_edges_apart(encode_kernel<F, K, NR, false, true, 1, false, 0, false, true>, p,
                                      crc_lds, items, edge_items, stream, kEncodePerCu, true)
                 : launch_edges_apart(encode_kernel<F, K, NR, false, false, 1, false, 0, false, true>, p,
                                      crc_lds, items, edge_items, stream, kEncodePerCu, true);
      else
        e = data ? launch_edges_apart(encode_kernel<F, K, NR, false, true>, p, lds, items, edge_items,
                                      stream, kEncodePerCu, true)
                 : launch_edges_apart(encode_kernel<F, K, NR>, p, lds, items, edge_items, stream,
                                      kEncodePerCu, true);
    } else {
      e = launch_edges_apart(encode_kernel<F, K, NR>, p, lds, items, edge_items, stream,
                             kEncodePerCu, true);
    }
  }
  if (e != hipSuccess || !crc) return e;
  return encode_crc_finish<K>(p, data, chunks, stream);
}

// LDS of a decode launch: two table slots.
template <class F, int K>
constexpr uint32_t decode_lds_bytes() {
  return 2 * table_slot_bytes(K, F::kW);
}

// The loader / consumer decode (decode_dma_kernel), launched like
// launch_encode_dma: items of W KiB, edge items in blocks of their own.
// Measured round 4 (tools/ab_bench.py, same process, profiles/r04j_ab.txt):
// W = 12 384.9 us against 401.0 for the stream kernel; W = 16 401.9 (its 75
// VGPRs leave no room for the edge blocks beside a 16-wave block; at 12
// waves both fit), R = 4 404.5, L = 8 401.3, cached DMA loads 402.6.
template <class F, int K, int R, bool NT, int L = 4, int W = 16, int PROBE = 0, int PER_CU = 1,
          int MODE = kDecode>
hipError_t launch_decode_dma(DecodeParams p, hipStream_t stream) {
  p.tile_ch = W / 4;
  const int64_t lim = MODE == kReconstruct ? static_cast<int64_t>(p.bs) : last_room(p.bs, p.obj_len, K);
  p.tiles = static_cast<uint32_t>(lim / (1024 * W));
  p.edge_tiles = (p.bs + kTile - 1) / kTile - p.tiles * p.tile_ch;
  const auto kern = decode_dma_kernel<F, K, R, NT, L, W, PROBE, MODE>;
  constexpr size_t lds = 2 * table_slot_bytes(K, F::kW) + R * 1024 * W;
  if (!lds_starts_at_zero(reinterpret_cast<const void*>(kern))) return hipErrorInvalidKernelFile;
  const int cus = device_cus();
  const uint32_t items = p.n_obj * p.tiles;
  const uint32_t edge_items =
      std::max(p.n_obj * p.edge_tiles, MODE == kReconstruct && p.headers ? p.n_obj : 0u);
  const uint32_t e = (std::min<uint32_t>(edge_items, static_cast<uint32_t>(cus)) + 7u) & ~7u;
  uint32_t g = std::min<uint32_t>((static_cast<uint32_t>(cus) * PER_CU) & ~7u, std::max(items, 1u));
  if (g >= 8) g &= ~7u;
  p.edge_blocks = edge_items ? e : 0;
  p.fused_edges = 1;
  p.xcd_split = xcd_split_for(static_cast<int>(g), kDecodeXcd);
  hipLaunchKernelGGL(kern, dim3(g + p.edge_blocks), dim3(W * 64), lds, stream, p);
  return hipGetLastError();
}

// A/B builds: the alternative decode launches (see launch_encode_ab).
template <class F, int K, int MODE>
hipError_t launch_decode_ab(DecodeParams p, hipStream_t stream, uint32_t edge_items) {
  constexpr size_t lds = decode_lds_bytes<F, K>();
  const int per_cu = MODE == kReconstruct ? ab_knob("ECAMD_REC_PER_CU", kReconstructPerCu)
                                          : ab_knob("ECAMD_DEC_PER_CU", kDecodePerCu);
  if (ab_knob("ECAMD_EDGE_SIDE", 0)) {
    p.fused_edges = 0;
    return fork_join(
        stream,
        [&](hipStream_t s) {
          return launch(decode_kernel<F, K, MODE>, p, lds, p.n_obj * p.tiles, s, per_cu, kDecodeXcd);
        },
        [&](hipStream_t s) { return launch(decode_edge_kernel<F, K, MODE>, p, lds, edge_items, s); });
  }
  p.fused_edges = 1;
  const uint32_t items = p.n_obj * p.tiles;
  if constexpr (K == 10 && MODE == kDecode) {
    if (ab_knob("ECAMD_DEC_NOCOMP", 0))  // memory-only probe: WRONG objects
      return launch_edges_apart(decode_kernel<F, K, MODE, true>, p, lds, items, edge_items, stream,
                                per_cu, kDecodeXcd);
    const int dring = ab_knob("ECAMD_DEC_DMA", 0), dl = ab_knob("ECAMD_DEC_DMA_L", 4);
    const int dw = ab_knob("ECAMD_DEC_DMA_W", 16);
    if (dring == 4 && dl == 4 && dw == 16) return launch_decode_dma<F, K, 4, true>(p, stream);
    if (dring == 3 && dl == 8 && dw == 16) return launch_decode_dma<F, K, 3, true, 8>(p, stream);
    if (dring == 3 && dl == 4 && dw == 16) return launch_decode_dma<F, K, 3, true, 4, 16>(p, stream);
    if (dring == 3 && dl == 2 && dw == 12) return launch_decode_dma<F, K, 3, true, 2, 12>(p, stream);
    if (dring == 3 && dl == 4 && dw == 8) return launch_decode_dma<F, K, 3, true, 4, 8, 0, 2>(p, stream);
    if (ab_knob("ECAMD_DEC_DMA_NOCOMP", 0) == 1) return launch_decode_dma<F, K, 3, true, 4, 12, 1>(p, stream);
    if (ab_knob("ECAMD_DEC_DMA_NOCOMP", 0) == 2) return launch_decode_dma<F, K, 3, true, 4, 12, 2>(p, stream);
    if (dring == 4 && dl == 4 && dw == 12) return launch_decode_dma<F, K, 4, true, 4, 12>(p, stream);
    if (dring == 4 && dl == 2 && dw == 8) return launch_decode_dma<F, K, 4, true, 2, 8>(p, stream);
    if (dring == 5 && dl == 2 && dw == 8) return launch_decode_dma<F, K, 5, true, 2, 8>(p, stream);
    if (dring == -3 && dl == 4 && dw == 16) return launch_decode_dma<F, K, 3, false>(p, stream);
    if (ab_knob("ECAMD_DEC_R3", 0))  // round 3: vector descriptor loads, old prologue
      return launch_edges_apart(decode_kernel<F, K, MODE, false, 0, false>, p, lds, items,
                                edge_items, stream, per_cu, kDecodeXcd);
    const int nb = ab_knob("ECAMD_DEC_NB", 0);  // inputs in flight per wave
    if (nb == 10)
      return launch_edges_apart(decode_kernel<F, K, MODE, false, 10>, p, lds, items, edge_items,
                                stream, per_cu, kDecodeXcd);
    if (nb == 2)
      return launch_edges_apart(decode_kernel<F, K, MODE, false, 2>, p, lds, items, edge_items,
                                stream, per_cu, kDecodeXcd);
  }
  if (per_cu != (MODE == kReconstruct ? kReconstructPerCu : kDecodePerCu))
    return launch_edges_apart(decode_kernel<F, K, MODE>, p, lds, items, edge_items, stream, per_cu,
                              kDecodeXcd);
  return hipErrorNotSupported;
}

// Decode / reconstruct: (reconstruct headers +) edge items, then the
// interior stream, in one launch.  A multi-pass decode runs each pass as a
// decode (the descriptor's copy_inputs / n_out say what the pass stores).
template <class F, int K, int MODE>
hipError_t launch_decode_mode(DecodeParams p, hipStream_t stream) {
  if constexpr (MODE == kDecodeGeneric) {
    return launch_decode_mode<F, K, kDecode>(p, stream);
  } else {
    const int64_t lim = MODE == kReconstruct ? static_cast<int64_t>(p.bs)
                                             : last_room(p.bs, p.obj_len, K);
    p.tile_ch = 1;
    p.tiles = static_cast<uint32_t>(lim / kTile);
    p.edge_tiles = (p.bs + kTile - 1) / kTile - p.tiles;
    constexpr size_t lds = decode_lds_bytes<F, K>();
    const uint32_t edge_items =
        std::max(p.n_obj * p.edge_tiles, MODE == kReconstruct && p.headers ? p.n_obj : 0u);
    // inline_crc32 reconstruct: the same launch with its chunks' partials,
    // then the finishing pass (no A/B forms)
    const bool crc = MODE == kReconstruct && p.crc_lanes != nullptr;
    if (MODE != kReconstruct && p.crc_lanes != nullptr) return hipErrorInvalidValue;
    if (crc) {
      p.fused_edges = 1;
      auto kern = decode_kernel<F, K, MODE>;
      if constexpr (kAB && K == 10 && MODE == kReconstruct)
        if (ab_knob("ECAMD_REC_CRC_FREE", 0)) kern = decode_kernel<F, K, MODE, false, 0, true, true>;
      hipError_t e = launch_edges_apart(kern, p, lds + kCrcLaneBytes, p.n_obj * p.tiles, edge_items,
                                        stream, kReconstructPerCu, kDecodeXcd);
      if (e != hipSuccess) return e;
      return crc_finish(p.out, 0, p.out_stride, p.crc_part, 1, 0, p.crc_lanes, p.crc_finish_tables,
                        p.n_obj, 1, p.bs, crc_chunks(p.tiles, p.tile_ch), stream);
    }
    if constexpr (kAB) {
      const hipError_t e = launch_decode_ab<F, K, MODE>(p, stream, edge_items);
      if (e != hipErrorNotSupported) return e;
    }
    // the loader / consumer decode when the batch has a 16 KiB item per CU
    if constexpr (K >= kDmaMinK && F::kRows <= kRowsPerPass) {
      const int cus = device_cus();
      if constexpr (MODE == kDecode) {
        if (dma_batch(K, p.bs, p.obj_len, p.n_obj, cus, p.direct) && !ab_knob("ECAMD_DEC_STREAM", 0))
          return launch_decode_dma<F, K, 3, true, 4, 12>(p, stream);
      } else if constexpr (kAB) {
        // reconstruct keeps the stream kernel: the loader / consumer form ran
        // 330.8 us against 259.9 (k=10 m=4 256 x 4 MiB) and 462.9 against
        // 447.0 (isa_l_rs_cauchy 12+4 128 x 16 MiB; tools/ab_bench.py
        // --reconstruct, profiles/r04r_ab_reconstruct.txt)
        const int rd = ab_knob("ECAMD_REC_DMA", 0);
        if (dma_batch(K, p.bs, static_cast<uint64_t>(K) * p.bs, p.n_obj, cus) && rd != 0) {
          if constexpr (K == 10) {  // shapes of the loader / consumer reconstruct
            if (rd == 3) return launch_decode_dma<F, K, 3, true, 4, 12, 1, 1, kReconstruct>(p, stream);
            if (rd == 4) return launch_decode_dma<F, K, 3, true, 4, 16, 0, 1, kReconstruct>(p, stream);
            if (rd == 5) return launch_decode_dma<F, K, 4, true, 4, 12, 0, 1, kReconstruct>(p, stream);
            if (rd == 6) return launch_decode_dma<F, K, 3, true, 2, 12, 0, 1, kReconstruct>(p, stream);
            if (rd == 7) return launch_decode_dma<F, K, 3, true, 4, 8, 0, 2, kReconstruct>(p, stream);
          }
          return launch_decode_dma<F, K, 3, true, 4, 12, 0, 1, kReconstruct>(p, stream);
        }
      }
    }
    p.fused_edges = 1;
    return launch_edges_apart(decode_kernel<F, K, MODE>, p, lds, p.n_obj * p.tiles, edge_items,
                              stream, MODE == kReconstruct ? kReconstructPerCu : kDecodePerCu,
                              kDecodeXcd);
  }
}

}  // namespace
}  // namespace ecamd
