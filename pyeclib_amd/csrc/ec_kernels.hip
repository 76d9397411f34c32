// gfx950 region kernels for the rs_vand erasure code (see ec_kernels.hpp).
//
// Hot loop replaced: liberasurecode_rs_vand's region_dot_product /
// region_multiply / region_xor (upstream src/builtin/rs_vand/
// liberasurecode_rs_vand.c), which walks one 16-bit word at a time through a
// 64 K-entry log/antilog table on one CPU thread.
//
// Arithmetic.  Multiplication by a constant c is GF(2)-linear, so
//   c * x = T[0][x & 15] ^ T[1][(x>>4) & 15] ^ T[2][(x>>8) & 15] ^ T[3][x>>12]
// with T[q][v] = c * (v << 4q).  One u64 table entry packs the products for
// up to four output rows, so four 8-byte LDS reads per input symbol feed all
// four parities at once.  A 16-entry x 8-byte table is 128 B = 32 LDS banks:
// the 32 lanes of a ds_read_b64 lane group can never hit one bank with two
// different addresses, so every lookup is conflict-free whatever the data.
//
// Addressing.  Table [c][q][v] sits at byte 512c + 128q + 8v.  For one input
// dword x (two symbols, eight nibbles) we build
//   ylo = (x << 3) & 0x78787878               nibbles 0,2,4,6 scaled by 8
//   yhi = ((x >> 1) & 0x78787878) | 0x80..80  nibbles 1,3,5,7 scaled by 8,
//                                             +128 for odd q
// and one v_perm_b32 per lookup assembles {y.byte_b, (b & 1)} into the final
// LDS byte offset; the per-input 512c lands in the ds_read immediate because
// the input loop is unrolled over a compile-time k.
//
// Memory.  Each lane moves 16 B per input per step (global_load_dwordx4,
// 1 KiB contiguous per wave-instruction); inputs are read once from HBM and
// every output byte is written once.  Fragment payloads inside an object
// start at j*bs, which is only 2-byte aligned in general (bs = 2*ceil(L/2k));
// the loads rely on gfx9's unaligned-access mode for those inputs.
#include "ec_kernels.hpp"

#include <cstdlib>

namespace ecamd {
namespace {

constexpr uint32_t kSel[4] = {0x0C0C0400u, 0x0C0C0501u, 0x0C0C0402u, 0x0C0C0503u};

// LDS is addressed by raw byte offsets: these kernels declare no static
// __shared__ data, so the dynamic allocation (the nibble tables of the current
// coefficient matrix) starts at LDS address 0.  Going through an
// address_space(3) pointer made from the integer keeps hipcc from adding the
// symbol base to every lookup address (one VALU op per lookup), and the
// compile-time `tab` folds into the ds_read offset field.
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

// Accumulate input dword x (symbols s_lo, s_hi) times the input column whose
// tables start at LDS byte `tab`.  NW = 1: tables hold <= 2 rows, read the
// low dword only (ds_read_b32).
template <int NW>
__device__ __forceinline__ void mac_dword(uint32_t tab, uint32_t x, uint2& s_lo, uint2& s_hi) {
  const uint32_t ylo = (x << 3) & 0x78787878u;
  const uint32_t yhi = ((x >> 1) & 0x78787878u) | 0x80808080u;
  constexpr uint32_t kB = 0x00000100u;  // byte0 = 0, byte1 = 1
  const uint32_t a0 = __builtin_amdgcn_perm(kB, ylo, kSel[0]);
  const uint32_t a1 = __builtin_amdgcn_perm(kB, yhi, kSel[0]);
  const uint32_t a2 = __builtin_amdgcn_perm(kB, ylo, kSel[1]);
  const uint32_t a3 = __builtin_amdgcn_perm(kB, yhi, kSel[1]);
  const uint32_t a4 = __builtin_amdgcn_perm(kB, ylo, kSel[2]);
  const uint32_t a5 = __builtin_amdgcn_perm(kB, yhi, kSel[2]);
  const uint32_t a6 = __builtin_amdgcn_perm(kB, ylo, kSel[3]);
  const uint32_t a7 = __builtin_amdgcn_perm(kB, yhi, kSel[3]);
  if constexpr (NW == 2) {
    const uint2 e0 = lds_u64(a0, tab), e1 = lds_u64(a1, tab), e2 = lds_u64(a2, tab), e3 = lds_u64(a3, tab);
    const uint2 e4 = lds_u64(a4, tab), e5 = lds_u64(a5, tab), e6 = lds_u64(a6, tab), e7 = lds_u64(a7, tab);
    s_lo.x = xor3(xor3(s_lo.x, e0.x, e1.x), e2.x, e3.x);
    s_lo.y = xor3(xor3(s_lo.y, e0.y, e1.y), e2.y, e3.y);
    s_hi.x = xor3(xor3(s_hi.x, e4.x, e5.x), e6.x, e7.x);
    s_hi.y = xor3(xor3(s_hi.y, e4.y, e5.y), e6.y, e7.y);
  } else {
    s_lo.x = xor3(xor3(s_lo.x, lds_u32(a0, tab), lds_u32(a1, tab)), lds_u32(a2, tab), lds_u32(a3, tab));
    s_hi.x = xor3(xor3(s_hi.x, lds_u32(a4, tab), lds_u32(a5, tab)), lds_u32(a6, tab), lds_u32(a7, tab));
  }
}

template <int NW>
__device__ __forceinline__ void mac_chunk(uint32_t tab, const uint4& x, uint2 (&s)[8]) {
  // The scheduling barriers stop hipcc from hoisting every LDS lookup of the
  // unrolled input loop ahead of the XORs that consume them (2 VGPRs each).
  mac_dword<NW>(tab, x.x, s[0], s[1]);
  __builtin_amdgcn_sched_barrier(0);
  mac_dword<NW>(tab, x.y, s[2], s[3]);
  __builtin_amdgcn_sched_barrier(0);
  mac_dword<NW>(tab, x.z, s[4], s[5]);
  __builtin_amdgcn_sched_barrier(0);
  mac_dword<NW>(tab, x.w, s[6], s[7]);
  __builtin_amdgcn_sched_barrier(0);
}

// Materialise all accumulators here: otherwise hipcc sinks the row 2-3
// XOR chains into the (runtime-conditional) store blocks and keeps every
// looked-up table word live until then.
__device__ __forceinline__ void pin(uint2 (&s)[8]) {
#pragma unroll
  for (int i = 0; i < 8; ++i) asm volatile("" : "+v"(s[i].x), "+v"(s[i].y));
}

// Output row r of 8 accumulated symbols as a 16-byte chunk.
__device__ __forceinline__ uint32_t pack_row(const uint2& lo, const uint2& hi, int r) {
  const uint32_t a = (r < 2) ? lo.x : lo.y;
  const uint32_t b = (r < 2) ? hi.x : hi.y;
  return __builtin_amdgcn_perm(b, a, (r & 1) ? 0x07060302u : 0x05040100u);
}
__device__ __forceinline__ uint4 row_chunk(const uint2 (&s)[8], int r) {
  return make_uint4(pack_row(s[0], s[1], r), pack_row(s[2], s[3], r), pack_row(s[4], s[5], r),
                    pack_row(s[6], s[7], r));
}

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

__device__ __forceinline__ void load_tables(const uint64_t* src, uint32_t k) {
  auto* dst = reinterpret_cast<__attribute__((address_space(3))) v4u*>(static_cast<uintptr_t>(0));
  for (uint32_t i = threadIdx.x; i < k * (kTableBytesPerInput / 16); i += blockDim.x)
    dst[i] = reinterpret_cast<const v4u*>(src)[i];
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
// output, so the main kernels run them with no bounds checks, unrolled over
// K and with the next item's loads in flight (register double buffering).
// Tiles [first_edge, tiles) -- at most two per object: the payload tail and
// the tile reaching the zero padding / the end of the object -- run in a
// separate launch with a rolled, bounds-checked loop, so their code adds no
// registers to the main kernels.

__device__ __forceinline__ void tile_of(uint32_t w, uint32_t per_obj, uint32_t first,
                                        uint32_t& o, uint32_t& tile, uint32_t& t) {
  o = w / per_obj;
  tile = first + (w - o * per_obj);
  t = (tile * kThreadsPerBlock + threadIdx.x) << 4;
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
  for (int j = 0; j < K; ++j)
    x[j] = ld_stream(obj + static_cast<uint64_t>(j) * p.bs);
}

// One interior item with its inputs already in `cur`; first issues the loads
// of the workgroup's next item into `nxt`, so they are in flight while this
// item's table lookups run.
template <int K, int NW>
__device__ __forceinline__ void encode_item(const EncodeParams& p, uint32_t w, uint32_t items,
                                            uint4 (&cur)[K], uint4 (&nxt)[K]) {
  uint32_t o, tile, t;
  tile_of(w, p.first_edge, 0, o, tile, t);
  const uint32_t wn = w + gridDim.x;
  if (wn < items) {
    uint32_t on, tn, ttn;
    tile_of(wn, p.first_edge, 0, on, tn, ttn);
    encode_load<K>(p, on, ttn, nxt);
  }
  if (tile == 0) encode_headers(p, o, K);
  uint2 s[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) s[i] = make_uint2(0, 0);
#pragma unroll
  for (int j = 0; j < K; ++j) mac_chunk<NW>(j * kTableBytesPerInput, cur[j], s);
  pin(s);

  uint8_t* par = p.parity + static_cast<uint64_t>(o) * p.stripe_stride + p.row0 * p.frag_stride +
                 kHeaderBytes + t;
#pragma unroll
  for (int r = 0; r < kRowsPerPass; ++r)
    if (r < static_cast<int>(p.nrows))
      st_stream(par + r * p.frag_stride, row_chunk(s, r));

  if (p.data != nullptr && p.row0 == 0) {
    uint8_t* dat = p.data + static_cast<uint64_t>(o) * p.stripe_stride + kHeaderBytes + t;
#pragma unroll
    for (int j = 0; j < K; ++j) st_stream(dat + j * p.frag_stride, cur[j]);
  }
}

template <int K, int NW>
__global__ void __launch_bounds__(kThreadsPerBlock) encode_kernel(EncodeParams p) {
  load_tables(p.tables, K);
  __syncthreads();
  const uint32_t items = p.n_obj * p.first_edge;
  uint4 xa[K], xb[K];
  uint32_t w = blockIdx.x;
  if (w < items) {
    uint32_t o, tile, t;
    tile_of(w, p.first_edge, 0, o, tile, t);
    encode_load<K>(p, o, t, xa);
  }
  while (w < items) {
    encode_item<K, NW>(p, w, items, xa, xb);
    w += gridDim.x;
    if (w >= items) break;
    encode_item<K, NW>(p, w, items, xb, xa);
    w += gridDim.x;
  }
}

// Edge tiles: payload tail (t + 16 > bs) and chunks reaching the zero padding
// past obj_len (liberasurecode's prepare_fragments_for_encode zero-fills).
template <int NW>
__global__ void __launch_bounds__(kThreadsPerBlock) encode_edge_kernel(EncodeParams p) {
  load_tables(p.tables, p.k);
  __syncthreads();
  const uint32_t n_edge = p.tiles - p.first_edge;
  const uint32_t items = p.n_obj * n_edge;
  for (uint32_t w = blockIdx.x; w < items; w += gridDim.x) {
    uint32_t o, tile, t;
    tile_of(w, n_edge, p.first_edge, o, tile, t);
    if (tile == 0) encode_headers(p, o, p.k);
    if (t >= p.bs) continue;
    const uint8_t* obj = p.objs + static_cast<uint64_t>(o) * p.obj_stride;
    const int64_t rem = static_cast<int64_t>(p.bs) - t;
    uint2 s[8];
    for (int i = 0; i < 8; ++i) s[i] = make_uint2(0, 0);
#pragma unroll 1
    for (uint32_t j = 0; j < p.k; ++j) {
      const uint4 x = load_clamped(obj, static_cast<uint64_t>(j) * p.bs + t, p.obj_len);
      mac_chunk<NW>(j * kTableBytesPerInput, x, s);
      if (p.data != nullptr && p.row0 == 0)
        store_partial(p.data + static_cast<uint64_t>(o) * p.stripe_stride + j * p.frag_stride +
                          kHeaderBytes + t,
                      x, rem);
    }
    pin(s);
    uint8_t* par = p.parity + static_cast<uint64_t>(o) * p.stripe_stride +
                   p.row0 * p.frag_stride + kHeaderBytes + t;
    for (uint32_t r = 0; r < p.nrows; ++r)
      store_partial(par + r * p.frag_stride, row_chunk(s, r), rem);
  }
}

// ---------------- decode / reconstruct ----------------

// (Re)load the table set of object o's descriptor if it differs from the one
// in LDS.  Workgroup-uniform; contains barriers.
__device__ __forceinline__ void ensure_tables(const DecodeParams& p, const ObjDesc& d,
                                              uint32_t& cur_table) {
  if (d.n_out == 0 || d.table == cur_table) return;
  __syncthreads();
  load_tables(p.tables + static_cast<uint64_t>(d.table) * p.k * (kTableBytesPerInput / 8), p.k);
  __syncthreads();
  cur_table = d.table;
}

__device__ __forceinline__ void reconstruct_header(const DecodeParams& p, const ObjDesc& d,
                                                   uint8_t* out) {
  if (threadIdx.x < 5)
    reinterpret_cast<uint4*>(out)[threadIdx.x] = reinterpret_cast<const uint4*>(
        p.headers + static_cast<uint64_t>(d.header) * kHeaderBytes)[threadIdx.x];
}

// Inputs are read through the cache (not nontemporal): decode reads the
// surviving data fragments' lines again for the line-aligned copies below.
template <int K>
__device__ __forceinline__ void decode_load(const DecodeParams& p, uint32_t o, uint32_t t,
                                            uint4 (&x)[K]) {
  const ObjDesc& d = p.desc[o];
  const uint8_t* frags = p.frags + static_cast<uint64_t>(o) * p.stripe_stride + kHeaderBytes + t;
#pragma unroll
  for (int j = 0; j < K; ++j) {
    const uint8_t* a = frags + d.in_idx[j] * p.frag_stride;
    x[j] = *reinterpret_cast<const uint4*>(a);
  }
}

// Decode output alignment.  Data fragment j of an object starts at byte
// j*bs, and bs = 2*ceil(L/2k) leaves it at an arbitrary even offset from a
// 128-B line, while lanes are aligned to the fragment payloads they read.
// A wave's 1 KiB store then covers 9 lines, 2 of them partial, and partial
// nontemporal line writes cost ~20% of the decode (tools/microbench.hip
// "dstream nt" 450 us vs "dshift nt" 395 us).  Staging in LDS (4 KiB per
// output per tile, barriers) and in-register 16-B realignment (DPP) were
// measured slower.  What works: the copies of surviving data fragments are
// re-read at the object's line phase -- lane chunk t - delta_j, so every
// wave's 1 KiB of copy stores is line-aligned -- and the re-read hits L2
// because the first read was a cached load ("mix c shift" 400 us).  Rebuilt
// rows (on average e*k/(k+m) of the k outputs) keep their natural offsets.
// One interior decode / reconstruct item with inputs in `cur`; prefetches
// the workgroup's next item (w + step) into `nxt`.  Items are grid-strided
// (the chip works on a few objects at a time: better DRAM locality than
// contiguous per-workgroup ranges, measured 513 -> 479 us at k=10 m=4), so
// the LDS tables are usually reloaded per item (5 KiB from L2).
template <int K, int NW>
__device__ __forceinline__ void decode_item(const DecodeParams& p, uint32_t w, uint32_t step,
                                            uint32_t end, uint32_t& cur_table, uint4 (&cur)[K],
                                            uint4 (&nxt)[K]) {
  const uint32_t bs = p.bs;
  uint32_t o, tile, t;
  tile_of(w, p.first_edge, 0, o, tile, t);
  if (w + step < end) {
    uint32_t on, tn, ttn;
    tile_of(w + step, p.first_edge, 0, on, tn, ttn);
    decode_load<K>(p, on, ttn, nxt);
  }
  const ObjDesc& d = p.desc[o];
  ensure_tables(p, d, cur_table);
  uint8_t* out = p.out + static_cast<uint64_t>(o) * p.out_stride;
  if (p.reconstruct && tile == 0) reconstruct_header(p, d, out);
  const uint32_t n_out = d.n_out;

  uint2 s[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) s[i] = make_uint2(0, 0);
  if (n_out != 0) {
#pragma unroll
    for (int j = 0; j < K; ++j) mac_chunk<NW>(j * kTableBytesPerInput, cur[j], s);
  }
  pin(s);

#pragma unroll
  for (int r = 0; r < kRowsPerPass; ++r) {
    if (r >= static_cast<int>(n_out)) break;
    uint8_t* dst = p.reconstruct ? out + kHeaderBytes + t
                                 : out + static_cast<uint64_t>(d.out_idx[r]) * bs + t;
    st_stream(dst, row_chunk(s, r));
  }
  if (d.copy_inputs) {
#pragma unroll
    for (int j = 0; j < K; ++j) {
      const uint32_t idx = d.in_idx[j];
      if (idx < K) st_stream(out + static_cast<uint64_t>(idx) * bs + t, cur[j]);
    }
  }
}

template <int K, int NW>
__global__ void __launch_bounds__(kThreadsPerBlock) decode_kernel(DecodeParams p) {
  const uint32_t end = p.n_obj * p.first_edge;
  const uint32_t begin = blockIdx.x, step = gridDim.x;
  uint32_t cur_table = 0xFFFFFFFFu;
  uint4 xa[K], xb[K];
  uint32_t w = begin;
  if (w < end) {
    uint32_t o, tile, t;
    tile_of(w, p.first_edge, 0, o, tile, t);
    decode_load<K>(p, o, t, xa);
  }
  while (w < end) {
    decode_item<K, NW>(p, w, step, end, cur_table, xa, xb);
    w += step;
    if (w >= end) break;
    decode_item<K, NW>(p, w, step, end, cur_table, xb, xa);
    w += step;
  }
}

// Interior decode with line-aligned copies (p.copy_shift).  No cross-item
// prefetch here: the shifted re-reads must follow the aligned reads closely
// to hit L2 (with a one-item prefetch distance they missed: 544 us).
template <int K, int NW>
__global__ void __launch_bounds__(kThreadsPerBlock) decode_shift_kernel(DecodeParams p) {
  const uint32_t end = p.n_obj * p.first_edge;
  uint32_t cur_table = 0xFFFFFFFFu;
  for (uint32_t w = blockIdx.x; w < end; w += gridDim.x) {
    uint32_t o, tile, t;
    tile_of(w, p.first_edge, 0, o, tile, t);
    const ObjDesc& d = p.desc[o];
    const uint8_t* fb = p.frags + static_cast<uint64_t>(o) * p.stripe_stride + kHeaderBytes;
    uint8_t* out = p.out + static_cast<uint64_t>(o) * p.out_stride;
    uint4 x[K], c[K];
    int32_t src[K];
#pragma unroll
    for (int j = 0; j < K; ++j)
      x[j] = *reinterpret_cast<const uint4*>(fb + d.in_idx[j] * p.frag_stride + t);
#pragma unroll
    for (int j = 0; j < K; ++j) {
      const uint32_t idx = d.in_idx[j];
      src[j] = -16;
      if (idx >= K || !d.copy_inputs) continue;
      const uint32_t delta = static_cast<uint32_t>(
          reinterpret_cast<uintptr_t>(out + static_cast<uint64_t>(idx) * p.bs) & 127u);
      src[j] = static_cast<int32_t>(t) - static_cast<int32_t>(delta);
      if (src[j] > -16)
        c[j] = *reinterpret_cast<const uint4*>(fb + idx * p.frag_stride + src[j]);
    }
    ensure_tables(p, d, cur_table);
    const uint32_t n_out = d.n_out;
    uint2 s[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) s[i] = make_uint2(0, 0);
    if (n_out != 0) {
#pragma unroll
      for (int j = 0; j < K; ++j) mac_chunk<NW>(j * kTableBytesPerInput, x[j], s);
    }
    pin(s);
#pragma unroll
    for (int r = 0; r < kRowsPerPass; ++r) {
      if (r >= static_cast<int>(n_out)) break;
      st_stream(out + static_cast<uint64_t>(d.out_idx[r]) * p.bs + t, row_chunk(s, r));
    }
#pragma unroll
    for (int j = 0; j < K; ++j) {
      if (src[j] <= -16) continue;  // not a data fragment, or nothing of this chunk is ours
      uint8_t* dst0 = out + static_cast<uint64_t>(d.in_idx[j]) * p.bs;
      if (src[j] >= 0) {
        st_stream(dst0 + src[j], c[j]);
      } else {  // the fragment's first chunk: only its payload bytes
        const uint32_t wv[4] = {c[j].x, c[j].y, c[j].z, c[j].w};
        for (int i = -src[j]; i < 16; ++i)
          dst0[src[j] + i] = static_cast<uint8_t>(wv[i >> 2] >> (8 * (i & 3)));
      }
    }
  }
}

// Edge tiles of decode / reconstruct: payload tail, and (decode) outputs
// that cross the end of the object.
template <int NW>
__global__ void __launch_bounds__(kThreadsPerBlock) decode_edge_kernel(DecodeParams p) {
  const uint32_t n_edge = p.tiles - p.first_edge;
  const uint32_t items = p.n_obj * n_edge;
  const uint32_t per = (items + gridDim.x - 1) / gridDim.x;
  const uint32_t begin = blockIdx.x * per;
  const uint32_t end = min(items, begin + per);
  uint32_t cur_table = 0xFFFFFFFFu;
  for (uint32_t w = begin; w < end; ++w) {
    uint32_t o, tile, t;
    tile_of(w, n_edge, p.first_edge, o, tile, t);
    const ObjDesc& d = p.desc[o];
    ensure_tables(p, d, cur_table);
    uint8_t* out = p.out + static_cast<uint64_t>(o) * p.out_stride;
    if (p.reconstruct && tile == 0) reconstruct_header(p, d, out);
    if (p.copy_shift && d.copy_inputs && tile == p.first_edge && threadIdx.x < 8) {
      // the interior's shifted copies stop up to 127 B short of its end
      const uint32_t te = p.first_edge * kThreadsPerBlock * 16 - 128 + 16 * threadIdx.x;
      const uint8_t* fb = p.frags + static_cast<uint64_t>(o) * p.stripe_stride + kHeaderBytes + te;
      for (uint32_t j = 0; j < p.k; ++j) {
        const uint32_t idx = d.in_idx[j];
        if (idx >= p.k) continue;
        const int64_t n = object_bytes(idx, p.bs, te, p.obj_len);
        if (n > 0)
          store_partial(out + static_cast<uint64_t>(idx) * p.bs + te,
                        *reinterpret_cast<const uint4*>(fb + idx * p.frag_stride), n);
      }
    }
    if (t >= p.bs) continue;
    const uint8_t* frags =
        p.frags + static_cast<uint64_t>(o) * p.stripe_stride + kHeaderBytes + t;
    uint2 s[8];
    for (int i = 0; i < 8; ++i) s[i] = make_uint2(0, 0);
#pragma unroll 1
    for (uint32_t j = 0; j < p.k; ++j) {
      const uint4 x = *reinterpret_cast<const uint4*>(frags + d.in_idx[j] * p.frag_stride);
      const uint32_t idx = d.in_idx[j];
      if (d.copy_inputs && idx < p.k) {
        const int64_t n = object_bytes(idx, p.bs, t, p.obj_len);
        if (n > 0) store_partial(out + static_cast<uint64_t>(idx) * p.bs + t, x, n);
      }
      if (d.n_out) mac_chunk<NW>(j * kTableBytesPerInput, x, s);
    }
    pin(s);
    for (uint32_t r = 0; r < d.n_out; ++r) {
      if (p.reconstruct) {
        store_partial(out + kHeaderBytes + t, row_chunk(s, r), static_cast<int64_t>(p.bs) - t);
      } else {
        const uint32_t idx = d.out_idx[r];
        const int64_t n = object_bytes(idx, p.bs, t, p.obj_len);
        if (n > 0) store_partial(out + static_cast<uint64_t>(idx) * p.bs + t, row_chunk(s, r), n);
      }
    }
  }
}

int grid_for(const void* kernel, size_t lds_bytes, uint32_t items) {
  int dev = 0, cus = 256, per_cu = 4;
  if (hipGetDevice(&dev) == hipSuccess) {
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    int b = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&b, kernel, kThreadsPerBlock, lds_bytes) ==
            hipSuccess &&
        b > 0)
      per_cu = b;
  }
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
template <typename Kern>
bool lds_starts_at_zero(Kern kern) {
  static const bool ok = [kern] {
    hipFuncAttributes attr{};
    return hipFuncGetAttributes(&attr, reinterpret_cast<const void*>(kern)) == hipSuccess &&
           attr.sharedSizeBytes == 0;
  }();
  return ok;
}

template <typename Kern, typename Params>
hipError_t launch(Kern kern, const Params& p, size_t lds, uint32_t items, hipStream_t stream) {
  if (items == 0) return hipSuccess;
  if (!lds_starts_at_zero(kern)) return hipErrorInvalidKernelFile;
  const int grid = grid_for(reinterpret_cast<const void*>(kern), lds, items);
  hipLaunchKernelGGL(kern, dim3(grid), dim3(kThreadsPerBlock), lds, stream, p);
  return hipGetLastError();
}

template <int K, int NW>
hipError_t launch_encode_k(EncodeParams p, hipStream_t stream) {
  const size_t lds = K * kTableBytesPerInput;
  split_tiles(p.bs, p.obj_len, K, false, p.tiles, p.first_edge);
  const hipError_t e = launch(encode_kernel<K, NW>, p, lds, p.n_obj * p.first_edge, stream);
  if (e != hipSuccess) return e;
  return launch(encode_edge_kernel<NW>, p, lds, p.n_obj * (p.tiles - p.first_edge), stream);
}

template <int K, int NW>
hipError_t launch_decode_k(DecodeParams p, hipStream_t stream) {
  const size_t lds_tables = K * kTableBytesPerInput;
  split_tiles(p.bs, p.obj_len, K, p.reconstruct != 0, p.tiles, p.first_edge);
  // Shifted interior copies leave up to 127 B before the interior's end to
  // the first edge tile, so decode always has one (and first_edge >= 1
  // keeps its start offset non-negative).
  if (!p.reconstruct && p.first_edge == p.tiles && p.first_edge > 0) --p.first_edge;
  p.copy_shift = !p.reconstruct && p.first_edge > 0 && std::getenv("ECAMD_DSHIFT");
  const uint32_t n = p.n_obj * p.first_edge;
  const hipError_t e = p.copy_shift ? launch(decode_shift_kernel<K, NW>, p, lds_tables, n, stream)
                                    : launch(decode_kernel<K, NW>, p, lds_tables, n, stream);
  if (e != hipSuccess) return e;
  return launch(decode_edge_kernel<NW>, p, lds_tables, p.n_obj * (p.tiles - p.first_edge), stream);
}

template <int K>
hipError_t dispatch_encode(const EncodeParams& p, hipStream_t s) {
  return p.nrows <= 2 ? launch_encode_k<K, 1>(p, s) : launch_encode_k<K, 2>(p, s);
}

template <int K>
hipError_t dispatch_decode(const DecodeParams& p, uint32_t max_rows, hipStream_t s) {
  return max_rows <= 2 ? launch_decode_k<K, 1>(p, s) : launch_decode_k<K, 2>(p, s);
}

#define ECAMD_K_CASES(X) \
  X(1) X(2) X(3) X(4) X(5) X(6) X(7) X(8) X(9) X(10) X(11) X(12) X(13) X(14) X(15) X(16) \
  X(17) X(18) X(19) X(20) X(21) X(22) X(23) X(24) X(25) X(26) X(27) X(28) X(29) X(30) X(31)

}  // namespace

hipError_t launch_encode(const EncodeParams& p, hipStream_t stream) {
  switch (p.k) {
#define X(K) \
  case K:    \
    return dispatch_encode<K>(p, stream);
    ECAMD_K_CASES(X)
#undef X
    default:
      return hipErrorInvalidValue;
  }
}

hipError_t launch_decode(const DecodeParams& p, hipStream_t stream) {
  // Every object's n_out is <= 4; the row count only selects the table word width.
  const uint32_t max_rows = p.m < kRowsPerPass ? p.m : kRowsPerPass;
  switch (p.k) {
#define X(K) \
  case K:    \
    return dispatch_decode<K>(p, p.reconstruct ? 1 : max_rows, stream);
    ECAMD_K_CASES(X)
#undef X
    default:
      return hipErrorInvalidValue;
  }
}

}  // namespace ecamd
