// Memory-pattern ceilings for the encode / decode streams on MI355X (dev tool,
// not the product; `make -C tools membench`).  No GF arithmetic: the inputs
// are XORed, so each kernel shows what the HBM side of an access pattern
// allows, beside a plain copy and a read-only sweep of the same bytes.
//
// Workload shape = bench.py's: 256 objects x 4 MiB (obj_stride 4 MiB),
// k = 10, m = 4, fragment payloads at 128-B-aligned fragment strides.
//   enc : 10 slices read at j*bs inside the object, 4 parity rows written
//   dec : 10 fragment payloads read, 10 object slices written at j*bs
// bs is a runtime argument, so bs = 419432 (the real, 8-mod-16 slices) and
// bs = 419456 (128-B-aligned slices) isolate the misalignment cost.
//
// Every shape is checked on the host against the buffers it touches before
// its first launch (round 2's compact-layout probe overran the fragment
// buffer by 2.85 MB: its stripes were sized for a different object count).
//
//   ./membench [reps] [sections]     sections: any of "base enc ceil wpb runs dec alt" (default all)
//   MB_RANDOM=1: random object bytes instead of a constant fill
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <algorithm>
#include <vector>

#define CHECK(x)                                                               \
  do {                                                                         \
    hipError_t e_ = (x);                                                       \
    if (e_ != hipSuccess) {                                                    \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      std::exit(1);                                                            \
    }                                                                          \
  } while (0)

namespace {

typedef unsigned int v4u __attribute__((ext_vector_type(4)));

template <bool NT>
__device__ __forceinline__ v4u ld(const uint8_t* p) {
  if constexpr (NT) return __builtin_nontemporal_load(reinterpret_cast<const v4u*>(p));
  return *reinterpret_cast<const v4u*>(p);
}
template <bool NT>
__device__ __forceinline__ void st(uint8_t* p, v4u v) {
  if constexpr (NT)
    __builtin_nontemporal_store(v, reinterpret_cast<v4u*>(p));
  else
    *reinterpret_cast<v4u*>(p) = v;
}

struct Shape {
  uint8_t* objs;
  uint8_t* frags;
  uint32_t bs, n_obj, tiles;
  uint64_t obj_stride, frag_stride, stripe_stride;
};

constexpr int K = 10, M = 4;

// Host-side bounds check of one shape against its buffers: tile span T bytes
// of payload positions per item (4096 * CH).  Exits on a violation.
struct Bufs {
  uint8_t *objs_base, *out_base, *frags_base;
  uint64_t obj_bytes, frag_bytes;
};
Bufs g_bufs;
void check_shape(const char* name, const Shape& s, uint64_t span, bool in_out = false) {
  const uint64_t obj_end = (s.objs - (in_out ? g_bufs.out_base : g_bufs.objs_base)) +
                           uint64_t(s.n_obj - 1) * s.obj_stride + uint64_t(K - 1) * s.bs +
                           uint64_t(s.tiles) * span;
  const uint64_t frag_end = (s.frags - g_bufs.frags_base) + uint64_t(s.n_obj - 1) * s.stripe_stride +
                            uint64_t(K + M - 1) * s.frag_stride + 80 + uint64_t(s.tiles) * span;
  const bool obj_ok = obj_end <= g_bufs.obj_bytes;
  const bool frag_ok = frag_end <= g_bufs.frag_bytes;
  if (!obj_ok || !frag_ok || uint64_t(s.tiles) * span > s.bs + 0ull) {
    std::fprintf(stderr, "shape %s out of bounds: obj end %llu / %llu, frag end %llu / %llu, "
                 "tile span %llu vs bs %u\n", name, (unsigned long long)obj_end,
                 (unsigned long long)g_bufs.obj_bytes, (unsigned long long)frag_end,
                 (unsigned long long)g_bufs.frag_bytes,
                 (unsigned long long)(uint64_t(s.tiles) * span), s.bs);
    std::exit(2);
  }
}

// Item order (item w = object w / tiles, tile w % tiles).
//   0 PLAIN: grid-stride over the item list.
//   1 XCD: the list cut into 8 contiguous ranges, range x walked by the blocks
//     with b % 8 == x (blocks are dealt round-robin over the 8 XCDs).
//   2 OBJECT: P = grid / n_obj blocks per object; block b takes object
//     b % n_obj, tiles c, c + P, c + 2P, ... (c = b / n_obj): every object
//     in flight at once, each block's items one fixed stride apart inside
//     one object (what a per-thread Horner CRC over the parity needs).
//   3 RANGE: block b takes the contiguous items [n b / G, n (b+1) / G)
//     (the fused-CRC encode's order).
struct Order {
  uint32_t begin, end, step;
};
template <int ORD>
__device__ __forceinline__ Order order(uint32_t items, uint32_t tiles = 1) {
  if constexpr (ORD == 0) return {blockIdx.x, items, gridDim.x};
  if constexpr (ORD == 1) {
    const uint32_t x = blockIdx.x & 7u;
    const uint32_t lo = uint32_t(uint64_t(items) * x / 8), hi = uint32_t(uint64_t(items) * (x + 1) / 8);
    return {lo + (blockIdx.x >> 3), hi, gridDim.x >> 3};
  }
  if constexpr (ORD == 2) {
    const uint32_t n_obj = items / tiles, per = gridDim.x / n_obj;  // host: grid % n_obj == 0
    const uint32_t o = blockIdx.x % n_obj, c = blockIdx.x / n_obj;
    return {o * tiles + c, o * tiles + tiles, per};
  }
  return {uint32_t(uint64_t(items) * blockIdx.x / gridDim.x),
          uint32_t(uint64_t(items) * (blockIdx.x + 1) / gridDim.x), 1u};
}

// ---- plain copy / read sweeps (grid-stride, 16 B per lane, CH units per lane
// per step, each unit one contiguous 1 KiB wave access) ----
template <int CH, bool NT>
__global__ void __launch_bounds__(256) copy_kernel(const uint8_t* src, uint8_t* dst, uint64_t n) {
  const uint64_t step = uint64_t(gridDim.x) * 256 * 16 * CH;
  const uint32_t wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  for (uint64_t b = uint64_t(blockIdx.x) * 256 * 16 * CH + wave * 1024 * CH + lane * 16; b < n;
       b += step) {
    v4u v[CH];
#pragma unroll
    for (int c = 0; c < CH; ++c) v[c] = ld<NT>(src + b + 1024 * c);
#pragma unroll
    for (int c = 0; c < CH; ++c) st<NT>(dst + b + 1024 * c, v[c]);
  }
}
template <int CH, bool NT>
__global__ void __launch_bounds__(256) read_kernel(const uint8_t* src, uint64_t n, uint32_t* sink) {
  const uint64_t step = uint64_t(gridDim.x) * 256 * 16 * CH;
  const uint32_t wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  uint32_t acc = 0;
  for (uint64_t b = uint64_t(blockIdx.x) * 256 * 16 * CH + wave * 1024 * CH + lane * 16; b < n;
       b += step) {
#pragma unroll
    for (int c = 0; c < CH; ++c) {
      const v4u v = ld<NT>(src + b + 1024 * c);
      acc ^= v.x ^ v.y ^ v.z ^ v.w;
    }
  }
  if (acc == 0x12345678u) sink[0] = acc;
}
template <int CH, bool NT>
__global__ void __launch_bounds__(256) write_kernel(uint8_t* dst, uint64_t n) {
  const uint64_t step = uint64_t(gridDim.x) * 256 * 16 * CH;
  const uint32_t wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  for (uint64_t b = uint64_t(blockIdx.x) * 256 * 16 * CH + wave * 1024 * CH + lane * 16; b < n;
       b += step) {
#pragma unroll
    for (int c = 0; c < CH; ++c) st<NT>(dst + b + 1024 * c, v4u{uint32_t(b), 1u, 2u, 3u});
  }
}

// ---- encode stream: item = (object, tile of 4096*CH payload positions);
// wave w of the block takes [x, x + 1024*CH) with x = tile*4096*CH + w*1024*CH.
// PF: the block's next item is loaded before this one is consumed.
// SROW: parity stored row-major (each row's CH KiB back to back: a store
// burst of CH KiB per row) instead of chunk-major. ----
template <int CH, bool NTL>
__device__ __forceinline__ void enc_load(const Shape& s, uint32_t w, v4u (&v)[K][CH]) {
  const uint32_t o = w / s.tiles, t = w - o * s.tiles;
  const uint32_t x = t * 4096 * CH + (threadIdx.x >> 6) * 1024 * CH + (threadIdx.x & 63) * 16;
  const uint8_t* src = s.objs + o * s.obj_stride + x;
#pragma unroll
  for (int j = 0; j < K; ++j)
#pragma unroll
    for (int c = 0; c < CH; ++c) v[j][c] = ld<NTL>(src + uint64_t(j) * s.bs + 1024 * c);
}
template <int CH, bool NTS, bool SROW>
__device__ __forceinline__ void enc_store(const Shape& s, uint32_t w, const v4u (&v)[K][CH]) {
  const uint32_t o = w / s.tiles, t = w - o * s.tiles;
  const uint32_t x = t * 4096 * CH + (threadIdx.x >> 6) * 1024 * CH + (threadIdx.x & 63) * 16;
  uint8_t* dst = s.frags + o * s.stripe_stride + K * s.frag_stride + 80 + x;
  v4u a[CH];
#pragma unroll
  for (int c = 0; c < CH; ++c) {
    a[c] = v[0][c];
#pragma unroll
    for (int j = 1; j < K; ++j) a[c] ^= v[j][c];
  }
  if constexpr (SROW) {
#pragma unroll
    for (int r = 0; r < M; ++r)
#pragma unroll
      for (int c = 0; c < CH; ++c) st<NTS>(dst + r * s.frag_stride + 1024 * c, a[c] + uint32_t(r));
  } else {
#pragma unroll
    for (int c = 0; c < CH; ++c)
#pragma unroll
      for (int r = 0; r < M; ++r) st<NTS>(dst + r * s.frag_stride + 1024 * c, a[c] + uint32_t(r));
  }
}
// MODE 1: loads only (XOR folded into a never-taken store), MODE 2: stores only
template <bool NTL, int MODE>
__global__ void __launch_bounds__(256) enc_half_kernel(Shape s, uint32_t* sink) {
  const uint32_t items = s.n_obj * s.tiles;
  uint32_t acc = 0;
  for (uint32_t w = blockIdx.x; w < items; w += gridDim.x) {
    v4u v[K][1];
    if constexpr (MODE == 1) {
      enc_load<1, NTL>(s, w, v);
#pragma unroll
      for (int j = 0; j < K; ++j) acc ^= v[j][0].x ^ v[j][0].y ^ v[j][0].z ^ v[j][0].w;
    } else {
#pragma unroll
      for (int j = 0; j < K; ++j) v[j][0] = v4u{w, uint32_t(j), 0u, 1u};
      enc_store<1, true, false>(s, w, v);
    }
  }
  if (acc == 0x12345678u) sink[0] = acc;
}

template <int CH, bool NTL, bool NTS, bool PF, int ORD = 0, bool SROW = false>
__global__ void __launch_bounds__(256) enc_kernel(Shape s) {
  const Order r = order<ORD>(s.n_obj * s.tiles, s.tiles);
  if constexpr (!PF) {
    for (uint32_t w = r.begin; w < r.end; w += r.step) {
      v4u v[K][CH];
      enc_load<CH, NTL>(s, w, v);
      enc_store<CH, NTS, SROW>(s, w, v);
    }
  } else {
    uint32_t w = r.begin;
    if (w >= r.end) return;
    v4u a[K][CH], b[K][CH];
    enc_load<CH, NTL>(s, w, a);
    while (true) {
      uint32_t wn = w + r.step < r.end ? w + r.step : w;
      enc_load<CH, NTL>(s, wn, b);
      enc_store<CH, NTS, SROW>(s, w, a);
      if (wn == w) break;
      w = wn;
      wn = w + r.step < r.end ? w + r.step : w;
      enc_load<CH, NTL>(s, wn, a);
      enc_store<CH, NTS, SROW>(s, w, b);
      if (wn == w) break;
      w = wn;
    }
  }
}

// The product kernel's stream shape without the lookups: NB input chunks in
// flight per wave, refilled as each is consumed, running over into the
// block's next item (ec_kernels_impl.hpp encode_interior).  CH chunks per
// wave per item, consumed chunk-major (all K inputs of chunk c, then c + 1).
template <int CH, int NB, int ORD>
__global__ void __launch_bounds__(256) enc_stream_kernel(Shape s) {
  constexpr int SL = K * CH;  // slots per item
  const Order r = order<ORD>(s.n_obj * s.tiles, s.tiles);
  uint32_t w = r.begin;
  if (w >= r.end) return;
  const uint32_t lanex = (threadIdx.x >> 6) * 1024 * CH + (threadIdx.x & 63) * 16;
  auto src_of = [&](uint32_t it, int slot) {
    const uint32_t o = it / s.tiles, t = it - o * s.tiles;
    const int c = slot / K, j = slot % K;
    return s.objs + o * s.obj_stride + uint64_t(j) * s.bs + t * 4096 * CH + lanex + 1024 * c;
  };
  v4u buf[NB];
#pragma unroll
  for (int i = 0; i < NB; ++i) buf[i] = ld<false>(src_of(w, i));
  while (true) {
    const uint32_t wn = w + r.step < r.end ? w + r.step : w;
    const uint32_t o = w / s.tiles, t = w - o * s.tiles;
    uint8_t* dst = s.frags + o * s.stripe_stride + K * s.frag_stride + 80 + t * 4096 * CH + lanex;
    v4u acc = v4u{0u, 0u, 0u, 0u};
#pragma unroll
    for (int i = 0; i < SL; ++i) {
      acc ^= buf[i % NB];
      if (i + NB < SL)
        buf[i % NB] = ld<false>(src_of(w, i + NB));
      else if (wn != w)
        buf[i % NB] = ld<false>(src_of(wn, i + NB - SL));
      if (i % K == K - 1) {
#pragma unroll
        for (int q = 0; q < M; ++q) st<true>(dst + q * s.frag_stride + 1024 * (i / K), acc + uint32_t(q));
        acc = v4u{0u, 0u, 0u, 0u};
      }
    }
    if (wn == w) break;
    w = wn;
  }
}

// The same stream through buffer instructions, as the product kernels issue
// them (ec_kernels_impl.hpp: one wave-uniform descriptor per object, the
// lane's 16*lane in voffset, every per-input / per-row offset in soffset).
// NTL: nontemporal loads; ST_NOP: the product's one wait state after each
// 16-B store.
typedef __amdgpu_buffer_rsrc_t Rsrc;
__device__ __forceinline__ Rsrc mk_rsrc(const void* base, int records = -1) {
  const uint64_t a = reinterpret_cast<uint64_t>(base);
  const uint32_t lo = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(a));
  const uint32_t hi = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(a >> 32));
  const int n = static_cast<int>(__builtin_amdgcn_readfirstlane(static_cast<uint32_t>(records)));
  return __builtin_amdgcn_make_buffer_rsrc(
      reinterpret_cast<void*>((static_cast<uint64_t>(hi) << 32) | lo), 0, n, 0x00020000);
}
template <int CH, int NB, int ORD, bool NTL, bool ST_NOP, int OCC = 1>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(OCC, 8)))
    enc_stream_buf_kernel(Shape s) {
  constexpr int SL = K * CH;  // slots per item
  const Order r = order<ORD>(s.n_obj * s.tiles, s.tiles);
  uint32_t w = r.begin;
  if (w >= r.end) return;
  const uint32_t lane16 = (threadIdx.x & 63) * 16;
  const uint32_t wx = __builtin_amdgcn_readfirstlane((threadIdx.x >> 6) * 1024 * CH);
  auto item_x = [&](uint32_t it) { return (it - it / s.tiles * s.tiles) * 4096 * CH + wx; };
  auto obj_of = [&](uint32_t it, int rec) { return mk_rsrc(s.objs + (it / s.tiles) * s.obj_stride, rec); };
  Rsrc cur = obj_of(w, -1);
  uint32_t x = item_x(w);
  v4u buf[NB];
#pragma unroll
  for (int i = 0; i < NB; ++i)
    buf[i] = __builtin_amdgcn_raw_buffer_load_b128(cur, lane16, (i % K) * s.bs + x + 1024 * (i / K),
                                                  NTL ? 2 : 0);
  while (true) {
    const uint32_t wn = w + r.step < r.end ? w + r.step : w;
    const Rsrc nxt = obj_of(wn, wn == w ? 0 : -1);
    const uint32_t xn = item_x(wn);
    const Rsrc par = mk_rsrc(s.frags + (w / s.tiles) * s.stripe_stride);
    v4u acc = v4u{0u, 0u, 0u, 0u};
#pragma unroll
    for (int i = 0; i < SL; ++i) {
      acc ^= buf[i % NB];
      if (i + NB < SL)
        buf[i % NB] = __builtin_amdgcn_raw_buffer_load_b128(
            cur, lane16, ((i + NB) % K) * s.bs + x + 1024 * ((i + NB) / K), NTL ? 2 : 0);
      else
        buf[i % NB] = __builtin_amdgcn_raw_buffer_load_b128(
            nxt, lane16, ((i + NB - SL) % K) * s.bs + xn + 1024 * ((i + NB - SL) / K), NTL ? 2 : 0);
      if (i % K == K - 1) {
#pragma unroll
        for (int q = 0; q < M; ++q) {
          __builtin_amdgcn_raw_buffer_store_b128(acc + uint32_t(q), par, lane16,
                                                 uint32_t(K + q) * uint32_t(s.frag_stride) + 80 + x + 1024 * (i / K), 2);
          if constexpr (ST_NOP) {
            __builtin_amdgcn_sched_barrier(0);
            asm volatile("s_nop 0");
            __builtin_amdgcn_sched_barrier(0);
          }
        }
        acc = v4u{0u, 0u, 0u, 0u};
      }
    }
    if (wn == w) break;
    w = wn;
    x = xn;
    cur = nxt;
  }
}

// The buf-stream encode in "runs": block b takes runs b, b + G, ... of RUN
// consecutive items (the order a per-thread Horner CRC over RUN tiles of one
// payload needs; RUN = 1 is the plain grid-stride order).
template <int RUN, bool NTL>
__global__ void __launch_bounds__(256) enc_stream_run_kernel(Shape s) {
  constexpr int NB = 5, SL = K;
  const uint32_t items = s.n_obj * s.tiles;
  const uint32_t G = gridDim.x;
  uint32_t w = blockIdx.x * RUN;
  if (w >= items) return;
  auto next = [&](uint32_t it) -> uint32_t {
    const uint32_t n = (it % RUN == RUN - 1) ? it + 1 + (G - 1) * RUN : it + 1;
    return n < items ? n : it;
  };
  const uint32_t lane16 = (threadIdx.x & 63) * 16;
  const uint32_t wx = __builtin_amdgcn_readfirstlane((threadIdx.x >> 6) * 1024);
  auto item_x = [&](uint32_t it) { return (it - it / s.tiles * s.tiles) * 4096 + wx; };
  auto obj_of = [&](uint32_t it, int rec) { return mk_rsrc(s.objs + (it / s.tiles) * s.obj_stride, rec); };
  Rsrc cur = obj_of(w, -1);
  uint32_t x = item_x(w);
  v4u buf[NB];
#pragma unroll
  for (int i = 0; i < NB; ++i)
    buf[i] = __builtin_amdgcn_raw_buffer_load_b128(cur, lane16, i * s.bs + x, NTL ? 2 : 0);
  while (true) {
    const uint32_t wn = next(w);
    const Rsrc nxt = obj_of(wn, wn == w ? 0 : -1);
    const uint32_t xn = item_x(wn);
    const Rsrc par = mk_rsrc(s.frags + (w / s.tiles) * s.stripe_stride);
    v4u acc = v4u{0u, 0u, 0u, 0u};
#pragma unroll
    for (int i = 0; i < SL; ++i) {
      acc ^= buf[i % NB];
      if (i + NB < SL)
        buf[i % NB] = __builtin_amdgcn_raw_buffer_load_b128(cur, lane16, (i + NB) * s.bs + x, NTL ? 2 : 0);
      else
        buf[i % NB] = __builtin_amdgcn_raw_buffer_load_b128(nxt, lane16, (i + NB - SL) * s.bs + xn, NTL ? 2 : 0);
    }
#pragma unroll
    for (int q = 0; q < M; ++q) {
      __builtin_amdgcn_raw_buffer_store_b128(acc + uint32_t(q), par, lane16,
                                             uint32_t(K + q) * uint32_t(s.frag_stride) + 80 + x, 2);
      __builtin_amdgcn_sched_barrier(0);
      asm volatile("s_nop 0");
      __builtin_amdgcn_sched_barrier(0);
    }
    if (wn == w) break;
    w = wn;
    x = xn;
    cur = nxt;
  }
}

// The product stream with WPB waves per block (WPB x 64 threads): an item is
// WPB KiB of payload positions, one 1 KiB chunk per wave.  Do 1 block of 8
// waves per CU behave like 1 block of 4 (fewer, larger blocks) or like 2
// blocks of 4 (the same waves)?
// SPREAD: consecutive items of a block alternate between the two halves of
// its XCD range (the footprint in flight doubles at the same wave count).
// HALF: each wave moves 512 B per chunk (lanes 0-31), an item WPB x 512 B.
template <int WPB, bool NTL, bool SPREAD = false, bool HALF = false>
__global__ void __launch_bounds__(WPB * 64) enc_stream_wpb_kernel(Shape s) {
  constexpr int NB = 5, SL = K;
  constexpr uint32_t CB = HALF ? 512u : 1024u;
  constexpr uint32_t T = WPB * CB;
  if (HALF && (threadIdx.x & 63) >= 32) return;
  const uint32_t tiles = s.bs / T;
  const uint32_t items = s.n_obj * tiles;
  // XCD-major split as order<1>
  const uint32_t xg = blockIdx.x & 7u;
  const uint32_t lo = uint32_t(uint64_t(items) * xg / 8), hi = uint32_t(uint64_t(items) * (xg + 1) / 8);
  uint32_t w = lo + (blockIdx.x >> 3);
  const uint32_t step = gridDim.x >> 3;
  if (w >= hi) return;
  const uint32_t lane16 = (threadIdx.x & 63) * 16;
  const uint32_t wx = __builtin_amdgcn_readfirstlane((threadIdx.x >> 6) * CB);
  const uint32_t half = (hi - lo) / 2;
  auto real = [&](uint32_t v) {
    if (!SPREAD) return v;
    const uint32_t d = v - lo;
    return (d & 1u) ? lo + half + d / 2 : lo + d / 2;
  };
  auto item_x = [&](uint32_t it) { it = real(it); return (it - it / tiles * tiles) * T + wx; };
  auto obj_of = [&](uint32_t it, int rec) {
    return mk_rsrc(s.objs + (real(it) / tiles) * s.obj_stride, rec);
  };
  Rsrc cur = obj_of(w, -1);
  uint32_t x = item_x(w);
  v4u buf[NB];
#pragma unroll
  for (int i = 0; i < NB; ++i)
    buf[i] = __builtin_amdgcn_raw_buffer_load_b128(cur, lane16, i * s.bs + x, NTL ? 2 : 0);
  while (true) {
    const uint32_t wn = w + step < hi ? w + step : w;
    const Rsrc nxt = obj_of(wn, wn == w ? 0 : -1);
    const uint32_t xn = item_x(wn);
    const Rsrc par = mk_rsrc(s.frags + (real(w) / tiles) * s.stripe_stride);
    v4u acc = v4u{0u, 0u, 0u, 0u};
#pragma unroll
    for (int i = 0; i < SL; ++i) {
      acc ^= buf[i % NB];
      if (i + NB < SL)
        buf[i % NB] = __builtin_amdgcn_raw_buffer_load_b128(cur, lane16, (i + NB) * s.bs + x, NTL ? 2 : 0);
      else
        buf[i % NB] = __builtin_amdgcn_raw_buffer_load_b128(nxt, lane16, (i + NB - SL) * s.bs + xn, NTL ? 2 : 0);
    }
#pragma unroll
    for (int q = 0; q < M; ++q) {
      __builtin_amdgcn_raw_buffer_store_b128(acc + uint32_t(q), par, lane16,
                                             uint32_t(K + q) * uint32_t(s.frag_stride) + 80 + x, 2);
      __builtin_amdgcn_sched_barrier(0);
      asm volatile("s_nop 0");
      __builtin_amdgcn_sched_barrier(0);
    }
    if (wn == w) break;
    w = wn;
    x = xn;
    cur = nxt;
  }
}

// Paired slices: lanes 0-31 read slice 2i and lanes 32-63 slice 2i+1 at the
// same 512 B of positions, so each load instruction moves two 512-B
// segments; a wave's chunk is 512 B of positions, an item 4 x 512 B.  NP
// pairs in flight per wave.  Parity rows 0-1 stored by lanes 0-31 and 2-3 by
// lanes 32-63 (as the real kernel would after a 32-lane swap).
template <int NP, bool NTL>
__global__ void __launch_bounds__(256) enc_pair_kernel(Shape s) {
  constexpr int SL = K / 2;  // pair slots per item
  constexpr uint32_t T = 4 * 512u;
  const uint32_t tiles = s.bs / T;
  const uint32_t items = s.n_obj * tiles;
  const uint32_t xg = blockIdx.x & 7u;
  const uint32_t lo = uint32_t(uint64_t(items) * xg / 8), hi = uint32_t(uint64_t(items) * (xg + 1) / 8);
  uint32_t w = lo + (blockIdx.x >> 3);
  const uint32_t step = gridDim.x >> 3;
  if (w >= hi) return;
  const uint32_t l = threadIdx.x & 63;
  const uint32_t hl = l >> 5;                  // 0: even slice, 1: odd slice
  const uint32_t voff = (l & 31) * 16 + hl * s.bs;
  const uint32_t wx = __builtin_amdgcn_readfirstlane((threadIdx.x >> 6) * 512);
  auto item_x = [&](uint32_t it) { return (it - it / tiles * tiles) * T + wx; };
  auto obj_of = [&](uint32_t it, int rec) { return mk_rsrc(s.objs + (it / tiles) * s.obj_stride, rec); };
  Rsrc cur = obj_of(w, -1);
  uint32_t x = item_x(w);
  v4u buf[NP];
#pragma unroll
  for (int i = 0; i < NP; ++i)
    buf[i] = __builtin_amdgcn_raw_buffer_load_b128(cur, voff, 2 * i * s.bs + x, NTL ? 2 : 0);
  while (true) {
    const uint32_t wn = w + step < hi ? w + step : w;
    const Rsrc nxt = obj_of(wn, wn == w ? 0 : -1);
    const uint32_t xn = item_x(wn);
    const Rsrc par = mk_rsrc(s.frags + (w / tiles) * s.stripe_stride);
    v4u acc = v4u{0u, 0u, 0u, 0u};
#pragma unroll
    for (int i = 0; i < SL; ++i) {
      acc ^= buf[i % NP];
      if (i + NP < SL)
        buf[i % NP] = __builtin_amdgcn_raw_buffer_load_b128(cur, voff, 2 * (i + NP) * s.bs + x, NTL ? 2 : 0);
      else
        buf[i % NP] = __builtin_amdgcn_raw_buffer_load_b128(nxt, voff, 2 * (i + NP - SL) * s.bs + xn, NTL ? 2 : 0);
    }
    const uint32_t soff_lane = (l & 31) * 16 + hl * 2 * uint32_t(s.frag_stride);
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      __builtin_amdgcn_raw_buffer_store_b128(acc + uint32_t(q), par, soff_lane,
                                             uint32_t(K + q) * uint32_t(s.frag_stride) + 80 + x, 2);
      __builtin_amdgcn_sched_barrier(0);
      asm volatile("s_nop 0");
      __builtin_amdgcn_sched_barrier(0);
    }
    if (wn == w) break;
    w = wn;
    x = xn;
    cur = nxt;
  }
}

// ---- decode stream: read the 10 data-fragment payloads (line-aligned),
// write them to the object's slices at j*bs + x. ----
template <bool NTL, bool NTS>
__global__ void __launch_bounds__(256) dec_kernel(Shape s) {
  const uint32_t items = s.n_obj * s.tiles;
  for (uint32_t w = blockIdx.x; w < items; w += gridDim.x) {
    const uint32_t o = w / s.tiles, t = w - o * s.tiles;
    const uint32_t x = t * 4096 + (threadIdx.x >> 6) * 1024 + (threadIdx.x & 63) * 16;
    const uint8_t* src = s.frags + o * s.stripe_stride + 80 + x;
    v4u v[K];
#pragma unroll
    for (int j = 0; j < K; ++j) v[j] = ld<NTL>(src + j * s.frag_stride);
    uint8_t* dst = s.objs + o * s.obj_stride + x;
#pragma unroll
    for (int j = 0; j < K; ++j) st<NTS>(dst + uint64_t(j) * s.bs, v[j] + 1u);
  }
}

// ---- the guide's ceilings (MI355X_MICROARCH.md, chip table: "6.29 TB/s
// measured (float4 copy)"; price table row ldsdma-fill: an LDS-DMA stream
// "chip 6.4 TB/s default policy, 6.5-6.8 nt"), rebuilt here so they run on
// the same box, in the same call, as the product kernels (round 6). ----

// One float4 per thread and U per block-stride, no loop: the textbook copy.
template <int U, bool NT>
__global__ void __launch_bounds__(256) copy_f4_kernel(const uint8_t* src, uint8_t* dst, uint64_t n16) {
  const uint64_t base = uint64_t(blockIdx.x) * 256 * U + threadIdx.x;
  v4u v[U];
#pragma unroll
  for (int u = 0; u < U; ++u)
    if (base + u * 256 < n16) v[u] = ld<NT>(src + (base + u * 256) * 16);
#pragma unroll
  for (int u = 0; u < U; ++u)
    if (base + u * 256 < n16) st<NT>(dst + (base + u * 256) * 16, v[u]);
}
template <int U, bool NT>
__global__ void __launch_bounds__(256) read_f4_kernel(const uint8_t* src, uint64_t n16, uint32_t* sink) {
  const uint64_t base = uint64_t(blockIdx.x) * 256 * U + threadIdx.x;
  uint32_t acc = 0;
#pragma unroll
  for (int u = 0; u < U; ++u)
    if (base + u * 256 < n16) {
      const v4u v = ld<NT>(src + (base + u * 256) * 16);
      acc ^= v.x ^ v.y ^ v.z ^ v.w;
    }
  if (acc == 0x12345678u) sink[0] = acc;
}

// LDS-DMA (buffer_load_dwordx4 ... lds) as the product issues it
// (ec_kernels_impl.hpp dma16): M0 = the wave's LDS destination, 1 KiB per
// wave-instruction.
typedef unsigned int v4u_s __attribute__((ext_vector_type(4)));
__device__ __forceinline__ v4u_s rsrc4(const void* base, uint32_t records) {
  const uint64_t a = reinterpret_cast<uint64_t>(base);
  v4u_s r;
  r.x = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(a));
  r.y = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(a >> 32)) & 0xFFFFu;
  r.z = __builtin_amdgcn_readfirstlane(records);
  r.w = 0x00020000u;
  return r;
}
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
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// Read-only LDS-DMA stream (the guide's ldsdma-fill row): L loader waves per
// block, no consumers; each wave keeps D 1-KiB DMAs in flight into a ring of
// D slots of its own.  Chunk c of wave (b, w) = b * L + w + i * grid * L.
template <int L, int D, bool NT>
__global__ void __launch_bounds__(L * 64) dma_read_kernel(const uint8_t* src, uint64_t n) {
  const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t lane16 = (threadIdx.x & 63) * 16;
  const v4u_s r = rsrc4(src, 0xFFFFFFFFu);
  const uint64_t chunks = n / 1024, stride = uint64_t(gridDim.x) * L;
  uint32_t slot = 0;
  for (uint64_t c = uint64_t(blockIdx.x) * L + wave; c < chunks; c += stride) {
    dma16<NT>(r, lane16, __builtin_amdgcn_readfirstlane(uint32_t(c * 1024)), (wave * D + slot) * 1024);
    slot = slot + 1 == D ? 0 : slot + 1;
    wait_vm<D - 1>();
  }
  wait_vm<0>();
}

// Copy through an LDS-DMA ring, the product's loader / consumer shape
// (decode_dma_kernel without the lookups): W waves per block, L of them
// loaders, R ring slots of W KiB; every wave reads its 1 KiB of the slot and
// stores it (nt) to dst.  Item = W KiB; one block per CU walks the items
// grid-stride.
template <int W, int L, int R, bool NT>
__global__ void __launch_bounds__(W * 64) dma_copy_kernel(const uint8_t* src, uint8_t* dst, uint64_t n) {
  constexpr uint32_t kSlot = 1024u * W;
  constexpr int kPer = W / L;
  const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t lane16 = (threadIdx.x & 63) * 16;
  const bool loader = wave < uint32_t(L);
  const uint32_t items = uint32_t(n / kSlot);
  const uint32_t n_items = blockIdx.x < items ? (items - blockIdx.x + gridDim.x - 1) / gridDim.x : 0;
  if (n_items == 0) return;
  auto issue = [&](uint32_t i, uint32_t ri) {
    if (!loader) return;
    const uint32_t it = blockIdx.x + (i < n_items ? i : 0) * gridDim.x;
    const v4u_s r = rsrc4(src, i < n_items ? 0xFFFFFFFFu : 0u);
    const uint32_t part = wave * (kSlot / L);
#pragma unroll
    for (int c = 0; c < kPer; ++c)
      dma16<NT>(r, lane16, __builtin_amdgcn_readfirstlane(it * kSlot + part + 1024 * c),
                ri * kSlot + part + 1024 * c);
  };
  const Rsrc out = mk_rsrc(dst), none = mk_rsrc(dst, 0);
#pragma unroll
  for (int t = 0; t < R - 1; ++t) {
    issue(t, t);
    if (loader) __builtin_amdgcn_raw_buffer_store_b128(v4u{0u, 0u, 0u, 0u}, none, lane16, 0, 2);
  }
  uint32_t ring = 0;
  for (uint32_t i = 0; i < n_items; ++i) {
    if (loader) wait_vm<1 + (R - 2) * (kPer + 1)>();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    issue(i + R - 1, ring == 0 ? R - 1 : ring - 1);
    const v4u x = *reinterpret_cast<const __attribute__((address_space(3))) v4u*>(
        static_cast<uintptr_t>(ring * kSlot + wave * 1024 + lane16));
    const uint32_t it = blockIdx.x + i * gridDim.x;
    __builtin_amdgcn_raw_buffer_store_b128(x + 1u, out, lane16, it * kSlot + wave * 1024, 2);
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_nop 0");
    __builtin_amdgcn_sched_barrier(0);
    ring = ring + 1 == R ? 0 : ring + 1;
  }
  if (loader) wait_vm<0>();
}

// The product's decode and encode memory patterns in the loader / consumer
// shape (ec_kernels_impl.hpp decode_dma_kernel / encode_dma_kernel) with the
// lookups left out.  Item = W KiB of payload positions of one object, one
// ring slot per input.
//   dma_dec: input j = fragment j's payload (line-aligned), stored at once to
//            the object's slice j at j * bs (bs = 8 mod 16 at 4 MiB: half the
//            slices misaligned); the product stores 6 present slices this way
//            and 4 rebuilt rows at the item's end -- the same bytes.
//   dma_enc: input j = the object's slice j (at j * bs), XORed; the 4 parity
//            rows stored line-aligned at the item's end.
// ORD: 0 grid-stride over the items, 1 XCD-split (encode's order).
template <int W, int L, int R, bool NT, int ORD = 0>
__global__ void __launch_bounds__(W * 64) dma_dec_kernel(Shape s) {
  constexpr uint32_t kSlot = 1024u * W;
  constexpr int kPer = W / L;
  const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t lane16 = (threadIdx.x & 63) * 16;
  const bool loader = wave < uint32_t(L);
  const Order rg = order<ORD>(s.n_obj * s.tiles, s.tiles);
  if (rg.begin >= rg.end) return;
  const uint32_t n_items = (rg.end - rg.begin + rg.step - 1) / rg.step;
  auto item_at = [&](uint32_t i, uint32_t& o, uint32_t& x0) {
    const uint32_t w = rg.begin + (i < n_items ? i : 0) * rg.step;
    o = __builtin_amdgcn_readfirstlane(w / s.tiles);
    x0 = (w - o * s.tiles) * kSlot;
  };
  auto issue = [&](uint32_t i, int j, uint32_t ri) {
    if (!loader) return;
    uint32_t o, x0;
    item_at(i, o, x0);
    const v4u_s r = rsrc4(s.frags + uint64_t(o) * s.stripe_stride, i < n_items ? 0xFFFFFFFFu : 0u);
    const uint32_t part = wave * (kSlot / L);
    const uint32_t soff = __builtin_amdgcn_readfirstlane(uint32_t(j) * uint32_t(s.frag_stride) + 80 + x0 + part);
#pragma unroll
    for (int c = 0; c < kPer; ++c) dma16<NT>(r, lane16, soff + 1024 * c, ri * kSlot + part + 1024 * c);
  };
  const Rsrc none = mk_rsrc(s.objs, 0);
#pragma unroll
  for (int t = 0; t < R - 1; ++t) {
    issue(t / K, t % K, t);
    if (loader) __builtin_amdgcn_raw_buffer_store_b128(v4u{0u, 0u, 0u, 0u}, none, lane16, 0, 2);
  }
  uint32_t ring = 0;
  for (uint32_t i = 0; i < n_items; ++i) {
    uint32_t o, x0;
    item_at(i, o, x0);
    const Rsrc out = mk_rsrc(s.objs + uint64_t(o) * s.obj_stride);
#pragma unroll
    for (int j = 0; j < K; ++j) {
      if (loader) wait_vm<1 + (R - 2) * (kPer + 1)>();
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
      const uint32_t rn = ring == 0 ? R - 1 : ring - 1;
      if (j + R - 1 < K)
        issue(i, j + R - 1, rn);
      else
        issue(i + 1, j + R - 1 - K, rn);
      const v4u x = *reinterpret_cast<const __attribute__((address_space(3))) v4u*>(
          static_cast<uintptr_t>(ring * kSlot + wave * 1024 + lane16));
      __builtin_amdgcn_raw_buffer_store_b128(x + 1u, out, lane16, uint32_t(j) * s.bs + x0 + wave * 1024, 2);
      __builtin_amdgcn_sched_barrier(0);
      asm volatile("s_nop 0");
      __builtin_amdgcn_sched_barrier(0);
      ring = ring + 1 == R ? 0 : ring + 1;
    }
  }
  if (loader) wait_vm<0>();
}

// DATA: the full stripe -- every input chunk also stored to its data
// fragment's (line-aligned) payload as it is read from the ring.
template <int W, int L, int R, bool NT, int ORD = 1, bool DATA = false>
__global__ void __launch_bounds__(W * 64) dma_enc_kernel(Shape s) {
  constexpr uint32_t kSlot = 1024u * W;
  constexpr int kPer = W / L;
  const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t lane16 = (threadIdx.x & 63) * 16;
  const bool loader = wave < uint32_t(L);
  const Order rg = order<ORD>(s.n_obj * s.tiles, s.tiles);
  if (rg.begin >= rg.end) return;
  const uint32_t n_items = (rg.end - rg.begin + rg.step - 1) / rg.step;
  auto item_at = [&](uint32_t i, uint32_t& o, uint32_t& x0) {
    const uint32_t w = rg.begin + (i < n_items ? i : 0) * rg.step;
    o = __builtin_amdgcn_readfirstlane(w / s.tiles);
    x0 = (w - o * s.tiles) * kSlot;
  };
  auto issue = [&](uint32_t i, int j, uint32_t ri) {
    if (!loader) return;
    uint32_t o, x0;
    item_at(i, o, x0);
    const v4u_s r = rsrc4(s.objs + uint64_t(o) * s.obj_stride, i < n_items ? 0xFFFFFFFFu : 0u);
    const uint32_t part = wave * (kSlot / L);
    const uint32_t soff = __builtin_amdgcn_readfirstlane(uint32_t(j) * s.bs + x0 + part);
#pragma unroll
    for (int c = 0; c < kPer; ++c) dma16<NT>(r, lane16, soff + 1024 * c, ri * kSlot + part + 1024 * c);
  };
#pragma unroll
  for (int t = 0; t < R - 1; ++t) issue(t / K, t % K, t);
  uint32_t ring = 0;
  for (uint32_t i = 0; i < n_items; ++i) {
    uint32_t o, x0;
    item_at(i, o, x0);
    const Rsrc par = mk_rsrc(s.frags + uint64_t(o) * s.stripe_stride);
    v4u acc = v4u{0u, 0u, 0u, 0u};
#pragma unroll
    for (int j = 0; j < K; ++j) {
      if (loader) wait_vm<kPer * (R - 2)>();
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
      const uint32_t rn = ring == 0 ? R - 1 : ring - 1;
      issue(i + (j + R - 1) / K, (j + R - 1) % K, rn);
      const v4u xin = *reinterpret_cast<const __attribute__((address_space(3))) v4u*>(
          static_cast<uintptr_t>(ring * kSlot + wave * 1024 + lane16));
      acc ^= xin;
      if constexpr (DATA) {
        __builtin_amdgcn_raw_buffer_store_b128(xin, par, lane16,
                                               uint32_t(j) * uint32_t(s.frag_stride) + 80 + x0 + wave * 1024, 2);
        __builtin_amdgcn_sched_barrier(0);
        asm volatile("s_nop 0");
        __builtin_amdgcn_sched_barrier(0);
      }
      ring = ring + 1 == R ? 0 : ring + 1;
    }
#pragma unroll
    for (int q = 0; q < M; ++q) {
      __builtin_amdgcn_raw_buffer_store_b128(acc + uint32_t(q), par, lane16,
                                             uint32_t(K + q) * uint32_t(s.frag_stride) + 80 + x0 + wave * 1024, 2);
      __builtin_amdgcn_sched_barrier(0);
      asm volatile("s_nop 0");
      __builtin_amdgcn_sched_barrier(0);
    }
  }
  if (loader) wait_vm<0>();
}

// One-shot forms of the decode / encode patterns (the float4 copy's shape):
// one block per item (object, 4 KiB tile), no loop -- the dispatcher keeps
// as many waves resident as fit and launches the next blocks in order, so
// the chip sweeps memory in one compact front.  Every input of the item in
// registers at once.
template <bool NTL, bool NTS, bool ENC>
__global__ void __launch_bounds__(256) oneshot_kernel(Shape s) {
  const uint32_t w = blockIdx.x;
  const uint32_t o = w / s.tiles, t = w - o * s.tiles;
  const uint32_t x = t * 4096 + (threadIdx.x >> 6) * 1024 + (threadIdx.x & 63) * 16;
  v4u v[K];
  if constexpr (ENC) {
    const uint8_t* src = s.objs + uint64_t(o) * s.obj_stride + x;
#pragma unroll
    for (int j = 0; j < K; ++j) v[j] = ld<NTL>(src + uint64_t(j) * s.bs);
    v4u acc = v[0];
#pragma unroll
    for (int j = 1; j < K; ++j) acc ^= v[j];
    uint8_t* dst = s.frags + uint64_t(o) * s.stripe_stride + K * s.frag_stride + 80 + x;
#pragma unroll
    for (int q = 0; q < M; ++q) st<NTS>(dst + q * s.frag_stride, acc + uint32_t(q));
  } else {
    const uint8_t* src = s.frags + uint64_t(o) * s.stripe_stride + 80 + x;
#pragma unroll
    for (int j = 0; j < K; ++j) v[j] = ld<NTL>(src + j * s.frag_stride);
    uint8_t* dst = s.objs + uint64_t(o) * s.obj_stride + x;
#pragma unroll
    for (int j = 0; j < K; ++j) st<NTS>(dst + uint64_t(j) * s.bs, v[j] + 1u);
  }
}

int g_cus = 256;
int g_reps = 20;

template <typename F>
double time_us(F launch) {
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  launch();
  launch();
  CHECK(hipDeviceSynchronize());
  CHECK(hipGetLastError());
  CHECK(hipEventRecord(e0, 0));
  for (int i = 0; i < g_reps; ++i) launch();
  CHECK(hipEventRecord(e1, 0));
  CHECK(hipEventSynchronize(e1));
  float ms = 0;
  CHECK(hipEventElapsedTime(&ms, e0, e1));
  CHECK(hipGetLastError());
  CHECK(hipEventDestroy(e0));
  CHECK(hipEventDestroy(e1));
  return ms * 1e3 / g_reps;
}

// Alternating form (bench.py's step): `other` then `timed`, g_reps times;
// the mean time of `timed` alone, from events around it.
template <typename A, typename B>
double time_alt_us(A other, B timed) {
  std::vector<hipEvent_t> ev(2 * g_reps);
  for (auto& e : ev) CHECK(hipEventCreate(&e));
  other();
  timed();
  CHECK(hipDeviceSynchronize());
  for (int i = 0; i < g_reps; ++i) {
    other();
    CHECK(hipEventRecord(ev[2 * i], 0));
    timed();
    CHECK(hipEventRecord(ev[2 * i + 1], 0));
  }
  CHECK(hipDeviceSynchronize());
  CHECK(hipGetLastError());
  double sum = 0;
  for (int i = 0; i < g_reps; ++i) {
    float ms = 0;
    CHECK(hipEventElapsedTime(&ms, ev[2 * i], ev[2 * i + 1]));
    sum += ms;
  }
  for (auto& e : ev) CHECK(hipEventDestroy(e));
  return sum * 1e3 / g_reps;
}

void report(const char* name, int bpc, double us, double bytes) {
  std::printf("%-52s bpc=%d %9.1f us %8.1f GB/s\n", name, bpc, us, bytes / us / 1e3);
  std::fflush(stdout);
}

bool want(const char* sections, const char* s) {
  return sections == nullptr || std::strstr(sections, s) != nullptr;
}

}  // namespace

int main(int argc, char** argv) {
  if (argc > 1) g_reps = std::atoi(argv[1]);
  const char* sections = argc > 2 ? argv[2] : nullptr;
  int dev = 0;
  CHECK(hipGetDevice(&dev));
  CHECK(hipDeviceGetAttribute(&g_cus, hipDeviceAttributeMultiprocessorCount, dev));
  const uint32_t n_obj = 256, L = 4u << 20;
  const uint32_t bs_real = 2 * ((L + 2 * K - 1) / (2 * K));  // 419432
  const uint32_t bs_al = (bs_real + 127) / 128 * 128;        // 419456
  const uint64_t obj_stride = L;
  const uint64_t fs = ((80 + (bs_al + 15) / 16 * 16) + 127) / 128 * 128;
  const uint64_t ss = fs * (K + M);
  // compact layout: many small objects holding the same bytes (10 slices of
  // 40 KiB), stripes of 14 fragments of 40 KiB + 128
  const uint32_t sbs = 40960, sobj = 10 * sbs, sfs = sbs + 128;
  const uint64_t sss = uint64_t(sfs) * (K + M);
  const uint32_t n_compact = uint32_t(uint64_t(n_obj) * obj_stride / sobj);
  const uint64_t obj_bytes = obj_stride * n_obj + (1 << 20);
  const uint64_t frag_bytes = std::max(ss * n_obj, sss * n_compact) + (1 << 20);
  uint8_t *objs, *frags_raw, *out;
  uint32_t* sink;
  CHECK(hipMalloc(&objs, obj_bytes));
  CHECK(hipMalloc(&out, obj_bytes));
  CHECK(hipMalloc(&frags_raw, frag_bytes));
  CHECK(hipMalloc(&sink, 64));
  CHECK(hipMemset(objs, 1, obj_bytes));
  if (const char* r = std::getenv("MB_RANDOM"); r != nullptr && r[0] == '1') {
    // random object bytes, as bench.py's (the constant fill flips no bus bits)
    std::vector<uint64_t> host(obj_bytes / 8);
    uint64_t x = 0x9E3779B97F4A7C15ull;
    for (auto& v : host) {
      x ^= x << 13;
      x ^= x >> 7;
      x ^= x << 17;
      v = x;
    }
    CHECK(hipMemcpy(objs, host.data(), host.size() * 8, hipMemcpyHostToDevice));
    std::printf("random object bytes\n");
  }
  CHECK(hipMemset(out, 0, obj_bytes));
  CHECK(hipMemset(frags_raw, 2, frag_bytes));
  uint8_t* frags = frags_raw + 48;  // payloads (80 B past each fragment start) 128-B aligned
  g_bufs = {objs, out, frags_raw, obj_bytes, frag_bytes};
  std::printf("CUs %d, reps %d, bs %u / aligned %u, frag_stride %llu\n", g_cus, g_reps, bs_real,
              bs_al, (unsigned long long)fs);

  const uint64_t n_copy = uint64_t(n_obj) * L;
  if (want(sections, "base")) {
    for (int bpc : {2, 4, 8}) {
      const int grid = g_cus * bpc;
      report("copy 1 GiB, 16 B/lane, nt", bpc,
             time_us([&] { copy_kernel<1, true><<<grid, 256>>>(objs, out, n_copy); }), 2.0 * n_copy);
      report("copy 1 GiB, 2x16 B/lane, nt", bpc,
             time_us([&] { copy_kernel<2, true><<<grid, 256>>>(objs, out, n_copy); }), 2.0 * n_copy);
      report("read 1 GiB, 16 B/lane, cached", bpc,
             time_us([&] { read_kernel<1, false><<<grid, 256>>>(objs, n_copy, sink); }), 1.0 * n_copy);
      report("read 1 GiB, 4x16 B/lane, cached", bpc,
             time_us([&] { read_kernel<4, false><<<grid, 256>>>(objs, n_copy, sink); }), 1.0 * n_copy);
      report("write 1 GiB, 16 B/lane, nt", bpc,
             time_us([&] { write_kernel<1, true><<<grid, 256>>>(out, n_copy); }), 1.0 * n_copy);
    }
  }
  if (want(sections, "roof")) {
    // the guide's copy and LDS-DMA stream beside this repo's best copy
    const uint64_t n16 = n_copy / 16;
    report("guide: float4 copy, 1/thread, default policy", 0,
           time_us([&] { copy_f4_kernel<1, false><<<n16 / 256, 256>>>(objs, out, n16); }), 2.0 * n_copy);
    report("guide: float4 copy, 1/thread, nt", 0,
           time_us([&] { copy_f4_kernel<1, true><<<n16 / 256, 256>>>(objs, out, n16); }), 2.0 * n_copy);
    report("guide: float4 copy, 4/thread, default policy", 0,
           time_us([&] { copy_f4_kernel<4, false><<<n16 / 1024, 256>>>(objs, out, n16); }), 2.0 * n_copy);
    report("guide: float4 copy, 4/thread, nt", 0,
           time_us([&] { copy_f4_kernel<4, true><<<n16 / 1024, 256>>>(objs, out, n16); }), 2.0 * n_copy);
    report("float4 read, 1/thread, default policy", 0,
           time_us([&] { read_f4_kernel<1, false><<<n16 / 256, 256>>>(objs, n16, sink); }), 1.0 * n_copy);
    report("float4 read, 4/thread, nt", 0,
           time_us([&] { read_f4_kernel<4, true><<<n16 / 1024, 256>>>(objs, n16, sink); }), 1.0 * n_copy);
    for (int bpc : {1, 2}) {
      const int grid = g_cus * bpc;
      report("best copy so far: 16 B/lane grid-stride, nt", bpc,
             time_us([&] { copy_kernel<1, true><<<grid * 2, 256>>>(objs, out, n_copy); }), 2.0 * n_copy);
      report("guide: LDS-DMA read stream L4 D8 nt", bpc,
             time_us([&] { dma_read_kernel<4, 8, true><<<grid, 256, 4 * 8 * 1024>>>(objs, n_copy); }), 1.0 * n_copy);
      report("guide: LDS-DMA read stream L4 D8 default", bpc,
             time_us([&] { dma_read_kernel<4, 8, false><<<grid, 256, 4 * 8 * 1024>>>(objs, n_copy); }), 1.0 * n_copy);
      report("guide: LDS-DMA read stream L4 D16 nt", bpc,
             time_us([&] { dma_read_kernel<4, 16, true><<<grid, 256, 4 * 16 * 1024>>>(objs, n_copy); }), 1.0 * n_copy);
      report("guide: LDS-DMA read stream L4 D4 nt", bpc,
             time_us([&] { dma_read_kernel<4, 4, true><<<grid, 256, 4 * 4 * 1024>>>(objs, n_copy); }), 1.0 * n_copy);
    }
    report("LDS-DMA copy W12 L4 R3 nt (product shape)", 1,
           time_us([&] { dma_copy_kernel<12, 4, 3, true><<<g_cus, 768, 3 * 12 * 1024>>>(objs, out, n_copy); }),
           2.0 * n_copy);
    report("LDS-DMA copy W12 L4 R4 nt", 1,
           time_us([&] { dma_copy_kernel<12, 4, 4, true><<<g_cus, 768, 4 * 12 * 1024>>>(objs, out, n_copy); }),
           2.0 * n_copy);
    report("LDS-DMA copy W8 L4 R4 nt", 1,
           time_us([&] { dma_copy_kernel<8, 4, 4, true><<<g_cus, 512, 4 * 8 * 1024>>>(objs, out, n_copy); }),
           2.0 * n_copy);
    report("LDS-DMA copy W8 L4 R4 nt", 2,
           time_us([&] { dma_copy_kernel<8, 4, 4, true><<<g_cus * 2, 512, 4 * 8 * 1024>>>(objs, out, n_copy); }),
           2.0 * n_copy);
    report("LDS-DMA copy W16 L4 R3 nt", 1,
           time_us([&] { dma_copy_kernel<16, 4, 3, true><<<g_cus, 1024, 3 * 16 * 1024>>>(objs, out, n_copy); }),
           2.0 * n_copy);
    report("LDS-DMA copy W16 L8 R4 nt", 1,
           time_us([&] { dma_copy_kernel<16, 8, 4, true><<<g_cus, 1024, 4 * 16 * 1024>>>(objs, out, n_copy); }),
           2.0 * n_copy);
  }
  if (want(sections, "dmapat")) {
    // the product's decode / encode memory patterns, loader / consumer shape
    for (uint32_t bs : {bs_real, bs_al}) {
      auto dec = [&](auto kern, int W, const char* name) {
        Shape d{out, frags, bs, n_obj, bs_real / (1024u * W), obj_stride, fs, ss};
        check_shape(name, d, 1024u * W, true);
        const double bytes = double(n_obj) * d.tiles * 1024.0 * W * (2 * K);
        report(name, 1, time_us([&] { kern<<<g_cus, W * 64, 5 * 1024 * W>>>(d); }), bytes);
      };
      const bool al = bs == bs_al;
      dec(dma_dec_kernel<12, 4, 3, true>, 12, al ? "dma dec W12 R3 aligned" : "dma dec W12 R3 real (product shape)");
      dec(dma_dec_kernel<16, 4, 3, true>, 16, al ? "dma dec W16 R3 aligned" : "dma dec W16 R3 real");
      dec(dma_dec_kernel<12, 4, 4, true>, 12, al ? "dma dec W12 R4 aligned" : "dma dec W12 R4 real");
      dec(dma_dec_kernel<16, 4, 3, true, 1>, 16, al ? "dma dec W16 R3 xcd aligned" : "dma dec W16 R3 xcd real");
      dec(dma_dec_kernel<8, 4, 4, true>, 8, al ? "dma dec W8 R4 aligned" : "dma dec W8 R4 real");
      dec(dma_dec_kernel<8, 4, 5, true>, 8, al ? "dma dec W8 R5 aligned" : "dma dec W8 R5 real");
    }
    auto enc = [&](auto kern, int W, const char* name) {
      Shape e{objs, frags, bs_real, n_obj, bs_real / (1024u * W), obj_stride, fs, ss};
      check_shape(name, e, 1024u * W);
      const double bytes = double(n_obj) * e.tiles * 1024.0 * W * (K + M);
      report(name, 1, time_us([&] { kern<<<g_cus, W * 64, 5 * 1024 * W>>>(e); }), bytes);
    };
    enc(dma_enc_kernel<12, 4, 3, true>, 12, "dma enc W12 R3 xcd (product shape)");
    enc(dma_enc_kernel<16, 4, 3, true>, 16, "dma enc W16 R3 xcd");
    enc(dma_enc_kernel<12, 4, 4, true>, 12, "dma enc W12 R4 xcd");
    enc(dma_enc_kernel<16, 4, 4, true>, 16, "dma enc W16 R4 xcd");
    enc(dma_enc_kernel<12, 4, 3, true, 0>, 12, "dma enc W12 R3 plain order");
    enc(dma_enc_kernel<8, 4, 3, true>, 8, "dma enc W8 R3 xcd");
    // slice misalignment (bs = 8 mod 16 at 4 MiB, k = 10: half the slices)
    for (uint32_t b : {bs_real + 2, bs_al}) {
      Shape e{objs, frags, b, n_obj, bs_real / 12288u, obj_stride, fs, ss};
      check_shape("enc mis", e, 12288u);
      const double bytes = double(n_obj) * e.tiles * 12288.0 * (K + M);
      report(b == bs_al ? "dma enc W12 R3 xcd, slices 128-B aligned" : "dma enc W12 R3 xcd, bs = 10 mod 16",
             1, time_us([&] { dma_enc_kernel<12, 4, 3, true><<<g_cus, 768, 5 * 12288>>>(e); }), bytes);
    }
    enc(dma_enc_kernel<8, 4, 4, true>, 8, "dma enc W8 R4 xcd");
    enc(dma_enc_kernel<8, 4, 5, true>, 8, "dma enc W8 R5 xcd");
    // the full stripe (k data + m parity fragments): bytes = L + (k + m) x payload
    auto full = [&](auto kern, int W, int R, const char* name) {
      Shape e{objs, frags, bs_real, n_obj, bs_real / (1024u * W), obj_stride, fs, ss};
      check_shape(name, e, 1024u * W);
      const double bytes = double(n_obj) * e.tiles * 1024.0 * W * (2 * K + M);
      report(name, 1, time_us([&] { kern<<<g_cus, W * 64, R * 1024 * W>>>(e); }), bytes);
    };
    full(dma_enc_kernel<12, 4, 3, true, 1, true>, 12, 3, "dma full stripe W12 R3 xcd (product shape)");
    full(dma_enc_kernel<16, 4, 3, true, 1, true>, 16, 3, "dma full stripe W16 R3 xcd");
    full(dma_enc_kernel<12, 4, 4, true, 1, true>, 12, 4, "dma full stripe W12 R4 xcd");
    full(dma_enc_kernel<8, 4, 4, true, 1, true>, 8, 4, "dma full stripe W8 R4 xcd");
    full(dma_enc_kernel<12, 4, 3, true, 0, true>, 12, 3, "dma full stripe W12 R3 plain order");
    full(dma_enc_kernel<8, 4, 5, true, 1, true>, 8, 5, "dma full stripe W8 R5 xcd");
    full(dma_enc_kernel<8, 4, 4, true, 0, true>, 8, 4, "dma full stripe W8 R4 plain order");
  }
  if (want(sections, "oneshot")) {
    for (uint32_t bs : {bs_real, bs_al}) {
      const bool al = bs == bs_al;
      Shape d{out, frags, bs, n_obj, bs_real / 4096, obj_stride, fs, ss};
      check_shape("oneshot dec", d, 4096, true);
      const double db = double(n_obj) * d.tiles * 4096.0 * (2 * K);
      const int g = n_obj * d.tiles;
      report(al ? "oneshot dec aligned nt/nt" : "oneshot dec real nt/nt", 0,
             time_us([&] { oneshot_kernel<true, true, false><<<g, 256>>>(d); }), db);
      report(al ? "oneshot dec aligned def/nt" : "oneshot dec real def/nt", 0,
             time_us([&] { oneshot_kernel<false, true, false><<<g, 256>>>(d); }), db);
      report(al ? "oneshot dec aligned def/def" : "oneshot dec real def/def", 0,
             time_us([&] { oneshot_kernel<false, false, false><<<g, 256>>>(d); }), db);
      Shape e{objs, frags, bs, n_obj, bs_real / 4096, obj_stride, fs, ss};
      check_shape("oneshot enc", e, 4096);
      const double eb = double(n_obj) * e.tiles * 4096.0 * (K + M);
      report(al ? "oneshot enc aligned nt/nt" : "oneshot enc real nt/nt", 0,
             time_us([&] { oneshot_kernel<true, true, true><<<g, 256>>>(e); }), eb);
      report(al ? "oneshot enc aligned def/nt" : "oneshot enc real def/nt", 0,
             time_us([&] { oneshot_kernel<false, true, true><<<g, 256>>>(e); }), eb);
    }
    for (int bpc : {2, 4, 8, 16}) {
      report("grid-stride copy 16 B/lane nt", bpc,
             time_us([&] { copy_kernel<1, true><<<g_cus * bpc, 256>>>(objs, out, n_copy); }), 2.0 * n_copy);
    }
  }
  Shape s{objs, frags, bs_real, n_obj, bs_real / 4096, obj_stride, fs, ss};
  const double enc_bytes = double(n_obj) * s.tiles * 4096 * (K + M);
    // run orders (the fused-CRC encode's candidates): runs of R items per block
  // the encode pattern's ceiling rows only (same kernels as "enc")
  if (want(sections, "ceil")) {
    for (int bpc : {1, 2, 3, 4}) {
      const int grid = g_cus * bpc;
      Shape s2 = s;
      s2.tiles = bs_real / 8192;
      const double b1 = double(n_obj) * s.tiles * 4096 * (K + M);
      const double b2 = double(n_obj) * s2.tiles * 8192 * (K + M);
      report("enc buf-stream CH1 NB5 xcd (product)", bpc,
             time_us([&] { enc_stream_buf_kernel<1, 5, 1, false, true><<<grid, 256>>>(s); }), b1);
      report("enc buf-stream CH1 NB5 xcd ld-nt", bpc,
             time_us([&] { enc_stream_buf_kernel<1, 5, 1, true, true><<<grid, 256>>>(s); }), b1);
      report("enc CH2 ld-nt", bpc, time_us([&] { enc_kernel<2, true, true, false><<<grid, 256>>>(s2); }), b2);
      report("enc buf-stream CH1 NB5 xcd, product budget (8 waves/SIMD) + 5 KiB LDS", bpc,
             time_us([&] { enc_stream_buf_kernel<1, 5, 1, false, true, 8><<<grid, 256, 5120>>>(s); }), b1);
      report("enc buf-stream CH1 NB5 xcd + 5 KiB LDS", bpc,
             time_us([&] { enc_stream_buf_kernel<1, 5, 1, false, true><<<grid, 256, 5120>>>(s); }), b1);
      report("enc buf-stream CH1 NB5 xcd, product budget", bpc,
             time_us([&] { enc_stream_buf_kernel<1, 5, 1, false, true, 8><<<grid, 256>>>(s); }), b1);
      report("enc buf-stream CH1 NB2 xcd ld-nt", bpc,
             time_us([&] { enc_stream_buf_kernel<1, 2, 1, true, true><<<grid, 256>>>(s); }), b1);
      report("enc buf-stream CH1 NB2 xcd", bpc,
             time_us([&] { enc_stream_buf_kernel<1, 2, 1, false, true><<<grid, 256>>>(s); }), b1);
    }
  }
  // waves per block: 1 x 8-wave blocks vs 2 x 4-wave blocks per CU
  if (want(sections, "wpb")) {
    const double b4 = double(n_obj) * (bs_real / 4096) * 4096 * (K + M);
    const double b8 = double(n_obj) * (bs_real / 8192) * 8192 * (K + M);
    for (int ntl = 0; ntl < 2; ++ntl) {
      auto r4 = [&](int bpc) {
        return time_us([&] {
          if (ntl) enc_stream_wpb_kernel<4, true><<<g_cus * bpc, 256>>>(s);
          else enc_stream_wpb_kernel<4, false><<<g_cus * bpc, 256>>>(s);
        });
      };
      auto r8 = [&](int bpc) {
        return time_us([&] {
          if (ntl) enc_stream_wpb_kernel<8, true><<<g_cus * bpc, 512>>>(s);
          else enc_stream_wpb_kernel<8, false><<<g_cus * bpc, 512>>>(s);
        });
      };
      report(ntl ? "enc wpb4 ld-nt" : "enc wpb4", 1, r4(1), b4);
      report(ntl ? "enc wpb4 ld-nt" : "enc wpb4", 2, r4(2), b4);
      report(ntl ? "enc wpb8 ld-nt" : "enc wpb8", 1, r8(1), b8);
      report(ntl ? "enc wpb8 ld-nt" : "enc wpb8", 2, r8(2), b8);
    }
    // footprint vs wave count (nontemporal loads)
    const double b2 = double(n_obj) * (bs_real / 2048) * 2048 * (K + M);
    report("enc wpb4 ld-nt SPREAD (2x footprint, 4 waves/CU)", 1,
           time_us([&] { enc_stream_wpb_kernel<4, true, true><<<g_cus, 256>>>(s); }), b4);
    report("enc wpb4 ld-nt HALF (512 B/wave, 4 waves/CU)", 1,
           time_us([&] { enc_stream_wpb_kernel<4, true, false, true><<<g_cus, 256>>>(s); }), b2);
    report("enc wpb4 ld-nt HALF (512 B/wave, 8 waves/CU)", 2,
           time_us([&] { enc_stream_wpb_kernel<4, true, false, true><<<g_cus * 2, 256>>>(s); }), b2);
    report("enc wpb8 ld-nt HALF (512 B/wave, 8 waves/CU)", 1,
           time_us([&] { enc_stream_wpb_kernel<8, true, false, true><<<g_cus, 512>>>(s); }), b4);    const double bp = double(n_obj) * (bs_real / 2048) * 2048 * (K + M);
    for (int bpc : {1, 2, 3}) {
      report("enc pairs NP5 ld-nt (2 x 512 B per load)", bpc,
             time_us([&] { enc_pair_kernel<5, true><<<g_cus * bpc, 256>>>(s); }), bp);
      report("enc pairs NP5 (2 x 512 B per load)", bpc,
             time_us([&] { enc_pair_kernel<5, false><<<g_cus * bpc, 256>>>(s); }), bp);
      report("enc pairs NP3 ld-nt", bpc,
             time_us([&] { enc_pair_kernel<3, true><<<g_cus * bpc, 256>>>(s); }), bp);
    }
  }
  if (want(sections, "runs")) {
    for (int bpc : {2, 4}) {
      const int grid = g_cus * bpc;
      const double b1 = double(n_obj) * s.tiles * 4096 * (K + M);
      report("enc runs R1 (grid-stride)", bpc, time_us([&] { enc_stream_run_kernel<1, false><<<grid, 256>>>(s); }), b1);
      report("enc runs R2", bpc, time_us([&] { enc_stream_run_kernel<2, false><<<grid, 256>>>(s); }), b1);
      report("enc runs R4", bpc, time_us([&] { enc_stream_run_kernel<4, false><<<grid, 256>>>(s); }), b1);
      report("enc runs R8", bpc, time_us([&] { enc_stream_run_kernel<8, false><<<grid, 256>>>(s); }), b1);
      report("enc runs R16", bpc, time_us([&] { enc_stream_run_kernel<16, false><<<grid, 256>>>(s); }), b1);
      report("enc runs R32", bpc, time_us([&] { enc_stream_run_kernel<32, false><<<grid, 256>>>(s); }), b1);
      report("enc runs R8 ld-nt", bpc, time_us([&] { enc_stream_run_kernel<8, true><<<grid, 256>>>(s); }), b1);
      report("enc buf-stream block ranges (CRC order)", bpc,
             time_us([&] { enc_stream_buf_kernel<1, 5, 3, false, true><<<grid, 256>>>(s); }), b1);
    }
  }
  if (want(sections, "enc")) {
    // the 10:4 encode mix split into its halves
    check_shape("enc halves", s, 4096);
    const double rb = double(n_obj) * s.tiles * 4096 * K, wb = double(n_obj) * s.tiles * 4096 * M;
    for (int bpc : {4, 8}) {
      const int grid = g_cus * bpc;
      report("enc reads only, cached", bpc, time_us([&] { enc_half_kernel<false, 1><<<grid, 256>>>(s, sink); }), rb);
      report("enc writes only, nt", bpc, time_us([&] { enc_half_kernel<true, 2><<<grid, 256>>>(s, sink); }), wb);
    }
    // compact layout (page-locality probe)
    Shape c{objs, frags, sbs, n_compact, sbs / 4096, sobj, sfs, sss};
    check_shape("enc compact", c, 4096);
    const double cb = double(c.n_obj) * c.tiles * 4096 * (K + M);
    for (int bpc : {2, 4, 8}) {
      const int grid = g_cus * bpc;
      report("enc compact 40 KiB slices, CH1", bpc,
             time_us([&] { enc_kernel<1, false, true, false><<<grid, 256>>>(c); }), cb);
      report("enc compact 40 KiB slices, CH1 PF", bpc,
             time_us([&] { enc_kernel<1, false, true, true><<<grid, 256>>>(c); }), cb);
    }
    // chunk width per wave (CH KiB of every slice), order, store burst
    for (int bpc : {1, 2, 4, 8}) {
      const int grid = g_cus * bpc;
      Shape s1 = s, s2 = s, s4 = s;
      s2.tiles = bs_real / 8192;
      s4.tiles = bs_real / 16384;
      check_shape("CH1", s1, 4096);
      check_shape("CH2", s2, 8192);
      check_shape("CH4", s4, 16384);
      const double b1 = double(n_obj) * s1.tiles * 4096 * (K + M);
      const double b2 = double(n_obj) * s2.tiles * 8192 * (K + M);
      const double b4 = double(n_obj) * s4.tiles * 16384 * (K + M);
      report("enc CH1", bpc, time_us([&] { enc_kernel<1, false, true, false><<<grid, 256>>>(s1); }), b1);
      report("enc CH1 xcd", bpc, time_us([&] { enc_kernel<1, false, true, false, 1><<<grid, 256>>>(s1); }), b1);
      report("enc CH1 object-major", bpc, time_us([&] { enc_kernel<1, false, true, false, 2><<<grid, 256>>>(s1); }), b1);
      report("enc CH1 block ranges", bpc, time_us([&] { enc_kernel<1, false, true, false, 3><<<grid, 256>>>(s1); }), b1);
      report("enc CH1 PF", bpc, time_us([&] { enc_kernel<1, false, true, true><<<grid, 256>>>(s1); }), b1);
      report("enc CH2", bpc, time_us([&] { enc_kernel<2, false, true, false><<<grid, 256>>>(s2); }), b2);
      report("enc CH2 xcd", bpc, time_us([&] { enc_kernel<2, false, true, false, 1><<<grid, 256>>>(s2); }), b2);
      report("enc CH2 object-major", bpc, time_us([&] { enc_kernel<2, false, true, false, 2><<<grid, 256>>>(s2); }), b2);
      report("enc CH2 row-burst stores", bpc,
             time_us([&] { enc_kernel<2, false, true, false, 0, true><<<grid, 256>>>(s2); }), b2);
      report("enc CH2 ld-nt", bpc, time_us([&] { enc_kernel<2, true, true, false><<<grid, 256>>>(s2); }), b2);
      if (bpc <= 4) {
        report("enc CH2 PF", bpc, time_us([&] { enc_kernel<2, false, true, true><<<grid, 256>>>(s2); }), b2);
        report("enc CH4", bpc, time_us([&] { enc_kernel<4, false, true, false><<<grid, 256>>>(s4); }), b4);
        report("enc CH4 row-burst stores", bpc,
               time_us([&] { enc_kernel<4, false, true, false, 0, true><<<grid, 256>>>(s4); }), b4);
      }
      // the product kernel's stream shape
      report("enc stream CH1 NB5", bpc, time_us([&] { enc_stream_kernel<1, 5, 0><<<grid, 256>>>(s1); }), b1);
      report("enc stream CH1 NB5 xcd", bpc, time_us([&] { enc_stream_kernel<1, 5, 1><<<grid, 256>>>(s1); }), b1);
      report("enc stream CH1 NB5 object-major", bpc, time_us([&] { enc_stream_kernel<1, 5, 2><<<grid, 256>>>(s1); }), b1);
      report("enc stream CH1 NB5 block ranges", bpc, time_us([&] { enc_stream_kernel<1, 5, 3><<<grid, 256>>>(s1); }), b1);
      report("enc stream CH1 NB10", bpc, time_us([&] { enc_stream_kernel<1, 10, 0><<<grid, 256>>>(s1); }), b1);
      report("enc buf-stream CH1 NB5 xcd (product)", bpc,
             time_us([&] { enc_stream_buf_kernel<1, 5, 1, false, true><<<grid, 256>>>(s1); }), b1);
      report("enc buf-stream CH1 NB5 xcd no-nop", bpc,
             time_us([&] { enc_stream_buf_kernel<1, 5, 1, false, false><<<grid, 256>>>(s1); }), b1);
      report("enc buf-stream CH1 NB5 plain", bpc,
             time_us([&] { enc_stream_buf_kernel<1, 5, 0, false, true><<<grid, 256>>>(s1); }), b1);
      report("enc buf-stream CH1 NB5 xcd ld-nt", bpc,
             time_us([&] { enc_stream_buf_kernel<1, 5, 1, true, true><<<grid, 256>>>(s1); }), b1);
      report("enc buf-stream CH2 NB5 xcd ld-nt", bpc,
             time_us([&] { enc_stream_buf_kernel<2, 5, 1, true, true><<<grid, 256>>>(s2); }), b2);
      report("enc buf-stream CH2 NB10 xcd ld-nt", bpc,
             time_us([&] { enc_stream_buf_kernel<2, 10, 1, true, true><<<grid, 256>>>(s2); }), b2);
      report("enc buf-stream CH2 NB10 plain ld-nt", bpc,
             time_us([&] { enc_stream_buf_kernel<2, 10, 0, true, true><<<grid, 256>>>(s2); }), b2);
      report("enc stream CH2 NB5", bpc, time_us([&] { enc_stream_kernel<2, 5, 0><<<grid, 256>>>(s2); }), b2);
      report("enc stream CH2 NB10", bpc, time_us([&] { enc_stream_kernel<2, 10, 0><<<grid, 256>>>(s2); }), b2);
      report("enc stream CH4 NB10", bpc, time_us([&] { enc_stream_kernel<4, 10, 0><<<grid, 256>>>(s4); }), b4);
    }
    // aligned slices (isolates the 8-mod-16 slice misalignment)
    Shape a = s;
    a.bs = bs_al;
    check_shape("enc aligned", a, 4096);
    for (int bpc : {2, 8}) {
      const int grid = g_cus * bpc;
      report("enc aligned CH1", bpc, time_us([&] { enc_kernel<1, false, true, false><<<grid, 256>>>(a); }), enc_bytes);
      Shape a2 = a;
      a2.tiles = bs_real / 8192;
      report("enc aligned CH2", bpc, time_us([&] { enc_kernel<2, false, true, false><<<grid, 256>>>(a2); }),
             double(n_obj) * a2.tiles * 8192 * (K + M));
    }
  }
  if (want(sections, "dec")) {
    for (uint32_t bs : {bs_real, bs_al}) {
      Shape d{out, frags, bs, n_obj, bs_real / 4096, obj_stride, fs, ss};
      check_shape("dec", d, 4096, true);
      const double bytes = double(n_obj) * d.tiles * 4096 * (2 * K);
      for (int bpc : {2, 4, 8}) {
        const int grid = g_cus * bpc;
        report(bs == bs_al ? "dec aligned ld-nt st-nt" : "dec real    ld-nt st-nt", bpc,
               time_us([&] { dec_kernel<true, true><<<grid, 256>>>(d); }), bytes);
      }
    }
  }
  if (want(sections, "alt")) {
    // bench.py's alternating step: encode after a decode pattern (and vice
    // versa), each timed alone with events around it
    Shape d{out, frags, bs_real, n_obj, bs_real / 4096, obj_stride, fs, ss};
    Shape s2 = s;
    s2.tiles = bs_real / 8192;
    const double dec_bytes = double(n_obj) * d.tiles * 4096 * (2 * K);
    const int g8 = g_cus * 8, g2 = g_cus * 2;
    report("alt: enc CH1 after dec", 8,
           time_alt_us([&] { dec_kernel<true, true><<<g2, 256>>>(d); },
                       [&] { enc_kernel<1, false, true, false><<<g8, 256>>>(s); }), enc_bytes);
    report("alt: enc CH2 after dec", 2,
           time_alt_us([&] { dec_kernel<true, true><<<g2, 256>>>(d); },
                       [&] { enc_kernel<2, false, true, false><<<g2, 256>>>(s2); }),
           double(n_obj) * s2.tiles * 8192 * (K + M));
    report("alt: dec after enc CH1", 2,
           time_alt_us([&] { enc_kernel<1, false, true, false><<<g8, 256>>>(s); },
                       [&] { dec_kernel<true, true><<<g2, 256>>>(d); }), dec_bytes);
    report("b2b: enc CH1", 8, time_us([&] { enc_kernel<1, false, true, false><<<g8, 256>>>(s); }), enc_bytes);
    report("b2b: dec", 2, time_us([&] { dec_kernel<true, true><<<g2, 256>>>(d); }), dec_bytes);
  }
  CHECK(hipFree(objs));
  CHECK(hipFree(out));
  CHECK(hipFree(frags_raw));
  CHECK(hipFree(sink));
  return 0;
}
