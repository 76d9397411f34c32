// Microbenchmark for the encode hot loop: separates the memory stream from
// the LDS/VALU work.  Not part of the product; built by `make -C tools`.
//
//   stream   : same loads/stores as encode (K x 16 B strided by bs, R x 16 B
//              out per lane), XOR instead of GF products      -> HBM roof
//   compute  : GF products on register data, no HBM traffic   -> LDS/VALU roof
//   full     : the product encode kernel (via launch_encode)
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <algorithm>
#include <vector>

#include "../pyeclib_amd/csrc/ec_kernels.hip"

using namespace ecamd;

namespace {

template <int K>
__global__ void __launch_bounds__(256) stream_kernel(const uint8_t* objs, uint8_t* par,
                                                     uint32_t bs, uint32_t n_obj,
                                                     uint64_t obj_stride, uint64_t frag_stride,
                                                     uint32_t tiles) {
  const uint32_t items = n_obj * tiles;
  for (uint32_t w = blockIdx.x; w < items; w += gridDim.x) {
    const uint32_t o = w / tiles, tile = w % tiles;
    const uint32_t t = (tile * 256 + threadIdx.x) * 16;
    const uint8_t* src = objs + o * obj_stride + t;
    uint4 acc = make_uint4(0, 0, 0, 0);
    uint4 x[K];
#pragma unroll
    for (int j = 0; j < K; ++j) x[j] = *reinterpret_cast<const uint4*>(src + uint64_t(j) * bs);
#pragma unroll
    for (int j = 0; j < K; ++j) {
      acc.x ^= x[j].x; acc.y ^= x[j].y; acc.z ^= x[j].z; acc.w ^= x[j].w;
    }
    uint8_t* dst = par + o * 4 * frag_stride + 80 + t;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      *reinterpret_cast<uint4*>(dst + r * frag_stride) = acc;
      acc.x += 1;
    }
  }
}

// Variants of the encode memory stream.  C = 16-B chunks per lane per input
// (adjacent), CONTIG = contiguous item ranges per workgroup (else grid
// stride), NT = nontemporal loads/stores.
template <int K, int C, bool CONTIG, bool NT, bool NTS = NT>
__global__ void __launch_bounds__(256) stream2_kernel(const uint8_t* objs, uint8_t* par,
                                                      uint32_t bs, uint32_t n_obj,
                                                      uint64_t obj_stride, uint64_t frag_stride,
                                                      uint32_t tiles, uint32_t out_off) {
  const uint32_t items = n_obj * tiles;
  const uint32_t per = (items + gridDim.x - 1) / gridDim.x;
  const uint32_t b0 = CONTIG ? blockIdx.x * per : blockIdx.x;
  const uint32_t b1 = CONTIG ? min(items, b0 + per) : items;
  const uint32_t st = CONTIG ? 1 : gridDim.x;
  for (uint32_t w = b0; w < b1; w += st) {
    const uint32_t o = w / tiles, tile = w % tiles;
    const uint32_t t = (tile * 256 * C + threadIdx.x * C) * 16;
    const uint8_t* src = objs + o * obj_stride + t;
    uint4 x[K][C];
#pragma unroll
    for (int j = 0; j < K; ++j)
#pragma unroll
      for (int c = 0; c < C; ++c) {
        const uint4* a = reinterpret_cast<const uint4*>(src + uint64_t(j) * bs + c * 16);
        if constexpr (NT) {
          x[j][c].x = __builtin_nontemporal_load(&a->x);
          x[j][c].y = __builtin_nontemporal_load(&a->y);
          x[j][c].z = __builtin_nontemporal_load(&a->z);
          x[j][c].w = __builtin_nontemporal_load(&a->w);
        } else {
          x[j][c] = *a;
        }
      }
    uint8_t* dst = par + o * 4 * frag_stride + out_off + t;
#pragma unroll
    for (int c = 0; c < C; ++c) {
      uint4 acc = make_uint4(0, 0, 0, 0);
#pragma unroll
      for (int j = 0; j < K; ++j) {
        acc.x ^= x[j][c].x; acc.y ^= x[j][c].y; acc.z ^= x[j][c].z; acc.w ^= x[j][c].w;
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        uint4* d = reinterpret_cast<uint4*>(dst + r * frag_stride + c * 16);
        if constexpr (NTS) {
          __builtin_nontemporal_store(acc.x, &d->x);
          __builtin_nontemporal_store(acc.y, &d->y);
          __builtin_nontemporal_store(acc.z, &d->z);
          __builtin_nontemporal_store(acc.w, &d->w);
        } else {
          *d = acc;
        }
        acc.x += 1;
      }
    }
  }
}

// Decode memory pattern: K aligned fragment payload reads -> K object slices.
template <int K, bool NT>
__global__ void __launch_bounds__(256) dstream_kernel(const uint8_t* frags, uint8_t* objs,
                                                      uint32_t bs, uint32_t n_obj,
                                                      uint64_t obj_stride, uint64_t fs,
                                                      uint32_t tiles) {
  const uint32_t items = n_obj * tiles;
  for (uint32_t w = blockIdx.x; w < items; w += gridDim.x) {
    const uint32_t o = w / tiles, tile = w % tiles;
    const uint32_t t = (tile * 256 + threadIdx.x) * 16;
    const uint8_t* src = frags + o * (K + 4) * fs + 128 + t;
    uint4 x[K];
#pragma unroll
    for (int j = 0; j < K; ++j) {
      const uint4* a = reinterpret_cast<const uint4*>(src + j * fs);
      if constexpr (NT) x[j] = ld_stream(a); else x[j] = *a;
    }
    uint8_t* dst = objs + o * obj_stride + t;
#pragma unroll
    for (int j = 0; j < K; ++j) {
      uint4* d = reinterpret_cast<uint4*>(dst + uint64_t(j) * bs);
      if constexpr (NT) st_stream(d, x[j]); else *d = x[j];
    }
  }
}

// Same pattern with the copy realigned on the load side: each lane loads
// fragment j at payload offset t - delta_j (unaligned) so that its store to
// the object lands on a 16-B boundary and every wave writes whole lines.
template <int K, bool NT, uint32_t MASK = 127>
__global__ void __launch_bounds__(256) dstream_shift_kernel(const uint8_t* frags, uint8_t* objs,
                                                            uint32_t bs, uint32_t n_obj,
                                                            uint64_t obj_stride, uint64_t fs,
                                                            uint32_t tiles) {
  const uint32_t items = n_obj * tiles;
  for (uint32_t w = blockIdx.x; w < items; w += gridDim.x) {
    const uint32_t o = w / tiles, tile = w % tiles;
    const uint32_t t = (tile * 256 + threadIdx.x) * 16;
    const uint8_t* src = frags + o * (K + 4) * fs + 128 + t;
    uint4 x[K];
#pragma unroll
    for (int j = 0; j < K; ++j) {
      const uint32_t delta = (j * bs) & MASK;
      const uint4* a = reinterpret_cast<const uint4*>(src + j * fs - delta);
      if constexpr (NT) x[j] = ld_stream(a); else x[j] = *a;
    }
    uint8_t* dst = objs + o * obj_stride + t;
#pragma unroll
    for (int j = 0; j < K; ++j) {
      const uint32_t delta = (j * bs) & MASK;
      uint4* d = reinterpret_cast<uint4*>(dst + uint64_t(j) * bs - delta);
      if constexpr (NT) st_stream(d, x[j]); else *d = x[j];
    }
  }
}

// Aligned loads; the copy is re-aligned to 16 B in registers: lane L's
// store chunk takes its low r bytes from lane L-1 (DPP wave_shr:1) and the
// rest from itself, so every store is a 16-B aligned dwordx4 except one
// partial chunk at each end of the wave's 1 KiB span.
__device__ __forceinline__ uint32_t wave_shr1(uint32_t v) {
  return static_cast<uint32_t>(__builtin_amdgcn_update_dpp(0, static_cast<int>(v), 0x138, 0xF, 0xF, false));
}
__device__ __forceinline__ uint4 funnel16(const uint4& prev, const uint4& own, uint32_t r) {
  // bytes [16 - r, 32 - r) of prev||own, r even in [2, 14]
  const uint32_t w[8] = {prev.x, prev.y, prev.z, prev.w, own.x, own.y, own.z, own.w};
  const uint32_t q = (16 - r) >> 2, b = (16 - r) & 3;
  uint32_t o[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    uint32_t lo = w[i], hi = w[i + 1];
    if (q == 1) { lo = w[i + 1]; hi = w[i + 2]; }
    if (q == 2) { lo = w[i + 2]; hi = w[i + 3]; }
    if (q == 3) { lo = w[i + 3]; hi = w[i + 4]; }
    o[i] = __builtin_amdgcn_alignbyte(hi, lo, b);
  }
  return make_uint4(o[0], o[1], o[2], o[3]);
}
template <int K>
__global__ void __launch_bounds__(256) dstream_dpp_kernel(const uint8_t* frags, uint8_t* objs,
                                                          uint32_t bs, uint32_t n_obj,
                                                          uint64_t obj_stride, uint64_t fs,
                                                          uint32_t tiles) {
  const uint32_t items = n_obj * tiles;
  const uint32_t lane = threadIdx.x & 63;
  for (uint32_t w = blockIdx.x; w < items; w += gridDim.x) {
    const uint32_t o = w / tiles, tile = w % tiles;
    const uint32_t t = (tile * 256 + threadIdx.x) * 16;
    const uint8_t* src = frags + o * (K + 4) * fs + 128 + t;
    uint4 x[K];
#pragma unroll
    for (int j = 0; j < K; ++j) x[j] = ld_stream(src + j * fs);
    uint8_t* dst = objs + o * obj_stride + t;
#pragma unroll
    for (int j = 0; j < K; ++j) {
      uint8_t* d = dst + uint64_t(j) * bs;
      const uint32_t r = static_cast<uint32_t>(reinterpret_cast<uintptr_t>(d) & 15u);
      if (r == 0) { st_stream(d, x[j]); continue; }
      const uint4 prev = make_uint4(wave_shr1(x[j].x), wave_shr1(x[j].y), wave_shr1(x[j].z),
                                    wave_shr1(x[j].w));
      const uint4 v = funnel16(prev, x[j], r);
      uint8_t* a = d - r;
      if (lane != 0) {
        st_stream(a, v);
      } else {
        const uint32_t wv[4] = {v.x, v.y, v.z, v.w};
        for (uint32_t i = r; i < 16; ++i) a[i] = static_cast<uint8_t>(wv[i >> 2] >> (8 * (i & 3)));
      }
      if (lane == 63) {
        const uint32_t wv[4] = {x[j].x, x[j].y, x[j].z, x[j].w};
        for (uint32_t i = 16 - r; i < 16; ++i) a[i + 16] = static_cast<uint8_t>(wv[i >> 2] >> (8 * (i & 3)));
      }
    }
  }
}

// Decode-shaped mix: K aligned loads (nt or cached), E rebuilt rows (XOR of
// all inputs) stored at their natural unaligned offsets, K-E copies either
// stored unaligned from the aligned loads (SHIFT=false) or re-loaded at the
// object's line phase (cached load, hopefully from L2) and stored aligned.
template <int K, int E, bool LNT, bool SHIFT>
__global__ void __launch_bounds__(256) dmix_kernel(const uint8_t* frags, uint8_t* objs,
                                                   uint32_t bs, uint32_t n_obj,
                                                   uint64_t obj_stride, uint64_t fs,
                                                   uint32_t tiles) {
  const uint32_t items = n_obj * tiles;
  for (uint32_t w = blockIdx.x; w < items; w += gridDim.x) {
    const uint32_t o = w / tiles, tile = w % tiles;
    const uint32_t t = (tile * 256 + threadIdx.x) * 16;
    const uint8_t* src = frags + o * (K + 4) * fs + 128 + t;
    uint4 x[K];
#pragma unroll
    for (int j = 0; j < K; ++j) {
      if constexpr (LNT) x[j] = ld_stream(src + j * fs);
      else x[j] = *reinterpret_cast<const uint4*>(src + j * fs);
    }
    uint4 acc = make_uint4(0, 0, 0, 0);
#pragma unroll
    for (int j = 0; j < K; ++j) {
      acc.x ^= x[j].x; acc.y ^= x[j].y; acc.z ^= x[j].z; acc.w ^= x[j].w;
    }
    uint8_t* dst = objs + o * obj_stride + t;
#pragma unroll
    for (int j = 0; j < E; ++j) {
      acc.x += j;
      st_stream(dst + uint64_t(j) * bs, acc);
    }
#pragma unroll
    for (int j = E; j < K; ++j) {
      if constexpr (SHIFT) {
        const uint32_t delta = (j * bs) & 127u;
        const uint4 v = *reinterpret_cast<const uint4*>(src + j * fs - delta);
        st_stream(dst + uint64_t(j) * bs - delta, v);
      } else {
        st_stream(dst + uint64_t(j) * bs, x[j]);
      }
    }
  }
}

// Reference streams: plain 16 B/lane copy and read-only sweep.
__global__ void __launch_bounds__(256) copy_kernel(const uint4* src, uint4* dst, uint64_t n) {
  for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += uint64_t(gridDim.x) * 256)
    dst[i] = src[i];
}
__global__ void __launch_bounds__(256) read_kernel(const uint4* src, uint64_t n, uint32_t* sink) {
  uint32_t acc = 0;
  for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += uint64_t(gridDim.x) * 256) {
    const uint4 v = src[i];
    acc ^= v.x ^ v.y ^ v.z ^ v.w;
  }
  if (acc == 0x9E3779B9u) sink[0] = acc;
}

template <int K>
__global__ void __launch_bounds__(256) compute_kernel(const uint64_t* tables, uint8_t* sink,
                                                      uint32_t iters) {
  load_tables(tables, K);
  __syncthreads();
  uint4 x[K];
#pragma unroll
  for (int j = 0; j < K; ++j)
    x[j] = make_uint4(threadIdx.x * 2654435761u + j, blockIdx.x ^ (j << 7), threadIdx.x + j * 77,
                      blockIdx.x * 31 + j);
  uint2 s[8];
  for (int i = 0; i < 8; ++i) s[i] = make_uint2(0, 0);
  for (uint32_t it = 0; it < iters; ++it) {
#pragma unroll
    for (int j = 0; j < K; ++j)  // opaque inputs: nothing hoists out of the loop
      asm volatile("" : "+v"(x[j].x), "+v"(x[j].y), "+v"(x[j].z), "+v"(x[j].w));
#pragma unroll
    for (int j = 0; j < K; ++j) mac_chunk<2>(j * kTableBytesPerInput, x[j], s);
    pin(s);
  }
  uint32_t v = 0;
  for (int i = 0; i < 8; ++i) v ^= s[i].x ^ s[i].y;
  if (v == 0x12345678u) sink[threadIdx.x] = 1;
}

#define CHECK(x)                                                          \
  do {                                                                    \
    hipError_t e_ = (x);                                                  \
    if (e_ != hipSuccess) {                                               \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      std::exit(1);                                                       \
    }                                                                     \
  } while (0)

template <typename F>
float time_ms(F f, int reps) {
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a));
  CHECK(hipEventCreate(&b));
  f();
  CHECK(hipDeviceSynchronize());
  CHECK(hipEventRecord(a));
  for (int i = 0; i < reps; ++i) f();
  CHECK(hipEventRecord(b));
  CHECK(hipEventSynchronize(b));
  float ms = 0;
  CHECK(hipEventElapsedTime(&ms, a, b));
  return ms / reps;
}

}  // namespace

int main(int argc, char** argv) {
  constexpr int K = 10;
  const int m = 4;
  const uint32_t n_obj = argc > 1 ? std::atoi(argv[1]) : 256;
  const uint64_t L = argc > 2 ? std::atoll(argv[2]) : (4u << 20);
  const uint32_t bs = static_cast<uint32_t>(((L + 2 * K - 1) / (2 * K)) * 2);
  const uint64_t obj_stride = (L + 255) / 256 * 256;
  const uint64_t fs = ((80 + (bs + 15) / 16 * 16) + 15) / 16 * 16;
  uint8_t *objs, *par;
  uint64_t* tables;
  CHECK(hipMalloc(&objs, n_obj * obj_stride));
  CHECK(hipMalloc(&par, n_obj * m * fs));
  CHECK(hipMalloc(&tables, K * 64 * 8));
  std::vector<uint64_t> ht(K * 64);
  for (size_t i = 0; i < ht.size(); ++i) ht[i] = i * 0x9E3779B97F4A7C15ull;
  CHECK(hipMemcpy(tables, ht.data(), ht.size() * 8, hipMemcpyHostToDevice));
  CHECK(hipMemset(objs, 7, n_obj * obj_stride));

  const double bytes = double(n_obj) * (L + m * (bs + 80.0));
  const uint32_t tiles = (bs / 16) / 256;  // interior tiles only
  int cus = 256;
  CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  const char* mode = argc > 3 ? argv[3] : "all";
  auto want = [&](const char* m) { return !std::strcmp(mode, "all") || !std::strcmp(mode, m); };
  if (want("copy")) {
    const uint64_t n16 = n_obj * obj_stride / 16;
    const uint64_t ncopy = std::min<uint64_t>(n16, n_obj * m * fs / 16);
    const uint4* src4 = reinterpret_cast<const uint4*>(objs);
    uint4* dst4 = reinterpret_cast<uint4*>(par);
    uint32_t* sink = reinterpret_cast<uint32_t*>(par);
    for (int per_cu : {4, 8}) {
      const dim3 grid(cus * per_cu);
      float ms = time_ms([&] {
        hipLaunchKernelGGL(copy_kernel, grid, dim3(256), 0, 0, src4, dst4, ncopy);
      }, 20);
      const double b = 2.0 * ncopy * 16;
      std::printf("copy    grid=%d/CU  %.1f us  %.1f GB/s\n", per_cu, ms * 1e3, b / (ms * 1e-3) / 1e9);
      ms = time_ms([&] {
        hipLaunchKernelGGL(read_kernel, grid, dim3(256), 0, 0, src4, n16, sink);
      }, 20);
      std::printf("read    grid=%d/CU  %.1f us  %.1f GB/s\n", per_cu, ms * 1e3,
                  n16 * 16.0 / (ms * 1e-3) / 1e9);
    }
  }
  for (int per_cu : {2, 4, 8}) {
    if (!want("stream")) break;
    float ms = time_ms([&] {
      hipLaunchKernelGGL(stream_kernel<K>, dim3(cus * per_cu), dim3(256), 0, 0, objs, par, bs,
                         n_obj, obj_stride, fs, tiles);
    }, 20);
    std::printf("stream  grid=%d/CU  %.1f us  %.1f GB/s\n", per_cu, ms * 1e3,
                bytes / (ms * 1e-3) / 1e9);
  }
  // compute: same number of (input chunk x table) MACs as one encode batch
  const uint64_t chunks = uint64_t(n_obj) * tiles * 256;  // lane-chunks of 16 B per input
  if (want("dstream")) {
    const uint64_t fsd = (128 + (bs + 15) / 16 * 16 + 127) / 128 * 128;
    uint8_t* frags;
    CHECK(hipMalloc(&frags, n_obj * (K + 4) * fsd + 256));
    const uint32_t tl = (bs / 16) / 256;
    const double db = double(n_obj) * (2.0 * K * bs);
    for (int per_cu : {4, 8}) {
      const dim3 grid(cus * per_cu);
      float ms = time_ms([&] {
        hipLaunchKernelGGL((dstream_kernel<K, true>), grid, dim3(256), 0, 0, frags, objs, bs,
                           n_obj, obj_stride, fsd, tl);
      }, 20);
      std::printf("dstream nt grid=%d/CU %.1f us %.1f GB/s\n", per_cu, ms * 1e3, db / (ms * 1e-3) / 1e9);
      ms = time_ms([&] {
        hipLaunchKernelGGL((dstream_kernel<K, false>), grid, dim3(256), 0, 0, frags, objs, bs,
                           n_obj, obj_stride, fsd, tl);
      }, 20);
      std::printf("dstream    grid=%d/CU %.1f us %.1f GB/s\n", per_cu, ms * 1e3, db / (ms * 1e-3) / 1e9);
      ms = time_ms([&] {
        hipLaunchKernelGGL((dstream_shift_kernel<K, true>), grid, dim3(256), 0, 0, frags, objs,
                           bs, n_obj, obj_stride, fsd, tl);
      }, 20);
      std::printf("dshift nt  grid=%d/CU %.1f us %.1f GB/s\n", per_cu, ms * 1e3, db / (ms * 1e-3) / 1e9);
      ms = time_ms([&] {
        hipLaunchKernelGGL((dstream_shift_kernel<K, true, 15>), grid, dim3(256), 0, 0, frags, objs,
                           bs, n_obj, obj_stride, fsd, tl);
      }, 20);
      std::printf("dshift16nt grid=%d/CU %.1f us %.1f GB/s\n", per_cu, ms * 1e3, db / (ms * 1e-3) / 1e9);
      ms = time_ms([&] {
        hipLaunchKernelGGL((dstream_dpp_kernel<K>), grid, dim3(256), 0, 0, frags, objs,
                           bs, n_obj, obj_stride, fsd, tl);
      }, 20);
      std::printf("ddpp nt    grid=%d/CU %.1f us %.1f GB/s\n", per_cu, ms * 1e3, db / (ms * 1e-3) / 1e9);
#define MIX(LNT, SH, NAME)                                                                  \
      ms = time_ms([&] {                                                                    \
        hipLaunchKernelGGL((dmix_kernel<K, 3, LNT, SH>), grid, dim3(256), 0, 0, frags, objs, \
                           bs, n_obj, obj_stride, fsd, tl);                                 \
      }, 20);                                                                               \
      std::printf(NAME "  grid=%d/CU %.1f us %.1f GB/s\n", per_cu, ms * 1e3, db / (ms * 1e-3) / 1e9);
      MIX(true, false, "mix nt plain ")
      MIX(false, false, "mix c  plain ")
      MIX(true, true, "mix nt shift ")
      MIX(false, true, "mix c  shift ")
      ms = time_ms([&] {
        hipLaunchKernelGGL((dstream_shift_kernel<K, false>), grid, dim3(256), 0, 0, frags, objs,
                           bs, n_obj, obj_stride, fsd, tl);
      }, 20);
      std::printf("dshift     grid=%d/CU %.1f us %.1f GB/s\n", per_cu, ms * 1e3, db / (ms * 1e-3) / 1e9);
    }
  }
  if (want("stream2")) {
    const uint64_t fs2 = (fs + 255) / 256 * 256;
    auto run = [&](auto kern, int C, const char* name, uint32_t off, int per_cu) {
      const uint32_t tl = (bs / 16) / (256 * C);
      const dim3 grid(cus * per_cu);
      float ms = time_ms([&] {
        hipLaunchKernelGGL(kern, grid, dim3(256), 0, 0, objs, par, bs, n_obj, obj_stride, fs2, tl,
                           off);
      }, 20);
      std::printf("stream2 %-22s off=%3u grid=%d/CU %.1f us %.1f GB/s\n", name, off, per_cu,
                  ms * 1e3, bytes / (ms * 1e-3) / 1e9);
    };
    for (int pc : {4, 8}) {
      run(stream2_kernel<K, 1, false, false, true>, 1, "C1 stride nt-store", 128, pc);
      run(stream2_kernel<K, 1, false, true, false>, 1, "C1 stride nt-load", 128, pc);
      run(stream2_kernel<K, 1, false, true, true>, 1, "C1 stride nt", 128, pc);
      run(stream2_kernel<K, 2, false, true, true>, 2, "C2 stride nt", 128, pc);
      run(stream2_kernel<K, 2, false, false, true>, 2, "C2 stride nt-store", 128, pc);
    }
    for (int pc : {4, 8}) {
      if (!std::getenv("MB_ALL")) break;
      for (uint32_t off : {80u, 128u}) {
        run(stream2_kernel<K, 1, false, false>, 1, "C1 stride", off, pc);
        run(stream2_kernel<K, 1, true, false>, 1, "C1 contig", off, pc);
        run(stream2_kernel<K, 2, false, false>, 2, "C2 stride", off, pc);
        run(stream2_kernel<K, 2, true, false>, 2, "C2 contig", off, pc);
        run(stream2_kernel<K, 1, false, true>, 1, "C1 stride nt", off, pc);
        run(stream2_kernel<K, 1, true, true>, 1, "C1 contig nt", off, pc);
        run(stream2_kernel<K, 2, true, true>, 2, "C2 contig nt", off, pc);
      }
    }
  }
  for (int per_cu : {4, 8}) {
    if (!want("compute")) break;
    const uint32_t blocks = cus * per_cu;
    const uint32_t iters = static_cast<uint32_t>(chunks / (uint64_t(blocks) * 256));
    float ms = time_ms([&] {
      hipLaunchKernelGGL(compute_kernel<K>, dim3(blocks), dim3(256), K * 512, 0, tables, par,
                         iters);
    }, 10);
    std::printf("compute grid=%d/CU  %.1f us  (%u iters)\n", per_cu, ms * 1e3, iters);
  }
  EncodeParams p{};
  p.objs = objs;
  p.obj_stride = obj_stride;
  p.obj_len = L;
  p.parity = par;
  p.frag_stride = fs;
  p.stripe_stride = m * fs;
  p.tables = tables;
  p.k = K;
  p.m = m;
  p.row0 = 0;
  p.nrows = m;
  p.bs = bs;
  p.n_obj = n_obj;
  if (!want("full")) return 0;
  float ms = time_ms([&] { CHECK(launch_encode(p, 0)); }, 20);
  std::printf("full encode  payload%%128=80  %.1f us  %.1f GB/s\n", ms * 1e3, bytes / (ms * 1e-3) / 1e9);
  // line-aligned payloads: fragment slots start 48 B into 256-B-aligned slots
  const uint64_t fs_al = (80 + (bs + 15) / 16 * 16 + 48 + 255) / 256 * 256;
  uint8_t* par2;
  CHECK(hipMalloc(&par2, n_obj * m * fs_al + 256));
  p.parity = par2 + 48;
  p.frag_stride = fs_al;
  p.stripe_stride = m * fs_al;
  ms = time_ms([&] { CHECK(launch_encode(p, 0)); }, 20);
  std::printf("full encode  payload%%128=0   %.1f us  %.1f GB/s\n", ms * 1e3, bytes / (ms * 1e-3) / 1e9);
  return 0;
}
