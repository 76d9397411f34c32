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
//   ./membench [reps]
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
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

// ---- encode stream: item = (object, tile of 4096*CH payload positions);
// wave w of the block takes [x, x + 1024*CH) with x = tile*4096*CH + w*1024*CH.
// PF: the block's next item is loaded before this one is consumed. ----
template <int CH, bool NTL, bool NTS>
__device__ __forceinline__ void enc_load(const Shape& s, uint32_t w, v4u (&v)[K][CH]) {
  const uint32_t o = w / s.tiles, t = w - o * s.tiles;
  const uint32_t x = t * 4096 * CH + (threadIdx.x >> 6) * 1024 * CH + (threadIdx.x & 63) * 16;
  const uint8_t* src = s.objs + o * s.obj_stride + x;
#pragma unroll
  for (int j = 0; j < K; ++j)
#pragma unroll
    for (int c = 0; c < CH; ++c) v[j][c] = ld<NTL>(src + uint64_t(j) * s.bs + 1024 * c);
}
template <int CH, bool NTL, bool NTS>
__device__ __forceinline__ void enc_store(const Shape& s, uint32_t w, const v4u (&v)[K][CH]) {
  const uint32_t o = w / s.tiles, t = w - o * s.tiles;
  const uint32_t x = t * 4096 * CH + (threadIdx.x >> 6) * 1024 * CH + (threadIdx.x & 63) * 16;
  uint8_t* dst = s.frags + o * s.stripe_stride + K * s.frag_stride + 80 + x;
#pragma unroll
  for (int c = 0; c < CH; ++c) {
    v4u a = v[0][c];
#pragma unroll
    for (int j = 1; j < K; ++j) a ^= v[j][c];
#pragma unroll
    for (int r = 0; r < M; ++r) {
      st<NTS>(dst + r * s.frag_stride + 1024 * c, a);
      a.x += 1;
    }
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
      enc_load<1, NTL, true>(s, w, v);
#pragma unroll
      for (int j = 0; j < K; ++j) acc ^= v[j][0].x ^ v[j][0].y ^ v[j][0].z ^ v[j][0].w;
    } else {
#pragma unroll
      for (int j = 0; j < K; ++j) v[j][0] = v4u{w, uint32_t(j), 0u, 1u};
      enc_store<1, NTL, true>(s, w, v);
    }
  }
  if (acc == 0x12345678u) sink[0] = acc;
}

template <int CH, bool NTL, bool NTS, bool PF>
__global__ void __launch_bounds__(256) enc_kernel(Shape s) {
  const uint32_t items = s.n_obj * s.tiles;
  if constexpr (!PF) {
    for (uint32_t w = blockIdx.x; w < items; w += gridDim.x) {
      v4u v[K][CH];
      enc_load<CH, NTL, NTS>(s, w, v);
      enc_store<CH, NTL, NTS>(s, w, v);
    }
  } else {
    uint32_t w = blockIdx.x;
    if (w >= items) return;
    v4u a[K][CH], b[K][CH];
    enc_load<CH, NTL, NTS>(s, w, a);
    while (true) {
      uint32_t wn = w + gridDim.x < items ? w + gridDim.x : w;
      enc_load<CH, NTL, NTS>(s, wn, b);
      enc_store<CH, NTL, NTS>(s, w, a);
      if (wn == w) break;
      w = wn;
      wn = w + gridDim.x < items ? w + gridDim.x : w;
      enc_load<CH, NTL, NTS>(s, wn, a);
      enc_store<CH, NTL, NTS>(s, w, b);
      if (wn == w) break;
      w = wn;
    }
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
  CHECK(hipEventRecord(e0, 0));
  for (int i = 0; i < g_reps; ++i) launch();
  CHECK(hipEventRecord(e1, 0));
  CHECK(hipEventSynchronize(e1));
  float ms = 0;
  CHECK(hipEventElapsedTime(&ms, e0, e1));
  CHECK(hipGetLastError());
  return ms * 1e3 / g_reps;
}

void report(const char* name, int bpc, double us, double bytes) {
  std::printf("%-44s bpc=%d %9.1f us %8.1f GB/s\n", name, bpc, us, bytes / us / 1e3);
  std::fflush(stdout);
}

}  // namespace

int main(int argc, char** argv) {
  if (argc > 1) g_reps = std::atoi(argv[1]);
  int dev = 0;
  CHECK(hipGetDevice(&dev));
  CHECK(hipDeviceGetAttribute(&g_cus, hipDeviceAttributeMultiprocessorCount, dev));
  const uint32_t n_obj = 256, L = 4u << 20;
  const uint32_t bs_real = 2 * ((L + 2 * K - 1) / (2 * K));  // 419432
  const uint32_t bs_al = (bs_real + 127) / 128 * 128;        // 419456
  const uint64_t obj_stride = L;
  const uint64_t fs = ((80 + (bs_al + 15) / 16 * 16) + 127) / 128 * 128;
  const uint64_t ss = fs * (K + M);
  const uint64_t obj_bytes = obj_stride * n_obj + (1 << 20);
  const uint64_t frag_bytes = ss * n_obj + (1 << 20);
  uint8_t *objs, *frags_raw, *out;
  uint32_t* sink;
  CHECK(hipMalloc(&objs, obj_bytes));
  CHECK(hipMalloc(&out, obj_bytes));
  CHECK(hipMalloc(&frags_raw, frag_bytes));
  CHECK(hipMalloc(&sink, 64));
  CHECK(hipMemset(objs, 1, obj_bytes));
  CHECK(hipMemset(out, 0, obj_bytes));
  CHECK(hipMemset(frags_raw, 2, frag_bytes));
  uint8_t* frags = frags_raw + 48;  // payloads (80 B past each fragment start) 128-B aligned
  std::printf("CUs %d, reps %d, bs %u / aligned %u, frag_stride %llu\n", g_cus, g_reps, bs_real,
              bs_al, (unsigned long long)fs);

  const uint64_t n_copy = uint64_t(n_obj) * L;
  for (int bpc : {2, 4, 8}) {
    const int grid = g_cus * bpc;
    report("copy 1 GiB, 16 B/lane, cached", bpc,
           time_us([&] { copy_kernel<1, false><<<grid, 256>>>(objs, out, n_copy); }), 2.0 * n_copy);
    report("copy 1 GiB, 16 B/lane, nt", bpc,
           time_us([&] { copy_kernel<1, true><<<grid, 256>>>(objs, out, n_copy); }), 2.0 * n_copy);
    report("copy 1 GiB, 2x16 B/lane, nt", bpc,
           time_us([&] { copy_kernel<2, true><<<grid, 256>>>(objs, out, n_copy); }), 2.0 * n_copy);
    report("read 1 GiB, 16 B/lane, nt", bpc,
           time_us([&] { read_kernel<1, true><<<grid, 256>>>(objs, n_copy, sink); }), 1.0 * n_copy);
    report("read 1 GiB, 4x16 B/lane, cached", bpc,
           time_us([&] { read_kernel<4, false><<<grid, 256>>>(objs, n_copy, sink); }), 1.0 * n_copy);
  }
  {
    // split the 10:4 encode mix into its halves, and a compact layout (many
    // small objects: 10 slices of 40 KiB, same bytes) to test page locality
    Shape s{objs, frags, bs_real, n_obj, bs_real / 4096, obj_stride, fs, ss};
    double rb = double(n_obj) * s.tiles * 4096 * K, wb = double(n_obj) * s.tiles * 4096 * M;
    for (int bpc : {4, 8}) {
      const int grid = g_cus * bpc;
      report("enc reads only, cached", bpc, time_us([&] { enc_half_kernel<false, 1><<<grid, 256>>>(s, sink); }), rb);
      report("enc reads only, nt", bpc, time_us([&] { enc_half_kernel<true, 1><<<grid, 256>>>(s, sink); }), rb);
      report("enc writes only, nt", bpc, time_us([&] { enc_half_kernel<true, 2><<<grid, 256>>>(s, sink); }), wb);
      const uint32_t sbs = 40960, sobj = 10 * sbs, sfs = sbs + 128;
      Shape c{objs, frags, sbs, uint32_t(uint64_t(n_obj) * obj_stride / sobj), sbs / 4096, sobj, sfs, uint64_t(sfs) * (K + M)};
      const double cb = double(c.n_obj) * c.tiles * 4096 * (K + M);
      report("enc compact 40 KiB slices, ld-cached st-nt PF", bpc,
             time_us([&] { enc_kernel<1, false, true, true><<<grid, 256>>>(c); }), cb);
    }
  }
  for (uint32_t bs : {bs_real, bs_al}) {
    Shape s{objs, frags, bs, n_obj, 0, obj_stride, fs, ss};
    const bool al = bs == bs_al;
    char name[128];
    for (int bpc : {2, 4, 8}) {
      const int grid = g_cus * bpc;
      s.tiles = bs_real / 4096;
      double bytes = double(n_obj) * s.tiles * 4096 * (K + M);
      std::snprintf(name, sizeof name, "enc %s ld-cached st-nt", al ? "aligned" : "real   ");
      report(name, bpc, time_us([&] { enc_kernel<1, false, true, false><<<grid, 256>>>(s); }), bytes);
      std::snprintf(name, sizeof name, "enc %s ld-cached st-nt PF", al ? "aligned" : "real   ");
      report(name, bpc, time_us([&] { enc_kernel<1, false, true, true><<<grid, 256>>>(s); }), bytes);
      std::snprintf(name, sizeof name, "enc %s ld-nt st-nt PF", al ? "aligned" : "real   ");
      report(name, bpc, time_us([&] { enc_kernel<1, true, true, true><<<grid, 256>>>(s); }), bytes);
      std::snprintf(name, sizeof name, "enc %s ld-cached st-cached PF", al ? "aligned" : "real   ");
      report(name, bpc, time_us([&] { enc_kernel<1, false, false, true><<<grid, 256>>>(s); }), bytes);
      s.tiles = bs_real / 8192;
      bytes = double(n_obj) * s.tiles * 8192 * (K + M);
      std::snprintf(name, sizeof name, "enc %s ld-cached st-nt CH2", al ? "aligned" : "real   ");
      report(name, bpc, time_us([&] { enc_kernel<2, false, true, false><<<grid, 256>>>(s); }), bytes);
      s.tiles = bs_real / 4096;
      bytes = double(n_obj) * s.tiles * 4096 * (2 * K);
      std::snprintf(name, sizeof name, "dec %s ld-nt st-nt", al ? "aligned" : "real   ");
      Shape d = s;
      d.objs = out;
      report(name, bpc, time_us([&] { dec_kernel<true, true><<<grid, 256>>>(d); }), bytes);
      std::snprintf(name, sizeof name, "dec %s ld-nt st-cached", al ? "aligned" : "real   ");
      report(name, bpc, time_us([&] { dec_kernel<true, false><<<grid, 256>>>(d); }), bytes);
      std::snprintf(name, sizeof name, "dec %s ld-cached st-cached", al ? "aligned" : "real   ");
      report(name, bpc, time_us([&] { dec_kernel<false, false><<<grid, 256>>>(d); }), bytes);
    }
  }
  return 0;
}
