// libpyeclib_amd.so: liberasurecode-shaped C ABI over the gfx950 kernels.
//
// Part 1 restates, entry point by entry point, what pyeclib's C binding
// expects from liberasurecode 1.8.0 (call sites in src/pyeclib_c/pyeclib_c.c,
// cited per function in include/erasurecode_amd.h): fragment layout and
// padding (upstream erasurecode_preprocessing.c), 80-byte headers and
// checksums (erasurecode_helpers.c), the decode fast path and partitioning
// (erasurecode.c), and the rs_vand backend's choice of the first k available
// fragments (liberasurecode_rs_vand.c).  The GF(2^16) region products -- the
// only data-proportional arithmetic -- run on the GPU; there is no CPU
// implementation of them in this library.
//
// Part 2 (ecamd_*) is the batched device-resident API used for throughput.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <cerrno>
#include <cstdlib>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <unordered_map>
#include <vector>

#include "crc32.hpp"
#include "ec_crc.hpp"
#include "ec_kernels.hpp"
#include "erasurecode_amd.h"
#include "gf16.hpp"
#include "gf8.hpp"

namespace ecamd {
namespace {

constexpr uint32_t kLibecVersion = 0x010800;  // fragment format written (1.8.0)

// What a backend id means here: the id written into fragment headers, the
// backend version stamped next to it ((major << 16) | (minor << 8) | rev, as
// liberasurecode's backends declare it) and the field width.  amd_rs_vand (11)
// writes liberasurecode_rs_vand's bytes, id 6 included, so the two ec_types
// read each other's fragments.  The ISA-L versions are UNPINNED (ISA-L's
// liberasurecode backends are not in this container; DESIGN.md, Oracle).
struct Code {
  uint8_t wire_id;
  uint32_t version;
  int w;
};
constexpr Code kRsVand{EC_BACKEND_LIBERASURECODE_RS_VAND, 0x00010000, 16};  // rs_vand 1.0.0
constexpr Code kIsalVand{EC_BACKEND_ISA_L_RS_VAND, 0x00020D00, 8};          // isa_l_rs_vand 2.13.0
constexpr Code kIsalCauchy{EC_BACKEND_ISA_L_RS_CAUCHY, 0x00020E01, 8};      // isa_l_rs_cauchy 2.14.1

const Code* code_of(int backend_id) {
  switch (backend_id) {
    case EC_BACKEND_LIBERASURECODE_RS_VAND:
    case EC_BACKEND_AMD_RS_VAND:
      return &kRsVand;
    case EC_BACKEND_ISA_L_RS_VAND:
      return &kIsalVand;
    case EC_BACKEND_ISA_L_RS_CAUCHY:
      return &kIsalCauchy;
    default:
      return nullptr;
  }
}
constexpr int kRing = 4;

inline uint64_t round16(uint64_t x) { return (x + 15) & ~uint64_t(15); }

inline void put32(uint8_t* p, uint32_t v) { std::memcpy(p, &v, 4); }
inline void put64(uint8_t* p, uint64_t v) { std::memcpy(p, &v, 8); }
inline uint32_t get32(const void* p) {
  uint32_t v;
  std::memcpy(&v, p, 4);
  return v;
}
inline uint64_t get64(const void* p) {
  uint64_t v;
  std::memcpy(&v, p, 8);
  return v;
}

bool write_legacy_crc() {
  const char* v = std::getenv("LIBERASURECODE_WRITE_LEGACY_CRC");
  if (!v) return false;
  return !std::strcmp(v, "1") || !strcasecmp(v, "yes") || !strcasecmp(v, "true") ||
         !strcasecmp(v, "on");
}

uint32_t hdr_crc(const void* p, size_t n, bool legacy) {
  return legacy ? crc32_legacy(0, p, n) : crc32(0, p, n);
}

// add_fragment_metadata (upstream erasurecode_helpers.c), header into h[0..80)
void make_header(uint8_t* h, const Code& code, uint32_t idx, uint32_t bs, uint64_t orig, int ct,
                 const uint8_t* payload, bool legacy) {
  std::memset(h, 0, kHeaderBytes);
  put32(h + 0, idx);
  put32(h + 4, bs);
  put32(h + 8, 0);
  put64(h + 12, orig);
  h[20] = static_cast<uint8_t>(ct);
  // no payload: the GPU CRC kernel patches chksum[0] and the metadata checksum
  if (ct == CHKSUM_CRC32 && payload) put32(h + 21, hdr_crc(payload, bs, legacy));
  h[53] = 0;
  h[54] = code.wire_id;
  put32(h + 55, code.version);
  put32(h + 59, LIBERASURECODE_FRAG_HEADER_MAGIC);
  put32(h + 63, kLibecVersion);
  put32(h + 67, hdr_crc(h, sizeof(fragment_metadata_t), legacy));
}

// is_invalid_fragment_header (upstream erasurecode_helpers.c)
bool header_invalid(const uint8_t* h) {
  const uint32_t ver = get32(h + 63);
  if (ver == 0) return true;
  if (ver < 0x010200) return false;
  if (get32(h + 59) != LIBERASURECODE_FRAG_HEADER_MAGIC) return true;
  const uint32_t stored = get32(h + 67);
  return stored != crc32(0, h, sizeof(fragment_metadata_t)) &&
         stored != crc32_legacy(0, h, sizeof(fragment_metadata_t));
}

int hip_errno(hipError_t e) { return e == hipErrorOutOfMemory ? -ENOMEM : -EBACKENDINITERR; }

struct DeviceGuard {
  int prev = -1;
  explicit DeviceGuard(int dev) {
    if (hipGetDevice(&prev) == hipSuccess && prev != dev) (void)hipSetDevice(dev);
    else prev = -1;
  }
  ~DeviceGuard() {
    if (prev >= 0) (void)hipSetDevice(prev);
  }
};

struct DevBuf {
  void* p = nullptr;
  size_t cap = 0;
  hipError_t ensure(size_t n) {
    if (n <= cap) return hipSuccess;
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
    hipError_t e = hipMalloc(&p, n);
    if (e == hipSuccess) cap = n;
    return e;
  }
  void release() {
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
  }
  uint8_t* b() const { return static_cast<uint8_t*>(p); }
};

// Descriptor/header upload slot: pinned staging + device copy + completion event.
struct RingSlot {
  uint8_t* host = nullptr;
  DevBuf dev;
  size_t cap = 0;
  hipEvent_t ev = nullptr;
  bool pending = false;
};

struct Instance {
  int k = 0, m = 0, ct = CHKSUM_NONE, backend_id = 0, device = 0;
  Code code = kRsVand;
  bool legacy_crc = false;
  uint32_t passes = 1;  // ceil(m / 4) table sets per decode pattern
  GfMatrix gen;
  std::mutex mu;
  hipStream_t stream = nullptr;
  DevBuf enc_tables;  // passes x k x 64 u64
  DevBuf pool;        // decode / reconstruct table sets
  uint32_t pool_slots = 0, pool_used = 0;
  std::unordered_map<uint64_t, uint32_t> pool_index;
  DevBuf scratch;  // single-object staging
  RingSlot ring[kRing];
  int ring_pos = 0;
  hipStream_t hstream[2] = {nullptr, nullptr};  // host-resident pipeline
  DevBuf hbuf[2];
  std::map<uint64_t, DevBuf> crc_tables;  // payload size -> CrcTables (device)

  // bytes of one table set (k inputs x up to 4 rows)
  size_t table_bytes() const { return static_cast<size_t>(k) * table_bytes_per_input(code.w); }

  ~Instance() {
    DeviceGuard g(device);
    if (stream) (void)hipStreamSynchronize(stream);
    for (auto& s : hstream)
      if (s) {
        (void)hipStreamSynchronize(s);
        (void)hipStreamDestroy(s);
      }
    for (auto& r : ring) {
      if (r.ev) {
        (void)hipEventSynchronize(r.ev);
        (void)hipEventDestroy(r.ev);
      }
      if (r.host) (void)hipHostFree(r.host);
      r.dev.release();
    }
    enc_tables.release();
    pool.release();
    scratch.release();
    for (auto& b : hbuf) b.release();
    for (auto& kv : crc_tables) kv.second.release();
    if (stream) (void)hipStreamDestroy(stream);
  }

  // Acquire a ring slot with at least n bytes; waits for its previous use.
  RingSlot* ring_acquire(size_t n, hipError_t* err) {
    RingSlot& r = ring[ring_pos];
    ring_pos = (ring_pos + 1) % kRing;
    *err = hipSuccess;
    if (r.pending) {
      *err = hipEventSynchronize(r.ev);
      r.pending = false;
      if (*err != hipSuccess) return nullptr;
    }
    if (!r.ev && (*err = hipEventCreateWithFlags(&r.ev, hipEventDisableTiming)) != hipSuccess)
      return nullptr;
    if (r.cap < n) {
      if (r.host) (void)hipHostFree(r.host);
      r.host = nullptr;
      r.cap = 0;
      const size_t cap = std::max<size_t>(round16(n), 4096);
      if ((*err = hipHostMalloc(reinterpret_cast<void**>(&r.host), cap, 0)) != hipSuccess)
        return nullptr;
      if ((*err = r.dev.ensure(cap)) != hipSuccess) return nullptr;
      r.cap = cap;
    }
    return &r;
  }
  hipError_t ring_commit(RingSlot* r, size_t n, hipStream_t s) {
    return hipMemcpyAsync(r->dev.p, r->host, n, hipMemcpyHostToDevice, s);
  }
  hipError_t ring_release(RingSlot* r, hipStream_t s) {
    hipError_t e = hipEventRecord(r->ev, s);
    r->pending = (e == hipSuccess);
    return e;
  }
};

std::mutex g_registry_mu;
std::map<int, std::shared_ptr<Instance>> g_registry;
int g_next_desc = 0;

std::shared_ptr<Instance> lookup(int desc) {
  std::lock_guard<std::mutex> lk(g_registry_mu);
  auto it = g_registry.find(desc);
  return it == g_registry.end() ? nullptr : it->second;
}

int gpu_available() {
  static std::once_flag once;
  static int avail = 0;
  std::call_once(once, [] {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return;
    for (int d = 0; d < n; ++d) {
      hipDeviceProp_t prop;
      if (hipGetDeviceProperties(&prop, d) == hipSuccess &&
          std::strncmp(prop.gcnArchName, "gfx950", 6) == 0)
        avail = 1;
    }
  });
  return avail;
}

// get_aligned_data_size (upstream erasurecode_helpers.c): the object is padded
// to a multiple of k * w/8 bytes and split into k equal payloads.
uint64_t blocksize_of(int k, int w, uint64_t len) {
  const uint64_t mult = static_cast<uint64_t>(k) * (w / 8);
  return ((len + mult - 1) / mult) * mult / k;
}

uint16_t gf_mul(int w, uint16_t a, uint16_t b) {
  return w == 16 ? Gf16::get().mul(a, b) : Gf8::get().mul(a, b);
}

bool gf_invert(int w, const GfMatrix& a, GfMatrix& out, int n) {
  return w == 16 ? invert(a, out, n) : invert8(a, out, n);
}

// Table set(s) for `nrows` rows of a k-column coefficient matrix, in the
// kernel's layout for the field (one set per 4 rows).
void build_tables(int w, const uint16_t* rows, int nrows, int k, uint8_t* out) {
  if (w == 16)
    build_nibble_tables(rows, nrows, k, reinterpret_cast<uint64_t*>(out));
  else
    build_nibble_tables8(rows, nrows, k, reinterpret_cast<uint32_t*>(out));
}

// Rows of a decode (dest < 0) or reconstruct (dest >= 0) matrix over the
// inputs `avail` (first k available fragment indices, ascending).
bool pattern_rows(const Instance& I, const int* avail, int dest, std::vector<uint16_t>& rows,
                  std::vector<int>& out_idx) {
  const int k = I.k, w = I.code.w;
  GfMatrix sub(static_cast<size_t>(k) * k), inv;
  for (int i = 0; i < k; ++i)
    std::memcpy(&sub[i * k], &I.gen[avail[i] * k], sizeof(uint16_t) * k);
  if (!gf_invert(w, sub, inv, k)) return false;
  rows.clear();
  out_idx.clear();
  if (dest < 0) {
    std::vector<bool> present(k, false);
    for (int i = 0; i < k; ++i)
      if (avail[i] < k) present[avail[i]] = true;
    for (int j = 0; j < k; ++j)
      if (!present[j]) {
        rows.insert(rows.end(), inv.begin() + j * k, inv.begin() + (j + 1) * k);
        out_idx.push_back(j);
      }
  } else if (dest < k) {
    rows.assign(inv.begin() + dest * k, inv.begin() + (dest + 1) * k);
    out_idx.push_back(dest);
  } else {
    rows.assign(k, 0);
    for (int c = 0; c < k; ++c) {
      uint16_t acc = 0;
      for (int j = 0; j < k; ++j) acc ^= gf_mul(w, I.gen[dest * k + j], inv[j * k + c]);
      rows[c] = acc;
    }
    out_idx.push_back(dest);
  }
  return true;
}

// Table slot for (avail set, dest): `passes` consecutive table sets in the pool.
int pool_slot(Instance& I, uint32_t avail_mask, const int* avail, int dest, uint32_t* slot,
              std::vector<int>& out_idx) {
  const uint64_t key = avail_mask | (static_cast<uint64_t>(dest + 1) << 32);
  std::vector<uint16_t> rows;
  auto it = I.pool_index.find(key);
  if (it != I.pool_index.end()) {
    *slot = it->second;
    // out_idx is cheap to recompute and not cached
    if (dest >= 0) {
      out_idx.assign(1, dest);
    } else {
      out_idx.clear();
      std::vector<bool> present(I.k, false);
      for (int i = 0; i < I.k; ++i)
        if (avail[i] < I.k) present[avail[i]] = true;
      for (int j = 0; j < I.k; ++j)
        if (!present[j]) out_idx.push_back(j);
    }
    return 0;
  }
  if (!pattern_rows(I, avail, dest, rows, out_idx)) return -EINSUFFFRAGS;
  const size_t set_bytes = I.table_bytes();
  if (I.pool_slots == 0) {
    const size_t slot_bytes = set_bytes * I.passes;
    I.pool_slots = static_cast<uint32_t>(std::max<size_t>(64, (size_t(32) << 20) / slot_bytes));
    hipError_t e = I.pool.ensure(slot_bytes * I.pool_slots);
    if (e != hipSuccess) {
      I.pool_slots = 0;
      return hip_errno(e);
    }
  }
  if (I.pool_used == I.pool_slots) {
    // Pool full: wait for every in-flight user of the pool, then recycle it.
    (void)hipDeviceSynchronize();
    I.pool_index.clear();
    I.pool_used = 0;
  }
  const uint32_t s = I.pool_used++;
  std::vector<uint8_t> host(set_bytes * I.passes, 0);
  const int nrows = static_cast<int>(out_idx.size());
  for (uint32_t p = 0; p * kRowsPerPass < static_cast<uint32_t>(nrows); ++p) {
    const int r0 = p * kRowsPerPass;
    const int nr = std::min(kRowsPerPass, nrows - r0);
    build_tables(I.code.w, &rows[static_cast<size_t>(r0) * I.k], nr, I.k, &host[p * set_bytes]);
  }
  // The slot is unused by any in-flight kernel, so a synchronous upload is safe.
  hipError_t e = hipMemcpy(I.pool.b() + static_cast<size_t>(s) * set_bytes * I.passes,
                           host.data(), host.size(), hipMemcpyHostToDevice);
  if (e != hipSuccess) return hip_errno(e);
  I.pool_index.emplace(key, s);
  *slot = s;
  return 0;
}

// First k available indices of a mask; returns count found.
int first_k(uint32_t mask, int k, int n, int* avail) {
  int c = 0;
  for (int i = 0; i < n && c < k; ++i)
    if (mask & (1u << i)) avail[c++] = i;
  return c;
}

struct DecodeJob {
  const uint8_t* frags;
  uint64_t frag_stride, stripe_stride, obj_len;
  uint8_t* out;
  uint64_t out_stride;
  int n_obj;
  const uint32_t* masks;
  const int* dest;            // reconstruct: per-object destination, else null
  const uint8_t* headers;     // reconstruct: n_obj headers (host), else null
};

// Shared decode / reconstruct launcher (caller holds I.mu, device set).
int run_decode(Instance& I, const DecodeJob& J, hipStream_t stream) {
  const int k = I.k, n = I.k + I.m;
  const uint64_t bs = blocksize_of(k, I.code.w, J.obj_len);
  if (bs == 0) return 0;
  if (J.frag_stride % 16 || J.frag_stride < kHeaderBytes + round16(bs)) return -EINVALIDPARAMS;
  if (J.stripe_stride % 16 || reinterpret_cast<uintptr_t>(J.frags) % 16) return -EINVALIDPARAMS;
  if (J.dest && (J.out_stride % 16 || reinterpret_cast<uintptr_t>(J.out) % 16))
    return -EINVALIDPARAMS;
  std::vector<ObjDesc> desc(static_cast<size_t>(J.n_obj));
  std::vector<uint32_t> slots(J.n_obj);
  std::vector<std::vector<int>> outs(J.n_obj);
  uint32_t max_rows = 0;
  for (int o = 0; o < J.n_obj; ++o) {
    int avail[kMaxFragments];
    if (first_k(J.masks[o], k, n, avail) < k) return -EINSUFFFRAGS;
    uint32_t amask = 0;
    for (int i = 0; i < k; ++i) amask |= 1u << avail[i];
    const int dest = J.dest ? J.dest[o] : -1;
    if (J.dest && (dest < 0 || dest >= n)) return -EINVALIDPARAMS;
    int rc = pool_slot(I, amask, avail, dest, &slots[o], outs[o]);
    if (rc < 0) return rc;
    ObjDesc& d = desc[o];
    std::memset(&d, 0, sizeof(d));
    for (int i = 0; i < k; ++i) d.in_idx[i] = static_cast<uint8_t>(avail[i]);
    d.header = o;
    max_rows = std::max<uint32_t>(max_rows, static_cast<uint32_t>(outs[o].size()));
  }
  const uint32_t passes = J.dest ? 1 : std::max<uint32_t>(1, (max_rows + 3) / 4);
  const size_t desc_bytes = sizeof(ObjDesc) * J.n_obj;
  const size_t hdr_bytes = J.headers ? static_cast<size_t>(J.n_obj) * kHeaderBytes : 0;
  for (uint32_t p = 0; p < passes; ++p) {
    for (int o = 0; o < J.n_obj; ++o) {
      ObjDesc& d = desc[o];
      const int total = static_cast<int>(outs[o].size());
      const int r0 = p * kRowsPerPass;
      const int nr = std::max(0, std::min(kRowsPerPass, total - r0));
      d.n_out = static_cast<uint8_t>(nr);
      for (int r = 0; r < nr; ++r) d.out_idx[r] = static_cast<uint8_t>(outs[o][r0 + r]);
      d.copy_inputs = (!J.dest && p == 0) ? 1 : 0;
      d.table = slots[o] * I.passes + p;
    }
    hipError_t e;
    RingSlot* r = I.ring_acquire(desc_bytes + hdr_bytes, &e);
    if (!r) return hip_errno(e);
    std::memcpy(r->host, desc.data(), desc_bytes);
    if (hdr_bytes) std::memcpy(r->host + desc_bytes, J.headers, hdr_bytes);
    if ((e = I.ring_commit(r, desc_bytes + hdr_bytes, stream)) != hipSuccess) return hip_errno(e);
    DecodeParams P{};
    P.frags = J.frags;
    P.frag_stride = J.frag_stride;
    P.stripe_stride = J.stripe_stride;
    P.obj_len = J.obj_len;
    P.out = J.out;
    P.out_stride = J.out_stride;
    P.desc = reinterpret_cast<const ObjDesc*>(r->dev.p);
    P.tables = reinterpret_cast<const uint32_t*>(I.pool.p);
    P.headers = hdr_bytes ? r->dev.b() + desc_bytes : nullptr;
    P.k = k;
    P.m = I.m;
    P.w = static_cast<uint32_t>(I.code.w);
    P.bs = static_cast<uint32_t>(bs);
    P.n_obj = J.n_obj;
    P.reconstruct = J.dest ? 1 : 0;
    e = launch_decode(P, stream);
    hipError_t e2 = I.ring_release(r, stream);
    if (e != hipSuccess) return hip_errno(e);
    if (e2 != hipSuccess) return hip_errno(e2);
  }
  return 0;
}

// Inline CRC-32 of `count` fragments per object (caller holds I.mu): payload
// checksum and metadata checksum patched into headers already written.
int run_crc(Instance& I, uint8_t* base, uint64_t frag_stride, uint64_t stripe_stride,
            uint32_t count, int n_obj, uint64_t bs, hipStream_t stream) {
  if (bs == 0 || n_obj == 0 || count == 0) return 0;
  const uint32_t steps = static_cast<uint32_t>((bs + 4095) / 4096);
  auto it = I.crc_tables.find(bs);
  if (it == I.crc_tables.end()) {
    if (I.crc_tables.size() >= 16) {  // bounded cache: wait for users, then drop it
      (void)hipDeviceSynchronize();
      for (auto& kv : I.crc_tables) kv.second.release();
      I.crc_tables.clear();
    }
    CrcTables host;
    build_crc_tables(static_cast<uint32_t>(bs), steps, &host);
    DevBuf buf;
    hipError_t e = buf.ensure(sizeof(CrcTables));
    if (e == hipSuccess) e = hipMemcpy(buf.p, &host, sizeof(CrcTables), hipMemcpyHostToDevice);
    if (e != hipSuccess) {
      buf.release();
      return hip_errno(e);
    }
    it = I.crc_tables.emplace(bs, buf).first;
  }
  CrcParams P{};
  P.frags = base;
  P.frag_stride = frag_stride;
  P.stripe_stride = stripe_stride;
  P.first = 0;
  P.count = count;
  P.n_obj = static_cast<uint32_t>(n_obj);
  P.bs = static_cast<uint32_t>(bs);
  P.steps = steps;
  P.tables = it->second.p;
  const hipError_t e = launch_crc(P, stream);
  return e == hipSuccess ? 0 : hip_errno(e);
}

int run_encode(Instance& I, const uint8_t* objs, uint64_t obj_stride, uint64_t obj_len, int n_obj,
               uint8_t* parity, uint8_t* data, uint64_t frag_stride, uint64_t stripe_stride,
               bool headers, hipStream_t stream) {
  const int k = I.k, m = I.m;
  const uint64_t bs = blocksize_of(k, I.code.w, obj_len);
  if (bs == 0 && !headers) return 0;
  if (frag_stride % 16 || frag_stride < kHeaderBytes + round16(bs)) return -EINVALIDPARAMS;
  if (stripe_stride % 16) return -EINVALIDPARAMS;
  if (n_obj > 1 && (obj_stride < obj_len || obj_stride % 16)) return -EINVALIDPARAMS;
  if (reinterpret_cast<uintptr_t>(parity) % 16 || reinterpret_cast<uintptr_t>(data) % 16)
    return -EINVALIDPARAMS;
  if (bs > 0xFFFFFFF0ull) return -EINVALIDPARAMS;
  const size_t hdr_bytes = headers ? static_cast<size_t>(k + m) * kHeaderBytes : 0;
  RingSlot* r = nullptr;
  hipError_t e;
  if (headers) {
    // the GPU CRC writes zlib crc32 only; the legacy variant stays host-side
    if (I.ct == CHKSUM_CRC32 && I.legacy_crc) return -EBACKENDNOTSUPP;
    r = I.ring_acquire(hdr_bytes, &e);
    if (!r) return hip_errno(e);
    for (int i = 0; i < k + m; ++i)
      make_header(r->host + i * kHeaderBytes, I.code, i, static_cast<uint32_t>(bs), obj_len, I.ct,
                  nullptr, I.legacy_crc);
    if ((e = I.ring_commit(r, hdr_bytes, stream)) != hipSuccess) return hip_errno(e);
  }
  for (uint32_t p = 0; p < I.passes; ++p) {
    EncodeParams P{};
    P.objs = objs;
    P.obj_stride = obj_stride;
    P.obj_len = obj_len;
    P.parity = parity;
    P.data = data;
    P.frag_stride = frag_stride;
    P.stripe_stride = stripe_stride;
    P.tables = reinterpret_cast<const uint32_t*>(I.enc_tables.b() + p * I.table_bytes());
    P.headers = r ? r->dev.b() : nullptr;
    P.k = k;
    P.m = m;
    P.w = static_cast<uint32_t>(I.code.w);
    P.row0 = p * kRowsPerPass;
    P.nrows = std::min<uint32_t>(kRowsPerPass, m - P.row0);
    P.bs = static_cast<uint32_t>(bs);
    P.n_obj = n_obj;
    if (bs == 0) {
      // header-only fragments: nothing for the kernel to compute
      break;
    }
    if ((e = launch_encode(P, stream)) != hipSuccess) {
      if (r) (void)I.ring_release(r, stream);
      return hip_errno(e);
    }
  }
  if (r && (e = I.ring_release(r, stream)) != hipSuccess) return hip_errno(e);
  if (headers && I.ct == CHKSUM_CRC32) {
    int rc = run_crc(I, parity, frag_stride, stripe_stride, m, n_obj, bs, stream);
    if (rc == 0 && data) rc = run_crc(I, data, frag_stride, stripe_stride, k, n_obj, bs, stream);
    if (rc < 0) return rc;
  }
  return 0;
}

char* alloc_fragment(uint64_t size) {
  void* p = nullptr;
  if (posix_memalign(&p, 16, size ? size : 16) != 0) return nullptr;
  std::memset(p, 0, size ? size : 16);
  return static_cast<char*>(p);
}

}  // namespace
}  // namespace ecamd

using namespace ecamd;

extern "C" {

int liberasurecode_backend_available(const ec_backend_id_t backend_id) {
  if (code_of(backend_id) == nullptr) return 0;
  return gpu_available();
}

int liberasurecode_instance_create(const ec_backend_id_t id, struct ec_args* args) {
  if (!args) return -EINVALIDPARAMS;
  if (args->k < 0 || args->m < 0) return -EINVALIDPARAMS;
  if (args->k + args->m > kMaxFragments) return -EINVALIDPARAMS;
  if (static_cast<int>(id) < 0 || id >= EC_BACKENDS_MAX) return -EBACKENDNOTSUPP;
  const Code* code = code_of(id);
  if (code == nullptr) return -EBACKENDNOTAVAIL;
  if (args->k < 1 || args->m < 1) return -EBACKENDINITERR;
  if (args->ct != CHKSUM_NONE && args->ct != CHKSUM_CRC32 && args->ct != 0)
    return -EINVALIDPARAMS;
  if (!gpu_available()) return -EBACKENDNOTAVAIL;

  auto I = std::make_shared<Instance>();
  I->k = args->k;
  I->m = args->m;
  I->ct = args->ct == CHKSUM_CRC32 ? CHKSUM_CRC32 : CHKSUM_NONE;
  I->backend_id = id;
  I->code = *code;
  I->legacy_crc = write_legacy_crc();
  I->passes = (I->m + kRowsPerPass - 1) / kRowsPerPass;
  if (hipGetDevice(&I->device) != hipSuccess) return -EBACKENDNOTAVAIL;
  I->gen = id == EC_BACKEND_ISA_L_RS_CAUCHY ? make_isal_cauchy_matrix(I->k, I->m)
           : id == EC_BACKEND_ISA_L_RS_VAND   ? make_isal_rs_matrix(I->k, I->m)
                                              : make_generator(I->k, I->m);
  {
    DeviceGuard g(I->device);
    if (hipStreamCreateWithFlags(&I->stream, hipStreamNonBlocking) != hipSuccess)
      return -EBACKENDINITERR;
    const size_t set_bytes = I->table_bytes();
    std::vector<uint8_t> host(set_bytes * I->passes, 0);
    for (uint32_t p = 0; p < I->passes; ++p) {
      const int r0 = p * kRowsPerPass;
      const int nr = std::min(kRowsPerPass, I->m - r0);
      build_tables(I->code.w, &I->gen[static_cast<size_t>(I->k + r0) * I->k], nr, I->k,
                   &host[p * set_bytes]);
    }
    hipError_t e = I->enc_tables.ensure(host.size());
    if (e == hipSuccess)
      e = hipMemcpy(I->enc_tables.p, host.data(), host.size(), hipMemcpyHostToDevice);
    if (e != hipSuccess) return hip_errno(e);
  }
  args->w = I->code.w;
  std::lock_guard<std::mutex> lk(g_registry_mu);
  const int desc = ++g_next_desc;
  g_registry.emplace(desc, std::move(I));
  return desc;
}

int liberasurecode_instance_destroy(int desc) {
  std::shared_ptr<Instance> I;
  {
    std::lock_guard<std::mutex> lk(g_registry_mu);
    auto it = g_registry.find(desc);
    if (it == g_registry.end()) return -EBACKENDNOTAVAIL;
    I = std::move(it->second);
    g_registry.erase(it);
  }
  std::lock_guard<std::mutex> lk(I->mu);  // wait for in-flight calls
  return 0;
}

int liberasurecode_encode(int desc, const char* orig_data, uint64_t orig_data_size,
                          char*** encoded_data, char*** encoded_parity, uint64_t* fragment_len) {
  if (!orig_data || !encoded_data || !encoded_parity || !fragment_len) return -EINVALIDPARAMS;
  auto I = lookup(desc);
  if (!I) return -EBACKENDNOTAVAIL;
  std::lock_guard<std::mutex> lk(I->mu);
  DeviceGuard g(I->device);
  const int k = I->k, m = I->m;
  const uint64_t bs = blocksize_of(k, I->code.w, orig_data_size);
  const uint64_t fl = bs + kHeaderBytes;
  char** dat = static_cast<char**>(std::calloc(k, sizeof(char*)));
  char** par = static_cast<char**>(std::calloc(m, sizeof(char*)));
  auto fail = [&](int rc) {
    for (int i = 0; dat && i < k; ++i) std::free(dat[i]);
    for (int i = 0; par && i < m; ++i) std::free(par[i]);
    std::free(dat);
    std::free(par);
    *encoded_data = nullptr;
    *encoded_parity = nullptr;
    return rc;
  };
  if (!dat || !par) return fail(-ENOMEM);
  uint64_t left = orig_data_size;
  const char* src = orig_data;
  for (int j = 0; j < k; ++j) {
    if (!(dat[j] = alloc_fragment(fl))) return fail(-ENOMEM);
    const uint64_t c = std::min(left, bs);
    if (c) std::memcpy(dat[j] + kHeaderBytes, src, c);
    src += c;
    left -= c;
  }
  for (int p = 0; p < m; ++p)
    if (!(par[p] = alloc_fragment(fl))) return fail(-ENOMEM);

  if (bs > 0) {
    const uint64_t fs = round16(kHeaderBytes + round16(bs));
    const uint64_t obj_bytes = round16(orig_data_size);
    hipError_t e = I->scratch.ensure(obj_bytes + fs * m);
    if (e != hipSuccess) return fail(hip_errno(e));
    uint8_t* d_obj = I->scratch.b();
    uint8_t* d_par = d_obj + obj_bytes;
    if ((e = hipMemcpyAsync(d_obj, orig_data, orig_data_size, hipMemcpyHostToDevice,
                            I->stream)) != hipSuccess)
      return fail(hip_errno(e));
    int rc = run_encode(*I, d_obj, obj_bytes, orig_data_size, 1, d_par, nullptr, fs, fs * m,
                        false, I->stream);
    if (rc < 0) return fail(rc);
    for (int p = 0; p < m; ++p)
      if ((e = hipMemcpyAsync(par[p] + kHeaderBytes, d_par + p * fs + kHeaderBytes, bs,
                              hipMemcpyDeviceToHost, I->stream)) != hipSuccess)
        return fail(hip_errno(e));
    if ((e = hipStreamSynchronize(I->stream)) != hipSuccess) return fail(hip_errno(e));
  }
  for (int j = 0; j < k; ++j)
    make_header(reinterpret_cast<uint8_t*>(dat[j]), I->code, j, static_cast<uint32_t>(bs),
                orig_data_size, I->ct, reinterpret_cast<uint8_t*>(dat[j]) + kHeaderBytes,
                I->legacy_crc);
  for (int p = 0; p < m; ++p)
    make_header(reinterpret_cast<uint8_t*>(par[p]), I->code, k + p, static_cast<uint32_t>(bs),
                orig_data_size, I->ct, reinterpret_cast<uint8_t*>(par[p]) + kHeaderBytes,
                I->legacy_crc);
  *encoded_data = dat;
  *encoded_parity = par;
  *fragment_len = fl;
  return 0;
}

int liberasurecode_encode_cleanup(int desc, char** encoded_data, char** encoded_parity) {
  auto I = lookup(desc);
  if (!I) return -EBACKENDNOTAVAIL;
  if (encoded_data) {
    for (int i = 0; i < I->k; ++i) std::free(encoded_data[i]);
    std::free(encoded_data);
  }
  if (encoded_parity) {
    for (int i = 0; i < I->m; ++i) std::free(encoded_parity[i]);
    std::free(encoded_parity);
  }
  return 0;
}

namespace {

// liberasurecode_get_fragment_metadata's checksum test, on a fragment whose
// header fields are already known to be readable.
bool payload_chksum_mismatch(const uint8_t* frag) {
  if (frag[20] != CHKSUM_CRC32) return false;
  const uint32_t size = get32(frag + 4);
  const uint32_t stored = get32(frag + 21);
  return stored != crc32(0, frag + kHeaderBytes, size) &&
         stored != crc32_legacy(0, frag + kHeaderBytes, size);
}

// is_invalid_fragment (upstream erasurecode.c), used by force_metadata_checks
bool fragment_invalid(const uint8_t* frag, uint8_t wire_id) {
  const uint32_t ver = get32(frag + 63);
  if (ver > kLibecVersion) return true;
  if (get32(frag + 59) != LIBERASURECODE_FRAG_HEADER_MAGIC) return true;
  if (frag[54] != wire_id) return true;
  if (frag[20] < CHKSUM_NONE || frag[20] > CHKSUM_MD5) return true;
  if (frag[53] == 1) return true;
  return payload_chksum_mismatch(frag);
}

struct Partition {
  const uint8_t* by_idx[kMaxFragments];
  int missing = 0;
};

// get_fragment_partition (upstream erasurecode_preprocessing.c)
int partition(const Instance& I, char** frags, int n, Partition& P) {
  const int total = I.k + I.m;
  for (int i = 0; i < kMaxFragments; ++i) P.by_idx[i] = nullptr;
  for (int i = 0; i < n; ++i) {
    const uint32_t idx = get32(frags[i]);
    if (idx >= static_cast<uint32_t>(total)) return -EBADHEADER;
    P.by_idx[idx] = reinterpret_cast<const uint8_t*>(frags[i]);
  }
  P.missing = 0;
  for (int i = 0; i < total; ++i) P.missing += P.by_idx[i] == nullptr;
  return P.missing > I.m ? -EINSUFFFRAGS : 0;
}

// Upload the first k available payloads into a [k+m][fs] device image.
int stage_fragments(Instance& I, const Partition& P, uint64_t bs, uint64_t fs, uint8_t* d_frags,
                    uint32_t* mask) {
  int c = 0;
  *mask = 0;
  for (int i = 0; i < I.k + I.m && c < I.k; ++i) {
    if (!P.by_idx[i]) continue;
    hipError_t e = hipMemcpyAsync(d_frags + i * fs + kHeaderBytes, P.by_idx[i] + kHeaderBytes, bs,
                                  hipMemcpyHostToDevice, I.stream);
    if (e != hipSuccess) return hip_errno(e);
    *mask |= 1u << i;
    ++c;
  }
  return c == I.k ? 0 : -EINSUFFFRAGS;
}

}  // namespace

int liberasurecode_decode(int desc, char** available_fragments, int num_fragments,
                          uint64_t fragment_len, int force_metadata_checks, char** out_data,
                          uint64_t* out_data_len) {
  if (!available_fragments || !out_data || !out_data_len) return -EINVALIDPARAMS;
  auto I = lookup(desc);
  if (!I) return -EBACKENDNOTAVAIL;
  std::lock_guard<std::mutex> lk(I->mu);
  DeviceGuard g(I->device);
  const int k = I->k;
  if (num_fragments < k) return -EINSUFFFRAGS;
  if (fragment_len < kHeaderBytes) return -EBADHEADER;
  for (int i = 0; i < num_fragments; ++i)
    if (!available_fragments[i] ||
        header_invalid(reinterpret_cast<const uint8_t*>(available_fragments[i])))
      return -EBADHEADER;
  if (force_metadata_checks) {
    int bad = 0;
    for (int i = 0; i < num_fragments; ++i)
      bad += fragment_invalid(reinterpret_cast<const uint8_t*>(available_fragments[i]),
                              I->code.wire_id);
    if (num_fragments - bad < k) return -EINSUFFFRAGS;
  }
  // fragments_to_string preconditions: consistent orig_data_size
  const uint64_t orig = get64(available_fragments[0] + 12);
  for (int i = 1; i < num_fragments; ++i)
    if (get64(available_fragments[i] + 12) != orig) return -EBADHEADER;
  Partition P;
  int rc = partition(*I, available_fragments, num_fragments, P);
  bool all_data = true;
  for (int j = 0; j < k; ++j) all_data &= P.by_idx[j] != nullptr;
  uint64_t bs = 0;
  for (int i = 0; i < k + I->m; ++i)
    if (P.by_idx[i]) {
      bs = get32(P.by_idx[i] + 4);
      break;
    }
  if (bs + kHeaderBytes > fragment_len) return -EBADHEADER;
  char* out = static_cast<char*>(alloc_fragment(orig));
  if (!out) return -ENOMEM;
  if (all_data && rc != -EBADHEADER) {
    // Fast path (fragments_to_string): every data fragment present, no GF work.
    uint64_t off = 0;
    for (int j = 0; j < k && off < orig; ++j) {
      const uint64_t c = std::min<uint64_t>(orig - off, get32(P.by_idx[j] + 4));
      std::memcpy(out + off, P.by_idx[j] + kHeaderBytes, c);
      off += c;
    }
    *out_data = out;
    *out_data_len = orig;
    return 0;
  }
  if (rc < 0) {
    std::free(out);
    return rc;
  }
  const uint64_t fs = round16(kHeaderBytes + round16(bs));
  const uint64_t obj_bytes = round16(orig);
  hipError_t e = I->scratch.ensure(fs * (k + I->m) + obj_bytes);
  if (e != hipSuccess) {
    std::free(out);
    return hip_errno(e);
  }
  uint8_t* d_frags = I->scratch.b();
  uint8_t* d_obj = d_frags + fs * (k + I->m);
  uint32_t mask = 0;
  rc = stage_fragments(*I, P, bs, fs, d_frags, &mask);
  if (rc == 0) {
    DecodeJob J{d_frags, fs, fs * (k + I->m), orig, d_obj, obj_bytes, 1, &mask, nullptr, nullptr};
    rc = run_decode(*I, J, I->stream);
  }
  if (rc == 0 && orig)
    if ((e = hipMemcpyAsync(out, d_obj, orig, hipMemcpyDeviceToHost, I->stream)) != hipSuccess)
      rc = hip_errno(e);
  if ((e = hipStreamSynchronize(I->stream)) != hipSuccess && rc == 0) rc = hip_errno(e);
  if (rc < 0) {
    std::free(out);
    return rc;
  }
  *out_data = out;
  *out_data_len = orig;
  return 0;
}

int liberasurecode_decode_cleanup(int desc, char* data) {
  (void)desc;
  std::free(data);
  return 0;
}

int liberasurecode_reconstruct_fragment(int desc, char** available_fragments, int num_fragments,
                                        uint64_t fragment_len, int destination_idx,
                                        char* out_fragment) {
  if (!available_fragments || !out_fragment) return -EINVALIDPARAMS;
  auto I = lookup(desc);
  if (!I) return -EBACKENDNOTAVAIL;
  std::lock_guard<std::mutex> lk(I->mu);
  DeviceGuard g(I->device);
  const int k = I->k, m = I->m;
  for (int i = 0; i < num_fragments; ++i)
    if (!available_fragments[i] ||
        header_invalid(reinterpret_cast<const uint8_t*>(available_fragments[i])))
      return -EBADHEADER;
  Partition P;
  int rc = partition(*I, available_fragments, num_fragments, P);
  if (rc < 0) return rc;
  if (destination_idx < 0 || destination_idx >= k + m) return -EINVALIDPARAMS;
  if (P.by_idx[destination_idx]) {
    std::memcpy(out_fragment, P.by_idx[destination_idx], fragment_len);
    return 0;
  }
  const uint8_t* any = nullptr;
  for (int i = 0; i < k + m && !any; ++i) any = P.by_idx[i];
  const uint64_t bs = get32(any + 4);
  const uint64_t orig = get64(any + 12);
  if (bs + kHeaderBytes > fragment_len) return -EBADHEADER;
  std::memset(out_fragment, 0, fragment_len);
  if (bs > 0) {
    const uint64_t fs = round16(kHeaderBytes + round16(bs));
    hipError_t e = I->scratch.ensure(fs * (k + m + 1));
    if (e != hipSuccess) return hip_errno(e);
    uint8_t* d_frags = I->scratch.b();
    uint8_t* d_out = d_frags + fs * (k + m);
    uint32_t mask = 0;
    rc = stage_fragments(*I, P, bs, fs, d_frags, &mask);
    if (rc == 0) {
      uint8_t hdr[kHeaderBytes] = {0};
      DecodeJob J{d_frags, fs, fs * (k + m), orig, d_out, fs, 1, &mask, &destination_idx, hdr};
      rc = run_decode(*I, J, I->stream);
    }
    if (rc == 0 &&
        (e = hipMemcpyAsync(out_fragment + kHeaderBytes, d_out + kHeaderBytes, bs,
                            hipMemcpyDeviceToHost, I->stream)) != hipSuccess)
      rc = hip_errno(e);
    if ((e = hipStreamSynchronize(I->stream)) != hipSuccess && rc == 0) rc = hip_errno(e);
    if (rc < 0) return rc;
  }
  make_header(reinterpret_cast<uint8_t*>(out_fragment), I->code, destination_idx,
              static_cast<uint32_t>(bs), orig, I->ct,
              reinterpret_cast<uint8_t*>(out_fragment) + kHeaderBytes, I->legacy_crc);
  return 0;
}

int liberasurecode_fragments_needed(int desc, int* fragments_to_reconstruct,
                                    int* fragments_to_exclude, int* fragments_needed) {
  auto I = lookup(desc);
  if (!I) return -EBACKENDNOTAVAIL;
  if (!fragments_to_reconstruct || !fragments_to_exclude || !fragments_needed)
    return -EINVALIDPARAMS;
  // liberasurecode_rs_vand_min_fragments: first k indices neither missing nor
  // excluded; -1 when fewer than k remain.
  uint64_t bm = 0;
  for (int* p = fragments_to_reconstruct; *p > -1; ++p) bm |= uint64_t(1) << (*p & 63);
  for (int* p = fragments_to_exclude; *p > -1; ++p) bm |= uint64_t(1) << (*p & 63);
  int j = 0;
  for (int i = 0; i < I->k + I->m; ++i) {
    if (!(bm & (uint64_t(1) << i))) fragments_needed[j++] = i;
    if (j == I->k) {
      fragments_needed[j] = -1;
      return 0;
    }
  }
  return -1;
}

int liberasurecode_get_fragment_metadata(char* fragment, fragment_metadata_t* fragment_metadata) {
  if (!fragment || !fragment_metadata) return -EINVALIDPARAMS;
  const uint8_t* f = reinterpret_cast<const uint8_t*>(fragment);
  if (get32(f + 59) != LIBERASURECODE_FRAG_HEADER_MAGIC) return -EBADHEADER;
  std::memcpy(fragment_metadata, f, sizeof(fragment_metadata_t));
  if (payload_chksum_mismatch(f)) fragment_metadata->chksum_mismatch = 1;
  return 0;
}

int liberasurecode_verify_stripe_metadata(int desc, char** fragments, int num_fragments) {
  auto I = lookup(desc);
  if (!I) return -EINVALIDPARAMS;
  if (!fragments || num_fragments <= 0) return -EINVALIDPARAMS;
  for (int i = 0; i < num_fragments; ++i) {
    if (!fragments[i]) return -EINVALIDPARAMS;
    const fragment_metadata_t* md = reinterpret_cast<const fragment_metadata_t*>(fragments[i]);
    if (md->backend_id != I->code.wire_id) return -EBADHEADER;
    if (md->chksum_type < CHKSUM_NONE || md->chksum_type >= CHKSUM_TYPES_MAX) return -EBADCHKSUM;
    if (md->chksum_mismatch == 1) return -EBADCHKSUM;
  }
  return 0;
}

int liberasurecode_get_aligned_data_size(int desc, uint64_t data_len) {
  auto I = lookup(desc);
  if (!I) return -EBACKENDNOTAVAIL;
  return static_cast<int>(blocksize_of(I->k, I->code.w, data_len) * I->k);
}

int liberasurecode_get_minimum_encode_size(int desc) {
  return liberasurecode_get_aligned_data_size(desc, 1);
}

int liberasurecode_get_fragment_size(int desc, int data_len) {
  auto I = lookup(desc);
  if (!I) return -EBACKENDNOTAVAIL;
  if (data_len < 0) return -EINVALIDPARAMS;
  return static_cast<int>(blocksize_of(I->k, I->code.w, static_cast<uint64_t>(data_len)));
}

uint32_t liberasurecode_get_version(void) { return kLibecVersion; }

/* ---------------- Part 2 ---------------- */

uint64_t ecamd_blocksize(int desc, uint64_t obj_len) {
  auto I = lookup(desc);
  return I ? blocksize_of(I->k, I->code.w, obj_len) : 0;
}

int ecamd_device(int desc) {
  auto I = lookup(desc);
  return I ? I->device : -EBACKENDNOTAVAIL;
}

int ecamd_encode_batch(int desc, const void* d_objs, uint64_t obj_stride, uint64_t obj_len,
                       int n_obj, void* d_parity, void* d_data, uint64_t frag_stride,
                       uint64_t stripe_stride, void* stream) {
  if (!d_objs || !d_parity || n_obj < 0) return -EINVALIDPARAMS;
  auto I = lookup(desc);
  if (!I) return -EBACKENDNOTAVAIL;
  if (n_obj == 0) return 0;
  if (obj_len == 0) return -EINVALIDPARAMS;
  std::lock_guard<std::mutex> lk(I->mu);
  DeviceGuard g(I->device);
  return run_encode(*I, static_cast<const uint8_t*>(d_objs), obj_stride, obj_len, n_obj,
                    static_cast<uint8_t*>(d_parity), static_cast<uint8_t*>(d_data), frag_stride,
                    stripe_stride, true, static_cast<hipStream_t>(stream));
}

int ecamd_decode_batch(int desc, const void* d_frags, uint64_t frag_stride,
                       uint64_t stripe_stride, uint64_t obj_len, int n_obj,
                       const uint32_t* h_avail, void* d_objs, uint64_t obj_stride, void* stream) {
  if (!d_frags || !h_avail || !d_objs || n_obj < 0) return -EINVALIDPARAMS;
  auto I = lookup(desc);
  if (!I) return -EBACKENDNOTAVAIL;
  if (n_obj == 0) return 0;
  if (n_obj > 1 && obj_stride < obj_len) return -EINVALIDPARAMS;
  std::lock_guard<std::mutex> lk(I->mu);
  DeviceGuard g(I->device);
  DecodeJob J{static_cast<const uint8_t*>(d_frags), frag_stride, stripe_stride, obj_len,
              static_cast<uint8_t*>(d_objs), obj_stride, n_obj, h_avail, nullptr, nullptr};
  return run_decode(*I, J, static_cast<hipStream_t>(stream));
}

int ecamd_reconstruct_batch(int desc, const void* d_frags, uint64_t frag_stride,
                            uint64_t stripe_stride, uint64_t obj_len, int n_obj,
                            const uint32_t* h_avail, const int* h_dest, void* d_out,
                            uint64_t out_stride, void* stream) {
  if (!d_frags || !h_avail || !h_dest || !d_out || n_obj < 0) return -EINVALIDPARAMS;
  auto I = lookup(desc);
  if (!I) return -EBACKENDNOTAVAIL;
  if (n_obj == 0) return 0;
  if (I->ct == CHKSUM_CRC32 && I->legacy_crc) return -EBACKENDNOTSUPP;
  std::lock_guard<std::mutex> lk(I->mu);
  DeviceGuard g(I->device);
  const uint64_t bs = blocksize_of(I->k, I->code.w, obj_len);
  std::vector<uint8_t> hdr(static_cast<size_t>(n_obj) * kHeaderBytes);
  for (int o = 0; o < n_obj; ++o) {
    if (h_dest[o] < 0 || h_dest[o] >= I->k + I->m) return -EINVALIDPARAMS;
    make_header(&hdr[static_cast<size_t>(o) * kHeaderBytes], I->code, h_dest[o], static_cast<uint32_t>(bs),
                obj_len, I->ct, nullptr, I->legacy_crc);
  }
  DecodeJob J{static_cast<const uint8_t*>(d_frags), frag_stride, stripe_stride, obj_len,
              static_cast<uint8_t*>(d_out), out_stride, n_obj, h_avail, h_dest, hdr.data()};
  int rc = run_decode(*I, J, static_cast<hipStream_t>(stream));
  if (rc == 0 && I->ct == CHKSUM_CRC32)
    rc = run_crc(*I, static_cast<uint8_t*>(d_out), 0, out_stride, 1, n_obj, bs,
                 static_cast<hipStream_t>(stream));
  return rc;
}

int ecamd_encode_host_batch(int desc, const void* h_objs, uint64_t obj_stride, uint64_t obj_len,
                            int n_obj, void* h_parity, uint64_t frag_stride) {
  if (!h_objs || !h_parity || n_obj < 0) return -EINVALIDPARAMS;
  auto I = lookup(desc);
  if (!I) return -EBACKENDNOTAVAIL;
  if (n_obj == 0) return 0;
  if (obj_stride < obj_len || obj_stride % 16 || frag_stride % 16) return -EINVALIDPARAMS;
  std::lock_guard<std::mutex> lk(I->mu);
  DeviceGuard g(I->device);
  const int m = I->m;
  // ~64 MiB of objects per chunk, two chunks in flight (one per stream).
  const int chunk = static_cast<int>(std::max<uint64_t>(1, (uint64_t(64) << 20) / obj_stride));
  const uint64_t in_bytes = static_cast<uint64_t>(chunk) * obj_stride;
  const uint64_t out_bytes = static_cast<uint64_t>(chunk) * m * frag_stride;
  hipError_t e = hipSuccess;
  for (int s = 0; s < 2; ++s) {
    if (!I->hstream[s] &&
        (e = hipStreamCreateWithFlags(&I->hstream[s], hipStreamNonBlocking)) != hipSuccess)
      return hip_errno(e);
    if ((e = I->hbuf[s].ensure(in_bytes + out_bytes)) != hipSuccess) return hip_errno(e);
  }
  int rc = 0;
  for (int o0 = 0, c = 0; o0 < n_obj && rc == 0; o0 += chunk, ++c) {
    const int n = std::min(chunk, n_obj - o0);
    hipStream_t s = I->hstream[c & 1];
    uint8_t* d_in = I->hbuf[c & 1].b();
    uint8_t* d_out = d_in + in_bytes;
    const uint8_t* src = static_cast<const uint8_t*>(h_objs) + static_cast<uint64_t>(o0) * obj_stride;
    const uint64_t nin = static_cast<uint64_t>(n - 1) * obj_stride + obj_len;
    if ((e = hipMemcpyAsync(d_in, src, nin, hipMemcpyHostToDevice, s)) != hipSuccess) {
      rc = hip_errno(e);
      break;
    }
    rc = run_encode(*I, d_in, obj_stride, obj_len, n, d_out, nullptr, frag_stride,
                    static_cast<uint64_t>(m) * frag_stride, true, s);
    if (rc < 0) break;
    uint8_t* dst = static_cast<uint8_t*>(h_parity) + static_cast<uint64_t>(o0) * m * frag_stride;
    if ((e = hipMemcpyAsync(dst, d_out, static_cast<uint64_t>(n) * m * frag_stride,
                            hipMemcpyDeviceToHost, s)) != hipSuccess)
      rc = hip_errno(e);
  }
  for (auto s : I->hstream)
    if ((e = hipStreamSynchronize(s)) != hipSuccess && rc == 0) rc = hip_errno(e);
  return rc;
}

}  // extern "C"
