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
#include <chrono>
#include <cerrno>
#include <cstdio>
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
#include "host_copy.hpp"

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
constexpr int kHostStreams = 4;  // host-resident pipeline streams (H2D / kernel / D2H in flight)
constexpr int kCrcPartSlots = 8;  // fused parity CRC partials: one buffer per stream

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

bool env_on(const char* name, bool dflt = false) {
  const char* v = std::getenv(name);
  if (v == nullptr || v[0] == 0) return dflt;
  return v[0] != '0';
}

long env_long(const char* name, long dflt) {
  const char* v = std::getenv(name);
  return (v == nullptr || *v == 0) ? dflt : std::atol(v);
}

// Runtime knobs, read from the environment once, when an instance is created
// -- never on the call path.  Each one selects between outputs that are
// identical (a staging path, a pool size, a launch form); none changes a byte
// written.  Tests and tools/ use them to reach every path.
struct Knobs {
  // objects up to this many bytes take the zero-copy single-object path (0:
  // never).  Measured round 2 (tools/single_ab.py, profiles/r02m_single_ab.txt
  // and r02n, k=10 m=4): faster than the DMA path up to 1 MiB on both boxes
  // -- 64 KiB encode 51-54 vs 97-105 us, decode 57-59 vs 91-93; 1 MiB 148 vs
  // 181-187, 163-167 vs 264-268.
  // Round 4 (tools/single_probe.py, profiles/r04e_single_probe.txt): with the
  // parallel host copies, 4 MiB encode 279 -> 215 us through pinned staging.
  size_t single_pinned_max = size_t(64) << 20;  // ECAMD_SINGLE_PINNED_MAX
  // In place (opt-in, ECAMD_REGISTER_CALLER=1): the kernels read the
  // caller's object (encode) and fragments (decode) and write the parity
  // (encode) and the rebuilt slices (decode) through the whole pages
  // strictly inside each caller buffer, registered with hipHostRegister for
  // the call (about 2.5 us each); the partial first and last pages, which
  // other heap objects share, never are (their bytes go through the staging
  // buffer).  Measured round 6 (tools/single_probe.py,
  // profiles/r06f_single_probe_in_place_all.txt, one box): 4 MiB encode
  // 185.3 -> 127.8 us, decode 181.0 -> 131.6 us.  Off by default: with it
  // on by default the GPU suite faulted once (profiles/r06k_*) exactly as in
  // round 4 -- hipErrorIllegalAddress in a later torch pageable copy of
  // 1.15 MB (a size the runtime pins on the fly), with no kernel of this
  // library in flight -- so registering callers' memory, whole pages or
  // not, is what exposes it.  CallerPin keeps a
  // process-wide registry so that no two of this library's registrations
  // share a page, and checks every unregistration.
  bool register_caller = false;
  // in-place calls only for objects of at least this many bytes
  // (ECAMD_DIRECT_MIN): below it the staging copy costs less than the
  // registration
  size_t direct_min = size_t(256) << 10;
  long pool_slots = 0;          // ECAMD_POOL_SLOTS: decode table-set slots (0 = from 32 MiB)
  bool host_staged = false;     // ECAMD_HOST_STAGED: copy-engine host pipeline
  bool host_staged_out = false; // ECAMD_HOST_STAGED_OUT: ... with outputs staged through HBM
  int host_streams = 3;         // ECAMD_HOST_STREAMS
  int host_chunk_mb = 32;       // ECAMD_HOST_CHUNK_MB
  bool edge_blocks = true;      // ECAMD_EDGE_BLOCKS=0: the round-2 launch form
  // ECAMD_UPLOAD_HOST_WAIT=0: a launch waits for its descriptor upload on the
  // GPU (hipStreamWaitEvent) instead of the host waiting for the copy before
  // the launch.  Round 5 (tools/timeline_gaps.py on fresh_probe.py's
  // back-to-back decodes with new masks per call): the GPU-side wait opened
  // an 11.6 us gap before every kernel, although each copy had long finished;
  // repeated masks (no upload) ran back to back with none.  The host is ahead
  // of the GPU there, so its wait for a 16 KiB copy costs nothing.
  bool upload_host_wait = true;
  static Knobs from_env() {
    Knobs k;
    k.single_pinned_max = static_cast<size_t>(
        std::max<long>(0, env_long("ECAMD_SINGLE_PINNED_MAX", static_cast<long>(k.single_pinned_max))));
    k.pool_slots = std::max<long>(0, env_long("ECAMD_POOL_SLOTS", 0));
    k.host_staged = env_on("ECAMD_HOST_STAGED");
    k.host_staged_out = env_on("ECAMD_HOST_STAGED_OUT");
    k.host_streams = static_cast<int>(env_long("ECAMD_HOST_STREAMS", k.host_streams));
    k.host_chunk_mb = static_cast<int>(std::max<long>(1, env_long("ECAMD_HOST_CHUNK_MB", k.host_chunk_mb)));
    k.edge_blocks = env_on("ECAMD_EDGE_BLOCKS", true);
    k.register_caller = env_on("ECAMD_REGISTER_CALLER", false);
    k.direct_min = static_cast<size_t>(
        std::max<long>(0, env_long("ECAMD_DIRECT_MIN", static_cast<long>(k.direct_min))));
    k.upload_host_wait = env_on("ECAMD_UPLOAD_HOST_WAIT", true);
    return k;
  }
};

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

// The HIP error behind the calling thread's last -EBACKENDINITERR (pyeclib
// reports it as "Unknown error"; ecamd_last_device_error hands the runtime's
// name and text to the binding, which appends them to the message).  Reset
// by every entry point that may launch (CallScope).
thread_local hipError_t t_last_hip = hipSuccess;
int hip_errno(hipError_t e) {
  t_last_hip = e;
  return e == hipErrorOutOfMemory ? -ENOMEM : -EBACKENDINITERR;
}

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

// Pinned, device-mapped host memory (same address on both sides) for the
// single-object calls: the kernels read and write it over PCIe, the host
// fills and drains it with memcpy -- no DMA copies, which from pageable
// Python bytes cost a staged transfer each (one per fragment on decode).
//
// The process's instances share one budget for these buffers
// (ECAMD_PINNED_TOTAL_MB, default 1024): a buffer that would take the total
// past it is not grown, and that call (and the instance's later ones of that
// size) takes the DMA path through HBM instead -- a Swift worker holding many
// policies' instances does not pin gigabytes of host memory (round-4 advice).
std::atomic<size_t>& pinned_total() {
  static std::atomic<size_t> t{0};
  return t;
}
size_t pinned_budget() {
  static const size_t b = static_cast<size_t>(std::max<long>(0, env_long("ECAMD_PINNED_TOTAL_MB", 1024)))
                          << 20;
  return b;
}

struct PinBuf {
  uint8_t* p = nullptr;
  size_t cap = 0;       // bytes held, counted in pinned_total()
  bool failed = false;  // allocation or mapping refused: use the DMA path
  uint8_t* ensure(size_t n) {
    if (failed) return nullptr;
    if (n <= cap) return p;
    const size_t want = std::max<size_t>((n + (1 << 20) - 1) & ~size_t((1 << 20) - 1), 1 << 20);
    const size_t grow = want - cap;  // the new buffer replaces the old one
    // reserve `grow` only if the total stays within the budget (a CAS loop:
    // the process total never passes it, even for an instant)
    size_t cur = pinned_total().load();
    do {
      if (cur + grow > pinned_budget()) return nullptr;  // over budget: the DMA path
    } while (!pinned_total().compare_exchange_weak(cur, cur + grow));
    free_buffer();
    void* h = nullptr;
    void* d = nullptr;
    if (hipHostMalloc(&h, want, hipHostMallocMapped) != hipSuccess) {
      (void)hipGetLastError();
      pinned_total().fetch_sub(want);
      failed = true;
      return nullptr;
    }
    if (hipHostGetDevicePointer(&d, h, 0) != hipSuccess || d != h) {
      (void)hipGetLastError();
      (void)hipHostFree(h);
      pinned_total().fetch_sub(want);
      failed = true;
      return nullptr;
    }
    p = static_cast<uint8_t*>(h);
    cap = want;
    return p;
  }
  void release() {
    pinned_total().fetch_sub(cap);
    free_buffer();
  }

 private:
  void free_buffer() {  // no accounting: the caller has moved cap
    if (p) (void)hipHostFree(p);
    p = nullptr;
    cap = 0;
  }
};

// Descriptor/header upload slot: pinned staging + device copy + completion event.
struct RingSlot {
  uint8_t* host = nullptr;
  DevBuf dev;
  size_t cap = 0;
  hipEvent_t cev = nullptr;  // the upload copy into `dev` done (on the upload stream)
  hipEvent_t ev = nullptr;
  bool pending = false;
};

// Device copy of a small per-call table (decode descriptors, encode headers)
// that usually repeats from call to call.  A call whose key differs from the
// previous call's uploads through the ring; the second call in a row with the
// same key uploads once into this buffer; later calls with that key launch
// with no host work and no host-to-device copy at all.
struct UploadCache {
  std::vector<uint8_t> last_key;  // key of the previous call
  std::vector<uint8_t> dev_key;   // key whose bytes are in `dev`
  uint64_t last_gen = 0, dev_gen = 0;
  bool dev_valid = false;
  uint32_t dev_passes = 1;  // decode: kernel passes the cached descriptors cover
  uint8_t* host = nullptr;
  size_t host_cap = 0;
  DevBuf dev;
  hipEvent_t fill_ev = nullptr;     // recorded after the H2D copy that filled `dev`
  hipStream_t fill_stream = nullptr;
  bool fill_done = false;           // that copy is known to be complete
  // (launches that read `dev` record no event -- an event record costs GPU
  // time between kernels; the instance's per-stream waits order a rewrite
  // after them, Instance::order_after_streams)
  void release() {  // the instance's streams are idle (~Instance)
    if (fill_ev) {
      (void)hipEventSynchronize(fill_ev);
      (void)hipEventDestroy(fill_ev);
      fill_ev = nullptr;
    }
    if (host) (void)hipHostFree(host);
    host = nullptr;
    host_cap = 0;
    dev.release();
    dev_valid = false;
  }
};

struct Instance {
  int k = 0, m = 0, ct = CHKSUM_NONE, backend_id = 0, device = 0;
  Code code = kRsVand;
  bool legacy_crc = false;
  Knobs knobs;
  uint32_t passes = 1;  // ceil(m / 4) table sets per decode pattern
  GfMatrix gen;
  std::mutex mu;
  hipStream_t stream = nullptr;
  hipStream_t ustream = nullptr;  // descriptor uploads (ring_commit)
  // The end of this instance's work on every stream a launch of it has been
  // queued on (a caller's streams, the instance's own), so that a device
  // buffer the instance rewrites or frees -- read only by launches on these
  // streams -- is rewritten after them: GPU-side where the rewrite is itself
  // queued, on the host where it is not.  That replaces a device-wide
  // synchronisation: other instances' and threads' work is not waited for,
  // and every error is returned.
  //   * A caller's stream handle is used only during a call on it (a caller
  //     may destroy its stream once the call returns).  While the instance
  //     has seen ONE caller stream, nothing is recorded: its work is ordered
  //     by the stream itself, and an end mark per call cost the bench's
  //     encode 2.4 % (6.5 us of 274; profiles/r05b_ab_endmark.txt).  When a
  //     second caller stream appears, the first one's calls are finished
  //     once with a device synchronise (its handle may be gone), and from
  //     then on every call records its end mark on its stream (CallScope).
  //   * The instance's own streams are valid while it lives: marked lazily,
  //     when something must wait for them.
  // Entries whose recorded work has completed are dropped -- whenever a
  // new stream would take the list past kMarkPrune entries, and before
  // every GPU-side ordering -- so a caller taking a new stream per call
  // holds at most about kMarkPrune plus its in-flight calls.
  struct StreamMark {
    hipStream_t s;
    hipEvent_t ev;
    bool own;       // the instance's own stream
    bool open;      // launched on during the current call
    bool recorded;  // ev marks the end of this instance's work on s
  };
  std::vector<StreamMark> marks;
  static constexpr size_t kMarkPrune = 16;
  bool multi = false;  // has seen two caller streams: caller calls are marked
  DevBuf enc_tables;  // passes x k x 64 u64
  // GF(2^16) with 4 < m <= 8: one eight-row table set (k x 1 KiB), so encode
  // reads the object once (ec_kernels_impl.hpp Gf16x8); the four-row passes
  // above remain for the fused inline-CRC encode
  bool wide = false;
  DevBuf enc_tables8;
  DevBuf pool;        // decode / reconstruct table sets
  uint32_t pool_slots = 0, pool_used = 0;
  uint64_t pool_gen = 1;  // bumped whenever slots are recycled
  // recorded where the pool was last recycled, after the waits for every
  // launch that could read the old table sets: the table copies (upload
  // stream) wait for it before overwriting a slot
  hipEvent_t pool_gen_ev = nullptr;
  bool pool_gen_pending = false;
  std::unordered_map<uint64_t, uint32_t> pool_index;
  // table sets of patterns new in this call: built on the host into
  // pool_stage (slots pool_stage_first..), uploaded by pool_commit with ONE
  // async copy on the upload stream ahead of its launch; pool_ev marks the
  // last such copy, which every launch that reads the pool waits for
  std::vector<uint8_t> pool_stage;
  uint32_t pool_stage_first = 0;
  hipEvent_t pool_ev = nullptr;  // on the upload stream
  bool pool_ev_pending = false;
  // host-side phase times of the last single-object call (ecamd_call_phases):
  // [0] copy in, [1] launch, [2] host work beside the kernel, [3] wait for
  // the kernel, [4] copy out, [5] headers; microseconds
  double phase_us[6] = {0, 0, 0, 0, 0, 0};
  DevBuf scratch;  // single-object staging
  PinBuf pin;      // single-object staging, zero-copy (small objects)
  uint64_t dma_calls = 0;     // single-object calls that staged through HBM (ecamd_instance_stats)
  uint64_t direct_calls = 0;  // single-object calls that used the caller's pages in place
  RingSlot ring[kRing];
  int ring_pos = 0;
  UploadCache dec_cache, rec_cache, hdr_cache;
  hipStream_t hstream[kHostStreams] = {};  // host-resident pipeline
  DevBuf hbuf[kHostStreams];
  hipEvent_t hdone[kHostStreams] = {};
  DevBuf crc_lanes;                       // CrcLaneTables (device), the instance's CRC variant
  std::map<uint64_t, DevBuf> crc_finish;  // payload size -> CrcFinishTables (device)
  // inline_crc32 chunk partials, one buffer per launch stream: a launch
  // reads and writes its own stream's buffer, so launches on different
  // streams (the staged host pipeline deals chunks over 3) never share one
  // and need no device-wide wait between them
  struct CrcPart {
    hipStream_t stream = nullptr;
    bool used = false;
    DevBuf buf;
  } crc_part[kCrcPartSlots];
  int crc_part_victim = 0;

  // bytes of one table set (k inputs x up to 4 rows)
  size_t table_bytes() const { return static_cast<size_t>(k) * table_bytes_per_input(code.w); }

  bool is_own(hipStream_t s) const {
    if (s == stream) return true;
    for (hipStream_t h : hstream)
      if (h && s == h) return true;
    return false;
  }
  // Finish the unmarked work of every caller stream but s (all of them
  // when !keep; single-stream mode: their handles may be gone) and forget them.
  hipError_t drop_unmarked_callers(hipStream_t s, bool keep = true) {
    auto gone = [&](const StreamMark& k) {
      return !k.own && !k.open && !k.recorded && !(keep && k.s == s);
    };
    bool any = false;
    for (auto& k : marks) any |= gone(k);
    if (!any) return hipSuccess;
    const hipError_t e = hipDeviceSynchronize();
    if (e != hipSuccess) return e;
    size_t j = 0;
    for (size_t i = 0; i < marks.size(); ++i) {
      StreamMark& k = marks[i];
      if (gone(k)) {
        (void)hipEventDestroy(k.ev);
        continue;
      }
      marks[j++] = k;
    }
    marks.resize(j);
    return hipSuccess;
  }
  // A launch of this instance is about to be queued on s (during a call).
  hipError_t note_stream(hipStream_t s) {
    for (auto& k : marks)
      if (k.s == s) {
        k.open = true;
        return hipSuccess;
      }
    const bool own = is_own(s);
    if (!own && !multi) {
      bool other = false;
      for (auto& k : marks) other |= !k.own;
      if (other) {  // a second caller stream
        const hipError_t e = drop_unmarked_callers(s);
        if (e != hipSuccess) return e;
        multi = true;
      }
    }
    hipEvent_t ev = nullptr;
    const hipError_t e = hipEventCreateWithFlags(&ev, hipEventDisableTiming);
    if (e != hipSuccess) return e;
    marks.push_back({s, ev, own, true, false});
    // a caller taking a new stream per call adds one entry per call: drop
    // the completed ones once the list passes a few (round-5 advice)
    if (marks.size() > kMarkPrune) prune_marks(s);
    return hipSuccess;
  }
  // End of a call: mark the end of its work on every caller stream it
  // launched on (those handles are the call's own, valid now) once the
  // instance has seen two caller streams.
  hipError_t end_call() {
    hipError_t first = hipSuccess;
    for (auto& k : marks) {
      if (!k.open) continue;
      k.open = false;
      if (k.own) continue;  // marked when something waits for it
      if (!multi) {
        k.recorded = false;  // single caller stream: unmarked
        continue;
      }
      const hipError_t e = hipEventRecord(k.ev, k.s);
      k.recorded = e == hipSuccess;
      if (e != hipSuccess && first == hipSuccess) first = e;
    }
    return first;
  }
  // Drop the caller entries (other than s's) whose recorded work has completed.
  void prune_marks(hipStream_t s) {
    size_t j = 0;
    for (size_t i = 0; i < marks.size(); ++i) {
      StreamMark& k = marks[i];
      if (k.s != s && !k.own && !k.open && k.recorded && hipEventQuery(k.ev) == hipSuccess) {
        (void)hipEventDestroy(k.ev);
        continue;
      }
      marks[j++] = k;
    }
    marks.resize(j);
  }
  // GPU-side: work queued on s from now on runs after everything this
  // instance queued so far on its other streams (s's own work is ordered
  // already): the current call's other streams and the instance's own
  // through a mark recorded now, earlier calls' caller streams through their
  // end marks -- or, unmarked, by a device synchronise.
  hipError_t order_after_streams(hipStream_t s) {
    prune_marks(s);
    hipError_t e = drop_unmarked_callers(s);
    if (e != hipSuccess) return e;
    for (auto& k : marks) {
      if (k.s == s) continue;
      if (k.open || k.own) {
        if ((e = hipEventRecord(k.ev, k.s)) != hipSuccess) return e;
        k.recorded = true;
      }
      if (!k.recorded) continue;
      if ((e = hipStreamWaitEvent(s, k.ev, 0)) != hipSuccess) return e;
    }
    return hipSuccess;
  }
  // Host-side: wait for everything queued so far on the instance's streams.
  hipError_t wait_streams() {
    hipError_t first = drop_unmarked_callers(nullptr, false);
    for (auto& k : marks) {
      if (k.open || k.own) {
        const hipError_t e = hipEventRecord(k.ev, k.s);
        if (e != hipSuccess && first == hipSuccess) first = e;
        k.recorded = e == hipSuccess;
      }
      if (!k.recorded) continue;
      const hipError_t e = hipEventSynchronize(k.ev);
      if (e != hipSuccess && first == hipSuccess) first = e;
    }
    return first;
  }

  ~Instance() {
    DeviceGuard g(device);
    (void)wait_streams();
    if (stream) (void)hipStreamSynchronize(stream);
    for (auto& s : hstream)
      if (s) {
        (void)hipStreamSynchronize(s);
        (void)hipStreamDestroy(s);
      }
    for (auto& e : hdone)
      if (e) (void)hipEventDestroy(e);
    for (auto& k : marks) (void)hipEventDestroy(k.ev);
    if (pool_gen_ev) (void)hipEventDestroy(pool_gen_ev);
    if (pool_ev) {
      (void)hipEventSynchronize(pool_ev);
      (void)hipEventDestroy(pool_ev);
    }
    dec_cache.release();
    rec_cache.release();
    hdr_cache.release();
    if (ustream) (void)hipStreamSynchronize(ustream);
    for (auto& r : ring) {
      if (r.ev) {
        (void)hipEventSynchronize(r.ev);
        (void)hipEventDestroy(r.ev);
      }
      if (r.cev) (void)hipEventDestroy(r.cev);
      if (r.host) (void)hipHostFree(r.host);
      r.dev.release();
    }
    enc_tables.release();
    enc_tables8.release();
    pool.release();
    scratch.release();
    pin.release();
    for (auto& b : hbuf) b.release();
    crc_lanes.release();
    for (auto& kv : crc_finish) kv.second.release();
    for (auto& c : crc_part) c.buf.release();
    if (stream) (void)hipStreamDestroy(stream);
    if (ustream) (void)hipStreamDestroy(ustream);
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
    // the slot's event only says that the launches reading its device bytes
    // have finished (nothing they wrote is read through it): no system-scope
    // fence, whose cache writeback cost a few us between kernels (round 5)
    if (!r.ev && (*err = hipEventCreateWithFlags(
                      &r.ev, hipEventDisableTiming | hipEventDisableSystemFence)) != hipSuccess)
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
  // Copy a slot's n bytes for a launch on s.  The copy runs on the
  // instance's upload stream, beside the kernels s is still running, and s
  // waits for it: a call with new descriptors then adds no copy between two
  // kernels on s (decode with erasure masks new every call, pyeclib_c.c:878;
  // the copy on s itself had cost that decode ~12 % over the cached-descriptor
  // call, BENCH_r04 decode_fresh_ms).  The slot's buffers are rewritten only
  // after ring_acquire's wait for the launch that read them, which ran after
  // this copy.
  hipError_t ensure_ustream() {
    return ustream ? hipSuccess : hipStreamCreateWithFlags(&ustream, hipStreamNonBlocking);
  }
  hipError_t ring_commit(RingSlot* r, size_t n, hipStream_t s) {
    hipError_t e = ensure_ustream();
    if (e != hipSuccess) return e;
    if (!r->cev && (e = hipEventCreateWithFlags(&r->cev, hipEventDisableTiming)) != hipSuccess)
      return e;
    if ((e = hipMemcpyAsync(r->dev.p, r->host, n, hipMemcpyHostToDevice, ustream)) != hipSuccess)
      return e;
    if ((e = hipEventRecord(r->cev, ustream)) != hipSuccess) return e;
    // After a pool recycle the upload stream may hold a GPU-side wait behind
    // queued kernels (pool_commit); a host wait would then block on them, so
    // the launch waits on the GPU instead (round-5 advice).
    const bool behind_gpu = pool_gen_pending && hipEventQuery(pool_gen_ev) != hipSuccess;
    if (knobs.upload_host_wait && !behind_gpu) return hipEventSynchronize(r->cev);
    return hipStreamWaitEvent(s, r->cev, 0);
  }
  hipError_t ring_release(RingSlot* r, hipStream_t s) {
    hipError_t e = hipEventRecord(r->ev, s);
    r->pending = (e == hipSuccess);
    return e;
  }
};

// Held by every entry point that may launch (after the instance lock): the
// call's end marks are recorded however it returns (Instance::end_call).
struct CallScope {
  Instance& I;
  explicit CallScope(Instance& i) : I(i) { t_last_hip = hipSuccess; }
  CallScope(const CallScope&) = delete;
  CallScope& operator=(const CallScope&) = delete;
  ~CallScope() { (void)I.end_call(); }
};

// Where one launch's small table came from (see UploadCache).
struct Upload {
  const uint8_t* dev = nullptr;
  RingSlot* ring = nullptr;     // ring slot to release after the launch, or
  UploadCache* cache = nullptr;  // cache whose event to record after the launch
};

// A launch on stream s may read the cache's device bytes only after the copy
// that filled them, which ran on C.fill_stream: other streams wait for it on
// the GPU (no host wait) until it is known to be complete.
hipError_t cache_ready(UploadCache& C, hipStream_t s) {
  if (C.fill_done) return hipSuccess;
  if (hipEventQuery(C.fill_ev) == hipSuccess) {
    C.fill_done = true;
    return hipSuccess;
  }
  return s == C.fill_stream ? hipSuccess : hipStreamWaitEvent(s, C.fill_ev, 0);
}

// Device bytes for (key, gen).  `build` fills n bytes of host memory; it is
// only called when the bytes are not already on the device.
template <class Build>
int upload(Instance& I, UploadCache& C, const std::vector<uint8_t>& key, uint64_t gen, size_t n,
           hipStream_t s, Build build, Upload* out) {
  *out = Upload{};
  hipError_t e;
  if (C.dev_valid && C.dev_gen == gen && C.dev_key == key && C.dev.cap >= n) {
    if ((e = cache_ready(C, s)) != hipSuccess) return hip_errno(e);
    out->dev = C.dev.b();
    out->cache = &C;
    return 0;
  }
  if (C.last_key == key && C.last_gen == gen) {
    // second call in a row with this key: make it resident.  The copy that
    // rewrites `dev` is queued on s behind every launch of this instance
    // that may still read the old bytes (launches that read the cache record
    // no event: the GPU-side waits cover them, once per new repeated key),
    // and the host staging buffer is rewritten only once its previous copy
    // has completed.
    if (C.dev_valid && (e = I.order_after_streams(s)) != hipSuccess) return hip_errno(e);
    if (C.fill_ev && !C.fill_done && (e = hipEventSynchronize(C.fill_ev)) != hipSuccess)
      return hip_errno(e);
    C.dev_valid = false;
    if (C.host_cap < n) {
      if (C.host) (void)hipHostFree(C.host);
      C.host = nullptr;
      C.host_cap = 0;
      if ((e = hipHostMalloc(reinterpret_cast<void**>(&C.host), n, 0)) != hipSuccess)
        return hip_errno(e);
      C.host_cap = n;
    }
    if ((e = C.dev.ensure(n)) != hipSuccess) return hip_errno(e);
    int rc = build(C.host);
    if (rc < 0) return rc;
    if ((e = hipMemcpyAsync(C.dev.p, C.host, n, hipMemcpyHostToDevice, s)) != hipSuccess)
      return hip_errno(e);
    if (!C.fill_ev && (e = hipEventCreateWithFlags(&C.fill_ev, hipEventDisableTiming)) != hipSuccess)
      return hip_errno(e);
    if ((e = hipEventRecord(C.fill_ev, s)) != hipSuccess) return hip_errno(e);
    C.fill_stream = s;
    C.fill_done = false;
    C.dev_key = key;
    C.dev_gen = gen;
    C.dev_valid = true;
    out->dev = C.dev.b();
    out->cache = &C;
    return 0;
  }
  RingSlot* r = I.ring_acquire(n, &e);
  if (!r) return hip_errno(e);
  int rc = build(r->host);
  if (rc < 0) return rc;
  if ((e = I.ring_commit(r, n, s)) != hipSuccess) return hip_errno(e);
  C.last_key = key;
  C.last_gen = gen;
  out->dev = r->dev.b();
  out->ring = r;
  return 0;
}

// After the launch(es) that read an Upload's bytes.
hipError_t upload_done(Instance& I, Upload& u, hipStream_t s) {
  if (u.ring) return I.ring_release(u.ring, s);
  return hipSuccess;
}

// The fused parity CRC's partials buffer for launches on stream s, at least
// `bytes` long.  A stream keeps its slot; a new stream takes a free slot, or
// -- all taken -- the round-robin victim, whose last user's queued work s
// then waits for on the GPU.  Growing a slot waits for its own stream only.
hipError_t crc_part_for(Instance& I, hipStream_t s, size_t bytes, uint32_t** out) {
  Instance::CrcPart* slot = nullptr;
  for (auto& c : I.crc_part)
    if (c.used && c.stream == s) {
      slot = &c;
      break;
    }
  hipError_t e;
  if (!slot) {
    for (auto& c : I.crc_part)
      if (!c.used) {
        slot = &c;
        break;
      }
    if (!slot) {
      slot = &I.crc_part[I.crc_part_victim];
      I.crc_part_victim = (I.crc_part_victim + 1) % kCrcPartSlots;
      // the victim's last stream is one of the instance's streams
      if ((e = I.order_after_streams(s)) != hipSuccess) return e;
    }
    slot->stream = s;
    slot->used = true;
  }
  if (bytes > slot->buf.cap) {
    if ((e = hipStreamSynchronize(s)) != hipSuccess) return e;
    if ((e = slot->buf.ensure(bytes)) != hipSuccess) return e;
  }
  *out = static_cast<uint32_t*>(slot->buf.p);
  return hipSuccess;
}

template <class T>
void key_append(std::vector<uint8_t>& key, const T* p, size_t n) {
  const uint8_t* b = reinterpret_cast<const uint8_t*>(p);
  key.insert(key.end(), b, b + n * sizeof(T));
}

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
//
// The rows are those of inverse(G[avail]) (liberasurecode_rs_vand's decode
// matrix), found without the k x k inversion: G's top is the identity, so
// with D the e missing data indices and P the e parity inputs, the parity
// equations read  par_P = A d_D + B d_present  (A = G[P][D], e x e;
// B = G[P][present]), hence  d_D = inv(A) par_P + inv(A) B d_present  (char 2).
// One e x e inversion (e <= m) and an e x e x (k - e) product replace a
// k x k Gauss-Jordan: measured round 3, per-call decode with erasures that
// change every call spent most of its host time here.  The inverse is unique,
// so the rows -- and every byte decoded -- are the same.
bool decode_rows(int k, int w, const GfMatrix& gen, const int* avail, int dest,
                 std::vector<uint16_t>& rows, std::vector<int>& out_idx) {
  int pos_of[kMaxFragments];  // input position of data index j, or -1
  for (int j = 0; j < k; ++j) pos_of[j] = -1;
  int par_pos[kMaxFragments], n_par = 0;
  for (int c = 0; c < k; ++c) {
    if (avail[c] < k)
      pos_of[avail[c]] = c;
    else
      par_pos[n_par++] = c;
  }
  int miss[kMaxFragments], e = 0;
  for (int j = 0; j < k; ++j)
    if (pos_of[j] < 0) miss[e++] = j;
  if (e != n_par) return false;  // k inputs: every missing data index has a parity input
  // R[t]: row of missing data index miss[t] over the k inputs
  std::vector<uint16_t> R(static_cast<size_t>(e) * k, 0);
  if (e > 0) {
    GfMatrix A(static_cast<size_t>(e) * e), Ainv;
    for (int r = 0; r < e; ++r)
      for (int t = 0; t < e; ++t) A[r * e + t] = gen[avail[par_pos[r]] * k + miss[t]];
    if (!gf_invert(w, A, Ainv, e)) return false;
    for (int t = 0; t < e; ++t) {
      uint16_t* row = &R[static_cast<size_t>(t) * k];
      for (int r = 0; r < e; ++r) row[par_pos[r]] = Ainv[t * e + r];
      for (int j = 0; j < k; ++j) {
        const int c = pos_of[j];
        if (c < 0) continue;
        uint16_t acc = 0;
        for (int r = 0; r < e; ++r)
          acc ^= gf_mul(w, Ainv[t * e + r], gen[avail[par_pos[r]] * k + j]);
        row[c] = acc;
      }
    }
  }
  int miss_t[kMaxFragments];  // index into R of missing data index j
  for (int t = 0; t < e; ++t) miss_t[miss[t]] = t;
  rows.clear();
  out_idx.clear();
  if (dest < 0) {
    for (int t = 0; t < e; ++t) {
      rows.insert(rows.end(), R.begin() + static_cast<size_t>(t) * k,
                  R.begin() + static_cast<size_t>(t + 1) * k);
      out_idx.push_back(miss[t]);
    }
  } else if (dest < k) {
    rows.assign(k, 0);
    if (pos_of[dest] >= 0)
      rows[pos_of[dest]] = 1;
    else
      rows.assign(R.begin() + static_cast<size_t>(miss_t[dest]) * k,
                  R.begin() + static_cast<size_t>(miss_t[dest] + 1) * k);
    out_idx.push_back(dest);
  } else {
    // parity row dest over the inputs: sum over data j of G[dest][j] * (row of d_j)
    rows.assign(k, 0);
    for (int j = 0; j < k; ++j) {
      const uint16_t g = gen[dest * k + j];
      if (g == 0) continue;
      if (pos_of[j] >= 0) {
        rows[pos_of[j]] ^= g;
      } else {
        const uint16_t* row = &R[static_cast<size_t>(miss_t[j]) * k];
        for (int c = 0; c < k; ++c) rows[c] ^= gf_mul(w, g, row[c]);
      }
    }
    out_idx.push_back(dest);
  }
  return true;
}

bool pattern_rows(const Instance& I, const int* avail, int dest, std::vector<uint16_t>& rows,
                  std::vector<int>& out_idx) {
  return decode_rows(I.k, I.code.w, I.gen, avail, dest, rows, out_idx);
}

// Table slot for (avail set, dest): `passes` consecutive table sets in the pool.
// Returns kPoolFull, touching nothing, when the pattern is not cached and every
// slot is taken: the caller must first launch the objects that already hold
// slots, then pool_recycle() and ask again.
constexpr int kPoolFull = 1;

void missing_rows(const Instance& I, const int* avail, int dest, std::vector<int>& out_idx) {
  if (dest >= 0) {
    out_idx.assign(1, dest);
    return;
  }
  out_idx.clear();
  bool present[kMaxFragments] = {false};
  for (int i = 0; i < I.k; ++i)
    if (avail[i] < I.k) present[avail[i]] = true;
  for (int j = 0; j < I.k; ++j)
    if (!present[j]) out_idx.push_back(j);
}

// Forget all patterns; the next table copies into the pool (queued on s, the
// recycling call's stream, or on any other stream after pool_gen_ev) run
// after every launch queued so far that may read the old sets.  No host wait.
// (Staged sets were committed by the flush that precedes every recycle.)
hipError_t pool_recycle(Instance& I, hipStream_t s) {
  hipError_t e = I.order_after_streams(s);
  if (e != hipSuccess) return e;
  if (!I.pool_gen_ev && (e = hipEventCreateWithFlags(&I.pool_gen_ev, hipEventDisableTiming)) != hipSuccess)
    return e;
  if ((e = hipEventRecord(I.pool_gen_ev, s)) != hipSuccess) return e;
  I.pool_gen_pending = true;
  I.pool_index.clear();
  I.pool_used = 0;
  I.pool_stage.clear();
  I.pool_ev_pending = false;
  ++I.pool_gen;
  return hipSuccess;
}

int pool_slot(Instance& I, uint32_t avail_mask, const int* avail, int dest, uint32_t* slot,
              std::vector<int>& out_idx) {
  const uint64_t key = avail_mask | (static_cast<uint64_t>(dest + 1) << 32);
  std::vector<uint16_t> rows;
  auto it = I.pool_index.find(key);
  if (it != I.pool_index.end()) {
    *slot = it->second;
    missing_rows(I, avail, dest, out_idx);  // cheap to recompute, not cached
    return 0;
  }
  const size_t set_bytes = I.table_bytes();
  if (I.pool_slots == 0) {
    const size_t slot_bytes = set_bytes * I.passes;
    // knob ECAMD_POOL_SLOTS (tests): force a small pool to exercise recycling
    const long forced = I.knobs.pool_slots;
    I.pool_slots = forced > 0 ? static_cast<uint32_t>(forced)
                              : static_cast<uint32_t>(
                                    std::max<size_t>(64, (size_t(32) << 20) / slot_bytes));
    hipError_t e = I.pool.ensure(slot_bytes * I.pool_slots);
    if (e != hipSuccess) {
      I.pool_slots = 0;
      return hip_errno(e);
    }
  }
  if (I.pool_used == I.pool_slots) return kPoolFull;
  if (!pattern_rows(I, avail, dest, rows, out_idx)) return -EINSUFFFRAGS;
  const uint32_t s = I.pool_used++;
  // staged for pool_commit: the new slots of a call are consecutive
  if (I.pool_stage.empty()) I.pool_stage_first = s;
  const size_t at = I.pool_stage.size();
  I.pool_stage.resize(at + set_bytes * I.passes, 0);
  uint8_t* host = I.pool_stage.data() + at;
  const int nrows = static_cast<int>(out_idx.size());
  for (uint32_t p = 0; p * kRowsPerPass < static_cast<uint32_t>(nrows); ++p) {
    const int r0 = p * kRowsPerPass;
    const int nr = std::min(kRowsPerPass, nrows - r0);
    build_tables(I.code.w, &rows[static_cast<size_t>(r0) * I.k], nr, I.k, &host[p * set_bytes]);
  }
  I.pool_index.emplace(key, s);
  *slot = s;
  return 0;
}

// Upload the table sets staged by pool_slot (one async copy through the ring)
// and order the launch about to be queued on `stream` after every table copy
// so far.  Call before every launch that reads the pool.
//
// Every table copy runs on the instance's upload stream, in order (round 5:
// they had run on the launch stream, where each one sat between two kernels;
// decode with erasure masks new every call brings new patterns now and then,
// pyeclib_c.c:878).  A copy that rewrites slots after a recycle first waits
// for the recycle's marker (pool_gen_ev, recorded behind every launch that
// could read the old sets); pool_ev marks the last copy, and a launch on any
// stream waits for it until it is known to be complete.  No kernel reads a
// slot before its copy, and no queued kernel reads a slot being rewritten.
hipError_t pool_commit(Instance& I, hipStream_t stream) {
  hipError_t e = hipSuccess;
  if (!I.pool_stage.empty()) {
    if ((e = I.ensure_ustream()) != hipSuccess) return e;
    bool behind_gpu = false;  // the copy waits for queued kernels (pool recycled)
    if (I.pool_gen_pending) {
      if (hipEventQuery(I.pool_gen_ev) == hipSuccess)
        I.pool_gen_pending = false;
      else if ((e = hipStreamWaitEvent(I.ustream, I.pool_gen_ev, 0)) != hipSuccess)
        return e;
      else
        behind_gpu = true;
    }
    const size_t n = I.pool_stage.size();
    RingSlot* r = I.ring_acquire(n, &e);
    if (!r) return e;
    std::memcpy(r->host, I.pool_stage.data(), n);
    const size_t slot_bytes = I.table_bytes() * I.passes;
    e = hipMemcpyAsync(I.pool.b() + static_cast<size_t>(I.pool_stage_first) * slot_bytes, r->host,
                       n, hipMemcpyHostToDevice, I.ustream);
    I.pool_stage.clear();
    if (e != hipSuccess) return e;
    if (!I.pool_ev && (e = hipEventCreateWithFlags(&I.pool_ev, hipEventDisableTiming)) != hipSuccess)
      return e;
    if ((e = hipEventRecord(I.pool_ev, I.ustream)) != hipSuccess) return e;
    if (I.knobs.upload_host_wait && !behind_gpu) {
      // as ring_commit: the host waits for the copy, the launch needs no wait
      if ((e = hipEventSynchronize(I.pool_ev)) != hipSuccess) return e;
      return I.ring_release(r, stream);
    }
    I.pool_ev_pending = true;
    // the launch waits for the copy; the slot's host buffer is reused only
    // after a marker on `stream` behind that wait
    if ((e = hipStreamWaitEvent(stream, I.pool_ev, 0)) != hipSuccess) return e;
    return I.ring_release(r, stream);
  }
  if (I.pool_ev_pending) {
    if (hipEventQuery(I.pool_ev) == hipSuccess)
      I.pool_ev_pending = false;
    else
      e = hipStreamWaitEvent(stream, I.pool_ev, 0);
  }
  return e;
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
  bool compact = false;       // object o's i-th input (ascending fragment index)
                              // at frags + o*stripe_stride + i*frag_stride
  bool no_copy = false;       // decode: store only the rebuilt slices (the caller
                              // copies the present data fragments itself)
  bool crc = false;           // reconstruct with inline_crc32: the launch sets each
                              // fragment's payload checksum (EncodeParams::crc_lanes)
  uint8_t* direct = nullptr;  // one object decoded in place (DecodeParams::direct)
  uint32_t direct_lo = 0, direct_hi = 0;
  const struct DirectIn* din = nullptr;  // its inputs read in place (DecodeParams::din)
};

// The first k available fragments of one object read in place: input c's
// payload (device-mapped) and its window; null = staged.
struct DirectIn {
  const uint8_t* p[32] = {};
  uint32_t lo[32] = {}, hi[32] = {};
};

// Descriptors of objects [o0, o1) of a job: `passes` arrays of (o1 - o0)
// ObjDesc (pass p handles missing rows 4p..4p+3), then the reconstruct headers.
struct DescBatch {
  std::vector<ObjDesc> base;          // per object: inputs, header row
  std::vector<uint32_t> slots;        // per object: pool slot
  std::vector<std::vector<int>> outs; // per object: output rows (all passes)
};

size_t desc_bytes_of(const DecodeJob& J, int n, uint32_t passes) {
  return sizeof(ObjDesc) * static_cast<size_t>(n) * passes +
         (J.headers ? static_cast<size_t>(n) * kHeaderBytes : 0);
}

void fill_descs(const Instance& I, const DecodeJob& J, const DescBatch& B, int o0, int o1,
                uint32_t passes, uint8_t* host) {
  const int n = o1 - o0;
  ObjDesc* out = reinterpret_cast<ObjDesc*>(host);
  for (uint32_t p = 0; p < passes; ++p)
    for (int o = o0; o < o1; ++o) {
      ObjDesc d = B.base[o];
      d.header = static_cast<uint32_t>(o - o0);
      const int total = static_cast<int>(B.outs[o].size());
      const int r0 = p * kRowsPerPass;
      const int nr = std::max(0, std::min(kRowsPerPass, total - r0));
      d.n_out = static_cast<uint8_t>(nr);
      for (int r = 0; r < nr; ++r) d.out_idx[r] = static_cast<uint8_t>(B.outs[o][r0 + r]);
      d.copy_inputs = (!J.dest && !J.no_copy && p == 0) ? 1 : 0;
      d.table = B.slots[o] * I.passes + p;
      out[static_cast<size_t>(p) * n + (o - o0)] = d;
    }
  if (J.headers)
    std::memcpy(host + sizeof(ObjDesc) * static_cast<size_t>(n) * passes,
                J.headers + static_cast<size_t>(o0) * kHeaderBytes,
                static_cast<size_t>(n) * kHeaderBytes);
}

uint32_t passes_of(const DecodeJob& J, const DescBatch& B, int o0, int o1) {
  if (J.dest) return 1;
  size_t rows = 0;
  for (int o = o0; o < o1; ++o) rows = std::max(rows, B.outs[o].size());
  return std::max<uint32_t>(1, static_cast<uint32_t>((rows + kRowsPerPass - 1) / kRowsPerPass));
}

const void* crc_lanes_for(Instance& I, hipError_t* err);
const void* crc_finish_for(Instance& I, uint64_t bs, hipError_t* err);
size_t crc_part_bytes(int n_obj, uint64_t bs, int rows);

// Launch the kernel passes for objects [o0, o1) whose descriptors (passes x
// n ObjDesc, then headers) are at `dev`.
hipError_t launch_range(Instance& I, const DecodeJob& J, int o0, int o1, uint32_t passes,
                        const uint8_t* dev, uint64_t bs, hipStream_t stream) {
  const int n = o1 - o0;
  if (hipError_t e = I.note_stream(stream); e != hipSuccess) return e;
  if (hipError_t e = pool_commit(I, stream); e != hipSuccess) return e;
  const void* crc_lanes = nullptr;
  const void* crc_fin = nullptr;
  uint32_t* crc_part = nullptr;
  if (J.crc) {
    hipError_t e;
    if (!(crc_lanes = crc_lanes_for(I, &e)) || !(crc_fin = crc_finish_for(I, bs, &e))) return e;
    if ((e = crc_part_for(I, stream, crc_part_bytes(n, bs, 1), &crc_part)) != hipSuccess) return e;
  }
  for (uint32_t p = 0; p < passes; ++p) {
    DecodeParams P{};
    P.crc_lanes = crc_lanes;
    P.crc_finish_tables = crc_fin;
    P.crc_part = crc_part;
    P.frags = J.frags + static_cast<uint64_t>(o0) * J.stripe_stride;
    P.frag_stride = J.frag_stride;
    P.stripe_stride = J.stripe_stride;
    P.obj_len = J.obj_len;
    P.out = J.out + static_cast<uint64_t>(o0) * J.out_stride;
    P.out_stride = J.out_stride;
    P.desc = reinterpret_cast<const ObjDesc*>(dev) + static_cast<size_t>(p) * n;
    P.tables = reinterpret_cast<const uint32_t*>(I.pool.p);
    P.headers = J.headers ? dev + sizeof(ObjDesc) * static_cast<size_t>(n) * passes : nullptr;
    P.k = I.k;
    P.m = I.m;
    P.w = static_cast<uint32_t>(I.code.w);
    P.bs = static_cast<uint32_t>(bs);
    P.n_obj = static_cast<uint32_t>(n);
    P.reconstruct = J.dest ? 1 : 0;
    P.compact = J.compact ? 1 : 0;
    // passes == 1: every missing data row of every object is in this pass, so
    // the kernel stores all k data slices unconditionally (DecodeMode kDecode)
    P.mode = J.dest ? 1u : (passes == 1 ? 0u : 2u);
    P.no_edge_blocks = I.knobs.edge_blocks ? 0u : 1u;
    P.direct = J.direct;
    P.direct_lo = J.direct_lo;
    P.direct_hi = J.direct_hi;
    if (J.din)
      for (int c = 0; c < 32; ++c) {
        P.din[c] = J.din->p[c];
        P.din_lo[c] = J.din->lo[c];
        P.din_hi[c] = J.din->hi[c];
      }
    hipError_t e = launch_decode(P, stream);
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}

// Upload the descriptors of [o0, o1) through the ring and launch them.
int flush_range(Instance& I, const DecodeJob& J, const DescBatch& B, int o0, int o1, uint64_t bs,
                hipStream_t stream) {
  if (o1 <= o0) return 0;
  const uint32_t passes = passes_of(J, B, o0, o1);
  const size_t n = desc_bytes_of(J, o1 - o0, passes);
  hipError_t e;
  RingSlot* r = I.ring_acquire(n, &e);
  if (!r) return hip_errno(e);
  fill_descs(I, J, B, o0, o1, passes, r->host);
  if ((e = I.ring_commit(r, n, stream)) != hipSuccess) return hip_errno(e);
  e = launch_range(I, J, o0, o1, passes, r->dev.b(), bs, stream);
  const hipError_t e2 = I.ring_release(r, stream);
  if (e != hipSuccess) return hip_errno(e);
  return e2 == hipSuccess ? 0 : hip_errno(e2);
}

// The kernels address an object's bytes and a stripe's fragments through
// buffer descriptors with 32-bit offsets (ec_kernels_impl.hpp): j*bs + x for
// object slices (decode's output descriptor holds 2^31 - 1 records, so that
// voffset 2^31 drops a store; encode's input descriptor 2^32 - 1),
// i*frag_stride + 80 + x inside a stripe (2^32 - 1 records), and 32-bit item
// indices.  A layout past those limits would wrap with no error, so it is
// refused (-EINVALIDPARAMS) before anything is launched: objects up to ~2 GiB
// decode and ~4 GiB encode.
bool layout_fits(int k, int m, uint64_t bs, uint64_t frag_stride, uint64_t n_obj,
                 bool decode = true) {
  if (bs > 0xFFFFFFF0ull) return false;
  const uint64_t slice_limit = decode ? 0x7FFFFFFFull : 0xFFFFFFF0ull;
  if (static_cast<uint64_t>(k) * bs + 16 > slice_limit) return false;
  if (static_cast<uint64_t>(k + m) * frag_stride > 0xFFFFFFF0ull) return false;
  return n_obj * (bs / 4096 + 1) < (1ull << 31);
}

// Shared decode / reconstruct launcher (caller holds I.mu, device set).
//
// Every object needs the table set of its erasure pattern in the device pool.
// When a batch brings more new patterns than the pool has free slots, the
// objects that already hold slots are launched first, then the pool is
// recycled (after a device-wide wait) and the rest of the batch continues --
// a slot is never rewritten while a launched or still-to-launch object of
// this call refers to it.  A batch whose masks repeat the previous call's
// reuses its device descriptors (UploadCache) without rebuilding them.
int run_decode(Instance& I, const DecodeJob& J, hipStream_t stream) {
  const int k = I.k, n = I.k + I.m;
  const uint64_t bs = blocksize_of(k, I.code.w, J.obj_len);
  if (bs == 0) return 0;
  if (J.frag_stride % 16 || J.frag_stride < kHeaderBytes + round16(bs)) return -EINVALIDPARAMS;
  if (J.stripe_stride % 16 || reinterpret_cast<uintptr_t>(J.frags) % 16) return -EINVALIDPARAMS;
  if (J.dest && (J.out_stride % 16 || reinterpret_cast<uintptr_t>(J.out) % 16))
    return -EINVALIDPARAMS;
  if (!layout_fits(k, I.m, bs, J.frag_stride, static_cast<uint64_t>(J.n_obj)))
    return -EINVALIDPARAMS;
  for (int o = 0; o < J.n_obj; ++o) {
    if (__builtin_popcount(J.masks[o] & ((n >= 32 ? 0u : (1u << n)) - 1u)) < k)
      return -EINSUFFFRAGS;
    if (J.dest && (J.dest[o] < 0 || J.dest[o] >= n)) return -EINVALIDPARAMS;
  }

  // cache key: everything the descriptor bytes depend on besides the pool
  // (this thread's buffers are reused from call to call: the per-object
  // vectors of a 256-object batch were 256+ allocations per call)
  thread_local std::vector<uint8_t> key;
  key.clear();
  key_append(key, J.masks, J.n_obj);
  if (J.dest) key_append(key, J.dest, J.n_obj);
  if (J.no_copy) key.push_back(1);
  if (J.headers) key_append(key, J.headers, static_cast<size_t>(J.n_obj) * kHeaderBytes);
  UploadCache& C = J.dest ? I.rec_cache : I.dec_cache;
  if (C.dev_valid && C.dev_gen == I.pool_gen && C.dev_key == key) {
    hipError_t ew = cache_ready(C, stream);
    if (ew != hipSuccess) return hip_errno(ew);
    Upload u{C.dev.b(), nullptr, &C};
    // passes: recorded in the key's cache entry by the build below
    const hipError_t e = launch_range(I, J, 0, J.n_obj, C.dev_passes, u.dev, bs, stream);
    const hipError_t e2 = upload_done(I, u, stream);
    if (e != hipSuccess) return hip_errno(e);
    return e2 == hipSuccess ? 0 : hip_errno(e2);
  }

  thread_local DescBatch B;
  B.base.resize(J.n_obj);
  B.slots.resize(J.n_obj);
  if (B.outs.size() < static_cast<size_t>(J.n_obj)) B.outs.resize(J.n_obj);
  int o0 = 0;  // first object not yet launched
  bool split = false;
  for (int o = 0; o < J.n_obj; ++o) {
    int avail[kMaxFragments];
    first_k(J.masks[o], k, n, avail);
    uint32_t amask = 0;
    for (int i = 0; i < k; ++i) amask |= 1u << avail[i];
    const int dest = J.dest ? J.dest[o] : -1;
    int rc = pool_slot(I, amask, avail, dest, &B.slots[o], B.outs[o]);
    if (rc == kPoolFull) {
      if ((rc = flush_range(I, J, B, o0, o, bs, stream)) < 0) return rc;
      o0 = o;
      split = true;
      if (const hipError_t er = pool_recycle(I, stream); er != hipSuccess) return hip_errno(er);
      rc = pool_slot(I, amask, avail, dest, &B.slots[o], B.outs[o]);
      if (rc == kPoolFull) return -ENOMEM;  // pool of zero slots
    }
    if (rc < 0) return rc;
    ObjDesc& d = B.base[o];
    std::memset(&d, 0, sizeof(d));
    for (int i = 0; i < k; ++i) d.in_idx[i] = static_cast<uint8_t>(avail[i]);
  }
  if (split) {
    C.last_key.clear();
    return flush_range(I, J, B, o0, J.n_obj, bs, stream);
  }
  const uint32_t passes = passes_of(J, B, 0, J.n_obj);
  Upload u;
  int rc = upload(I, C, key, I.pool_gen, desc_bytes_of(J, J.n_obj, passes), stream,
                  [&](uint8_t* host) {
                    fill_descs(I, J, B, 0, J.n_obj, passes, host);
                    return 0;
                  },
                  &u);
  if (rc < 0) return rc;
  if (u.cache) C.dev_passes = passes;
  const hipError_t e = launch_range(I, J, 0, J.n_obj, passes, u.dev, bs, stream);
  const hipError_t e2 = upload_done(I, u, stream);
  if (e != hipSuccess) return hip_errno(e);
  return e2 == hipSuccess ? 0 : hip_errno(e2);
}

// inline_crc32 tables on the device (zlib's CRC, or the legacy one when the
// instance writes legacy CRCs): the lane tables once per instance, the
// finishing tables per payload size (a bounded cache, ~12 KiB per size:
// when full, wait for the instance's own launches -- its users -- then drop
// it).  Null on failure (*err set).
constexpr size_t kCrcTableSizes = 64;
const void* crc_lanes_for(Instance& I, hipError_t* err) {
  *err = hipSuccess;
  if (I.crc_lanes.p) return I.crc_lanes.p;
  std::unique_ptr<CrcLaneTables> host(new CrcLaneTables);
  build_crc_lane_tables(I.legacy_crc, host.get());
  hipError_t e = I.crc_lanes.ensure(sizeof(CrcLaneTables));
  if (e == hipSuccess) e = hipMemcpy(I.crc_lanes.p, host.get(), sizeof(CrcLaneTables), hipMemcpyHostToDevice);
  if (e != hipSuccess) {
    I.crc_lanes.release();
    *err = e;
    return nullptr;
  }
  return I.crc_lanes.p;
}

const void* crc_finish_for(Instance& I, uint64_t bs, hipError_t* err) {
  *err = hipSuccess;
  auto it = I.crc_finish.find(bs);
  if (it == I.crc_finish.end()) {
    if (I.crc_finish.size() >= kCrcTableSizes) {
      if ((*err = I.wait_streams()) != hipSuccess) return nullptr;
      for (auto& kv : I.crc_finish) kv.second.release();
      I.crc_finish.clear();
    }
    std::unique_ptr<CrcFinishTables> host(new CrcFinishTables);
    build_crc_finish_tables(static_cast<uint32_t>(bs), I.legacy_crc, host.get());
    DevBuf buf;
    hipError_t e = buf.ensure(sizeof(CrcFinishTables));
    if (e == hipSuccess) e = hipMemcpy(buf.p, host.get(), sizeof(CrcFinishTables), hipMemcpyHostToDevice);
    if (e != hipSuccess) {
      buf.release();
      *err = e;
      return nullptr;
    }
    it = I.crc_finish.emplace(bs, buf).first;
  }
  return it->second.p;
}

// 1 KiB chunk partials of `rows` fragments per object (the launches store at
// most bs / 1024 chunks per fragment).
size_t crc_part_bytes(int n_obj, uint64_t bs, int rows) {
  return static_cast<size_t>(n_obj) * (bs / 1024 + 1) * rows * sizeof(uint32_t);
}

// One object's encode in place: the object read through its whole pages
// (EncodeParams::direct) and parity rows written into theirs
// (EncodeParams::dpar); null = staged.
struct Direct {
  const uint8_t* p = nullptr;
  uint32_t lo = 0, hi = 0;
  uint8_t* par[kMaxFragments] = {};
  uint32_t plo[kMaxFragments] = {}, phi[kMaxFragments] = {};
};

int run_encode(Instance& I, const uint8_t* objs, uint64_t obj_stride, uint64_t obj_len, int n_obj,
               uint8_t* parity, uint8_t* data, uint64_t frag_stride, uint64_t stripe_stride,
               bool headers, hipStream_t stream, const Direct* dir = nullptr) {
  const int k = I.k, m = I.m;
  const uint64_t bs = blocksize_of(k, I.code.w, obj_len);
  if (bs == 0 && !headers) return 0;
  if (frag_stride % 16 || frag_stride < kHeaderBytes + round16(bs)) return -EINVALIDPARAMS;
  if (stripe_stride % 16) return -EINVALIDPARAMS;
  if (n_obj > 1 && (obj_stride < obj_len || obj_stride % 16)) return -EINVALIDPARAMS;
  if (reinterpret_cast<uintptr_t>(parity) % 16 || reinterpret_cast<uintptr_t>(data) % 16)
    return -EINVALIDPARAMS;
  if (!layout_fits(k, m, bs, frag_stride, static_cast<uint64_t>(n_obj), false))
    return -EINVALIDPARAMS;
  const size_t hdr_bytes = headers ? static_cast<size_t>(k + m) * kHeaderBytes : 0;
  Upload u;
  hipError_t e;
  if (headers) {
    // headers depend only on (obj_len) for a given instance; with
    // inline_crc32 their chksum[0] is 0 here and the finishing pass sets it
    std::vector<uint8_t> key;
    key_append(key, &obj_len, 1);
    int rc = upload(I, I.hdr_cache, key, 0, hdr_bytes, stream,
                    [&](uint8_t* host) {
                      for (int i = 0; i < k + m; ++i)
                        make_header(host + i * kHeaderBytes, I.code, i, static_cast<uint32_t>(bs),
                                    obj_len, I.ct, nullptr, I.legacy_crc);
                      return 0;
                    },
                    &u);
    if (rc < 0) return rc;
  }
  // inline_crc32: every launch stores its chunks' CRC partials, and the
  // launcher runs the finishing pass (parity rows; data fragments too)
  const bool crc = headers && I.ct == CHKSUM_CRC32 && bs > 0;
  // in place: the plain parity encode of one object only (the stream kernel)
  if (dir && (n_obj != 1 || crc || data)) return -EINVALIDPARAMS;
  // those forms (and the full stripe) run the loader / consumer kernel for
  // k >= 4, whose input offsets j * bs + x are 32-bit (ec_kernels_impl.hpp
  // launch_encode_k)
  if ((crc || data) && k >= kDmaMinK && static_cast<uint64_t>(k) * bs + 65536u > 0xFFFFFFFFull)
    return -EINVALIDPARAMS;
  const void* crc_lanes = nullptr;
  const void* crc_fin = nullptr;
  uint32_t* crc_part = nullptr;
  if ((e = I.note_stream(stream)) != hipSuccess) {
    (void)upload_done(I, u, stream);
    return hip_errno(e);
  }
  if (crc) {
    hipError_t te;
    if (!(crc_lanes = crc_lanes_for(I, &te)) || !(crc_fin = crc_finish_for(I, bs, &te))) {
      (void)upload_done(I, u, stream);
      return hip_errno(te);
    }
    // parity partials, then room for the data fragments' (full stripe)
    if ((e = crc_part_for(I, stream, crc_part_bytes(n_obj, bs, m + (data ? k : 0)), &crc_part)) !=
        hipSuccess) {
      (void)upload_done(I, u, stream);
      return hip_errno(e);
    }
  }
  // one eight-row pass for 4 < m <= 8 (the inline CRC keeps four-row passes)
  const bool wide = I.wide && !crc;
  const uint32_t passes = wide ? 1 : I.passes;
  for (uint32_t p = 0; p < passes; ++p) {
    EncodeParams P{};
    P.crc_lanes = crc_lanes;
    P.crc_finish_tables = crc_fin;
    P.crc_part = crc_part;
    if (crc && data) P.crc_part_data = crc_part + crc_part_bytes(n_obj, bs, m) / sizeof(uint32_t);
    P.objs = objs;
    P.obj_stride = obj_stride;
    P.obj_len = obj_len;
    P.parity = parity;
    P.data = data;
    P.frag_stride = frag_stride;
    P.stripe_stride = stripe_stride;
    P.tables = wide ? reinterpret_cast<const uint32_t*>(I.enc_tables8.p)
                    : reinterpret_cast<const uint32_t*>(I.enc_tables.b() + p * I.table_bytes());
    P.headers = u.dev;
    P.k = k;
    P.m = m;
    P.w = static_cast<uint32_t>(I.code.w);
    P.row0 = p * kRowsPerPass;
    P.nrows = wide ? static_cast<uint32_t>(m) : std::min<uint32_t>(kRowsPerPass, m - P.row0);
    P.bs = static_cast<uint32_t>(bs);
    P.n_obj = n_obj;
    P.no_edge_blocks = I.knobs.edge_blocks ? 0u : 1u;
    if (dir) {
      P.direct = dir->p;
      P.direct_lo = dir->lo;
      P.direct_hi = dir->hi;
      for (uint32_t q = 0; q < 8; ++q) {
        const uint32_t r = P.row0 + q;
        if (r >= static_cast<uint32_t>(m)) break;
        P.dpar[q] = dir->par[r];
        P.dpar_lo[q] = dir->plo[r];
        P.dpar_hi[q] = dir->phi[r];
      }
    }
    if (bs == 0) {
      // header-only fragments: nothing for the kernel to compute
      break;
    }
    if ((e = launch_encode(P, stream)) != hipSuccess) {
      (void)upload_done(I, u, stream);
      return hip_errno(e);
    }
  }
  if ((e = upload_done(I, u, stream)) != hipSuccess) return hip_errno(e);
  return 0;
}

// Host-resident pipelines.  The caller's objects / fragments are in (pinned)
// host memory; chunks of objects go H2D -> kernels -> D2H, chunk c on stream
// c % kHostStreams, so one chunk's H2D, another's kernels and a third's D2H
// are in flight together (PCIe Gen5 x16 is full duplex: the bound is
// max(H2D bytes, D2H bytes) / link rate).  `in` / `out` describe the host
// arrays: object o's input at in + o*in_stride (in_last bytes for the final
// object of a chunk), output at out + o*out_stride (out_last likewise).
// Device staging per stream: in buffer at +kInSkew, out buffer at +kOutSkew
// past 256-B boundaries so fragment payloads (80 B after a fragment's start)
// and objects sit on 128-B lines when the strides are multiples of 128.
struct HostSide {
  const uint8_t* in;
  uint64_t in_stride, in_last, in_skew;
  uint8_t* out;
  uint64_t out_stride, out_last, out_skew;
};

// Pinned (page-locked, device-mapped) host memory covering [p, p + n)?
bool device_mapped(const void* p, uint64_t n) {
  hipPointerAttribute_t a{};
  if (hipPointerGetAttributes(&a, p) != hipSuccess) {
    (void)hipGetLastError();
    return false;
  }
  if (a.type != hipMemoryTypeHost || a.devicePointer == nullptr) return false;
  return a.devicePointer == p && n > 0;
}

template <class Run>
int host_pipeline(Instance& I, int n_obj, const HostSide& H, Run run) {
  // Both host arrays pinned and mapped (the default path): the kernels run
  // on them directly -- every load and store crosses PCIe from the CUs, no
  // staging copies -- in one launch on one stream.  Measured round 2
  // (tools/host_ab.py, k=10 m=4, 256 x 4 MiB): encode 50.4 GiB/s, decode
  // 40.5, against 39.7 / 27.4 for the copy-engine pipeline below (whose
  // H2D and D2H copies, run together, reach only 36 GiB/s each way).
  // Knob ECAMD_HOST_STAGED=1 forces the copy-engine pipeline.
  const uint64_t in_total = static_cast<uint64_t>(n_obj - 1) * H.in_stride + H.in_last;
  const uint64_t out_total = static_cast<uint64_t>(n_obj - 1) * H.out_stride + H.out_last;
  if (!I.knobs.host_staged && device_mapped(H.in, in_total) &&
      device_mapped(H.out, out_total)) {
    if (!I.hstream[0]) {
      hipError_t e = hipStreamCreateWithFlags(&I.hstream[0], hipStreamNonBlocking);
      if (e != hipSuccess) return hip_errno(e);
    }
    int rc = run(const_cast<uint8_t*>(H.in), H.out, 0, n_obj, I.hstream[0]);
    const hipError_t e = hipStreamSynchronize(I.hstream[0]);
    return rc < 0 ? rc : (e == hipSuccess ? 0 : hip_errno(e));
  }
  // Otherwise chunks go H2D (copy engine) -> kernels -> host.  Outputs: when
  // the host output array is pinned and mapped, the kernels write it
  // directly over PCIe (posted writes) while the copy engine moves the next
  // chunks' inputs H2D; ECAMD_HOST_STAGED_OUT=1 stages outputs through HBM +
  // D2H copies instead (measured round 2: 44.8 / 30.4 GiB/s vs 39.7 / 27.4
  // direct-out, both below the direct path above).
  const bool out_direct = !I.knobs.host_staged_out && device_mapped(H.out, out_total);
  // ~32 MiB of input per chunk, at least 2 chunks per stream when the batch
  // allows, so the three stages overlap for most of the batch.
  // Knobs ECAMD_HOST_CHUNK_MB / ECAMD_HOST_STREAMS: tuning (tools/host_ab.py).
  const int nstreams = std::max(1, std::min(kHostStreams, I.knobs.host_streams));
  const uint64_t chunk_bytes = static_cast<uint64_t>(I.knobs.host_chunk_mb) << 20;
  int chunk = static_cast<int>(std::max<uint64_t>(1, chunk_bytes / H.in_stride));
  chunk = std::min(chunk, std::max(1, (n_obj + 2 * nstreams - 1) / (2 * nstreams)));
  const uint64_t in_cap = (static_cast<uint64_t>(chunk) * H.in_stride + H.in_skew + 255) & ~255ull;
  const uint64_t out_cap = out_direct ? 0 : static_cast<uint64_t>(chunk) * H.out_stride + H.out_skew;
  hipError_t e = hipSuccess;
  for (int s = 0; s < nstreams; ++s) {
    if (!I.hstream[s] &&
        (e = hipStreamCreateWithFlags(&I.hstream[s], hipStreamNonBlocking)) != hipSuccess)
      return hip_errno(e);
    if ((e = I.hbuf[s].ensure(in_cap + out_cap)) != hipSuccess) return hip_errno(e);
  }
  int rc = 0;
  for (int o0 = 0, c = 0; o0 < n_obj && rc == 0; o0 += chunk, ++c) {
    const int n = std::min(chunk, n_obj - o0);
    const int si = c % nstreams;
    hipStream_t s = I.hstream[si];
    uint8_t* d_in = I.hbuf[si].b() + H.in_skew;
    uint8_t* d_out = out_direct ? H.out + static_cast<uint64_t>(o0) * H.out_stride
                                : I.hbuf[si].b() + in_cap + H.out_skew;
    const uint64_t nin = static_cast<uint64_t>(n - 1) * H.in_stride + H.in_last;
    if ((e = hipMemcpyAsync(d_in, H.in + static_cast<uint64_t>(o0) * H.in_stride, nin,
                            hipMemcpyHostToDevice, s)) != hipSuccess) {
      rc = hip_errno(e);
      break;
    }
    if ((rc = run(d_in, d_out, o0, n, s)) < 0) break;
    if (out_direct) continue;
    const uint64_t nout = static_cast<uint64_t>(n - 1) * H.out_stride + H.out_last;
    if ((e = hipMemcpyAsync(H.out + static_cast<uint64_t>(o0) * H.out_stride, d_out, nout,
                            hipMemcpyDeviceToHost, s)) != hipSuccess)
      rc = hip_errno(e);
  }
  for (auto s : I.hstream)
    if (s && (e = hipStreamSynchronize(s)) != hipSuccess && rc == 0) rc = hip_errno(e);
  return rc;
}

// zero = false: the caller writes every byte (decode's object buffer).
char* alloc_fragment(uint64_t size, bool zero = true) {
  void* p = nullptr;
  if (posix_memalign(&p, 16, size ? size : 16) != 0) return nullptr;
  if (zero) std::memset(p, 0, size ? size : 16);
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
  I->knobs = Knobs::from_env();
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
    I->wide = I->code.w == 16 && I->m > kRowsPerPass && I->m <= kRowsWide;
    if (I->wide) {
      std::vector<uint16_t> t8(static_cast<size_t>(I->k) * 4 * 16 * kRowsWide, 0);
      build_nibble_tables_x8(&I->gen[static_cast<size_t>(I->k) * I->k], I->m, I->k, t8.data());
      const size_t bytes = t8.size() * sizeof(uint16_t);
      e = I->enc_tables8.ensure(bytes);
      if (e == hipSuccess) e = hipMemcpy(I->enc_tables8.p, t8.data(), bytes, hipMemcpyHostToDevice);
      if (e != hipSuccess) return hip_errno(e);
    }
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

namespace {

// Phase clock of the single-object calls (Instance::phase_us).
struct PhaseClock {
  double* out;
  std::chrono::steady_clock::time_point t = std::chrono::steady_clock::now();
  explicit PhaseClock(double* o) : out(o) {
    for (int i = 0; i < 6; ++i) out[i] = 0;
  }
  void mark(int phase) {
    const auto now = std::chrono::steady_clock::now();
    out[phase] += std::chrono::duration<double, std::micro>(now - t).count();
    t = now;
  }
};

// Page ranges [first, end) that CallerPin holds registered, process-wide.
// The runtime pins whole pages, so two registrations whose ranges share a
// page -- neighbouring heap objects, or one buffer passed by two threads --
// would pin it twice and release it out of order; a registration is refused
// (the call copies instead) while any page of its range is held.  After a
// failed unregistration nothing more is registered in the process.
struct PinRegistry {
  std::mutex mu;
  std::map<uintptr_t, uintptr_t> live;
  bool broken = false;
};
PinRegistry* const g_pins = new PinRegistry;  // never destroyed (exit-time calls)
constexpr uintptr_t kPage = 4096;

// The whole pages strictly inside a caller's host buffer, used in place by
// the kernels for one call (opt-in, Knobs::register_caller): registered
// (mapped) with hipHostRegister, unregistered by unpin() after the call's
// stream synchronize -- its result is the call's.  Only pages that belong
// to the buffer alone are registered (round 6): the partial first and last
// pages, which other heap objects share, never are; the kernels take the
// bytes outside [lo, hi) from the staging buffer instead (EncodeParams /
// DecodeParams::direct).  pin() fails, and the call stages everything, when
// the buffer holds too few whole pages, a page is held by another live
// registration (PinRegistry), or the mapping is not the host address.
struct CallerPin {
  void* host = nullptr;
  uintptr_t first = 0;
  uint32_t lo = 0, hi = 0;  // the registered bytes, as offsets into the buffer
  bool pin(const void* p, size_t n) {
    const uintptr_t base = reinterpret_cast<uintptr_t>(p);
    const uintptr_t a = (base + kPage - 1) & ~(kPage - 1);
    const uintptr_t b = (base + n) & ~(kPage - 1);
    if (n == 0 || b <= a || b - a < 16 * kPage || n > 0xFFFFFFFFull) return false;
    PinRegistry& R = *g_pins;
    std::lock_guard<std::mutex> lk(R.mu);
    if (R.broken) return false;
    auto it = R.live.lower_bound(a);
    if (it != R.live.end() && it->first < b) return false;
    if (it != R.live.begin() && std::prev(it)->second > a) return false;
    void* h = reinterpret_cast<void*>(a);
    if (hipHostRegister(h, b - a, hipHostRegisterMapped) != hipSuccess) {
      (void)hipGetLastError();
      return false;
    }
    void* d = nullptr;
    if (hipHostGetDevicePointer(&d, h, 0) != hipSuccess || d != h) {
      // the kernels address the buffer by its host address
      (void)hipGetLastError();
      if (hipHostUnregister(h) != hipSuccess) {
        (void)hipGetLastError();
        R.broken = true;
        R.live.emplace(a, b);  // still held: keep every later range off it
      }
      return false;
    }
    R.live.emplace(a, b);
    host = h;
    first = a;
    lo = static_cast<uint32_t>(a - base);
    hi = static_cast<uint32_t>(b - base);
    return true;
  }
  hipError_t unpin() {
    if (!host) return hipSuccess;
    PinRegistry& R = *g_pins;
    std::lock_guard<std::mutex> lk(R.mu);
    const hipError_t e = hipHostUnregister(host);
    host = nullptr;
    if (e != hipSuccess) {
      (void)hipGetLastError();
      R.broken = true;  // the range stays in `live`
      return e;
    }
    R.live.erase(first);
    return hipSuccess;
  }
  CallerPin() = default;
  CallerPin(const CallerPin&) = delete;
  CallerPin& operator=(const CallerPin&) = delete;
  ~CallerPin() { (void)unpin(); }  // error paths, after their stream synchronize
};

// Bytes of the last data slice inside an object of len bytes (the stream
// kernels' interior tiles end at room / 4 KiB * 4 KiB of every payload).
int64_t last_room_of(int k, uint64_t bs, uint64_t len) {
  const int64_t room = static_cast<int64_t>(len) - static_cast<int64_t>(k - 1) * static_cast<int64_t>(bs);
  return std::max<int64_t>(0, std::min<int64_t>(room, static_cast<int64_t>(bs)));
}

// Byte ranges [a, b) of an object, sorted and merged (the staging copies of
// an in-place call).
struct Ranges {
  std::vector<std::pair<uint64_t, uint64_t>> v;
  void add(int64_t a, int64_t b, uint64_t limit) {
    a = std::max<int64_t>(a, 0);
    b = std::min<int64_t>(b, static_cast<int64_t>(limit));
    if (a < b) v.emplace_back(a, b);
  }
  void merge() {
    std::sort(v.begin(), v.end());
    size_t j = 0;
    for (size_t i = 0; i < v.size(); ++i) {
      if (j && v[i].first <= v[j - 1].second)
        v[j - 1].second = std::max(v[j - 1].second, v[i].second);
      else
        v[j++] = v[i];
    }
    v.resize(j);
  }
};

// The bytes of an object of `len` bytes (k slices of bs, the stream
// kernels' interior tiles of 4 KiB up to `room` bytes of the last slice)
// that an in-place launch does NOT take through the window [lo, hi): every
// 1 KiB interior chunk of slice j not inside the window, and the edge items'
// bytes (from tiles * 4 KiB to the slice end).  `rows`: the slices
// concerned (null: all k).  clip: each range kept inside its own slice (the
// copies out of a decode's staging, whose other slices hold nothing); else
// 16 B of margin each side (the copies into an encode's staging: the edge
// loads read aligned 16-B units).
void outside_window(int k, uint64_t bs, uint64_t len, uint32_t lo, uint32_t hi, const bool* rows,
                    bool clip, Ranges& R) {
  int64_t room = static_cast<int64_t>(len) - static_cast<int64_t>(k - 1) * static_cast<int64_t>(bs);
  room = std::max<int64_t>(0, std::min<int64_t>(room, static_cast<int64_t>(bs)));
  const uint64_t tiles = static_cast<uint64_t>(room) / 4096;
  const int64_t mg = clip ? 0 : 16;
  for (int j = 0; j < k; ++j) {
    if (rows && !rows[j]) continue;
    const int64_t s0 = static_cast<int64_t>(j * bs);
    const uint64_t lim = clip ? std::min<uint64_t>(s0 + bs, len) : len;
    for (uint64_t c = 0; c < tiles * 4; ++c) {
      const int64_t a = s0 + static_cast<int64_t>(c * 1024);
      if (a >= lo && a + 1024 <= hi) continue;
      R.add(a - mg, a + 1024 + mg, lim);
    }
    R.add(s0 + static_cast<int64_t>(tiles * 4096) - mg, s0 + static_cast<int64_t>(bs) + mg, lim);
  }
  R.merge();
}

// liberasurecode_encode's work for one object, into k + m caller-provided
// fragments of bs + 80 bytes (caller holds I.mu, device set).  The kernel
// reads the caller's object in place over PCIe (CallerPin) -- or, when it
// does not register, a copy in pinned, device-mapped staging (host_copy:
// parallel for large objects); while it runs, the host fills the data
// fragments from the object (prepare_fragments_for_encode's copy), then
// copies the parity out.  Objects past the single_pinned_max knob that do not
// register take DMA copies through HBM instead.
int encode_into(Instance& I, const char* data, uint64_t len, uint8_t* const* frags) {
  const int k = I.k, m = I.m;
  PhaseClock clk(I.phase_us);
  const uint64_t bs = blocksize_of(k, I.code.w, len);
  thread_local std::vector<CopyJob> jobs;
  auto data_fragments = [&] {  // payloads = the object's slices, zero padded
    jobs.clear();
    uint64_t left = len;
    const char* src = data;
    for (int j = 0; j < k; ++j) {
      const uint64_t c = std::min(left, bs);
      if (c) jobs.push_back({frags[j] + kHeaderBytes, src, c});
      if (c < bs) jobs.push_back({frags[j] + kHeaderBytes + c, nullptr, bs - c});
      src += c;
      left -= c;
    }
    host_copy(jobs.data(), static_cast<int>(jobs.size()));
  };
  if (bs > 0) {
    const uint64_t fs = round16(kHeaderBytes + round16(bs));
    const uint64_t obj_bytes = round16(len);
    // In place (opt-in, Knobs::register_caller): the kernel reads the
    // caller's object through its whole interior pages (CallerPin) and takes
    // the few bytes outside them -- the chunks at the ends, the edge items --
    // from the staging buffer, to which only those are copied.  Otherwise
    // the whole object is staged.  The parity goes through staging either way.
    CallerPin src;
    const bool can_pin = len <= I.knobs.single_pinned_max;
    uint8_t* pin = can_pin ? I.pin.ensure(obj_bytes + fs * m) : nullptr;
    I.dma_calls += pin == nullptr;
    const bool want_direct = pin && I.knobs.register_caller && len >= I.knobs.direct_min;
    const bool direct = want_direct && src.pin(data, len);
    I.direct_calls += direct;
    Direct dir;
    if (direct) {
      dir.p = reinterpret_cast<const uint8_t*>(data);
      dir.lo = src.lo;
      dir.hi = src.hi;
    }
    // the parity fragments' payloads in place too (up to 8 rows, the
    // stream kernel's per-pass limit), each through its own whole pages
    CallerPin parpin[8];
    bool any_par = false;
    for (int p = 0; want_direct && p < std::min(m, 8); ++p)
      if (parpin[p].pin(frags[k + p] + kHeaderBytes, bs)) {
        dir.par[p] = frags[k + p] + kHeaderBytes;
        dir.plo[p] = parpin[p].lo;
        dir.phi[p] = parpin[p].hi;
        any_par = true;
      }
    hipError_t e = hipSuccess;
    if (!pin && (e = I.scratch.ensure(obj_bytes + fs * m)) != hipSuccess) return hip_errno(e);
    uint8_t* base = pin ? pin : I.scratch.b();
    uint8_t* d_obj = base;
    uint8_t* d_par = base + obj_bytes;
    if (direct) {
      thread_local Ranges R;
      R.v.clear();
      outside_window(k, bs, len, src.lo, src.hi, nullptr, false, R);
      jobs.clear();
      for (const auto& r : R.v) jobs.push_back({d_obj + r.first, data + r.first, r.second - r.first});
      if (obj_bytes > len) jobs.push_back({d_obj + len, nullptr, obj_bytes - len});
      host_copy(jobs.data(), static_cast<int>(jobs.size()));
    } else if (pin) {
      const CopyJob in[2] = {{d_obj, data, len}, {d_obj + len, nullptr, obj_bytes - len}};
      host_copy(in, 2);
    } else if ((e = hipMemcpyAsync(d_obj, data, len, hipMemcpyHostToDevice, I.stream)) != hipSuccess) {
      return hip_errno(e);
    }
    clk.mark(0);
    int rc = run_encode(I, d_obj, obj_bytes, len, 1, d_par, nullptr, fs, fs * m, false, I.stream,
                        direct || any_par ? &dir : nullptr);
    if (rc < 0) {
      (void)hipStreamSynchronize(I.stream);
      return rc;
    }
    clk.mark(1);
    data_fragments();  // on the host, beside the kernel
    clk.mark(2);
    if (!pin)
      for (int p = 0; p < m; ++p)
        if ((e = hipMemcpyAsync(frags[k + p] + kHeaderBytes, d_par + p * fs + kHeaderBytes, bs,
                                hipMemcpyDeviceToHost, I.stream)) != hipSuccess) {
          (void)hipStreamSynchronize(I.stream);
          return hip_errno(e);
        }
    if ((e = hipStreamSynchronize(I.stream)) != hipSuccess) return hip_errno(e);
    if ((e = src.unpin()) != hipSuccess) return hip_errno(e);
    for (auto& pp : parpin)
      if ((e = pp.unpin()) != hipSuccess) return hip_errno(e);
    clk.mark(3);
    if (pin) {
      // a row written in place: only its chunks outside the window and its
      // edge bytes came through staging
      const uint64_t tiles = static_cast<uint64_t>(last_room_of(k, bs, len)) / 4096;
      jobs.clear();
      for (int p = 0; p < m; ++p) {
        uint8_t* dst = frags[k + p] + kHeaderBytes;
        const uint8_t* from = d_par + p * fs + kHeaderBytes;
        if (!dir.par[p]) {
          jobs.push_back({dst, from, bs});
          continue;
        }
        for (uint64_t c = 0; c < tiles * 4; ++c) {
          const uint64_t a = c * 1024;
          if (a >= dir.plo[p] && a + 1024 <= dir.phi[p]) continue;
          jobs.push_back({dst + a, from + a, 1024});
        }
        if (tiles * 4096 < bs) jobs.push_back({dst + tiles * 4096, from + tiles * 4096, bs - tiles * 4096});
      }
      host_copy(jobs.data(), static_cast<int>(jobs.size()));
    }
    clk.mark(4);
  } else {
    data_fragments();
  }
  for (int i = 0; i < k + m; ++i)
    make_header(frags[i], I.code, i, static_cast<uint32_t>(bs), len, I.ct,
                frags[i] + kHeaderBytes, I.legacy_crc);
  clk.mark(5);
  return 0;
}

}  // namespace

int liberasurecode_encode(int desc, const char* orig_data, uint64_t orig_data_size,
                          char*** encoded_data, char*** encoded_parity, uint64_t* fragment_len) {
  if (!orig_data || !encoded_data || !encoded_parity || !fragment_len) return -EINVALIDPARAMS;
  auto I = lookup(desc);
  if (!I) return -EBACKENDNOTAVAIL;
  std::lock_guard<std::mutex> lk(I->mu);
  DeviceGuard g(I->device);
  CallScope cs(*I);
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
  uint8_t* frags[kMaxFragments];
  for (int j = 0; j < k; ++j) {
    if (!(dat[j] = alloc_fragment(fl, false))) return fail(-ENOMEM);
    frags[j] = reinterpret_cast<uint8_t*>(dat[j]);
  }
  for (int p = 0; p < m; ++p) {
    if (!(par[p] = alloc_fragment(fl, false))) return fail(-ENOMEM);
    frags[k + p] = reinterpret_cast<uint8_t*>(par[p]);
  }
  const int rc = encode_into(*I, orig_data, orig_data_size, frags);
  if (rc < 0) return fail(rc);
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
// (`pinned`: d_frags is the zero-copy staging buffer, filled on the host.)
// (`din`, pinned only: inputs read in place by the kernel -- only their
// bytes outside the window, and the edge bytes from `tiles` 4 KiB on, are
// staged.)
int stage_fragments(Instance& I, const Partition& P, uint64_t bs, uint64_t fs, uint8_t* d_frags,
                    uint32_t* mask, bool pinned, const DirectIn* din = nullptr, uint64_t tiles = 0) {
  int c = 0;
  *mask = 0;
  thread_local std::vector<CopyJob> jobs;
  jobs.clear();
  for (int i = 0; i < I.k + I.m && c < I.k; ++i) {
    if (!P.by_idx[i]) continue;
    if (pinned && din && din->p[c]) {
      uint8_t* dst = d_frags + i * fs + kHeaderBytes;
      const uint8_t* from = P.by_idx[i] + kHeaderBytes;
      for (uint64_t x = 0; x < tiles * 4096; x += 1024)
        if (!(x >= din->lo[c] && x + 1024 <= din->hi[c])) jobs.push_back({dst + x, from + x, 1024});
      if (tiles * 4096 < bs) jobs.push_back({dst + tiles * 4096, from + tiles * 4096, bs - tiles * 4096});
    } else if (pinned) {
      jobs.push_back({d_frags + i * fs + kHeaderBytes, P.by_idx[i] + kHeaderBytes, bs});
    } else {
      hipError_t e = hipMemcpyAsync(d_frags + i * fs + kHeaderBytes, P.by_idx[i] + kHeaderBytes,
                                    bs, hipMemcpyHostToDevice, I.stream);
      if (e != hipSuccess) return hip_errno(e);
    }
    *mask |= 1u << i;
    ++c;
  }
  if (pinned) host_copy(jobs.data(), static_cast<int>(jobs.size()));
  return c == I.k ? 0 : -EINSUFFFRAGS;
}

// liberasurecode_decode's checks and partition (caller holds I.mu): the
// decoded length and the fragments by index, or -errno.
struct DecodeIn {
  Partition P;
  int part_rc = 0;  // partition()'s result (-EINSUFFFRAGS / -EBADHEADER) for the GF path
  bool all_data = true;
  uint64_t orig = 0, bs = 0;
};

int decode_prepare(Instance& I, char** frags, int n, uint64_t fragment_len, int force_checks,
                   DecodeIn& D) {
  const int k = I.k;
  if (n < k) return -EINSUFFFRAGS;
  if (fragment_len < kHeaderBytes) return -EBADHEADER;
  for (int i = 0; i < n; ++i)
    if (!frags[i] || header_invalid(reinterpret_cast<const uint8_t*>(frags[i]))) return -EBADHEADER;
  if (force_checks) {
    int bad = 0;
    for (int i = 0; i < n; ++i)
      bad += fragment_invalid(reinterpret_cast<const uint8_t*>(frags[i]), I.code.wire_id);
    if (n - bad < k) return -EINSUFFFRAGS;
  }
  // fragments_to_string preconditions: consistent orig_data_size, and every
  // payload size field inside the fragment buffer (a corrupt or crafted size
  // must not make the copies below read past it)
  D.orig = get64(frags[0] + 12);
  for (int i = 0; i < n; ++i) {
    if (get64(frags[i] + 12) != D.orig) return -EBADHEADER;
    if (static_cast<uint64_t>(get32(frags[i] + 4)) + kHeaderBytes > fragment_len) return -EBADHEADER;
  }
  D.part_rc = partition(I, frags, n, D.P);
  D.all_data = true;
  for (int j = 0; j < k; ++j) D.all_data &= D.P.by_idx[j] != nullptr;
  D.bs = 0;
  for (int i = 0; i < k + I.m; ++i)
    if (D.P.by_idx[i]) {
      D.bs = get32(D.P.by_idx[i] + 4);
      break;
    }
  if (D.bs + kHeaderBytes > fragment_len) return -EBADHEADER;
  if (!(D.all_data && D.part_rc != -EBADHEADER) && D.part_rc < 0) return D.part_rc;
  return 0;
}

// Decode into `out` (D.orig bytes; caller holds I.mu, device set).
int decode_into(Instance& I, const DecodeIn& D, uint8_t* out) {
  const int k = I.k;
  PhaseClock clk(I.phase_us);
  const uint64_t orig = D.orig, bs = D.bs;
  if (D.all_data && D.part_rc != -EBADHEADER) {
    // Fast path (fragments_to_string): every data fragment present, no GF work.
    thread_local std::vector<CopyJob> jobs;
    jobs.clear();
    uint64_t off = 0;
    for (int j = 0; j < k && off < orig; ++j) {
      const uint64_t c = std::min<uint64_t>(orig - off, get32(D.P.by_idx[j] + 4));
      jobs.push_back({out + off, D.P.by_idx[j] + kHeaderBytes, c});
      off += c;
    }
    if (off < orig) jobs.push_back({out + off, nullptr, orig - off});  // short size fields
    host_copy(jobs.data(), static_cast<int>(jobs.size()));
    clk.mark(4);
    return 0;
  }
  const uint64_t fs = round16(kHeaderBytes + round16(bs));
  const uint64_t obj_bytes = round16(orig);
  // In place (opt-in, Knobs::register_caller): the rebuilt slices' chunks
  // inside the caller's whole interior pages are stored there by the kernel
  // (CallerPin); the rest of them -- the chunks at the object's ends, the
  // edge items -- go to the staging buffer at the same offsets and are
  // copied out after it.  The present slices are copied by the host, from
  // their fragments straight into the caller's buffer, beside the kernel.
  const size_t need = fs * (k + I.m) + obj_bytes;
  uint8_t* pin = orig <= I.knobs.single_pinned_max ? I.pin.ensure(need) : nullptr;
  I.dma_calls += pin == nullptr;
  CallerPin dst;
  const bool want_direct = pin && I.knobs.register_caller && orig >= I.knobs.direct_min;
  const bool direct = want_direct && dst.pin(out, orig);
  I.direct_calls += direct;
  // the inputs -- the first k available fragments -- in place through their
  // own whole pages, each one that registers
  CallerPin inpin[kMaxFragments];
  thread_local DirectIn din;
  din = DirectIn{};
  bool any_in = false;
  for (int i = 0, c = 0; want_direct && k <= kDinMax && i < k + I.m && c < k; ++i) {
    if (!D.P.by_idx[i]) continue;
    if (inpin[c].pin(D.P.by_idx[i] + kHeaderBytes, bs)) {
      din.p[c] = D.P.by_idx[i] + kHeaderBytes;
      din.lo[c] = inpin[c].lo;
      din.hi[c] = inpin[c].hi;
      any_in = true;
    }
    ++c;
  }
  const uint64_t tiles = static_cast<uint64_t>(last_room_of(k, bs, orig)) / 4096;
  hipError_t e = hipSuccess;
  if (!pin && (e = I.scratch.ensure(need)) != hipSuccess) return hip_errno(e);
  uint8_t* d_frags = pin ? pin : I.scratch.b();
  uint8_t* d_obj = d_frags + fs * (k + I.m);
  uint32_t mask = 0;
  int rc = stage_fragments(I, D.P, bs, fs, d_frags, &mask, pin != nullptr, any_in ? &din : nullptr, tiles);
  clk.mark(0);
  // Through the pinned staging buffer, the kernel stores only the rebuilt
  // data slices: the present ones go from their fragments straight into the
  // caller's buffer on the host while it runs (round 5: the kernel had
  // stored the whole object over PCIe and the host copied all of it out --
  // 4 MiB decode, 4 data fragments missing: 6 of 10 slices twice over the
  // link and through the staging copy)
  const bool split = pin != nullptr;
  if (rc == 0) {
    DecodeJob J{d_frags, fs, fs * (k + I.m), orig, d_obj, obj_bytes, 1, &mask, nullptr, nullptr};
    J.no_copy = split;
    if (direct) {
      J.direct = out;
      J.direct_lo = dst.lo;
      J.direct_hi = dst.hi;
    }
    if (any_in) J.din = &din;
    rc = run_decode(I, J, I.stream);
  }
  if (rc == 0 && orig && !pin)
    if ((e = hipMemcpyAsync(out, d_obj, orig, hipMemcpyDeviceToHost, I.stream)) != hipSuccess)
      rc = hip_errno(e);
  clk.mark(1);
  thread_local std::vector<CopyJob> jobs;
  bool rebuilt[kMaxFragments];
  for (int j = 0; j < k; ++j) rebuilt[j] = D.P.by_idx[j] == nullptr;
  auto slices = [&](bool present) {  // data slice j of the object: present or rebuilt
    jobs.clear();
    if (!present && direct) {  // only what the kernel did not store in place
      thread_local Ranges R;
      R.v.clear();
      outside_window(k, bs, orig, dst.lo, dst.hi, rebuilt, true, R);
      for (const auto& r : R.v) jobs.push_back({out + r.first, d_obj + r.first, r.second - r.first});
    } else {
      for (int j = 0; j < k; ++j) {
        const uint64_t at = static_cast<uint64_t>(j) * bs;
        if (at >= orig || !rebuilt[j] != present) continue;
        const uint8_t* src = present ? D.P.by_idx[j] + kHeaderBytes : d_obj + at;
        jobs.push_back({out + at, src, std::min(bs, orig - at)});
      }
    }
    host_copy(jobs.data(), static_cast<int>(jobs.size()));
  };
  if (rc == 0 && orig && split) slices(true);
  clk.mark(2);
  if ((e = hipStreamSynchronize(I.stream)) != hipSuccess && rc == 0) rc = hip_errno(e);
  if ((e = dst.unpin()) != hipSuccess && rc == 0) rc = hip_errno(e);
  for (auto& ip : inpin)
    if ((e = ip.unpin()) != hipSuccess && rc == 0) rc = hip_errno(e);
  clk.mark(3);
  if (rc == 0 && orig && split) slices(false);
  clk.mark(4);
  return rc;
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
  CallScope cs(*I);
  DecodeIn D;
  int rc = decode_prepare(*I, available_fragments, num_fragments, fragment_len,
                          force_metadata_checks, D);
  if (rc < 0) return rc;
  char* out = static_cast<char*>(alloc_fragment(D.orig, false));
  if (!out) return -ENOMEM;
  if ((rc = decode_into(*I, D, reinterpret_cast<uint8_t*>(out))) < 0) {
    std::free(out);
    return rc;
  }
  *out_data = out;
  *out_data_len = D.orig;
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
  CallScope cs(*I);
  const int k = I->k, m = I->m;
  if (fragment_len < kHeaderBytes) return -EBADHEADER;
  for (int i = 0; i < num_fragments; ++i)
    if (!available_fragments[i] ||
        header_invalid(reinterpret_cast<const uint8_t*>(available_fragments[i])) ||
        static_cast<uint64_t>(get32(available_fragments[i] + 4)) + kHeaderBytes > fragment_len)
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
    const size_t need = fs * (k + m + 1);
    uint8_t* pin = orig <= I->knobs.single_pinned_max ? I->pin.ensure(need) : nullptr;
    I->dma_calls += pin == nullptr;
    hipError_t e = hipSuccess;
    if (!pin && (e = I->scratch.ensure(need)) != hipSuccess) return hip_errno(e);
    uint8_t* d_frags = pin ? pin : I->scratch.b();
    uint8_t* d_out = d_frags + fs * (k + m);
    uint32_t mask = 0;
    rc = stage_fragments(*I, P, bs, fs, d_frags, &mask, pin != nullptr);
    if (rc == 0) {
      uint8_t hdr[kHeaderBytes] = {0};
      DecodeJob J{d_frags, fs, fs * (k + m), orig, d_out, fs, 1, &mask, &destination_idx, hdr};
      rc = run_decode(*I, J, I->stream);
    }
    if (rc == 0 && !pin &&
        (e = hipMemcpyAsync(out_fragment + kHeaderBytes, d_out + kHeaderBytes, bs,
                            hipMemcpyDeviceToHost, I->stream)) != hipSuccess)
      rc = hip_errno(e);
    if ((e = hipStreamSynchronize(I->stream)) != hipSuccess && rc == 0) rc = hip_errno(e);
    if (rc < 0) return rc;
    if (pin) std::memcpy(out_fragment + kHeaderBytes, d_out + kHeaderBytes, bs);
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

int ecamd_call_phases(int desc, double* us, int n) {
  auto I = lookup(desc);
  if (!I) return -EBACKENDNOTAVAIL;
  if (!us || n < 0) return -EINVALIDPARAMS;
  std::lock_guard<std::mutex> lk(I->mu);
  const int c = std::min(n, 6);
  for (int i = 0; i < c; ++i) us[i] = I->phase_us[i];
  return c;
}

int ecamd_instance_stats(int desc, uint64_t* out, int n) {
  auto I = lookup(desc);
  if (!I) return -EBACKENDNOTAVAIL;
  if (!out || n < 0) return -EINVALIDPARAMS;
  std::lock_guard<std::mutex> lk(I->mu);
  const uint64_t v[5] = {I->marks.size(), pinned_total().load(), I->dma_calls, pinned_budget(),
                         I->direct_calls};
  const int c = std::min(n, 5);
  for (int i = 0; i < c; ++i) out[i] = v[i];
  return c;
}

int ecamd_last_device_error(char* buf, uint64_t n) {
  const hipError_t e = t_last_hip;
  if (buf && n) std::snprintf(buf, n, "%s: %s", hipGetErrorName(e), hipGetErrorString(e));
  return static_cast<int>(e);
}

int ecamd_encode_into(int desc, const char* data, uint64_t data_len, char** fragments,
                      uint64_t fragment_len) {
  if (!data || !fragments) return -EINVALIDPARAMS;
  auto I = lookup(desc);
  if (!I) return -EBACKENDNOTAVAIL;
  std::lock_guard<std::mutex> lk(I->mu);
  DeviceGuard g(I->device);
  CallScope cs(*I);
  if (fragment_len != blocksize_of(I->k, I->code.w, data_len) + kHeaderBytes)
    return -EINVALIDPARAMS;
  uint8_t* frags[kMaxFragments];
  for (int i = 0; i < I->k + I->m; ++i) {
    if (!fragments[i]) return -EINVALIDPARAMS;
    frags[i] = reinterpret_cast<uint8_t*>(fragments[i]);
  }
  return encode_into(*I, data, data_len, frags);
}

int ecamd_decode_into(int desc, char** available_fragments, int num_fragments,
                      uint64_t fragment_len, int force_metadata_checks, char* out,
                      uint64_t out_len) {
  if (!available_fragments || (!out && out_len)) return -EINVALIDPARAMS;
  auto I = lookup(desc);
  if (!I) return -EBACKENDNOTAVAIL;
  std::lock_guard<std::mutex> lk(I->mu);
  DeviceGuard g(I->device);
  CallScope cs(*I);
  DecodeIn D;
  const int rc = decode_prepare(*I, available_fragments, num_fragments, fragment_len,
                                force_metadata_checks, D);
  if (rc < 0) return rc;
  if (out_len != D.orig) return -EINVALIDPARAMS;
  return decode_into(*I, D, reinterpret_cast<uint8_t*>(out));
}

uint64_t ecamd_blocksize(int desc, uint64_t obj_len) {
  auto I = lookup(desc);
  return I ? blocksize_of(I->k, I->code.w, obj_len) : 0;
}

int ecamd_layout_supported(int k, int m, int w, uint64_t obj_len, uint64_t frag_stride,
                           uint64_t n_obj) {
  if (k < 1 || m < 1 || k + m > kMaxFragments || (w != 8 && w != 16)) return -EINVALIDPARAMS;
  return layout_fits(k, m, blocksize_of(k, w, obj_len), frag_stride, n_obj) ? 0 : -EINVALIDPARAMS;
}

int ecamd_decode_matrix(int backend_id, int k, int m, const int* avail, int dest, uint16_t* rows,
                        int* out_idx) {
  const Code* code = code_of(backend_id);
  if (!code || !avail || !rows || !out_idx || k < 1 || m < 1 || k + m > kMaxFragments ||
      dest < -1 || dest >= k + m)
    return -EINVALIDPARAMS;
  for (int c = 0; c < k; ++c)
    if (avail[c] < 0 || avail[c] >= k + m || (c > 0 && avail[c] <= avail[c - 1]))
      return -EINVALIDPARAMS;
  const GfMatrix gen = code->w == 16 ? make_generator(k, m)
                       : backend_id == EC_BACKEND_ISA_L_RS_CAUCHY ? make_isal_cauchy_matrix(k, m)
                                                                  : make_isal_rs_matrix(k, m);
  std::vector<uint16_t> r;
  std::vector<int> o;
  if (!decode_rows(k, code->w, gen, avail, dest, r, o)) return -EINSUFFFRAGS;
  std::memcpy(rows, r.data(), r.size() * sizeof(uint16_t));
  std::memcpy(out_idx, o.data(), o.size() * sizeof(int));
  return static_cast<int>(o.size());
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
  CallScope cs(*I);
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
  CallScope cs(*I);
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
  std::lock_guard<std::mutex> lk(I->mu);
  DeviceGuard g(I->device);
  CallScope cs(*I);
  const uint64_t bs = blocksize_of(I->k, I->code.w, obj_len);
  std::vector<uint8_t> hdr(static_cast<size_t>(n_obj) * kHeaderBytes);
  for (int o = 0; o < n_obj; ++o) {
    if (h_dest[o] < 0 || h_dest[o] >= I->k + I->m) return -EINVALIDPARAMS;
    make_header(&hdr[static_cast<size_t>(o) * kHeaderBytes], I->code, h_dest[o], static_cast<uint32_t>(bs),
                obj_len, I->ct, nullptr, I->legacy_crc);
  }
  DecodeJob J{static_cast<const uint8_t*>(d_frags), frag_stride, stripe_stride, obj_len,
              static_cast<uint8_t*>(d_out), out_stride, n_obj, h_avail, h_dest, hdr.data()};
  J.crc = I->ct == CHKSUM_CRC32 && bs > 0;
  return run_decode(*I, J, static_cast<hipStream_t>(stream));
}

int ecamd_encode_host_batch(int desc, const void* h_objs, uint64_t obj_stride, uint64_t obj_len,
                            int n_obj, void* h_parity, uint64_t frag_stride) {
  if (!h_objs || !h_parity || n_obj < 0) return -EINVALIDPARAMS;
  auto I = lookup(desc);
  if (!I) return -EBACKENDNOTAVAIL;
  if (n_obj == 0) return 0;
  if (obj_len == 0) return -EINVALIDPARAMS;
  if (obj_stride < obj_len || obj_stride % 16 || frag_stride % 16) return -EINVALIDPARAMS;
  const uint64_t bs = blocksize_of(I->k, I->code.w, obj_len);
  if (frag_stride < kHeaderBytes + round16(bs)) return -EINVALIDPARAMS;
  std::lock_guard<std::mutex> lk(I->mu);
  DeviceGuard g(I->device);
  CallScope cs(*I);
  const int m = I->m;
  const uint64_t ps = static_cast<uint64_t>(m) * frag_stride;
  const HostSide H{static_cast<const uint8_t*>(h_objs), obj_stride, obj_len, 0,
                   static_cast<uint8_t*>(h_parity), ps, ps, 48};
  return host_pipeline(*I, n_obj, H, [&](uint8_t* d_in, uint8_t* d_out, int, int n, hipStream_t s) {
    return run_encode(*I, d_in, obj_stride, obj_len, n, d_out, nullptr, frag_stride, ps, true, s);
  });
}

int ecamd_decode_host_batch(int desc, const void* h_frags, uint64_t frag_stride, uint64_t obj_len,
                            int n_obj, const uint32_t* h_avail, void* h_objs,
                            uint64_t obj_stride) {
  if (!h_frags || !h_avail || !h_objs || n_obj < 0) return -EINVALIDPARAMS;
  auto I = lookup(desc);
  if (!I) return -EBACKENDNOTAVAIL;
  if (n_obj == 0) return 0;
  if (obj_len == 0 || obj_stride < obj_len || obj_stride % 16 || frag_stride % 16)
    return -EINVALIDPARAMS;
  const uint64_t bs = blocksize_of(I->k, I->code.w, obj_len);
  if (frag_stride < kHeaderBytes + round16(bs)) return -EINVALIDPARAMS;
  std::lock_guard<std::mutex> lk(I->mu);
  DeviceGuard g(I->device);
  CallScope cs(*I);
  const uint64_t gs = static_cast<uint64_t>(I->k) * frag_stride;
  const HostSide H{static_cast<const uint8_t*>(h_frags), gs, gs, 48,
                   static_cast<uint8_t*>(h_objs), obj_stride, obj_len, 0};
  return host_pipeline(*I, n_obj, H, [&](uint8_t* d_in, uint8_t* d_out, int o0, int n,
                                         hipStream_t s) {
    DecodeJob J{d_in, frag_stride, gs, obj_len, d_out, obj_stride, n, h_avail + o0,
                nullptr, nullptr, true};
    return run_decode(*I, J, s);
  });
}

int ecamd_reconstruct_host_batch(int desc, const void* h_frags, uint64_t frag_stride,
                                 uint64_t obj_len, int n_obj, const uint32_t* h_avail,
                                 const int* h_dest, void* h_out, uint64_t out_stride) {
  if (!h_frags || !h_avail || !h_dest || !h_out || n_obj < 0) return -EINVALIDPARAMS;
  auto I = lookup(desc);
  if (!I) return -EBACKENDNOTAVAIL;
  if (n_obj == 0) return 0;
  const uint64_t bs = blocksize_of(I->k, I->code.w, obj_len);
  if (obj_len == 0 || frag_stride % 16 || out_stride % 16 ||
      frag_stride < kHeaderBytes + round16(bs) || out_stride < kHeaderBytes + round16(bs))
    return -EINVALIDPARAMS;
  std::lock_guard<std::mutex> lk(I->mu);
  DeviceGuard g(I->device);
  CallScope cs(*I);
  std::vector<uint8_t> hdr(static_cast<size_t>(n_obj) * kHeaderBytes);
  for (int o = 0; o < n_obj; ++o) {
    if (h_dest[o] < 0 || h_dest[o] >= I->k + I->m) return -EINVALIDPARAMS;
    make_header(&hdr[static_cast<size_t>(o) * kHeaderBytes], I->code, h_dest[o],
                static_cast<uint32_t>(bs), obj_len, I->ct, nullptr, I->legacy_crc);
  }
  const uint64_t gs = static_cast<uint64_t>(I->k) * frag_stride;
  const HostSide H{static_cast<const uint8_t*>(h_frags), gs, gs, 48,
                   static_cast<uint8_t*>(h_out), out_stride, kHeaderBytes + bs, 48};
  return host_pipeline(*I, n_obj, H, [&](uint8_t* d_in, uint8_t* d_out, int o0, int n,
                                         hipStream_t s) {
    DecodeJob J{d_in, frag_stride, gs, obj_len, d_out, out_stride, n, h_avail + o0,
                h_dest + o0, hdr.data() + static_cast<size_t>(o0) * kHeaderBytes, true};
    J.crc = I->ct == CHKSUM_CRC32 && bs > 0;
    return run_decode(*I, J, s);
  });
}

}  // extern "C"
