// Launch interface of the gfx950 region kernels (ec_kernels_impl.hpp).
//
// All kernels compute outputs[r] = XOR_c M[r][c] * inputs[c] over the code's
// field -- GF(2^16) on little-endian 16-bit symbols (liberasurecode_rs_vand)
// or GF(2^8) on bytes (ISA-L layout: isa_l_rs_vand / isa_l_rs_cauchy) -- 16
// bytes per lane per input, with M supplied as nibble lookup tables
// (gf16.hpp / gf8.hpp: build_nibble_tables*) staged in LDS.  They differ
// only in where inputs come from and where outputs go:
//   encode      inputs  = k slices of a contiguous object (zero padded past
//                         obj_len: liberasurecode's prepare_fragments_for_encode)
//               outputs = m parity payloads (+ optional data fragments)
//   decode      inputs  = first k available fragments of each object
//               outputs = the object bytes (present data copied, missing
//                         data rebuilt): liberasurecode_decode
//   reconstruct inputs  = first k available fragments
//               outputs = one fragment payload per object
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

namespace ecamd {

constexpr int kHeaderBytes = 80;
constexpr int kThreadsPerBlock = 256;
constexpr int kRowsPerPass = 4;  // one table entry carries the products of 4 rows

// Table bytes per input column: 4 nibble positions x 16 values x u64
// (GF(2^16)) or 2 nibble positions x 16 values x u32 (GF(2^8)).
__host__ __device__ constexpr uint32_t table_bytes_per_input(uint32_t w) {
  return w == 16 ? 512u : 128u;
}

// Decode keeps one table set per wave in LDS; a slot is rounded up to 256 B
// so that its base fits the second byte of an LDS address (ec_kernels_impl.hpp,
// kb), and 4 slots of the largest set (k = 31, GF(2^16)) stay below 64 KiB.
__host__ __device__ constexpr uint32_t table_slot_bytes(uint32_t k, uint32_t w) {
  return (k * table_bytes_per_input(w) + 255u) & ~255u;
}

// A/B builds.  The product library has no tuning switches: every launch
// takes the measured default, and nothing is read from the environment on
// the launch path.  `make -C pyeclib_amd/csrc ab` builds a separate library
// (tools/build/libpyeclib_amd_ab.so, -DECAMD_AB) in which the launchers also
// instantiate the alternative kernels of past A/B runs -- including the
// memory-only probes ECAMD_ENC_NOCOMP / ECAMD_DEC_NOCOMP, whose output is
// WRONG -- selected by name through ecamd_ab_set() (tools/ab_bench.py).
#ifdef ECAMD_AB
constexpr bool kAB = true;
int ab_knob(const char* name, int dflt);  // ec_dispatch.cpp
#else
constexpr bool kAB = false;
inline int ab_knob(const char*, int dflt) { return dflt; }
#endif

struct EncodeParams {
  const uint8_t* objs;      // object o at objs + o * obj_stride
  uint64_t obj_stride;
  uint64_t obj_len;
  uint8_t* parity;          // parity fragment (o, p) at parity + o*stripe_stride + p*frag_stride
  uint8_t* data;            // optional data fragments (o, j), same strides
  uint64_t frag_stride;
  uint64_t stripe_stride;
  const uint32_t* tables;   // k * table_bytes_per_input(w) bytes for this pass
  const uint8_t* headers;   // (k + m) * 80 precomputed headers, or null
  uint32_t k, m, w;         // w = field bits (16 or 8)
  uint32_t row0, nrows;     // parity rows handled by this pass
  uint32_t bs;              // payload bytes per fragment
  uint32_t n_obj;
  uint32_t tiles, edge_tiles;  // set by the launcher: interior / edge items per object
  uint32_t tile_ch;            // set by the launcher: an interior item spans tile_ch * 4 KiB
                               // (edge items 4 KiB each, from tiles * tile_ch * 4 KiB on)
  uint32_t xcd_split;          // set by the launcher (item_range)
  uint32_t fused_edges;        // set by the launcher: edge items run in the interior launch
  uint32_t edge_blocks;        // set by the launcher: blocks [0, edge_blocks) run only the edge
                               // items; 0 = every block runs its share of them first
  uint32_t no_edge_blocks;     // caller: 1 = never run the edge items in blocks of their own
                               // (the round-2 launch form; instance knob ECAMD_EDGE_BLOCKS=0)
  // inline_crc32 (crc_lanes null: none).  The launch takes the raw CRC of
  // every 1 KiB chunk of the interior it writes -- parity rows into
  // crc_part[(o * chunks + c) * m + row], with the full stripe the data
  // fragments into crc_part_data[(o * chunks + c) * k + j], chunks = the
  // interior's 1 KiB chunks per payload (<= bs / 1024) -- and the launcher
  // then runs the finishing pass (ec_crc.hpp) over those fragments.
  const void* crc_lanes;         // CrcLaneTables (crc32.hpp), device memory
  const void* crc_finish_tables; // CrcFinishTables for bs, device memory
  uint32_t* crc_part;
  uint32_t* crc_part_data;
  // One object read in place (ecamd_encode_into, the caller's whole pages
  // registered; n_obj = 1, stream kernel only): an interior 1 KiB input
  // chunk at object offset c with [c, c + 1024) inside [direct_lo,
  // direct_hi) is loaded from `direct` (the caller's object, device-mapped);
  // every other input byte -- those chunks and the edge items -- from objs,
  // the staged copy, which the caller fills for exactly those bytes.
  // null = off.
  const uint8_t* direct;
  uint32_t direct_lo, direct_hi;
  // Parity row q of this pass written in place (ecamd_encode_into, the
  // caller's parity fragments' whole pages registered; stream kernel only):
  // its 1 KiB interior chunk at payload offset x with [x, x + 1024) inside
  // [dpar_lo[q], dpar_hi[q]) is stored to dpar[q] + x (the fragment's
  // payload, device-mapped); every other parity byte to `parity` as usual.
  // null = that row staged.
  uint8_t* dpar[8];
  uint32_t dpar_lo[8], dpar_hi[8];
};

// Loader / consumer kernels (ec_kernels_impl.hpp encode_dma_kernel ...):
// taken for k >= kDmaMinK when a launch has a kDmaItem interior item for
// every CU and the input offsets j * bs + x fit 32 bits.
constexpr int kDmaMinK = 4;
constexpr uint32_t kDmaItem = 16 * 1024;
inline bool dma_batch(uint32_t k, uint32_t bs, uint64_t obj_len, uint32_t n_obj, int cus,
                      const void* direct = nullptr) {
  if (k < static_cast<uint32_t>(kDmaMinK) || direct != nullptr) return false;
  if (static_cast<uint64_t>(k) * bs + 65536u > 0xFFFFFFFFull) return false;
  int64_t room = static_cast<int64_t>(obj_len) - static_cast<int64_t>(k - 1) * bs;
  if (room > static_cast<int64_t>(bs)) room = bs;
  if (room < 0) room = 0;
  return static_cast<uint64_t>(room) / kDmaItem * n_obj >= static_cast<uint64_t>(cus);
}

// Per-object decode / reconstruct descriptor (device memory).
struct ObjDesc {
  uint8_t in_idx[32];   // fragment index of input c (first k available)
  uint8_t out_idx[4];   // destination of output row r (data index, or fragment
                        // index for reconstruct)
  uint8_t n_out;        // rows in this pass
  uint8_t copy_inputs;  // decode pass 0: copy present data inputs to the object
  uint8_t pad[2];
  uint32_t table;       // table set index (k * table_bytes_per_input(w) bytes each)
  uint32_t header;      // reconstruct: header row index, else unused
  uint32_t pad2;
};

struct DecodeParams {
  const uint8_t* frags;     // fragment (o, i) at frags + o*stripe_stride + i*frag_stride
  uint64_t frag_stride;
  uint64_t stripe_stride;
  uint64_t obj_len;
  uint8_t* out;             // decode: object o at out + o*out_stride
                            // reconstruct: fragment o at out + o*out_stride
  uint64_t out_stride;
  const ObjDesc* desc;
  const uint32_t* tables;   // table sets
  const uint8_t* headers;   // reconstruct: header rows (80 B), else null
  uint32_t k, m, w;
  uint32_t bs;
  uint32_t n_obj;
  uint32_t reconstruct;     // 1 = write fragment payload + header
  uint32_t compact;         // 1 = input c of object o at frags + o*stripe_stride
                            //     + c*frag_stride (only the k inputs are present)
  uint32_t mode;            // kernel variant (ec_kernels_impl.hpp DecodeMode): 0 = decode
                            // with every missing row in this pass, 1 = reconstruct,
                            // 2 = generic (multi-pass decode)
  uint32_t tiles, edge_tiles;  // set by the launcher: interior / edge items per object
  uint32_t xcd_split;          // set by the launcher (item_range)
  uint32_t fused_edges;        // set by the launcher: edge items run in the interior launch
  uint32_t edge_blocks;        // set by the launcher (see EncodeParams)
  uint32_t no_edge_blocks;     // caller (see EncodeParams)
  uint32_t tile_ch;            // set by the launcher: 4 KiB tiles per interior item
  // reconstruct with inline_crc32 (crc_lanes null: none): the raw CRC of every
  // 1 KiB interior chunk of fragment o into crc_part[o * chunks + c], then the
  // finishing pass (see EncodeParams)
  const void* crc_lanes;
  const void* crc_finish_tables;
  uint32_t* crc_part;
  // One object decoded in place (ecamd_decode_into, the caller's output
  // pages registered; n_obj = 1, MODE kDecode, stream kernel only): a
  // rebuilt row's 1 KiB interior chunk at object offset c with [c, c + 1024)
  // inside [direct_lo, direct_hi) is stored to `direct` (the caller's
  // buffer, device-mapped); every other output byte to `out` (staging, at
  // the same offset), which the caller copies out.  null = off.
  uint8_t* direct;
  uint32_t direct_lo, direct_hi;
  // Input c (of the first k available) of that object read in place: its
  // 1 KiB interior chunk at payload offset x with [x, x + 1024) inside
  // [din_lo[c], din_hi[c]) is loaded from din[c] + x (the caller's fragment
  // payload, device-mapped); every other input byte from `frags` (staged).
  // null = that input staged.
  const uint8_t* din[32];
  uint32_t din_lo[32], din_hi[32];
};
constexpr int kDinMax = 16;  // inputs read in place only for k <= 16

// Dispatch on (p.w, p.k) to the per-k instantiations (ec_dispatch.cpp).
hipError_t launch_encode(const EncodeParams& p, hipStream_t stream);
hipError_t launch_decode(const DecodeParams& p, hipStream_t stream);


}  // namespace ecamd
