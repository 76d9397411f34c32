// Launch interface of the gfx950 region kernels (ec_kernels.hip).
//
// All kernels compute outputs[r] = XOR_c M[r][c] * inputs[c] over GF(2^16)
// on little-endian 16-bit symbols, 16 bytes (8 symbols) per lane per input,
// with M supplied as nibble lookup tables (gf16.hpp: build_nibble_tables)
// staged in LDS.  They differ only in where inputs come from and where
// outputs go:
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
constexpr int kTableBytesPerInput = 512;  // 4 nibble positions x 16 values x u64
constexpr int kRowsPerPass = 4;           // one u64 table entry carries 4 products

struct EncodeParams {
  const uint8_t* objs;      // object o at objs + o * obj_stride
  uint64_t obj_stride;
  uint64_t obj_len;
  uint8_t* parity;          // parity fragment (o, p) at parity + o*stripe_stride + p*frag_stride
  uint8_t* data;            // optional data fragments (o, j), same strides
  uint64_t frag_stride;
  uint64_t stripe_stride;
  const uint64_t* tables;   // k * 64 entries for this pass
  const uint8_t* headers;   // (k + m) * 80 precomputed headers, or null
  uint32_t k, m;
  uint32_t row0, nrows;     // parity rows handled by this pass
  uint32_t bs;              // payload bytes per fragment
  uint32_t n_obj;
  uint32_t tiles, first_edge;  // set by the launcher (ec_kernels.hip: split_tiles)
};

// Per-object decode / reconstruct descriptor (device memory).
struct ObjDesc {
  uint8_t in_idx[32];   // fragment index of input c (first k available)
  uint8_t out_idx[4];   // destination of output row r (data index, or fragment
                        // index for reconstruct)
  uint8_t n_out;        // rows in this pass
  uint8_t copy_inputs;  // decode pass 0: copy present data inputs to the object
  uint8_t pad[2];
  uint32_t table;       // table set index (k * 64 u64 each, per pass)
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
  const uint64_t* tables;   // table sets
  const uint8_t* headers;   // reconstruct: header rows (80 B), else null
  uint32_t k, m;
  uint32_t bs;
  uint32_t n_obj;
  uint32_t reconstruct;     // 1 = write fragment payload + header
  uint32_t tiles, first_edge;  // set by the launcher (ec_kernels.hip: split_tiles)
  uint32_t copy_shift;      // set by the launcher: interior copies are line-aligned
};

hipError_t launch_encode(const EncodeParams& p, hipStream_t stream);
hipError_t launch_decode(const DecodeParams& p, hipStream_t stream);

// Number of 256-chunk tiles per fragment payload.
inline uint32_t tiles_per_fragment(uint32_t bs) {
  const uint32_t chunks = (bs + 15) / 16;
  return (chunks + kThreadsPerBlock - 1) / kThreadsPerBlock;
}

}  // namespace ecamd
