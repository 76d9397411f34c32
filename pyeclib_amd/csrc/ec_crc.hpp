// Launch interface of the GPU payload CRC's finishing pass (ec_crc.hip).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

namespace ecamd {

// liberasurecode's set_checksum / set_metadata_chksum for fragments whose
// payloads a region kernel has just written (encode parity, full-stripe data
// fragments, reconstructed fragments).  That kernel left, per fragment, one
// raw CRC per 1 KiB chunk of its interior -- chunks [0, chunks), i.e. bytes
// [0, 1024 chunks) -- at part[(o * chunks + c) * part_rows + part_row0 + r];
// the payload past them (the edge items' bytes) is read back here.  The
// fragment's header (80 bytes, already written) gets chksum[0] and its
// metadata checksum.
struct CrcFinishParams {
  uint8_t* frags;           // fragment (o, r) at frags + o*stripe_stride + r*frag_stride
  uint64_t frag_stride;
  uint64_t stripe_stride;
  const uint32_t* part;
  uint32_t part_rows, part_row0;
  const void* lanes;        // CrcLaneTables (crc32.hpp), device memory
  const void* tables;       // CrcFinishTables for bs, device memory
  uint32_t n_obj, count;    // fragments r = 0 .. count - 1 of every object
  uint32_t bs, chunks;
};
hipError_t launch_crc_finish(const CrcFinishParams& p, hipStream_t stream);

}  // namespace ecamd
