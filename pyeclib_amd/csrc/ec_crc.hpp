// Launch interface of the GPU payload CRC (ec_crc.hip).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

namespace ecamd {

struct CrcParams {
  uint8_t* frags;           // fragment (o, i) at frags + o*stripe_stride + i*frag_stride,
                            // 80-byte header already written, payload at +80
  uint64_t frag_stride;
  uint64_t stripe_stride;
  uint32_t first, count;    // fragments first .. first+count-1 of every object
  uint32_t n_obj;
  uint32_t bs;              // payload bytes
  uint32_t steps;           // ceil(bs / 4096)
  const void* tables;       // CrcTables for (bs, steps), device memory
};

// Writes chksum[0] = crc32(0, payload, bs) and the metadata checksum into
// each fragment's header.
hipError_t launch_crc(const CrcParams& p, hipStream_t stream);

}  // namespace ecamd
