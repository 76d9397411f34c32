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

// Finishing pass of the encode kernel's fused parity CRC: parity rows
// row0 .. row0+nrows-1 of every object.  The encode launch left, per object
// and row, one raw CRC per run of its interior 4 KiB tiles -- block b of a
// `grid`-block launch took the interior items [n*b/grid, n*(b+1)/grid), n =
// n_obj * tiles, split at object boundaries -- stored at the run's first
// tile: part[(o * (tiles + edge_tiles) + tile) * m + row].  The edge tiles'
// raw CRC is taken here, from the parity payload the encode wrote.
struct CrcFinishParams {
  uint8_t* parity;          // parity fragment (o, r) at parity + o*stripe_stride + r*frag_stride
  uint64_t frag_stride;
  uint64_t stripe_stride;
  const uint32_t* part;
  const void* maps;         // CrcTables (its raw16 / z4096 / level maps), device memory
  const void* tables;       // CrcFinishTables for (bs, tiles + edge_tiles), device memory
  uint32_t n_obj, m, row0, nrows;
  uint32_t bs, tiles, edge_tiles, grid;
  uint32_t tile_ch;         // 4 KiB tiles per interior item of the encode launch (runs
                            // are cut at item boundaries; `tiles` counts 4 KiB tiles)
};
hipError_t launch_crc_finish(const CrcFinishParams& p, hipStream_t stream);

}  // namespace ecamd
