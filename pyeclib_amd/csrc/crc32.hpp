// CRC-32 (IEEE 802.3, reflected 0xEDB88320) as used in fragment headers.
//
// liberasurecode >= 1.6.2 writes zlib-compatible crc32(0, buf, len) for both
// the payload checksum (chksum[0] when chksum_type == CHKSUM_CRC32) and the
// 59-byte metadata checksum (upstream src/erasurecode_helpers.c:
// set_checksum / set_metadata_chksum), and on verification also accepts its
// older "alt" variant, whose table walk used a signed int accumulator so the
// right shift is arithmetic (upstream src/utils/chksum/crc32.c:
// liberasurecode_crc32_alt; launchpad bug 1666320).
#pragma once

#include <cstddef>
#include <cstdint>

namespace ecamd {

uint32_t crc32(uint32_t crc, const void* buf, size_t len);
uint32_t crc32_legacy(uint32_t crc, const void* buf, size_t len);

}  // namespace ecamd
