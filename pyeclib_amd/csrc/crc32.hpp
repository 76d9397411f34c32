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

namespace ecamd {

// Tables for the GPU payload CRC (ec_crc.hip).  A zlib CRC-32 register is
// GF(2)-linear in the message: with raw(M) the register after M from a zero
// start, crc32(0, M) = raw(M) ^ Z_n(0xFFFFFFFF) ^ 0xFFFFFFFF, where Z_n
// appends n zero bytes, and raw(A || B) = Z_|B|(raw(A)) ^ raw(B).  Every
// linear map is stored as nibble tables [q 0..7][v 0..15] (u32) so that
// map(r) = XOR_q T[q][nibble_q(r)] -- eight conflict-free LDS lookups.
struct CrcTables {
  uint32_t raw16[32][16];     // raw CRC of a 16-byte chunk, per nibble position
  uint32_t z4096[8][16];      // Z_4096
  uint32_t level[8][8][16];   // Z_{16 * 2^l}, l = 0..7 (lane tree)
  uint32_t z8192[8][16];      // Z_8192, Z_12288, Z_16384: the loader / consumer encode's
  uint32_t z12288[8][16];     // wave tree and Horner steps (12 / 16 KiB items)
  uint32_t z16384[8][16];
  uint32_t unshift[8][16];    // Z_pad^-1: drops the zero padding past the payload
  uint32_t t0[256];           // bytewise table (header metadata CRC)
  uint32_t init_term;         // Z_bs(0xFFFFFFFF) ^ 0xFFFFFFFF
  uint32_t pad[3];
};
static_assert(sizeof(CrcTables) % 16 == 0, "CrcTables is copied to LDS in 16-B pieces");

// Tables for payloads of `bs` bytes processed in `steps` rounds of 4 KiB.
void build_crc_tables(uint32_t bs, uint32_t steps, CrcTables* out);

// The encode kernel's fused parity CRC (ec_kernels_impl.hpp) leaves one raw
// CRC per run of 4 KiB tiles; the finishing pass (ec_crc.hip) shifts each to
// the end of the zero-padded payload, XORs them, removes the padding and
// folds in the init / final XORs.
constexpr int kCrcPowBits = 20;  // tiles_total < 2^20 (payloads < 4 GiB)
struct CrcFinishTables {
  uint32_t pow[kCrcPowBits][8][16];  // Z_{4096 * 2^i}
  uint32_t unshift[8][16];           // Z_pad^-1, pad = tiles_total * 4096 - bs
  uint32_t t0[256];                  // bytewise table (header metadata CRC)
  uint32_t init_term;                // Z_bs(0xFFFFFFFF) ^ 0xFFFFFFFF
  uint32_t pad[3];
};
static_assert(sizeof(CrcFinishTables) % 16 == 0, "copied to LDS in 16-B pieces");

void build_crc_finish_tables(uint32_t bs, uint32_t tiles_total, CrcFinishTables* out);

}  // namespace ecamd
