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

// Tables for the GPU payload CRC.  A CRC-32 register is GF(2)-linear in the
// message: with raw(M) the register after M from a zero start,
// crc32(0, M) = raw(M) ^ Z_n(0xFFFFFFFF) ^ 0xFFFFFFFF, where Z_n appends n
// zero bytes, and raw(A || B) = Z_|B|(raw(A)) ^ raw(B).  That holds for the
// legacy variant too (its arithmetic shift is linear as well), with its own
// Z.  Every linear map is stored as nibble tables -- map(r) = XOR_q
// T[q][nibble_q(r)] -- eight LDS lookups.
//
// The kernels take the raw CRC of each 1 KiB chunk a wave holds (lane l
// holding bytes [16 l, 16 l + 16)): raw(chunk) = XOR_l Z_{16 (63 - l)}(
// raw16(piece_l)), i.e. per lane the 32 lookups of raw16 and the 8 of its
// own lane map, then an XOR across the wave (no shifts between lanes).
struct CrcLaneTables {
  uint32_t raw16[32][16];     // raw CRC of a 16-byte piece, per nibble position
  uint32_t lane[8][16][64];   // Z_{16 (63 - l)}: [q][v][lane], lane-minor, so the
                              // 64 lanes of a lookup hit 64 different banks
  // The matrix-core form (round 6, crc_device.hpp mfma_*): the chunk's 8192
  // bits times a 0/1 matrix on v_mfma_i32_32x32x32_i8, one bit plane of the
  // 16 bytes per instruction, the parity of each sum in bit 7 of its i32.
  uint32_t mst[4][16][64];    // second stage: lane l's 16 row sums -> Z_{16 (31 - r)}
                              // of its column's bit, by nibble [q][v][lane]
  int8_t mfb[8][64][16];      // B operands: [bit plane][lane][byte]; read into
                              // registers from device memory, never copied to LDS
};
static_assert(sizeof(CrcLaneTables) % 16 == 0, "copied to LDS in 16-B pieces");
// What the kernels copy to LDS: everything before mfb.
constexpr unsigned kCrcLdsBytes = static_cast<unsigned>(offsetof(CrcLaneTables, mfb));
static_assert(kCrcLdsBytes % 16 == 0, "copied to LDS in 16-B pieces");

// The finishing pass (ec_crc.hip) shifts every chunk's raw CRC to the end
// of the bs-byte payload -- chunk c ends at 1024 (c + 1), so by Z_r after
// Z_{1024 a}, r = bs mod 1024 -- XORs them with the payload tail's (read
// back, end-aligned: no zero padding to remove), and folds in the init /
// final XORs.  The header's metadata checksum was computed on the host with
// chksum[0] = 0; the checksum of the same 59 bytes with chksum[0] = c
// differs from it by meta(c), a linear map of c (the init and final terms
// cancel between two messages of one length).
constexpr int kCrcPowBits = 22;  // bs / 1024 < 2^22 (payloads < 4 GiB)
struct CrcFinishTables {
  uint32_t pow[kCrcPowBits][8][16];  // Z_{1024 * 2^i}
  uint32_t zr[8][16];                // Z_{bs mod 1024}
  uint32_t meta[8][16];              // c (header bytes 21..24) -> metadata checksum change
  uint32_t z16[6][8][16];            // Z_{16 * 2^k}: the lane tree of an edge chunk
  uint32_t init_term;                // Z_bs(0xFFFFFFFF) ^ 0xFFFFFFFF
  uint32_t pad[3];
};
static_assert(sizeof(CrcFinishTables) % 16 == 0, "copied to LDS in 16-B pieces");

void build_crc_lane_tables(bool legacy, CrcLaneTables* out);
void build_crc_finish_tables(uint32_t bs, bool legacy, CrcFinishTables* out);

}  // namespace ecamd
