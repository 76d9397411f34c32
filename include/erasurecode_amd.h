/*
 * erasurecode_amd.h -- C ABI of libpyeclib_amd.so, the MI355X-native
 * Reed-Solomon backend behind pyeclib's ECDriver.
 *
 * Part 1 mirrors, name for name and argument for argument, the liberasurecode
 * 1.8.0 entry points that pyeclib's C binding binds (the upstream header is
 * <liberasurecode/erasurecode.h>, included at src/pyeclib_c/pyeclib_c.c:34).
 * Each declaration cites the pyeclib call site it serves, so the library can
 * be linked in place of -lerasurecode (pyproject.toml:46-51) without touching
 * pyeclib_c.c.  The GF(2^16) region arithmetic behind encode / decode /
 * reconstruct runs in hand-written gfx950 kernels; fragments (80-byte header
 * included) are byte-compatible with backend liberasurecode_rs_vand (id 6).
 *
 * Part 2 adds batched, device-resident entry points (ecamd_*) for callers
 * that keep objects in HBM.  Plain pointers and sizes only; `stream` is a
 * hipStream_t passed as void* (NULL = default stream).
 *
 * Errors are negative errno-style values from LIBERASURECODE_ERROR_CODES
 * (pyeclib maps them at pyeclib_c.c:125-183); no entry point aborts.
 */
#ifndef ERASURECODE_AMD_H
#define ERASURECODE_AMD_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---------- types (liberasurecode erasurecode.h, 1.8.0) ---------- */

typedef enum {
    EC_BACKEND_NULL = 0,
    EC_BACKEND_JERASURE_RS_VAND = 1,
    EC_BACKEND_JERASURE_RS_CAUCHY = 2,
    EC_BACKEND_FLAT_XOR_HD = 3,
    EC_BACKEND_ISA_L_RS_VAND = 4,
    EC_BACKEND_SHSS = 5,
    EC_BACKEND_LIBERASURECODE_RS_VAND = 6,  /* served by the MI355X kernels */
    EC_BACKEND_ISA_L_RS_CAUCHY = 7,
    EC_BACKEND_LIBPHAZR = 8,
    EC_BACKEND_ISA_L_RS_VAND_INV = 9,
    EC_BACKEND_ISA_L_RS_LRC = 10,
    EC_BACKEND_AMD_RS_VAND = 11,            /* new ec_type 'amd_rs_vand': same code, same bytes */
    EC_BACKENDS_MAX
} ec_backend_id_t;

typedef enum {
    CHKSUM_NONE = 1,
    CHKSUM_CRC32 = 2,
    CHKSUM_MD5 = 3,
    CHKSUM_TYPES_MAX
} ec_checksum_type_t;

typedef enum {
    EBACKENDNOTSUPP = 200,
    EECMETHODNOTIMPL = 201,
    EBACKENDINITERR = 202,
    EBACKENDINUSE = 203,
    EBACKENDNOTAVAIL = 204,
    EBADCHKSUM = 205,
    EINVALIDPARAMS = 206,
    EBADHEADER = 207,
    EINSUFFFRAGS = 208
} LIBERASURECODE_ERROR_CODES;

struct ec_args {
    int k;   /* data fragments */
    int m;   /* parity fragments */
    int w;   /* word size in bits; set to 16 by this backend */
    int hd;  /* hamming distance (= m for RS) */
    union {
        struct { uint64_t arg1; } null_args;
        struct { uint64_t x, y; uint64_t z, a; } reserved; /* .x = local_parity (pyeclib_c.c:254) */
    } priv_args1;
    void *priv_args2;
    ec_checksum_type_t ct;  /* CHKSUM_NONE or CHKSUM_CRC32 (pyeclib_c.c:248) */
};

#define LIBERASURECODE_MAX_CHECKSUM_LEN 8
#define LIBERASURECODE_FRAG_HEADER_MAGIC 0xb0c5ecc

typedef struct __attribute__((__packed__)) fragment_metadata {
    uint32_t idx;
    uint32_t size;
    uint32_t frag_backend_metadata_size;
    uint64_t orig_data_size;
    uint8_t chksum_type;
    uint32_t chksum[LIBERASURECODE_MAX_CHECKSUM_LEN];
    uint8_t chksum_mismatch;
    uint8_t backend_id;
    uint32_t backend_version;
} fragment_metadata_t; /* 59 bytes */

typedef struct __attribute__((__packed__)) fragment_header_s {
    fragment_metadata_t meta;
    uint32_t magic;
    uint32_t libec_version;
    uint32_t metadata_chksum;
    uint8_t padding[9];
} fragment_header_t; /* 80 bytes */

/* ---------- Part 1: liberasurecode-compatible entry points ---------- */

/* pyeclib_c.c:1209 (check_backend_available).  1 iff id is 6 or 11 and a
 * gfx950 device is visible. */
int liberasurecode_backend_available(const ec_backend_id_t backend_id);

/* pyeclib_c.c:259.  Returns a descriptor > 0, or -errno. */
int liberasurecode_instance_create(const ec_backend_id_t id, struct ec_args *args);

/* pyeclib_c.c:322.  Double destroy returns -EBACKENDNOTAVAIL. */
int liberasurecode_instance_destroy(int desc);

/* pyeclib_c.c:537.  Allocates k data + m parity fragments of *fragment_len
 * bytes each (80-byte header + payload); release with _encode_cleanup. */
int liberasurecode_encode(int desc, const char *orig_data, uint64_t orig_data_size,
                          char ***encoded_data, char ***encoded_parity,
                          uint64_t *fragment_len);

/* pyeclib_c.c:562 */
int liberasurecode_encode_cleanup(int desc, char **encoded_data, char **encoded_parity);

/* pyeclib_c.c:878.  *out_data is allocated; release with _decode_cleanup. */
int liberasurecode_decode(int desc, char **available_fragments, int num_fragments,
                          uint64_t fragment_len, int force_metadata_checks,
                          char **out_data, uint64_t *out_data_len);

/* pyeclib_c.c:919 */
int liberasurecode_decode_cleanup(int desc, char *data);

/* pyeclib_c.c:735.  Caller allocates out_fragment (fragment_len bytes). */
int liberasurecode_reconstruct_fragment(int desc, char **available_fragments,
                                        int num_fragments, uint64_t fragment_len,
                                        int destination_idx, char *out_fragment);

/* pyeclib_c.c:640.  -1 terminated lists in and out. */
int liberasurecode_fragments_needed(int desc, int *fragments_to_reconstruct,
                                    int *fragments_to_exclude, int *fragments_needed);

/* pyeclib_c.c:1085 */
int liberasurecode_get_fragment_metadata(char *fragment, fragment_metadata_t *fragment_metadata);

/* pyeclib_c.c:1163.  fragments point at fragment_metadata_t blocks. */
int liberasurecode_verify_stripe_metadata(int desc, char **fragments, int num_fragments);

/* erasurecode.h helper; aligned size = ceil(len / 2k) * 2k for w = 16. */
int liberasurecode_get_aligned_data_size(int desc, uint64_t data_len);

/* pyeclib_c.c:412 */
int liberasurecode_get_minimum_encode_size(int desc);

/* pyeclib_c.c:441/:457/:477.  Payload bytes per fragment (header excluded). */
int liberasurecode_get_fragment_size(int desc, int data_len);

/* pyeclib_c.c:310/:1218.  Version of the fragment format written (1.8.0). */
uint32_t liberasurecode_get_version(void);

/* ---------- Part 2: device-resident batch API (MI355X) ---------- */

/* Payload bytes per fragment for objects of obj_len bytes. */
uint64_t ecamd_blocksize(int desc, uint64_t obj_len);

/* liberasurecode_encode (pyeclib_c.c:537) into caller-allocated fragments:
 * the same k + m fragments (80-byte header + payload each), written into
 * fragments[0 .. k+m-1], each fragment_len = blocksize + 80 bytes (else
 * -EINVALIDPARAMS).  A binding that owns its output objects (pyeclib_c wraps
 * liberasurecode's buffers in new bytes objects, pyeclib_c.c:544-560) can
 * hand their storage here and skip that copy.  Synchronous; 0 or -errno. */
int ecamd_encode_into(int desc, const char *data, uint64_t data_len, char **fragments,
                      uint64_t fragment_len);

/* Host-side phases of the instance's last single-object encode / decode,
 * in microseconds: [0] staging copy in, [1] launch, [2] host work beside the
 * kernel (encode: the data fragments), [3] wait for the kernel, [4] copy
 * out, [5] headers.  Returns the count written (<= n) or -errno. */
int ecamd_call_phases(int desc, double *us, int n);

/* Bookkeeping of an instance, for tests: [0] stream end marks held (a
 * caller that takes a new stream per call must not grow it), [1] pinned
 * staging bytes held by the process, [2] single-object calls of this
 * instance that staged through HBM instead (over the pinned budget or past
 * the size limit), [3] the process's pinned budget in bytes
 * (ECAMD_PINNED_TOTAL_MB), [4] single-object calls of this instance that
 * used the caller's pages in place (ECAMD_REGISTER_CALLER).  Returns the
 * count written (<= n) or -errno. */
int ecamd_instance_stats(int desc, uint64_t *out, int n);

/* The device-runtime error behind the calling thread's last -EBACKENDINITERR
 * from an entry point (pyeclib maps that code to "Unknown error",
 * pyeclib_c.c:170-173): its name and text into buf (NUL-terminated, at most
 * n bytes); returns the runtime's error code, 0 when the last call had none. */
int ecamd_last_device_error(char *buf, uint64_t n);

/* liberasurecode_decode (pyeclib_c.c:878) into a caller buffer of exactly
 * the decoded length (orig_data_size of the fragments' headers; else
 * -EINVALIDPARAMS).  Same checks, fast path and errors; synchronous. */
int ecamd_decode_into(int desc, char **available_fragments, int num_fragments,
                      uint64_t fragment_len, int force_metadata_checks, char *out,
                      uint64_t out_len);

/* Encode n_obj objects of obj_len bytes resident in HBM.
 *   d_objs:   object o at d_objs + o*obj_stride (obj_stride % 16 == 0)
 *   d_parity: parity fragment p of object o (80-byte header + payload) at
 *             d_parity + o*stripe_stride + p*frag_stride
 *   d_data:   optional (may be NULL): data fragment j of object o, headers
 *             included, at d_data + o*stripe_stride + j*frag_stride
 *   frag_stride % 16 == 0, frag_stride >= 80 + round_up(blocksize, 16);
 *   stripe_stride % 16 == 0.  A full-stripe layout [n_obj][k+m][frag_stride]
 *   is d_data = base, d_parity = base + k*frag_stride,
 *   stripe_stride = (k+m)*frag_stride.
 * Asynchronous on `stream`; returns 0 or -errno.
 * Streams: an instance orders the rewrite of its own device buffers (cached
 * descriptors, decode table pool) after its earlier launches on every stream
 * it was given, with GPU-side event waits -- never a device-wide
 * synchronisation -- so a stream passed to any ecamd_* call must remain valid
 * until the instance is destroyed (liberasurecode_instance_destroy waits for
 * the instance's work on those streams). */
int ecamd_encode_batch(int desc, const void *d_objs, uint64_t obj_stride, uint64_t obj_len,
                       int n_obj, void *d_parity, void *d_data, uint64_t frag_stride,
                       uint64_t stripe_stride, void *stream);

/* Decode n_obj objects from fragments resident in HBM.
 *   d_frags:  fragment i of object o at d_frags + o*stripe_stride + i*frag_stride
 *   h_avail:  host array of n_obj bitmasks; bit i set = fragment i usable
 *   d_objs:   output, object o at d_objs + o*obj_stride (obj_len bytes)
 * Uses the first k available fragments of each object (liberasurecode's
 * choice); present data fragments are copied, missing ones rebuilt. */
int ecamd_decode_batch(int desc, const void *d_frags, uint64_t frag_stride,
                       uint64_t stripe_stride, uint64_t obj_len, int n_obj,
                       const uint32_t *h_avail, void *d_objs, uint64_t obj_stride, void *stream);

/* Rebuild one fragment per object (index h_dest[o], header included) into
 * d_out + o*out_stride from the first k available fragments. */
int ecamd_reconstruct_batch(int desc, const void *d_frags, uint64_t frag_stride,
                            uint64_t stripe_stride, uint64_t obj_len, int n_obj,
                            const uint32_t *h_avail, const int *h_dest, void *d_out,
                            uint64_t out_stride, void *stream);

/* Host-resident encode: objects in host memory, parity fragments written
 * back to host memory.  Synchronous.  When both host arrays are pinned
 * (hipHostMalloc / hipHostRegister, device-mapped) the kernels read and write
 * them directly over PCIe; otherwise chunks of objects are copied H2D on three
 * streams, kernels write the outputs (pinned) or HBM + D2H copies (pageable).
 * Parity fragment p of object o at
 * h_parity + (o*m + p)*frag_stride; objects as in ecamd_encode_batch.
 * Replaces, for a batch, the host side of pyeclib_c_encode
 * (src/pyeclib_c/pyeclib_c.c:512-565): bytes in, fragments out. */
int ecamd_encode_host_batch(int desc, const void *h_objs, uint64_t obj_stride, uint64_t obj_len,
                            int n_obj, void *h_parity, uint64_t frag_stride);

/* Host-resident decode (the read path: Swift fetches k fragments per object).
 *   h_frags:  the k fragments used for object o, in ascending fragment index,
 *             fragment i of the group at h_frags + (o*k + i)*frag_stride
 *             (80-byte header + payload)
 *   h_avail:  n_obj bitmasks; the k lowest set bits name the fragments in
 *             h_frags (liberasurecode uses the first k available)
 *   h_objs:   output, object o at h_objs + o*obj_stride (obj_len bytes)
 * Paths as ecamd_encode_host_batch; synchronous.  Replaces, for a
 * batch, pyeclib_c_decode (src/pyeclib_c/pyeclib_c.c:770-922). */
int ecamd_decode_host_batch(int desc, const void *h_frags, uint64_t frag_stride, uint64_t obj_len,
                            int n_obj, const uint32_t *h_avail, void *h_objs,
                            uint64_t obj_stride);

/* Host-resident reconstruct: inputs as ecamd_decode_host_batch; fragment
 * h_dest[o] (header included) written to h_out + o*out_stride.  Replaces,
 * for a batch, pyeclib_c_reconstruct (src/pyeclib_c/pyeclib_c.c:681-758). */
int ecamd_reconstruct_host_batch(int desc, const void *h_frags, uint64_t frag_stride,
                                 uint64_t obj_len, int n_obj, const uint32_t *h_avail,
                                 const int *h_dest, void *h_out, uint64_t out_stride);

/* Device ordinal used by this process (hipGetDevice at create time). */
int ecamd_device(int desc);

/* The decode matrix the kernels apply for one erasure pattern (needs no GPU;
 * liberasurecode_rs_vand's decode: rows of inverse(G[avail]), the first k
 * available fragments avail[0..k-1] ascending).  dest = -1: one row per
 * missing data fragment; dest >= 0: the row rebuilding fragment dest.
 * rows: up to k rows x k u16 coefficients (GF(2^16); GF(2^8) values for the
 * ISA-L codes); out_idx: the fragment index each row produces.  Returns the
 * row count, or -EINVALIDPARAMS / -EINSUFFFRAGS (singular submatrix). */
int ecamd_decode_matrix(int backend_id, int k, int m, const int *avail, int dest, uint16_t *rows,
                        int *out_idx);

/* Does a batch layout fit the kernels' 32-bit buffer offsets?  0, or
 * -EINVALIDPARAMS when it does not: k*blocksize + 16 (an object's slices;
 * decode's output window holds 2^31 - 1 bytes), (k+m)*frag_stride (a stripe's
 * fragments) or the batch's 4 KiB work items pass their limit.  Every
 * encode / decode / reconstruct entry point (single object or batch) applies
 * it and returns -EINVALIDPARAMS instead of launching; needs no GPU.  w = 16
 * (rs_vand) or 8 (ISA-L codes). */
int ecamd_layout_supported(int k, int m, int w, uint64_t obj_len, uint64_t frag_stride,
                           uint64_t n_obj);

#ifdef __cplusplus
}
#endif

#endif /* ERASURECODE_AMD_H */
