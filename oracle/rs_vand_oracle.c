/*
 * oracle/rs_vand_oracle.c -- TEST INFRASTRUCTURE ONLY.
 *
 * Scalar CPU restatement of the `ECDriver(ec_type='liberasurecode_rs_vand')`
 * hot path, used exclusively as the checker in tests/, by
 * __graft_entry__.smoke() and as bench.py's `cpu_baseline` leg.  Nothing in
 * the product (pyeclib_amd/, include/) links, loads or calls this file.
 *
 * Provenance.  The arithmetic does not live in /root/reference: pyeclib's C
 * binding (src/pyeclib_c/pyeclib_c.c:34) includes <liberasurecode/erasurecode.h>
 * and links -lerasurecode (pyproject.toml:46-51); the library is the external,
 * un-vendored liberasurecode, pinned at 1.8.0 (Dockerfile:14, ChangeLog:19).
 * Its source is absent from this container, so this file restates its
 * published algorithm, function by function, naming the upstream file each
 * piece follows:
 *   src/builtin/rs_vand/rs_galois.c              -> gf_init/gf_mul/gf_div
 *   src/builtin/rs_vand/liberasurecode_rs_vand.c -> vand_nonsys/make_systematic/
 *                                                   gj_invert/region_* / encode/
 *                                                   decode/reconstruct rows
 *   src/erasurecode_preprocessing.c              -> aligned size, payload split
 *   src/erasurecode_helpers.c / _postprocessing  -> 80-byte header, checksums
 *   src/erasurecode.c                            -> encode/decode/reconstruct
 *                                                   driver logic, fast path
 * and the pyeclib call sites that pin the boundary:
 *   pyeclib_c.c:537 (encode), :878 (decode), :735 (reconstruct),
 *   :441/:412 (fragment size / minimum encode size), :1085 (metadata).
 *
 * PARITY STATUS: pinned against the reference's own invariants (round trip,
 * reconstruct == original fragment incl. header, fragment-size formula,
 * metadata fields, parity row 0 == XOR of data) and against an independent
 * numpy restatement (oracle/oracle_np.py).  Byte-equality with a real
 * liberasurecode build is UNPINNED in this container.
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <pthread.h>
#include <zlib.h>

/* ---- constants (erasurecode.h / rs_galois.c, liberasurecode 1.8.0) ---- */
#define ORC_W 16
#define ORC_FIELD (1 << 16)
#define ORC_GROUP (ORC_FIELD - 1)
#define ORC_POLY 0x1100B
#define ORC_HDR 80
#define ORC_META 59
#define ORC_MAGIC 0xB0C5ECCu
#define ORC_BACKEND_ID 6
#define ORC_BACKEND_VER 0x00010000u
#define ORC_CHKSUM_NONE 1
#define ORC_CHKSUM_CRC32 2
#define ORC_MAX_FRAGS 32

#define ORC_EBADCHKSUM 205
#define ORC_EINVALIDPARAMS 206
#define ORC_EBADHEADER 207
#define ORC_EINSUFFFRAGS 208

/* ---- GF(2^16) log / antilog (rs_galois.c: rs_galois_init_tables) ---- */
static int g_log[ORC_FIELD];
static int g_ilog_store[ORC_GROUP * 3];
static int *g_ilog = &g_ilog_store[ORC_GROUP];
static pthread_once_t g_once = PTHREAD_ONCE_INIT;

static void gf_build(void)
{
    int x = 1;
    for (int i = 0; i < ORC_GROUP; i++) {
        g_log[x] = i;
        g_ilog_store[i] = x;
        g_ilog_store[i + ORC_GROUP] = x;
        g_ilog_store[i + 2 * ORC_GROUP] = x;
        x <<= 1;
        if (x & ORC_FIELD)
            x ^= ORC_POLY;
    }
}

static void gf_init(void) { pthread_once(&g_once, gf_build); }

/* rs_galois_mult */
static int gf_mul(int a, int b)
{
    if (a == 0 || b == 0)
        return 0;
    return g_ilog[g_log[a] + g_log[b]];
}

/* rs_galois_div */
static int gf_div(int a, int b)
{
    if (a == 0)
        return 0;
    if (b == 0)
        return -1;
    return g_ilog[g_log[a] - g_log[b]];
}

static int gf_inv(int a) { return gf_div(1, a); }

/* ---- generator (liberasurecode_rs_vand.c) ---- */
/* create_non_systematic_vand_matrix: row 0 = [1,0..0], row i = i^j */
static int *vand_nonsys(int k, int m)
{
    int rows = k + m, cols = k;
    int *mat = (int *)malloc(sizeof(int) * rows * cols);
    if (!mat)
        return NULL;
    mat[0] = 1;
    for (int j = 1; j < cols; j++)
        mat[j] = 0;
    for (int i = 1; i < rows; i++) {
        int acc = 1;
        for (int j = 0; j < cols; j++) {
            mat[i * cols + j] = acc;
            acc = gf_mul(acc, i);
        }
    }
    return mat;
}

/* make_systematic_matrix: column operations until the top k x k block is I,
 * then scale each parity column so that the first parity row is all ones. */
static int *make_systematic(int k, int m)
{
    int rows = k + m, cols = k;
    int *mat = vand_nonsys(k, m);
    if (!mat)
        return NULL;
    for (int i = 1; i < cols; i++) {
        int r = i;
        while (r < rows && mat[r * cols + i] == 0)
            r++;
        if (r != i && r < rows) {
            for (int c = 0; c < cols; c++) {
                int t = mat[r * cols + c];
                mat[r * cols + c] = mat[i * cols + c];
                mat[i * cols + c] = t;
            }
        }
        int d = mat[i * cols + i];
        if (d != 1) {
            int s = gf_inv(d);
            for (int rr = 0; rr < rows; rr++)
                mat[rr * cols + i] = gf_mul(mat[rr * cols + i], s);
        }
        for (int j = 0; j < cols; j++) {
            int v = mat[i * cols + j];
            if (j != i && v != 0)
                for (int rr = 0; rr < rows; rr++)
                    mat[rr * cols + j] ^= gf_mul(mat[rr * cols + i], v);
        }
    }
    for (int j = 0; j < cols; j++) {
        int v = mat[k * cols + j];
        if (v != 1) {
            int s = gf_inv(v);
            for (int rr = k; rr < rows; rr++)
                mat[rr * cols + j] = gf_mul(mat[rr * cols + j], s);
        }
    }
    return mat;
}

/* gaussj_inversion (any correct inverse: the decoded bytes are unique) */
static int gj_invert(const int *in, int *out, int n)
{
    int w = 2 * n;
    int *a = (int *)calloc((size_t)n * w, sizeof(int));
    if (!a)
        return -1;
    for (int i = 0; i < n; i++) {
        for (int j = 0; j < n; j++)
            a[i * w + j] = in[i * n + j];
        a[i * w + n + i] = 1;
    }
    for (int i = 0; i < n; i++) {
        int p = i;
        while (p < n && a[p * w + i] == 0)
            p++;
        if (p == n) {
            free(a);
            return -1;
        }
        if (p != i)
            for (int c = 0; c < w; c++) {
                int t = a[p * w + c];
                a[p * w + c] = a[i * w + c];
                a[i * w + c] = t;
            }
        int d = a[i * w + i];
        if (d != 1) {
            int s = gf_inv(d);
            for (int c = 0; c < w; c++)
                a[i * w + c] = gf_mul(a[i * w + c], s);
        }
        for (int r = 0; r < n; r++) {
            int v = a[r * w + i];
            if (r != i && v != 0)
                for (int c = 0; c < w; c++)
                    a[r * w + c] ^= gf_mul(a[i * w + c], v);
        }
    }
    for (int i = 0; i < n; i++)
        for (int j = 0; j < n; j++)
            out[i * n + j] = a[i * w + n + j];
    free(a);
    return 0;
}

/* ---- region ops: little-endian 16-bit words (region_xor/region_multiply) ---- */
static void region_dot(const uint8_t *const *src, uint8_t *dst, const int *row, int n, uint64_t bs)
{
    memset(dst, 0, bs);
    for (int c = 0; c < n; c++) {
        int coef = row[c];
        const uint8_t *s = src[c];
        if (coef == 0)
            continue;
        for (uint64_t t = 0; t + 1 < bs; t += 2) {
            int x = s[t] | (s[t + 1] << 8);
            int y = (coef == 1) ? x : gf_mul(x, coef);
            dst[t] ^= (uint8_t)(y & 0xFF);
            dst[t + 1] ^= (uint8_t)(y >> 8);
        }
    }
}

/* ---- sizes (erasurecode_preprocessing.c: get_aligned_data_size) ---- */
uint64_t orc_blocksize(int k, uint64_t len)
{
    uint64_t mult = (uint64_t)k * (ORC_W / 8);
    uint64_t aligned = ((len + mult - 1) / mult) * mult;
    return aligned / (uint64_t)k;
}

uint64_t orc_fragment_len(int k, uint64_t len) { return orc_blocksize(k, len) + ORC_HDR; }

/* ---- header (erasurecode_helpers.c: add_fragment_metadata et al.) ---- */
static void put32(uint8_t *p, uint32_t v)
{
    p[0] = v & 0xFF; p[1] = (v >> 8) & 0xFF; p[2] = (v >> 16) & 0xFF; p[3] = v >> 24;
}
static uint32_t get32(const uint8_t *p)
{
    return p[0] | (p[1] << 8) | (p[2] << 16) | ((uint32_t)p[3] << 24);
}
static uint64_t get64(const uint8_t *p) { return get32(p) | ((uint64_t)get32(p + 4) << 32); }

static void write_header(uint8_t *frag, int idx, uint64_t bs, uint64_t orig, int ct, uint32_t libec)
{
    memset(frag, 0, ORC_HDR);
    put32(frag + 0, (uint32_t)idx);
    put32(frag + 4, (uint32_t)bs);
    put32(frag + 8, 0);
    put32(frag + 12, (uint32_t)(orig & 0xFFFFFFFFu));
    put32(frag + 16, (uint32_t)(orig >> 32));
    frag[20] = (uint8_t)ct;
    if (ct == ORC_CHKSUM_CRC32)
        put32(frag + 21, (uint32_t)crc32(0L, frag + ORC_HDR, (uInt)bs));
    frag[53] = 0;
    frag[54] = ORC_BACKEND_ID;
    put32(frag + 55, ORC_BACKEND_VER);
    put32(frag + 59, ORC_MAGIC);
    put32(frag + 63, libec);
    put32(frag + 67, (uint32_t)crc32(0L, frag, ORC_META));
}

/* is_invalid_fragment_header: metadata checksum over the 59-byte meta block */
static int header_invalid(const uint8_t *frag)
{
    uint32_t ver = get32(frag + 63);
    if (ver == 0)
        return 1;
    if (ver < 0x010200)
        return 0;
    return get32(frag + 67) != (uint32_t)crc32(0L, frag, ORC_META);
}

int orc_generator(int k, int m, int *out)
{
    gf_init();
    int *g = make_systematic(k, m);
    if (!g)
        return -1;
    memcpy(out, g, sizeof(int) * (k + m) * k);
    free(g);
    return 0;
}

int orc_gf_mul(int a, int b) { gf_init(); return gf_mul(a, b); }
int orc_gf_div(int a, int b) { gf_init(); return gf_div(a, b); }
int orc_invert(const int *in, int *out, int n) { gf_init(); return gj_invert(in, out, n); }
uint32_t orc_crc32(const uint8_t *p, uint64_t n) { return (uint32_t)crc32(0L, p, (uInt)n); }

/* liberasurecode_crc32_alt (upstream src/utils/chksum/crc32.c), the CRC
 * written when LIBERASURECODE_WRITE_LEGACY_CRC is set: the reflected
 * 0xEDB88320 table walk with a signed accumulator, so its right shift is
 * arithmetic (launchpad bug 1666320). */
uint32_t orc_crc32_legacy(const uint8_t *p, uint64_t n)
{
    static uint32_t t[256];
    static int ready;
    if (!ready) {
        for (uint32_t i = 0; i < 256; i++) {
            uint32_t c = i;
            for (int b = 0; b < 8; b++) c = (c & 1) ? 0xEDB88320u ^ (c >> 1) : c >> 1;
            t[i] = c;
        }
        ready = 1;
    }
    int32_t c = (int32_t)0xFFFFFFFFu;
    while (n--) c = (int32_t)(t[((uint32_t)c ^ *p++) & 0xFF] ^ (uint32_t)(c >> 8));
    return (uint32_t)c ^ 0xFFFFFFFFu;
}

/* liberasurecode_encode: out receives k+m fragments of orc_fragment_len bytes */
int orc_encode(int k, int m, int ct, uint32_t libec, const uint8_t *data, uint64_t len, uint8_t *out)
{
    gf_init();
    if (k <= 0 || m <= 0 || k + m > ORC_MAX_FRAGS)
        return -ORC_EINVALIDPARAMS;
    uint64_t bs = orc_blocksize(k, len);
    uint64_t fl = bs + ORC_HDR;
    int *g = make_systematic(k, m);
    if (!g)
        return -12;
    memset(out, 0, fl * (uint64_t)(k + m));
    uint64_t rem = len;
    const uint8_t *p = data;
    for (int j = 0; j < k; j++) {
        uint64_t n = rem > bs ? bs : rem;
        if (n)
            memcpy(out + j * fl + ORC_HDR, p, n);
        p += n;
        rem -= n;
    }
    const uint8_t *src[ORC_MAX_FRAGS];
    for (int j = 0; j < k; j++)
        src[j] = out + j * fl + ORC_HDR;
    for (int r = 0; r < m; r++)
        region_dot(src, out + (uint64_t)(k + r) * fl + ORC_HDR, g + (k + r) * k, k, bs);
    for (int i = 0; i < k + m; i++)
        write_header(out + i * fl, i, bs, len, ct, libec);
    free(g);
    return 0;
}

/* partition + first-k-available rows: shared by decode and reconstruct */
static int partition(int k, int m, const uint8_t *const *frags, int n,
                     const uint8_t **by_idx, int *avail)
{
    for (int i = 0; i < k + m; i++)
        by_idx[i] = NULL;
    for (int i = 0; i < n; i++) {
        uint32_t idx = get32(frags[i]);
        if (idx >= (uint32_t)(k + m))
            return -ORC_EBADHEADER;
        by_idx[idx] = frags[i];
    }
    int na = 0;
    for (int i = 0; i < k + m && na < k; i++)
        if (by_idx[i])
            avail[na++] = i;
    return na == k ? 0 : -ORC_EINSUFFFRAGS;
}

/* inverse of the k x k submatrix of G formed by the first k available rows */
static int decode_matrix(int k, int m, const int *avail, int *inv)
{
    int *g = make_systematic(k, m);
    int *sub = (int *)malloc(sizeof(int) * k * k);
    for (int i = 0; i < k; i++)
        memcpy(sub + i * k, g + avail[i] * k, sizeof(int) * k);
    int rc = gj_invert(sub, inv, k);
    free(sub);
    free(g);
    return rc;
}

/* liberasurecode_decode: out must hold orig_data_size bytes */
int orc_decode(int k, int m, const uint8_t *const *frags, int n, uint64_t fl, uint8_t *out, uint64_t *out_len)
{
    gf_init();
    if (n < k)
        return -ORC_EINSUFFFRAGS;
    if (fl < ORC_HDR)
        return -ORC_EBADHEADER;
    for (int i = 0; i < n; i++)
        if (header_invalid(frags[i]))
            return -ORC_EBADHEADER;
    const uint8_t *by_idx[ORC_MAX_FRAGS];
    int avail[ORC_MAX_FRAGS];
    int rc = partition(k, m, frags, n, by_idx, avail);
    uint64_t orig = get64(frags[0] + 12);
    uint64_t bs = get32(frags[0] + 4);
    if (rc < 0)
        return rc;
    uint8_t *rebuilt[ORC_MAX_FRAGS] = {0};
    int need = 0;
    for (int j = 0; j < k; j++)
        need |= by_idx[j] == NULL;
    if (need) {
        int *inv = (int *)malloc(sizeof(int) * k * k);
        if (decode_matrix(k, m, avail, inv) < 0) {
            free(inv);
            return -ORC_EINSUFFFRAGS;
        }
        const uint8_t *src[ORC_MAX_FRAGS];
        for (int i = 0; i < k; i++)
            src[i] = by_idx[avail[i]] + ORC_HDR;
        for (int j = 0; j < k; j++)
            if (!by_idx[j]) {
                rebuilt[j] = (uint8_t *)malloc(bs ? bs : 1);
                region_dot(src, rebuilt[j], inv + j * k, k, bs);
            }
        free(inv);
    }
    uint64_t off = 0;
    for (int j = 0; j < k && off < orig; j++) {
        const uint8_t *pl = rebuilt[j] ? rebuilt[j] : by_idx[j] + ORC_HDR;
        uint64_t c = orig - off > bs ? bs : orig - off;
        memcpy(out + off, pl, c);
        off += c;
    }
    for (int j = 0; j < k; j++)
        free(rebuilt[j]);
    *out_len = orig;
    return 0;
}

/* liberasurecode_reconstruct_fragment: out receives fl bytes */
int orc_reconstruct(int k, int m, int ct, uint32_t libec, const uint8_t *const *frags, int n,
                    uint64_t fl, int dest, uint8_t *out)
{
    gf_init();
    for (int i = 0; i < n; i++)
        if (header_invalid(frags[i]))
            return -ORC_EBADHEADER;
    const uint8_t *by_idx[ORC_MAX_FRAGS];
    int avail[ORC_MAX_FRAGS];
    int rc = partition(k, m, frags, n, by_idx, avail);
    if (rc < 0)
        return rc;
    if (dest < 0 || dest >= k + m)
        return -ORC_EINVALIDPARAMS;
    if (by_idx[dest]) {
        memcpy(out, by_idx[dest], fl);
        return 0;
    }
    uint64_t orig = get64(frags[0] + 12);
    uint64_t bs = get32(frags[0] + 4);
    int *inv = (int *)malloc(sizeof(int) * k * k);
    if (decode_matrix(k, m, avail, inv) < 0) {
        free(inv);
        return -ORC_EINSUFFFRAGS;
    }
    int row[ORC_MAX_FRAGS];
    if (dest < k) {
        memcpy(row, inv + dest * k, sizeof(int) * k);
    } else {
        int *g = make_systematic(k, m);
        for (int c = 0; c < k; c++) {
            int acc = 0;
            for (int j = 0; j < k; j++)
                acc ^= gf_mul(g[dest * k + j], inv[j * k + c]);
            row[c] = acc;
        }
        free(g);
    }
    const uint8_t *src[ORC_MAX_FRAGS];
    for (int i = 0; i < k; i++)
        src[i] = by_idx[avail[i]] + ORC_HDR;
    memset(out, 0, fl);
    region_dot(src, out + ORC_HDR, row, k, bs);
    write_header(out, dest, bs, orig, ct, libec);
    free(inv);
    return 0;
}
