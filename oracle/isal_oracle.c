/*
 * oracle/isal_oracle.c -- TEST INFRASTRUCTURE ONLY.
 *
 * Scalar CPU restatement of the GF(2^8) Reed-Solomon codes that pyeclib
 * reaches as ec_type 'isa_l_rs_vand' (backend id 4) and 'isa_l_rs_cauchy'
 * (id 7) (src/pyeclib/enums.py:13,16): liberasurecode 1.8.0's ISA-L backends
 * over ISA-L v2.32.0 (pinned at /root/reference Dockerfile:14-15).  Used only
 * by tests/ as the checker for the GPU path; nothing in the product links it.
 *
 * Provenance.  Neither ISA-L nor liberasurecode is in /root/reference or in
 * this container, so this restates their published algorithms:
 *   ISA-L erasure_code/ec_base.c     -> gf8 tables (poly 0x11D, generator 2),
 *                                       gf_gen_rs_matrix, gf_gen_cauchy1_matrix,
 *                                       gf_invert_matrix, ec_encode_data (byte
 *                                       dot products)
 *   liberasurecode isa_l_common.c    -> encode with rows k..k+m-1; decode and
 *                                       reconstruct from the first k available
 *                                       fragments (inverse rows; parity rows =
 *                                       generator row x inverse)
 *   erasurecode_helpers.c            -> aligned size = ceil(len / k) * k (w = 8),
 *                                       the 80-byte header (same layout as
 *                                       rs_vand_oracle.c)
 * PARITY STATUS: unpinned against a real ISA-L / liberasurecode build (none
 * here); pinned by round trips, reconstruct == encode byte for byte,
 * systematic identity rows and an independent numpy restatement
 * (oracle/oracle_np.py).  The header's backend_version values are the
 * liberasurecode ISA-L backend versions as remembered (2.13.0 / 2.14.1) and
 * are UNPINNED.
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <zlib.h>

#define O8_HDR 80
#define O8_META 59
#define O8_MAGIC 0xB0C5ECCu
#define O8_MAX_FRAGS 32
#define O8_CHKSUM_CRC32 2
#define O8_EINVALIDPARAMS 206
#define O8_EBADHEADER 207
#define O8_EINSUFFFRAGS 208

enum { O8_VAND = 4, O8_CAUCHY = 7 };

static uint8_t g8_log[256], g8_exp[512];
static int g8_ready;

static void g8_init(void)
{
    if (g8_ready)
        return;
    int x = 1;
    for (int i = 0; i < 255; i++) {
        g8_exp[i] = g8_exp[i + 255] = (uint8_t)x;
        g8_log[x] = (uint8_t)i;
        x <<= 1;
        if (x & 0x100)
            x ^= 0x11D;
    }
    g8_ready = 1;
}

static uint8_t g8_mul(uint8_t a, uint8_t b)
{
    if (!a || !b)
        return 0;
    return g8_exp[g8_log[a] + g8_log[b]];
}

static uint8_t g8_inv(uint8_t a) { return g8_exp[255 - g8_log[a]]; }

/* (k+m) x k generator; kind = O8_VAND (gf_gen_rs_matrix) or O8_CAUCHY */
static void gen_matrix(int kind, int k, int m, uint8_t *a)
{
    memset(a, 0, (size_t)(k + m) * k);
    for (int i = 0; i < k; i++)
        a[i * k + i] = 1;
    if (kind == O8_CAUCHY) {
        for (int i = k; i < k + m; i++)
            for (int j = 0; j < k; j++)
                a[i * k + j] = g8_inv((uint8_t)(i ^ j));
        return;
    }
    uint8_t gen = 1;
    for (int i = k; i < k + m; i++) {
        uint8_t p = 1;
        for (int j = 0; j < k; j++) {
            a[i * k + j] = p;
            p = g8_mul(p, gen);
        }
        gen = g8_mul(gen, 2);
    }
}

/* gf_invert_matrix: Gauss-Jordan with row swaps; -1 when singular */
static int invert(const uint8_t *in, uint8_t *out, int n)
{
    uint8_t a[O8_MAX_FRAGS][2 * O8_MAX_FRAGS];
    for (int i = 0; i < n; i++) {
        for (int j = 0; j < n; j++) {
            a[i][j] = in[i * n + j];
            a[i][n + j] = (uint8_t)(i == j);
        }
    }
    for (int c = 0; c < n; c++) {
        int p = c;
        while (p < n && !a[p][c])
            p++;
        if (p == n)
            return -1;
        if (p != c)
            for (int j = 0; j < 2 * n; j++) {
                uint8_t t = a[p][j];
                a[p][j] = a[c][j];
                a[c][j] = t;
            }
        uint8_t s = g8_inv(a[c][c]);
        for (int j = 0; j < 2 * n; j++)
            a[c][j] = g8_mul(a[c][j], s);
        for (int r = 0; r < n; r++) {
            uint8_t f = a[r][c];
            if (r == c || !f)
                continue;
            for (int j = 0; j < 2 * n; j++)
                a[r][j] ^= g8_mul(f, a[c][j]);
        }
    }
    for (int i = 0; i < n; i++)
        for (int j = 0; j < n; j++)
            out[i * n + j] = a[i][n + j];
    return 0;
}

/* ec_encode_data for one output row */
static void dot(const uint8_t *const *src, uint8_t *dst, const uint8_t *row, int n, uint64_t bs)
{
    memset(dst, 0, bs);
    for (int c = 0; c < n; c++) {
        uint8_t coef = row[c];
        if (!coef)
            continue;
        for (uint64_t t = 0; t < bs; t++)
            dst[t] ^= g8_mul(src[c][t], coef);
    }
}

uint64_t o8_blocksize(int k, uint64_t len) { return (len + (uint64_t)k - 1) / (uint64_t)k; }

static void put32(uint8_t *p, uint32_t v)
{
    p[0] = v & 0xFF; p[1] = (v >> 8) & 0xFF; p[2] = (v >> 16) & 0xFF; p[3] = v >> 24;
}
static uint32_t get32(const uint8_t *p)
{
    return p[0] | (p[1] << 8) | (p[2] << 16) | ((uint32_t)p[3] << 24);
}

static uint32_t backend_version(int kind) { return kind == O8_CAUCHY ? 0x00020E01u : 0x00020D00u; }

static void write_header(uint8_t *f, int kind, int idx, uint64_t bs, uint64_t orig, int ct,
                         uint32_t libec)
{
    memset(f, 0, O8_HDR);
    put32(f + 0, (uint32_t)idx);
    put32(f + 4, (uint32_t)bs);
    put32(f + 12, (uint32_t)(orig & 0xFFFFFFFFu));
    put32(f + 16, (uint32_t)(orig >> 32));
    f[20] = (uint8_t)ct;
    if (ct == O8_CHKSUM_CRC32)
        put32(f + 21, (uint32_t)crc32(0L, f + O8_HDR, (uInt)bs));
    f[54] = (uint8_t)kind;
    put32(f + 55, backend_version(kind));
    put32(f + 59, O8_MAGIC);
    put32(f + 63, libec);
    put32(f + 67, (uint32_t)crc32(0L, f, O8_META));
}

int o8_generator(int kind, int k, int m, uint8_t *out)
{
    g8_init();
    if (k <= 0 || m <= 0 || k + m > O8_MAX_FRAGS)
        return -O8_EINVALIDPARAMS;
    gen_matrix(kind, k, m, out);
    return 0;
}

int o8_gf_mul(int a, int b) { g8_init(); return g8_mul((uint8_t)a, (uint8_t)b); }

int o8_encode(int kind, int k, int m, int ct, uint32_t libec, const uint8_t *data, uint64_t len,
              uint8_t *out)
{
    g8_init();
    if (k <= 0 || m <= 0 || k + m > O8_MAX_FRAGS)
        return -O8_EINVALIDPARAMS;
    uint64_t bs = o8_blocksize(k, len), fl = bs + O8_HDR;
    uint8_t g[O8_MAX_FRAGS * O8_MAX_FRAGS];
    gen_matrix(kind, k, m, g);
    memset(out, 0, fl * (uint64_t)(k + m));
    uint64_t rem = len;
    for (int j = 0; j < k; j++) {
        uint64_t n = rem > bs ? bs : rem;
        if (n)
            memcpy(out + j * fl + O8_HDR, data + (uint64_t)j * bs, n);
        rem -= n;
    }
    const uint8_t *src[O8_MAX_FRAGS];
    for (int j = 0; j < k; j++)
        src[j] = out + j * fl + O8_HDR;
    for (int r = 0; r < m; r++)
        dot(src, out + (uint64_t)(k + r) * fl + O8_HDR, g + (k + r) * k, k, bs);
    for (int i = 0; i < k + m; i++)
        write_header(out + i * fl, kind, i, bs, len, ct, libec);
    return 0;
}

/* first k available fragments (index order) and the inverse of their rows */
static int prepare(int kind, int k, int m, const uint8_t *const *frags, int n,
                   const uint8_t **by_idx, int *avail, uint8_t *inv)
{
    for (int i = 0; i < k + m; i++)
        by_idx[i] = NULL;
    for (int i = 0; i < n; i++) {
        uint32_t idx = get32(frags[i]);
        if (idx >= (uint32_t)(k + m))
            return -O8_EBADHEADER;
        by_idx[idx] = frags[i];
    }
    int na = 0;
    for (int i = 0; i < k + m && na < k; i++)
        if (by_idx[i])
            avail[na++] = i;
    if (na < k)
        return -O8_EINSUFFFRAGS;
    uint8_t g[O8_MAX_FRAGS * O8_MAX_FRAGS], sub[O8_MAX_FRAGS * O8_MAX_FRAGS];
    gen_matrix(kind, k, m, g);
    for (int i = 0; i < k; i++)
        memcpy(sub + i * k, g + avail[i] * k, (size_t)k);
    return invert(sub, inv, k) ? -O8_EINSUFFFRAGS : 0;
}

int o8_decode(int kind, int k, int m, const uint8_t *const *frags, int n, uint8_t *out,
              uint64_t *out_len)
{
    g8_init();
    const uint8_t *by_idx[O8_MAX_FRAGS];
    int avail[O8_MAX_FRAGS];
    uint8_t inv[O8_MAX_FRAGS * O8_MAX_FRAGS];
    int rc = prepare(kind, k, m, frags, n, by_idx, avail, inv);
    if (rc < 0)
        return rc;
    uint64_t orig = get32(frags[0] + 12) | ((uint64_t)get32(frags[0] + 16) << 32);
    uint64_t bs = get32(frags[0] + 4);
    const uint8_t *src[O8_MAX_FRAGS];
    for (int i = 0; i < k; i++)
        src[i] = by_idx[avail[i]] + O8_HDR;
    uint8_t *tmp = (uint8_t *)malloc(bs ? bs : 1);
    uint64_t off = 0;
    for (int j = 0; j < k && off < orig; j++) {
        const uint8_t *pl = by_idx[j] ? by_idx[j] + O8_HDR : NULL;
        if (!pl) {
            dot(src, tmp, inv + j * k, k, bs);
            pl = tmp;
        }
        uint64_t c = orig - off > bs ? bs : orig - off;
        memcpy(out + off, pl, c);
        off += c;
    }
    free(tmp);
    *out_len = orig;
    return 0;
}

int o8_reconstruct(int kind, int k, int m, int ct, uint32_t libec, const uint8_t *const *frags,
                   int n, uint64_t fl, int dest, uint8_t *out)
{
    g8_init();
    const uint8_t *by_idx[O8_MAX_FRAGS];
    int avail[O8_MAX_FRAGS];
    uint8_t inv[O8_MAX_FRAGS * O8_MAX_FRAGS];
    int rc = prepare(kind, k, m, frags, n, by_idx, avail, inv);
    if (rc < 0)
        return rc;
    if (dest < 0 || dest >= k + m)
        return -O8_EINVALIDPARAMS;
    if (by_idx[dest]) {
        memcpy(out, by_idx[dest], fl);
        return 0;
    }
    uint64_t orig = get32(frags[0] + 12) | ((uint64_t)get32(frags[0] + 16) << 32);
    uint64_t bs = get32(frags[0] + 4);
    uint8_t row[O8_MAX_FRAGS];
    if (dest < k) {
        memcpy(row, inv + dest * k, (size_t)k);
    } else {
        uint8_t g[O8_MAX_FRAGS * O8_MAX_FRAGS];
        gen_matrix(kind, k, m, g);
        for (int c = 0; c < k; c++) {
            uint8_t acc = 0;
            for (int j = 0; j < k; j++)
                acc ^= g8_mul(g[dest * k + j], inv[j * k + c]);
            row[c] = acc;
        }
    }
    const uint8_t *src[O8_MAX_FRAGS];
    for (int i = 0; i < k; i++)
        src[i] = by_idx[avail[i]] + O8_HDR;
    memset(out, 0, fl);
    dot(src, out + O8_HDR, row, k, bs);
    write_header(out, kind, dest, bs, orig, ct, libec);
    return 0;
}
