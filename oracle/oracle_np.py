"""TEST INFRASTRUCTURE ONLY -- an independent numpy restatement of the
liberasurecode_rs_vand arithmetic, used to cross-check the C oracle.

It shares no code and no algorithm choices with rs_vand_oracle.c:
  * GF(2^16) products are carry-less multiplications reduced modulo the
    primitive polynomial 0x1100B (rs_galois.c builds log/antilog tables
    instead);
  * the systematic generator is computed in closed form as
    G = V * inverse(V_top), then every parity column is scaled so the first
    parity row is all ones (liberasurecode_rs_vand.c: make_systematic_matrix
    reaches the same unique matrix by column operations);
  * region products are vectorised over little-endian uint16 symbol arrays.

The GF(2^8) half restates the ISA-L matrices (isa_l_rs_vand /
isa_l_rs_cauchy) the same way -- carry-less products modulo 0x11D, Cauchy
entries as x^254 (the multiplicative inverse), no shared tables -- to check
oracle/isal_oracle.c.

Only tests/ may import it.
"""
from __future__ import annotations

import numpy as np

POLY = 0x1100B


def gf_mul(a: int, b: int) -> int:
    r = 0
    while b:
        if b & 1:
            r ^= a
        b >>= 1
        a <<= 1
        if a & 0x10000:
            a ^= POLY
    return r


def gf_pow(a: int, e: int) -> int:
    r = 1
    for _ in range(e):
        r = gf_mul(r, a)
    return r


def gf_inv(a: int) -> int:
    # a^(2^16 - 2) by square-and-multiply
    r, base, e = 1, a, 0xFFFE
    while e:
        if e & 1:
            r = gf_mul(r, base)
        base = gf_mul(base, base)
        e >>= 1
    return r


def mat_inv(mat: list[list[int]]) -> list[list[int]]:
    n = len(mat)
    a = [row[:] + [1 if i == j else 0 for j in range(n)] for i, row in enumerate(mat)]
    for c in range(n):
        p = next((r for r in range(c, n) if a[r][c]), None)
        if p is None:
            raise ValueError("singular")
        a[c], a[p] = a[p], a[c]
        s = gf_inv(a[c][c])
        a[c] = [gf_mul(v, s) for v in a[c]]
        for r in range(n):
            if r != c and a[r][c]:
                f = a[r][c]
                a[r] = [x ^ gf_mul(f, y) for x, y in zip(a[r], a[c])]
    return [row[n:] for row in a]


def mat_mul(x: list[list[int]], y: list[list[int]]) -> list[list[int]]:
    out = []
    for row in x:
        o = []
        for j in range(len(y[0])):
            acc = 0
            for t, v in enumerate(row):
                acc ^= gf_mul(v, y[t][j])
            o.append(acc)
        out.append(o)
    return out


def generator(k: int, m: int) -> list[list[int]]:
    v = [[gf_pow(i, j) for j in range(k)] for i in range(k + m)]  # 0^0 = 1
    g = mat_mul(v, mat_inv(v[:k]))
    for j in range(k):
        s = gf_inv(g[k][j])
        for r in range(k, k + m):
            g[r][j] = gf_mul(g[r][j], s)
    return g


def _mul_table(c: int) -> np.ndarray:
    """c * x for every 16-bit x, built from the 16 basis products (linearity)."""
    basis = [gf_mul(c, 1 << b) for b in range(16)]
    x = np.arange(1 << 16, dtype=np.uint32)
    out = np.zeros(1 << 16, dtype=np.uint16)
    for b in range(16):
        out ^= np.where((x >> b) & 1, basis[b], 0).astype(np.uint16)
    return out


def region_dot(srcs: list[np.ndarray], row: list[int]) -> np.ndarray:
    """sum_c row[c] * srcs[c] over GF(2^16); srcs are uint16 symbol arrays."""
    acc = np.zeros_like(srcs[0])
    for s, c in zip(srcs, row):
        if c:
            acc ^= _mul_table(c)[s]
    return acc


def encode_payloads(k: int, m: int, data: bytes) -> list[bytes]:
    """Data + parity payloads (no headers), zero padded to the 2k alignment."""
    mult = 2 * k
    bs = ((len(data) + mult - 1) // mult) * mult // k
    buf = np.zeros(k * bs, dtype=np.uint8)
    buf[: len(data)] = np.frombuffer(data, dtype=np.uint8)
    syms = [buf[j * bs:(j + 1) * bs].view("<u2") for j in range(k)]
    g = generator(k, m)
    par = [region_dot(syms, g[k + r]) for r in range(m)]
    return [s.tobytes() for s in syms] + [p.astype("<u2").tobytes() for p in par]


# ---------------- GF(2^8), ISA-L layout ----------------

POLY8 = 0x11D


def gf8_mul(a: int, b: int) -> int:
    r = 0
    while b:
        if b & 1:
            r ^= a
        b >>= 1
        a <<= 1
        if a & 0x100:
            a ^= POLY8
    return r


def gf8_inv(a: int) -> int:
    r, base, e = 1, a, 254  # a^(2^8 - 2)
    while e:
        if e & 1:
            r = gf8_mul(r, base)
        base = gf8_mul(base, base)
        e >>= 1
    return r


def isal_generator(kind: str, k: int, m: int) -> list[list[int]]:
    """kind 'vand': rows k.. are 2^((i-k) j); 'cauchy': 1 / (i ^ j)."""
    rows = [[int(i == j) for j in range(k)] for i in range(k)]
    for i in range(k, k + m):
        if kind == "cauchy":
            rows.append([gf8_inv(i ^ j) for j in range(k)])
        else:
            g = 1
            for _ in range(i - k):
                g = gf8_mul(g, 2)
            row, p = [], 1
            for _ in range(k):
                row.append(p)
                p = gf8_mul(p, g)
            rows.append(row)
    return rows


def _mul_table8(c: int) -> np.ndarray:
    return np.array([gf8_mul(c, x) for x in range(256)], dtype=np.uint8)


def isal_encode_payloads(kind: str, k: int, m: int, data: bytes) -> list[bytes]:
    bs = (len(data) + k - 1) // k
    buf = np.zeros(k * bs, dtype=np.uint8)
    buf[: len(data)] = np.frombuffer(data, dtype=np.uint8)
    slices = [buf[j * bs:(j + 1) * bs] for j in range(k)]
    g = isal_generator(kind, k, m)
    out = [s.tobytes() for s in slices]
    for r in range(m):
        acc = np.zeros(bs, dtype=np.uint8)
        for s, c in zip(slices, g[k + r]):
            if c:
                acc ^= _mul_table8(c)[s]
        out.append(acc.tobytes())
    return out
