"""The decode rows the kernels apply (ecamd_decode_matrix; no GPU): the
runtime finds them with one e x e inversion instead of liberasurecode_rs_vand's
k x k Gauss-Jordan (ec_runtime.cpp decode_rows), so here every row is checked
against the definition with the independent numpy restatement (oracle_np):
a decode row for missing data j times G[avail] is the unit vector e_j, a
reconstruct row for fragment d times G[avail] is G[d].  Exhaustive over the
erasure patterns of small codes, sampled for larger ones."""
import ctypes
import itertools
import random

import pytest

from oracle import oracle_np as N
from pyeclib_amd import _native

RS_VAND, ISAL_VAND, ISAL_CAUCHY = 6, 4, 7


def rows_of(backend, k, m, avail, dest):
    a = (ctypes.c_int * k)(*avail)
    rows = (ctypes.c_uint16 * (k * k))()
    out = (ctypes.c_int * k)()
    n = _native.lib.ecamd_decode_matrix(backend, k, m, a, dest, rows, out)
    return n, [list(rows[i * k:(i + 1) * k]) for i in range(max(n, 0))], list(out[:max(n, 0)])


def field(backend):
    return (N.gf_mul if backend == RS_VAND else N.gf8_mul)


def generator(backend, k, m):
    if backend == RS_VAND:
        return N.generator(k, m)
    return N.isal_generator("cauchy" if backend == ISAL_CAUCHY else "vand", k, m)


def apply(mul, row, mat_rows):
    k = len(mat_rows[0])
    out = [0] * k
    for c, coef in enumerate(row):
        if coef:
            for j in range(k):
                out[j] ^= mul(coef, mat_rows[c][j])
    return out


def check_pattern(backend, k, m, avail, G):
    mul = field(backend)
    sub = [G[i] for i in avail]
    n, rows, out = rows_of(backend, k, m, avail, -1)
    missing = [j for j in range(k) if j not in avail]
    assert n == len(missing) and out == missing
    for j, row in zip(out, rows):
        assert apply(mul, row, sub) == [int(i == j) for i in range(k)], (avail, j)
    for d in [i for i in range(k + m) if i not in avail]:
        n, rows, out = rows_of(backend, k, m, avail, d)
        assert n == 1 and out == [d]
        assert apply(mul, rows[0], sub) == G[d], (avail, d)


@pytest.mark.parametrize("backend,k,m", [(RS_VAND, 4, 2), (RS_VAND, 6, 3), (ISAL_CAUCHY, 5, 3),
                                         (ISAL_VAND, 4, 2)])
def test_every_pattern_small_codes(backend, k, m):
    G = generator(backend, k, m)
    for avail in itertools.combinations(range(k + m), k):
        check_pattern(backend, k, m, list(avail), G)


@pytest.mark.parametrize("backend,k,m", [(RS_VAND, 10, 4), (RS_VAND, 12, 4), (RS_VAND, 20, 8),
                                         (ISAL_CAUCHY, 12, 4), (RS_VAND, 28, 4)])
def test_sampled_patterns(backend, k, m):
    G = generator(backend, k, m)
    rng = random.Random(k * 100 + m)
    pats = {tuple(range(k)), tuple(range(m, k + m))}
    while len(pats) < 12:
        pats.add(tuple(sorted(rng.sample(range(k + m), k))))
    for avail in pats:
        check_pattern(backend, k, m, list(avail), G)


def test_bad_arguments():
    bad = -_native.EINVALIDPARAMS
    assert rows_of(RS_VAND, 4, 2, [0, 1, 1, 2], -1)[0] == bad      # not ascending
    assert rows_of(RS_VAND, 4, 2, [0, 1, 2, 6], -1)[0] == bad      # index out of range
    assert rows_of(RS_VAND, 4, 2, [0, 1, 2, 3], 6)[0] == bad       # dest out of range
    assert rows_of(99, 4, 2, [0, 1, 2, 3], -1)[0] == bad           # unknown backend
    assert rows_of(RS_VAND, 4, 2, [0, 1, 2, 3], -1)[0] == 0        # nothing missing
