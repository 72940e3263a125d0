"""CPU emulation of the large-body chunk combine (crc32_chunk_combine_kernel,
rpc_amd/csrc/crc32_kernels.hip) against zlib.

The kernel folds the RAW chunk CRCs of a body as
    crc = ~(A_L(F) ^ XOR_k A_{(nch-1-k)*chunk}(raw_k))
with every shift A_n applied map by map from the nibble tables
NIB[k][i][j] = A_{2^k bytes}(j << 4i).  Here the same tables, the same
thread-strided Horner (step map A_{NT*chunk}), the same per-thread shift to the
body end and the same per-block split are run in Python with a small NT, and
the result is compared with zlib.crc32 of the body (zlib 1.2.11 is the
reference's arithmetic).
"""
import random
import zlib

import pytest

POLY = 0xEDB88320
X0 = 0x80000000


def mulmod(a, b):
    m, p = X0, 0
    for _ in range(32):
        if a & m:
            p ^= b
        m >>= 1
        b = (b >> 1) ^ POLY if b & 1 else b >> 1
    return p


def build_nib(maps=40):
    nib, sq = [], X0 >> 8  # x^8: one zero byte; squared: x^(8 * 2^k)
    for _ in range(maps):
        nib.append([[mulmod(sq, j << (4 * i)) for j in range(16)] for i in range(8)])
        sq = mulmod(sq, sq)
    return nib


NIB = build_nib()


def nib_apply(k, v):
    r = 0
    for i in range(8):
        r ^= NIB[k][i][(v >> (4 * i)) & 15]
    return r


def nib_shift(nbytes, v):  # the kernel's nib_shift: one map per set bit of nbytes
    k = 0
    while nbytes:
        if nbytes & 1:
            v = nib_apply(k, v)
        nbytes >>= 1
        k += 1
    return v


def crc0(data: bytes) -> int:
    """Raw register from state 0, no conditioning: crc0(M) = ~crc(M) ^ A_|M|(F)."""
    return (~zlib.crc32(data) & 0xFFFFFFFF) ^ nib_shift(len(data), 0xFFFFFFFF)


def combine_emulated(body: bytes, chunk: int, nt: int, splits: int) -> int:
    L = len(body)
    nch = (L + chunk - 1) // chunk
    # end-aligned chunks (expand_chunks / the contiguous fast path)
    raw = []
    for k in range(nch):
        end = L - (nch - 1 - k) * chunk
        raw.append(crc0(body[max(0, end - chunk):end]))
    out = 0
    pb = (nch + splits - 1) // splits
    for s in range(splits):
        c0, c1 = s * pb, min(s * pb + pb, nch)
        if c0 >= c1:
            continue
        block = 0
        for t in range(nt):
            acc, k = 0, c0 + t
            while k < c1:
                acc = nib_shift(nt * chunk, acc) ^ raw[k]
                k += nt
            if c0 + t < c1:
                kl = c0 + t + (c1 - 1 - (c0 + t)) // nt * nt
                acc = nib_shift((nch - 1 - kl) * chunk, acc)
            block ^= acc
        if s == 0:
            block ^= ~nib_shift(L, 0xFFFFFFFF) & 0xFFFFFFFF
        out ^= block  # splits == 1: plain store; splits > 1: atomicXor into zeroed out
    return out


def test_nib_shift_is_zlib_combine():
    rnd = random.Random(5)
    for _ in range(30):
        a = rnd.randbytes(rnd.randint(0, 64))
        b = rnd.randbytes(rnd.randint(0, 3000))
        assert nib_shift(len(b), zlib.crc32(a)) ^ zlib.crc32(b) == zlib.crc32(a + b)


@pytest.mark.parametrize("L,chunk,nt,splits", [
    (1, 16, 4, 1), (4096, 1024, 4, 1), (5000, 1024, 4, 1), (5000, 1024, 2, 3), (70 * 64 + 3, 64, 8, 1),
    (70 * 64 + 3, 64, 8, 4), (33 * 48, 48, 4, 2), (256 * 16, 16, 16, 1), (1000, 4096, 4, 1),
])
def test_combine_matches_zlib(L, chunk, nt, splits):
    body = random.Random(L * 31 + chunk).randbytes(L)
    assert combine_emulated(body, chunk, nt, splits) == zlib.crc32(body)
