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


# ---- big-body route fold (big_combine_kernel) --------------
# crc = ~XOR_k A_{(nch-1-k) chunk}(raw_k) with raw_0 ^= A_{len0}(F) (zlib's
# pre-conditioning enters with chunk 0: Tq[len0 mod 4096] then one A_{2^k} map per
# set bit of len0 >> 12); thread t runs Horner over chunks t, t + NT, ... with the
# step map A_{NT chunk}, then shifts by A_{j chunk}, j = (nch - 1 - t) mod NT, one
# doubling map A_{chunk 2^i} per set bit of j (the kernel has NT = 1024 and maps
# i < 10); an empty body folds to 0.


def big_fold_emulated(body: bytes, chunk: int, nt: int) -> int:
    L = len(body)
    nch = (L + chunk - 1) // chunk
    if nch == 0:
        return 0
    raw = []
    for k in range(nch):
        end = L - (nch - 1 - k) * chunk
        raw.append(crc0(body[max(0, end - chunk):end]))
    len0 = L - (nch - 1) * chunk
    seed = nib_shift(len0 & 4095, 0xFFFFFFFF)  # Tq[len0 & 4095]
    q, k = len0 >> 12, 12
    while q:
        if q & 1:
            seed = nib_apply(k, seed)
        q >>= 1
        k += 1
    dbl = [lambda v, i=i: nib_shift(chunk << i, v) for i in range(nt.bit_length())]
    out = 0
    for t in range(nt):
        acc, kk = 0, t
        while kk < nch:
            acc = nib_shift(nt * chunk, acc) ^ raw[kk] ^ (seed if kk == 0 else 0)
            kk += nt
        if t < nch:
            j, i = (nch - 1 - t) % nt, 0
            while j:
                if j & 1:
                    acc = dbl[i](acc)
                j >>= 1
                i += 1
        out ^= acc
    return ~out & 0xFFFFFFFF


@pytest.mark.parametrize("L,chunk,nt", [
    (0, 4080, 8), (1, 4080, 8), (4080, 4080, 8), (4081, 4080, 8), (8176, 8176, 8), (8177, 8176, 4),
    (9000, 8176, 4), (5 * 8176 + 7, 8176, 2), (40000, 4080, 4), (33000, 16368, 4), (12345, 8176, 1),
])
def test_big_fold_matches_zlib(L, chunk, nt):
    """The route's fold algebra (seeded chunk 0, doubling maps) equals zlib.crc32."""
    body = random.Random(L * 7 + chunk).randbytes(L)
    assert big_fold_emulated(body, chunk, nt) == zlib.crc32(body)


# ---- address-aligned route chunks (big_*_aligned_kernel) ----
# A body at absolute address s is cut at multiples of the power-of-two chunk C:
# chunk k = [max(s, (s // C + k) C), min(e, (s // C + k + 1) C)).  The fold:
#   G   = XOR_{k < nch-1} A_{(nch-2-k) C}(raw_k), raw_0 ^= A_{len0}(F), by the
#         same thread-strided Horner (step A_{NT C}) and A_{j C} shifts;
#   crc = ~(A_t(G) ^ raw_last), t = the last chunk's length; one chunk:
#         crc = ~(raw_0 ^ A_{len0}(F)).


def aligned_fold_emulated(body: bytes, start: int, chunk: int, nt: int) -> int:
    L = len(body)
    if L == 0:
        return 0
    s, e = start, start + L
    nch = (e - 1) // chunk - s // chunk + 1
    blk0 = s - s % chunk
    pieces = [(max(s, blk0 + k * chunk), min(e, blk0 + (k + 1) * chunk)) for k in range(nch)]
    raw = [crc0(body[a - s:b - s]) for a, b in pieces]
    len0 = pieces[0][1] - pieces[0][0]
    seed = nib_shift(len0 & ~4095, nib_shift(len0 & 4095, 0xFFFFFFFF))  # A_{4096 q}(Tq[len0 mod 4096])
    if nch == 1:
        return ~(raw[0] ^ seed) & 0xFFFFFFFF
    m = nch - 1
    g = 0
    for t in range(nt):
        acc, kk = 0, t
        while kk < m:
            acc = nib_shift(nt * chunk, acc) ^ raw[kk] ^ (seed if kk == 0 else 0)
            kk += nt
        if t < m:
            acc = nib_shift(((m - 1 - t) % nt) * chunk, acc)
        g ^= acc
    t_last = pieces[-1][1] - pieces[-1][0]
    return ~(nib_shift(t_last, g) ^ raw[-1]) & 0xFFFFFFFF


@pytest.mark.parametrize("L,start,chunk,nt", [
    (1, 0, 4096, 4), (1, 4095, 4096, 4), (2, 4095, 4096, 4), (4096, 0, 4096, 4), (4096, 16, 4096, 4),
    (8192, 0, 8192, 8), (8193, 8191, 8192, 8), (9000, 5, 8192, 2), (5 * 8192 + 7, 12345, 8192, 4),
    (40000, 100, 4096, 4), (33000, 16384 - 3, 16384, 1), (70000, 8192 * 3, 8192, 3),
])
def test_aligned_fold_matches_zlib(L, start, chunk, nt):
    """The aligned route's chunking and fold algebra equal zlib.crc32 at any body
    alignment (single chunk, body inside one block, head + interior + tail)."""
    body = random.Random(L * 11 + start).randbytes(L)
    assert aligned_fold_emulated(body, start, chunk, nt) == zlib.crc32(body)


# ---- span mode (big_combine_aligned_kernel span branch) -----
# The bodies lie in a 4 KiB-aligned stream; the span pass CRCs every whole 4 KiB
# block (RAW) and the fold takes a body's interior blocks from it.  The ragged
# chunk pass CRCs each body's first and last partial blocks (pieces 2b, 2b + 1).


def span_fold_emulated(mem: bytes, s: int, L: int, nt: int, rs: int = 0) -> int:
    """big_combine_aligned_kernel's span branch; rs > 0: with round values of rs
    blocks (the product's 32), whole rounds from the round table."""
    if L == 0:
        return 0
    e = s + L
    j0, j1 = s >> 12, (e - 1) >> 12
    nch = j1 - j0 + 1
    head = crc0(mem[s:e if nch == 1 else (j0 + 1) << 12])
    tail = crc0(mem[j1 << 12:e]) if nch > 1 else 0
    len0 = (e if nch == 1 else (j0 + 1) << 12) - s
    seed = nib_shift(len0 & ~4095, nib_shift(len0 & 4095, 0xFFFFFFFF))
    if nch == 1:
        return ~(head ^ seed) & 0xFFFFFFFF
    m = nch - 1
    raw = [0] + [crc0(mem[(j0 + k) << 12:(j0 + k + 1) << 12]) for k in range(1, m)]  # G' leaves chunk 0 out
    g = 0
    ja, jb = j0 + 1, j1
    ra, rb = (ja + rs - 1) // rs if rs else 0, jb // rs if rs else 0
    if rs and m > 1 and ra < rb:
        # whole rounds (their crc0 as the span pass stores it), thread-strided Horner
        # with A_{nt * rs * 4096}, then the <= rs - 1 blocks before / after them
        blk = lambda j: crc0(mem[j << 12:(j + 1) << 12])  # noqa: E731
        rv = [crc0(mem[(r * rs) << 12:((r + 1) * rs) << 12]) for r in range(ra, rb)]
        nA, nR, nC = ra * rs - ja, rb - ra, jb - rb * rs
        for t in range(nt):
            acc, kk = 0, t
            while kk < nR:
                acc = nib_shift(nt * rs * 4096, acc) ^ rv[kk]
                kk += nt
            if t < nR:
                acc = nib_shift(((nR - 1 - t) % nt) * rs * 4096 + nC * 4096, acc)
            g ^= acc
        for u in range(nA):
            g ^= nib_shift((jb - 1 - (ja + u)) * 4096, blk(ja + u))
        for u in range(nC):
            g ^= nib_shift((nC - 1 - u) * 4096, blk(rb * rs + u))
        g ^= nib_shift((m - 1) * 4096, head ^ seed)
        return ~(nib_shift(e - (j1 << 12), g) ^ tail) & 0xFFFFFFFF
    for t in range(nt):
        acc, kk = 0, t
        while kk < m:
            acc = nib_shift(nt * 4096, acc) ^ raw[kk]
            kk += nt
        if t < m:
            acc = nib_shift(((m - 1 - t) % nt) * 4096, acc)
        g ^= acc
    g ^= nib_shift((m - 1) * 4096, head ^ seed)  # thread 0 adds the head at the end
    return ~(nib_shift(e - (j1 << 12), g) ^ tail) & 0xFFFFFFFF


@pytest.mark.parametrize("L,start,nt", [
    (0, 5, 4), (1, 0, 4), (1, 4095, 4), (3, 4094, 4), (4096, 0, 4), (4096, 7, 4), (4097, 4095, 2),
    (8192, 0, 4), (8193, 4093, 3), (5 * 4096 + 6, 1234, 4), (40000, 4096 * 2 + 1, 4), (12288, 4096, 1),
])
def test_span_fold_matches_zlib(L, start, nt):
    """Span mode: interior blocks from the block table, the partial first / last
    blocks from the piece pass -- equal to zlib.crc32 of the body."""
    rnd = random.Random(L * 13 + start)
    mem = bytearray(rnd.randbytes(start + L + 4096))
    assert span_fold_emulated(bytes(mem), start, L, nt) == zlib.crc32(bytes(mem[start:start + L]))


@pytest.mark.parametrize("L,start,nt,rs", [
    (4096 * 9, 5, 2, 4),            # rounds of 4 blocks: one whole round inside, blocks around it
    (4096 * 8, 0, 2, 4),            # body starting on a round boundary (its head is a whole block)
    (4096 * 12 - 1, 4096 * 4, 3, 4),
    (4096 * 40 + 77, 123, 4, 4),    # several rounds per thread
    (4096 * 7, 4096 * 3 + 1, 2, 4), # interior shorter than a round: per-block fold
    (4096 * 70 + 3, 4096 * 31, 2, 32),  # the product's 32-block rounds: one whole round
])
def test_span_fold_round_values_matches_zlib(L, start, nt, rs):
    """Span mode with round values (BigRoute.rnd): whole rounds from the round
    table, the blocks before and after them from the block table."""
    rnd = random.Random(L * 7 + start)
    mem = bytearray(rnd.randbytes(start + L + 4096))
    assert span_fold_emulated(bytes(mem), start, L, nt, rs) == zlib.crc32(bytes(mem[start:start + L]))
