"""CPU emulation of the dense span mode (crc32_rows.h kRowsSpanBnd,
crc32_kernels.hip dense_plan_kernel / dense_fold_kernel) against zlib.

A dense ragged batch -- bodies back to back, in order, each of >= 64 bytes -- is
read as one uniform stream of 4 KiB blocks.  Per block the span pass stores
W = crc0(block) and, for each body boundary b inside it (at most one per 64-B
segment: bodies are >= 64 B), three words computed from values the lanes hold
anyway:
    P1  = XOR over the segments before b's segment in its 1 KiB quarter of
          A_{64(15-lo')}(c_lo')                 (in-quarter exclusive XOR scan)
    cap = X_tb ^ (w_tb & ~low_u)                (the segment's chain state at
          b's dword, its bytes at or after b removed)
    Qp  = XOR over the quarters before b's of A_{1024(3-h)}(v_h)
The span pass stores eq = P1 ^ A_{64(15-lo)}(A_{4(16-tb)}(cap)) and Qp; the fold
then forms, per boundary, E(b) = crc0(block with bytes >= b zeroed)
    E = A_{1024(3-hi)}(eq) ^ Qp
and per body [s, e) over blocks j0 .. j1 (D = j1 - j0 > 0):
    Y = A_{4096 D}(Tq[4096 - s_off] ^ W[j0] ^ E(s)) ^ X ^ E(e)
    X = XOR over the blocks j in between of A_{4096 (j1 - j)}(W[j])
(E(e) is W[j1] when e ends its block; D = 0: Y = Tq ^ E(s) ^ E(e)), then the
inverse shift of the z = 4096 - e_off bytes past e.  Every step here is the
kernels' arithmetic on the kernels' stored values, lane by lane, and the result
is compared with zlib.crc32 of each body (zlib 1.2.11 is the reference's
arithmetic).
"""
import random
import zlib

import pytest

POLY = 0xEDB88320
X0 = 0x80000000
M32 = 0xFFFFFFFF


def mulmod(a, b):
    m, p = X0, 0
    for _ in range(32):
        if a & m:
            p ^= b
        m >>= 1
        b = (b >> 1) ^ POLY if b & 1 else b >> 1
    return p


def xpow8(nbytes):
    """x^(8 nbytes) mod P."""
    r, sq, n = X0, X0 >> 1, 8 * nbytes
    while n:
        if n & 1:
            r = mulmod(r, sq)
        sq = mulmod(sq, sq)
        n >>= 1
    return r


def xinv8(nbytes):
    """x^(-8 nbytes) mod P (P has a constant term: x is invertible)."""
    c = X0
    for _ in range(8 * nbytes):
        c = (((c ^ POLY) << 1) | 1) & M32 if c & X0 else (c << 1) & M32
    return c


def A(n, s):
    return mulmod(xpow8(n), s)


def crc0(data: bytes) -> int:
    return (~zlib.crc32(data, M32)) & M32


def T4(x):  # the slice-by-4 table step: crc0 of x's 4 bytes (little-endian)
    return crc0(x.to_bytes(4, "little"))


def plan(lens, anchor_pad):
    """dense_plan_kernel: boundary g at stream offset rel_g (g = n: the last end);
    per block {first, cnt, offsets}; per boundary its offset in its block."""
    rel = [anchor_pad]
    for L in lens:
        rel.append(rel[-1] + L)
    nblocks = (rel[-1] + 4095) // 4096
    first = [None] * nblocks
    cnt = [0] * nblocks
    for g, r in enumerate(rel):
        j = r >> 12
        if j < nblocks:
            if first[j] is None:
                first[j] = g
            cnt[j] += 1
    nxt = len(rel)
    for j in range(nblocks - 1, -1, -1):  # empty blocks: first = the next boundary
        if first[j] is None:
            first[j] = nxt
        nxt = first[j]
    return rel, nblocks, first, cnt


def span_block(block: bytes, offs):
    """The span pass on one 4 KiB block (lane L = 64-B segment L) with boundaries
    at block offsets `offs`: W and {offset: (P1, cap, Qp)}."""
    words = [[int.from_bytes(block[64 * L + 4 * t:64 * L + 4 * t + 4], "little") for t in range(16)]
             for L in range(64)]
    bnd = {o >> 6: o & 63 for o in offs}  # segment -> offset in it (one per segment)
    c, cap = [0] * 64, [0] * 64
    for L in range(64):
        w = words[L]
        tb, u = (bnd[L] >> 2, bnd[L] & 3) if L in bnd else (16, 0)
        nm = (M32 << (8 * u)) & M32  # bytes at or after the boundary in its dword
        x = w[0]
        if tb == 0:
            cap[L] = x ^ (w[0] & nm)
        for t in range(1, 16):
            x = T4(x) ^ w[t]
            if tb == t:
                cap[L] = x ^ (w[t] & nm)
        c[L] = T4(x)
    d1 = [A(64 * (15 - (L & 15)), c[L]) for L in range(64)]  # merge step 1 (ST1)
    v = [0] * 4
    for L in range(64):
        v[L >> 4] ^= d1[L]
    vs = [A(1024 * (3 - h), v[h]) for h in range(4)]  # merge step 2 (ST2, distributed)
    W = vs[0] ^ vs[1] ^ vs[2] ^ vs[3]
    out = {}
    for k, rr in bnd.items():
        hi, lo = k >> 4, k & 15
        p1 = 0
        for lo2 in range(lo):
            p1 ^= d1[16 * hi + lo2]
        qp = 0
        for h in range(hi):
            qp ^= vs[h]
        out[64 * k + rr] = (p1, cap[k], qp)
    return W, out


def boundary_e(off, p1, cap, qp):
    """E(b) = crc0(block with bytes >= b zeroed): the span pass stores
    eq = P1 ^ A_{64(15-lo)}(A_{4(16-tb)}(cap)) (its span_m4 and st1_map lookups)
    and Qp; dense_fold_kernel adds the quarter shift A_{1024(3-hi)}."""
    k, rr = off >> 6, off & 63
    hi, lo, tb = k >> 4, k & 15, rr >> 2
    eq = p1 ^ A(64 * (15 - lo), A(4 * (16 - tb), cap))
    return A(1024 * (3 - hi), eq) ^ qp


def dense_emulated(stream: bytes, anchor_pad: int, lens):
    rel, nblocks, first, cnt = plan(lens, anchor_pad)
    padded = stream + bytes(4096 * nblocks - len(stream))  # the last block's range-checked tail reads zeros
    W, E = [], {}
    for j in range(nblocks):
        offs = [rel[g] - 4096 * j for g in range(first[j], first[j] + cnt[j])]
        w, bnd = span_block(padded[4096 * j:4096 * j + 4096], offs)
        W.append(w)
        for g in range(first[j], first[j] + cnt[j]):
            o = rel[g] - 4096 * j
            E[g] = boundary_e(o, *bnd[o])
    crcs = []
    tq = lambda h: A(h, M32)  # Tq[h] = A_h(0xFFFFFFFF)
    for i, L in enumerate(lens):
        s, e = rel[i], rel[i] + L
        j0, r0 = s >> 12, s & 4095
        j1 = (e - 1) >> 12
        e_off = e - 4096 * j1
        Ee = W[j1] if e_off == 4096 else E[i + 1]
        acc = tq(4096 - r0) ^ E[i]
        if j1 == j0:
            acc ^= Ee
        else:  # the fold's closed form of the Horner over the blocks j0 .. j1
            X = 0
            for j in range(j0 + 1, j1):  # the in-between blocks (dealt over the wave's lanes)
                dd = j1 - j
                X ^= A(65536 * (dd >> 4), A(4096 * (dd & 15), W[j]))
            D = j1 - j0
            acc = A(65536 * (D >> 4), A(4096 * (D & 15), acc ^ W[j0])) ^ X ^ Ee
        z = 4096 - e_off
        crcs.append((~mulmod(xinv8(z), acc)) & M32)
    return crcs


@pytest.mark.parametrize("seed,nb,maxlen,pad", [(1, 12, 300, 0), (2, 6, 9000, 5), (3, 40, 128, 15),
                                                 (4, 3, 20000, 7), (5, 25, 700, 0)])
def test_dense_span_matches_zlib(seed, nb, maxlen, pad):
    rnd = random.Random(seed)
    lens = [rnd.randint(64, maxlen) for _ in range(nb)]
    if seed == 5:  # bodies ending and starting exactly on block boundaries
        lens = [4096 - pad, 64, 4032, 8192, 100, 3996, 4096]
    if seed == 3:  # boundaries at every dword phase of a segment, and at segment starts
        lens = [64 + (k % 7) for k in range(nb)]
    body = bytes(rnd.getrandbits(8) for _ in range(sum(lens)))
    stream = bytes(rnd.getrandbits(8) for _ in range(pad)) + body  # foreign bytes before the first body
    got = dense_emulated(stream, pad, lens)
    o = 0
    for L, g in zip(lens, got):
        assert g == zlib.crc32(body[o:o + L]), (L, o)
        o += L
