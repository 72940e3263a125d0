"""CPU emulation of the one-wave drop-in kernel (crc32_scalar_kernel,
rpc_amd/csrc/crc32_scalar.hip) against zlib.

For a body of len <= 4096 bytes the kernel picks seg = the smallest power of
two >= 4 with 64 * seg >= len, right-aligns the body in a virtual buffer V of
64 * seg bytes (stale bytes before it masked to zero), computes each lane's
crc0 of V[L*seg, +seg) with slice-by-4 tables, folds six pair levels
(left group shifted by A_{seg*2^b} via the nibble maps, XOR the right group),
and returns ~(A_len(0xFFFFFFFF) ^ crc0(V)).  Here the same tables and steps
run in Python, and the result is compared with zlib.crc32 (the reference's
arithmetic, crc.c:4-9, zlib 1.2.11).
"""
import random
import zlib

import pytest

from test_combine_emu import POLY, nib_apply, nib_shift


def byte_table():
    t = []
    for b in range(256):
        c = b
        for _ in range(8):
            c = (c >> 1) ^ POLY if c & 1 else c >> 1
        t.append(c)
    return t


T0 = byte_table()
T = [T0]
for _k in range(3):
    T.append([(T[-1][v] >> 8) ^ T0[T[-1][v] & 0xFF] for v in range(256)])


def seg_log2(n):  # scalar_seg_log2
    g = 2
    while (64 << g) < n:
        g += 1
    return g


def emulate(body: bytes, stale: int = 0xA5) -> int:
    n = len(body)
    g = seg_log2(n)
    seg = 1 << g
    vbytes = 64 * seg
    off0 = vbytes - n
    stage = bytes([stale]) * off0 + body  # what the pinned staging holds
    lanes = []
    for lane in range(64):
        s = 0
        for d in range(seg // 4):
            pos = lane * seg + 4 * d
            w = int.from_bytes(stage[pos:pos + 4], "little")
            keep = 0xFFFFFFFF if pos >= off0 else (0 if pos + 4 <= off0 else (0xFFFFFFFF << (8 * (off0 - pos))) & 0xFFFFFFFF)
            x = s ^ (w & keep)
            s = T[3][x & 0xFF] ^ T[2][(x >> 8) & 0xFF] ^ T[1][(x >> 16) & 0xFF] ^ T[0][x >> 24]
        lanes.append(s)
    for b in range(6):  # pair levels: lanes exchange across lane bit b
        sh = [nib_apply(g + b, v) for v in lanes]
        mine = [lanes[L] if (L >> b) & 1 else sh[L] for L in range(64)]
        lanes = [mine[L] ^ mine[L ^ (1 << b)] for L in range(64)]
    assert len(set(lanes)) == 1  # every lane holds crc0(V)
    seed = nib_shift(n, 0xFFFFFFFF)  # Tq[len] = A_len(0xFFFFFFFF)
    return ~(seed ^ lanes[0]) & 0xFFFFFFFF


@pytest.mark.parametrize("n", [0, 1, 3, 4, 5, 68, 255, 256, 257, 511, 512, 513, 1023, 1024, 1025, 2047, 2048,
                               2049, 4095, 4096])
def test_scalar_kernel_algebra_matches_zlib(n):
    rnd = random.Random(n)
    body = bytes(rnd.randrange(256) for _ in range(n))
    assert emulate(body) == zlib.crc32(body)
    assert emulate(body, stale=0xFF) == zlib.crc32(body)


def test_segment_sizes():
    assert [seg_log2(n) for n in (0, 256, 257, 512, 513, 1024, 1025, 2048, 2049, 4096)] == [2, 2, 3, 3, 4, 4, 5, 5, 6, 6]
