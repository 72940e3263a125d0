"""CPU oracle pinned against the reference's golden vectors (tests/golden, generated
from the compiled reference crc.c + zlib 1.2.11) and against Python zlib."""
import zlib

import numpy as np
import pytest

from oracle import oracle


def test_kats(golden):
    for k in golden["kats"]:
        b = bytes.fromhex(k["hex"])
        assert oracle.crc32(b) == k["crc"], k["name"]
        assert oracle.crc32_bitwise(b) == k["crc"], k["name"]


def test_check_value():
    assert oracle.crc32(b"123456789") == 0xCBF43926  # CRC-32/ISO-HDLC check value


def test_random_bodies(golden):
    for r in golden["random_bodies"]:
        data = oracle.splitmix_bytes(r["len"], r["seed"])
        assert oracle.crc32(data) == r["crc"], r


def test_json_c0(golden):
    g = golden["json_c0"]
    buf, offs, lens = oracle.json_bodies(g["n"], g["body_len"], g["seed"])
    got = oracle.crc32_batch(buf, offs, lens)
    assert got.tolist() == g["crcs"]
    # bodies are printable JSON
    text = buf[:g["body_len"]].tobytes().decode()
    assert text.startswith('{"jsonrpc":"2.0"') and text.endswith("}")


def test_frames(golden):
    for f in golden["frames"]:
        hdr = bytes.fromhex(f["header_hex"])
        body = f["body"].encode()
        assert int.from_bytes(hdr[8:12], "big") == oracle.crc32(body)


def test_combine(golden):
    for c in golden["combine"]:
        assert oracle.combine(c["a_crc"], c["b_crc"], c["len_b"]) == c["crc_ab"]


def test_edges(golden):
    e = golden["edges"]
    assert oracle.crc32(None, 5) == e["null_len5"] == 0
    # zlib's uInt length: size_t 2**32 + 3 is read as 3 bytes (only 3 bytes exist here)
    assert oracle.crc32(bytes(3), 2**32 + 3) == e["zeros3"]


def test_zlib_agreement_random():
    rng = np.random.default_rng(5)
    for n in [0, 1, 7, 100, 4096, 70001]:
        b = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
        assert oracle.crc32(b) == (zlib.crc32(b) & 0xFFFFFFFF)


def test_splitmix_numpy_matches_c():
    for n, seed in [(1, 3), (15, 4), (4096, 0x5EED0003), (100003, 9)]:
        assert np.array_equal(oracle.splitmix_bytes(n, seed), oracle.splitmix_bytes_c(n, seed))


def test_loguniform_lengths():
    ln = oracle.loguniform_lengths(200000)
    assert ln.min() >= 64 and ln.max() <= 65536
    # log-uniform: median near 64 * 1024 ** 0.5 = 2048
    assert 1700 < np.median(ln) < 2500
    assert 8500 < ln.mean() < 10500  # mean ~9446 B


@pytest.mark.skipif(not oracle.ref_available(), reason="oracle/_ref not built (needs /root/reference)")
def test_ref_matches_oracle():
    ref = oracle.load_ref()
    rng = np.random.default_rng(11)
    for n in [0, 1, 3, 64, 1000, 4096, 65537]:
        b = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
        assert ref.crc32(b) == oracle.crc32(b)
    assert ref.crc32(None, 7) == 0
    buf, offs, lens = oracle.json_bodies(8, 4096)
    sec, out = ref.batch_timed(buf, offs, lens, threads=2, reps=1)
    assert sec >= 0 and np.array_equal(out, oracle.crc32_batch(buf, offs, lens))
