"""Generates tests/golden/crc32_golden.json (committed fixture).

Expected CRCs come from the REFERENCE ITSELF: /root/reference/crc.c compiled by
oracle/Makefile into oracle/_ref/libref_crc.so and linked against the image's
system zlib 1.2.11 (exactly how the reference links it, CMakeLists.txt:44-45).
Every value is cross-checked against Python's zlib.crc32 (same libz 1.2.11).
Inputs are either literal bytes (hex) or a generator spec (splitmix64 seed +
length, JSON-RPC body spec) that tests regenerate with oracle.oracle.

Run in this container (needs oracle/_ref):  python tests/golden/make_golden.py
"""
import json
import os
import sys
import zlib

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

import numpy as np  # noqa: E402

from oracle import oracle  # noqa: E402

ref = oracle.load_ref()
if ref is None:
    sys.exit("oracle/_ref/libref_crc.so missing: run `make -C oracle` with /root/reference present")


def rcrc(b: bytes) -> int:
    v = ref.crc32(b)
    assert v == (zlib.crc32(b) & 0xFFFFFFFF), b[:32]
    return v


kats = []
for name, b in [
    ("empty", b""),
    ("a", b"a"),
    ("abc", b"abc"),
    ("check_123456789", b"123456789"),
    ("jsonrpc_ping", b'{"jsonrpc":"2.0","method":"ping","params":{},"id":1}'),
    ("zeros_4096", bytes(4096)),
    ("ff_64", b"\xff" * 64),
    ("request_add_i32", b'{"jsonrpc":"2.0","method":"add_i32","params":{"a":10,"b":20},"id":1}'),
    ("response_add_i32", b'{"jsonrpc":"2.0","id":1,"result":30}'),
]:
    kats.append({"name": name, "hex": b.hex(), "crc": rcrc(b)})

# Random bodies: splitmix64 stream (seed) truncated to len.
lengths = sorted(set(list(range(0, 80)) + [
    95, 96, 97, 127, 128, 129, 255, 256, 257, 511, 512, 513, 1000, 1023, 1024, 1025, 1100, 2047, 2048, 2049,
    3000, 4080, 4095, 4096, 4097, 4100, 4111, 4112, 5000, 8191, 8192, 8193, 12288, 16383, 16384, 16385,
    20000, 32768, 65535, 65536, 65537, 100000, 131072, 262144, 262147, 1 << 20, (1 << 20) + 5]))
random_bodies = []
for i, L in enumerate(lengths):
    seed = 0x60D0000 + i
    data = oracle.splitmix_bytes(L, seed).tobytes()
    random_bodies.append({"seed": seed, "len": L, "crc": rcrc(data)})

# JSON-RPC-shaped bodies of config C0 (first 16 of 1024 x 4096, seed 0x5EED0001).
buf, offs, lens = oracle.json_bodies(16, 4096, 0x5EED0001)
json_c0 = [rcrc(buf[int(o):int(o) + int(l)].tobytes()) for o, l in zip(offs, lens)]

# Wire frames captured from the reference server in the survey.
frames = [
    {"name": "request", "header_hex": "0001000000000044073c75a7",
     "body": '{"jsonrpc":"2.0","method":"add_i32","params":{"a":10,"b":20},"id":1}'},
    {"name": "response", "header_hex": "0001000000000024fb07505c", "body": '{"jsonrpc":"2.0","id":1,"result":30}'},
    {"name": "ping", "header_hex": "000100010000000000000000", "body": ""},
    {"name": "pong", "header_hex": "000100020000000000000000", "body": ""},
]
for f in frames:
    hdr = bytes.fromhex(f["header_hex"])
    body = f["body"].encode()
    assert int.from_bytes(hdr[4:8], "big") == len(body)
    assert int.from_bytes(hdr[8:12], "big") == rcrc(body)

combine = []
for a, b in [(b"1234", b"56789"), (b"", b"abc"), (b"abc", b""), (bytes(100), b"x" * 333),
             (oracle.splitmix_bytes(5000, 1).tobytes(), oracle.splitmix_bytes(70000, 2).tobytes())]:
    combine.append({"a_hex_len": len(a), "a_crc": rcrc(a), "b_crc": rcrc(b), "len_b": len(b), "crc_ab": rcrc(a + b)})

edges = {
    "null_len5": ref.crc32(None, 5),          # crc.c:6-7 with Z_NULL -> 0
    "zeros3": rcrc(bytes(3)),                 # CRC of 3 zero bytes; == rpc_crc32(p, 2**32 + 3)
}

out = {
    "provenance": "reference crc.c (compiled from /root/reference/crc.c) + system zlib 1.2.11; "
                  "cross-checked with python zlib.crc32",
    "kats": kats,
    "random_bodies": random_bodies,
    "json_c0": {"n": 16, "body_len": 4096, "seed": 0x5EED0001, "crcs": json_c0},
    "frames": frames,
    "combine": combine,
    "edges": edges,
}
with open(os.path.join(HERE, "crc32_golden.json"), "w") as f:
    json.dump(out, f, indent=1)
print("wrote", len(kats), "kats,", len(random_bodies), "random bodies")
