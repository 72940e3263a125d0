"""oracle/oracle.py -- Python handle on the CPU checkers.  TEST INFRASTRUCTURE ONLY.

Only tests/, ``__graft_entry__.smoke()`` and bench.py's ``cpu_baseline`` leg may
import this module, and only as the checker / baseline -- never as the thing
measured or shipped.  The product package ``rpc_amd`` never imports it.

* ``liboracle.so``   our plain-C restatement of zlib 1.2.11 CRC-32
                     (crc32_oracle.c; reference crc.c:4-14 semantics).
* ``_ref/libref_crc.so`` (optional) the reference's own crc.c compiled in this
                     container + system libz, with a threaded timing harness.

Also holds the deterministic synthetic-input generators shared by tests and
bench (splitmix64 counter stream; JSON-RPC-shaped bodies; log-uniform lengths).
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ORACLE_SO = os.path.join(HERE, "liboracle.so")
REF_SO = os.path.join(HERE, "_ref", "libref_crc.so")


def _build():
    subprocess.run(["make", "-s", "-C", HERE, "oracle"], check=True)


if not os.path.exists(ORACLE_SO):
    _build()

_o = ctypes.CDLL(ORACLE_SO)
_o.oracle_rpc_crc32.restype = ctypes.c_uint32
_o.oracle_rpc_crc32.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
_o.oracle_crc32_bitwise.restype = ctypes.c_uint32
_o.oracle_crc32_bitwise.argtypes = [ctypes.c_void_p, ctypes.c_uint64]
_o.oracle_crc32_combine.restype = ctypes.c_uint32
_o.oracle_crc32_combine.argtypes = [ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint64]
_o.oracle_crc32_batch.restype = None
_o.oracle_crc32_batch.argtypes = [ctypes.c_void_p] * 3 + [ctypes.c_uint64, ctypes.c_void_p]
_o.oracle_crc32_uniform.restype = None
_o.oracle_crc32_uniform.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint64,
                                    ctypes.c_void_p]
_o.oracle_splitmix_fill.restype = None
_o.oracle_splitmix_fill.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint64]


def _addr(data):
    if data is None:
        return None, None
    if isinstance(data, np.ndarray):
        a = np.ascontiguousarray(data)
        return a.ctypes.data, a
    b = bytes(data)
    buf = ctypes.create_string_buffer(b, len(b))
    return ctypes.addressof(buf), buf


def crc32(data, length=None) -> int:
    """oracle rpc_crc32 (crc.c:4-9 semantics incl. NULL->0 and uInt length)."""
    addr, keep = _addr(data)
    if length is None:
        length = 0 if data is None else len(data) if not isinstance(data, np.ndarray) else data.nbytes
    return int(_o.oracle_rpc_crc32(addr, length))


def crc32_bitwise(data) -> int:
    addr, keep = _addr(data)
    n = data.nbytes if isinstance(data, np.ndarray) else len(data)
    return int(_o.oracle_crc32_bitwise(addr, n))


def combine(crc1: int, crc2: int, len2: int) -> int:
    return int(_o.oracle_crc32_combine(crc1, crc2, len2))


def crc32_batch(buf: np.ndarray, offsets, lengths) -> np.ndarray:
    off = np.ascontiguousarray(offsets, dtype=np.uint64)
    ln = np.ascontiguousarray(lengths, dtype=np.uint32)
    out = np.empty(off.shape[0], dtype=np.uint32)
    b = np.ascontiguousarray(buf)
    _o.oracle_crc32_batch(b.ctypes.data, off.ctypes.data, ln.ctypes.data, off.shape[0], out.ctypes.data)
    return out


def crc32_uniform(buf: np.ndarray, n: int, body_len: int, stride: int | None = None) -> np.ndarray:
    stride = body_len if stride is None else stride
    out = np.empty(n, dtype=np.uint32)
    b = np.ascontiguousarray(buf)
    _o.oracle_crc32_uniform(b.ctypes.data, n, body_len, stride, out.ctypes.data)
    return out


# ---- frame verdicts (the reference's receive-side decisions) -------------------

FRAME_BAD_CRC, FRAME_OK, FRAME_CONTROL, FRAME_TOO_LARGE, FRAME_MALFORMED, FRAME_RECV_ERR = 0, 1, 2, 3, 4, 5
MAX_BODY_LEN = 1024  # rpc.h:17
RPC_TYPE_PING, RPC_TYPE_PONG = 1, 2  # rpc.h:12-13


def frame_verdict(stream: bytes, off: int, role: str = "server", lift_cap: bool = False) -> tuple[int, int]:
    """(verdict, body crc) of the frame at ``off``, restating the reference's order:
    parse the 12-byte big-endian header (rpc_server_main.c:165-169 / rpc_async.c:296-300);
    a server answers PING from the header alone (rpc_server_main.c:172-187), a client
    consumes PONG the same way (rpc_async.c:303-309); a body_len over MAX_BODY_LEN drops
    the peer before the body is read (rpc_server_main.c:189-195, rpc_async.c:312-315);
    a client that gets body_len 0 enters its BODY state, whose recv(fd, buf, 0) on the
    non-blocking socket returns 0 once anything more (or a FIN) is pending -- taken for
    a closed peer (rpc_async.c:330-349), so the call ends with RPC_RECV_ERR
    (rpc_types.h:26) and the empty body is never verified: RECV_ERR (the server reads
    the empty body and verifies it, rpc_server_main.c:198-227); otherwise the body is read and
    rpc_crc32_verify decides (rpc_server_main.c:227, rpc_async.c:219).  MALFORMED: the
    frame does not fit the stream (our bound)."""
    if off + 12 > len(stream):
        return FRAME_MALFORMED, 0
    h = stream[off:off + 12]
    typ = int.from_bytes(h[2:4], "big")
    blen = int.from_bytes(h[4:8], "big")
    hcrc = int.from_bytes(h[8:12], "big")
    if (role == "server" and typ == RPC_TYPE_PING) or (role == "client" and typ == RPC_TYPE_PONG):
        return FRAME_CONTROL, 0
    if blen > MAX_BODY_LEN and not lift_cap:
        return FRAME_TOO_LARGE, 0
    if blen == 0 and role == "client":
        return FRAME_RECV_ERR, 0
    if off + 12 + blen > len(stream):
        return FRAME_MALFORMED, 0
    c = crc32(np.frombuffer(stream, dtype=np.uint8)[off + 12:off + 12 + blen]) if blen else 0
    return (FRAME_OK if c == hcrc else FRAME_BAD_CRC), c


def crc32_uniform_mt(buf: np.ndarray, n: int, body_len: int, threads: int = 16) -> np.ndarray:
    """crc32_uniform over `threads` threads (the C oracle releases the GIL)."""
    from concurrent.futures import ThreadPoolExecutor

    out = np.empty(n, dtype=np.uint32)
    b = np.ascontiguousarray(buf)
    step = (n + threads - 1) // threads

    def part(k):
        lo, hi = k * step, min(n, (k + 1) * step)
        if lo < hi:
            _o.oracle_crc32_uniform(b.ctypes.data + lo * body_len, hi - lo, body_len, body_len,
                                    out.ctypes.data + lo * 4)

    with ThreadPoolExecutor(threads) as ex:
        list(ex.map(part, range(threads)))
    return out


def crc32_batch_mt(buf: np.ndarray, offsets, lengths, threads: int = 16) -> np.ndarray:
    """crc32_batch over `threads` threads."""
    from concurrent.futures import ThreadPoolExecutor

    off = np.ascontiguousarray(offsets, dtype=np.uint64)
    ln = np.ascontiguousarray(lengths, dtype=np.uint32)
    n = off.shape[0]
    out = np.empty(n, dtype=np.uint32)
    b = np.ascontiguousarray(buf)
    step = (n + threads - 1) // threads

    def part(k):
        lo, hi = k * step, min(n, (k + 1) * step)
        if lo < hi:
            _o.oracle_crc32_batch(b.ctypes.data, off.ctypes.data + lo * 8, ln.ctypes.data + lo * 4, hi - lo,
                                  out.ctypes.data + lo * 4)

    with ThreadPoolExecutor(threads) as ex:
        list(ex.map(part, range(threads)))
    return out


# ---- synthetic inputs (shared with bench.py and the device datagen kernel) ----

GOLDEN = 0x9E3779B97F4A7C15
M64 = (1 << 64) - 1


def _mix64(z: np.ndarray) -> np.ndarray:
    z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
    z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
    return z ^ (z >> np.uint64(31))


def splitmix_words(nwords: int, seed: int, word_offset: int = 0) -> np.ndarray:
    k = np.arange(word_offset + 1, word_offset + nwords + 1, dtype=np.uint64)
    with np.errstate(over="ignore"):
        z = np.uint64(seed & M64) + k * np.uint64(GOLDEN)
        return _mix64(z)


def splitmix_bytes(nbytes: int, seed: int) -> np.ndarray:
    """Bytes of the counter-based splitmix64 stream (== rpc_crc32_fill_random_device)."""
    w = splitmix_words((nbytes + 7) // 8, seed)
    return w.view(np.uint8)[:nbytes].copy()


def splitmix_bytes_c(nbytes: int, seed: int) -> np.ndarray:
    out = np.empty(nbytes, dtype=np.uint8)
    _o.oracle_splitmix_fill(out.ctypes.data, nbytes, seed, 0)
    return out


_PRINTABLE = np.array([c for c in range(0x20, 0x7F) if c not in (ord('"'), ord("\\"))], dtype=np.uint8)


def json_bodies(n: int, body_len: int, seed: int = 0x5EED0001):
    """Config C0 bodies: JSON-RPC text padded to exactly body_len bytes
    ({"jsonrpc":"2.0","method":"echo","params":{"s":"<printable>"},"id":N}),
    printable filler 0x20-0x7E without '"' and '\\' from splitmix64."""
    buf = np.empty(n * body_len, dtype=np.uint8)
    rnd = splitmix_bytes(n * body_len, seed)
    prefix = b'{"jsonrpc":"2.0","method":"echo","params":{"s":"'
    for i in range(n):
        suffix = b'"},"id":' + str(i + 1).encode() + b"}"
        fill = body_len - len(prefix) - len(suffix)
        if fill < 0:
            raise ValueError("body_len too small for the JSON envelope")
        row = buf[i * body_len:(i + 1) * body_len]
        row[:len(prefix)] = np.frombuffer(prefix, dtype=np.uint8)
        row[len(prefix):len(prefix) + fill] = _PRINTABLE[rnd[i * body_len:i * body_len + fill] % len(_PRINTABLE)]
        row[len(prefix) + fill:] = np.frombuffer(suffix, dtype=np.uint8)
    offsets = np.arange(n, dtype=np.uint64) * np.uint64(body_len)
    lengths = np.full(n, body_len, dtype=np.uint32)
    return buf, offsets, lengths


def loguniform_lengths(n: int, seed: int = 0x5EED0004, lo: int = 64, hi: int = 65536) -> np.ndarray:
    """Config C2 lengths: log-uniform integers in [lo, hi]."""
    w = splitmix_words(n, seed)
    u = (w >> np.uint64(11)).astype(np.float64) * (1.0 / (1 << 53))
    ln = np.floor(lo * np.exp(u * np.log(hi / lo))).astype(np.int64)
    return np.clip(ln, lo, hi).astype(np.uint32)


# ---- the compiled reference (optional) -------------------------------------

class Ref:
    """The reference crc.c (+ libz) built into oracle/_ref by oracle/Makefile."""

    def __init__(self, path: str = REF_SO):
        self.path = path
        self.lib = ctypes.CDLL(path)
        self.lib.ref_rpc_crc32.restype = ctypes.c_uint32
        self.lib.ref_rpc_crc32.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
        self.lib.ref_crc32_batch_timed.restype = ctypes.c_double
        self.lib.ref_crc32_batch_timed.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                                   ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint64,
                                                   ctypes.c_void_p, ctypes.c_int, ctypes.c_int]

    def crc32(self, data, length=None) -> int:
        addr, keep = _addr(data)
        if length is None:
            length = 0 if data is None else (data.nbytes if isinstance(data, np.ndarray) else len(data))
        return int(self.lib.ref_rpc_crc32(addr, length))

    def batch_timed(self, buf: np.ndarray, offsets=None, lengths=None, n=0, body_len=0, stride=0,
                    threads=1, reps=1):
        """Returns (seconds, crcs) for `reps` passes over the batch on `threads` threads."""
        b = np.ascontiguousarray(buf)
        if offsets is not None:
            off = np.ascontiguousarray(offsets, dtype=np.uint64)
            ln = np.ascontiguousarray(lengths, dtype=np.uint32)
            n = off.shape[0]
            op, lp = off.ctypes.data, ln.ctypes.data
        else:
            op = lp = None
        out = np.empty(n, dtype=np.uint32)
        sec = self.lib.ref_crc32_batch_timed(b.ctypes.data, op, lp, n, body_len, stride, out.ctypes.data,
                                             threads, reps)
        return sec, out


def ref_available() -> bool:
    return os.path.exists(REF_SO)


def load_ref() -> Ref | None:
    return Ref() if ref_available() else None
