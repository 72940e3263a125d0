"""rpc_amd -- MI355X-native body checksum for KlinLike/RPC.

Python mirror of the reference interface ``crc.h`` (``rpc_crc32`` at crc.h:8,
``rpc_crc32_verify`` at crc.h:11) plus the batched host/device API of
``include/rpccrc.h``.  Every CRC is computed by the HIP kernels in
``rpc_amd/csrc`` through ``rpc_amd/lib/librpccrc.so``; importing this package
fails if that library is missing, and the calls fail (raise or, for the two
drop-in functions, abort in C) if no HIP device is usable.  There is no CPU
implementation here.

Device-buffer functions take torch tensors on the current HIP device (torch is
only plumbing for device memory and streams) and run on torch's current stream
unless ``stream`` (a ``torch.cuda.Stream``) is given.
"""
from __future__ import annotations

import ctypes
from typing import Iterable, Optional, Sequence

import numpy as np

from . import _lib, rx_ring
from ._lib import RpcCrcError, check, lib
from .rx_ring import RxRing

__all__ = [
    "RpcCrcError",
    "rpc_crc32",
    "rpc_crc32_verify",
    "crc32_batch",
    "verify_batch",
    "crc32_combine",
    "device_batch",
    "device_uniform",
    "device_large",
    "frames_verify",
    "frames_stamp",
    "RxRing",
    "fill_random",
    "stream_read",
    "set_options",
    "set_ragged_path",
    "device_info",
    "device_status",
    "device_clear_status",
    "RPC_HEADER_LEN",
    "RPC_TYPE_DATA",
    "RPC_TYPE_PING",
    "RPC_TYPE_PONG",
    "MAX_BODY_LEN",
    "FRAME_BAD_CRC",
    "FRAME_OK",
    "FRAME_CONTROL",
    "FRAME_TOO_LARGE",
    "FRAME_MALFORMED",
    "FRAME_RECV_ERR",
]

# reference rpc.h:11-17
RPC_TYPE_DATA = 0
RPC_TYPE_PING = 1
RPC_TYPE_PONG = 2
RPC_HEADER_LEN = 12
MAX_BODY_LEN = 1024

# frame verdicts and flags (include/rpccrc.h RPC_FRAME_* / RPC_FRAMES_*)
FRAME_BAD_CRC = 0
FRAME_OK = 1
FRAME_CONTROL = 2
FRAME_TOO_LARGE = 3
FRAME_MALFORMED = 4
FRAME_RECV_ERR = 5  # client role, body_len 0: rpc_async.c:330-349 drops the connection (RPC_RECV_ERR)
FRAMES_SERVER = 0x1
FRAMES_CLIENT = 0x2
FRAMES_LIFT_CAP = 0x4


def _as_buffer(data) -> tuple[Optional[int], int, object]:
    """(address, nbytes, keepalive) for bytes-like / numpy input; None -> NULL."""
    if data is None:
        return None, 0, None
    if isinstance(data, np.ndarray):
        arr = np.ascontiguousarray(data)
        return arr.ctypes.data, arr.nbytes, arr
    mv = memoryview(data).cast("B")
    if mv.readonly:
        buf = ctypes.create_string_buffer(bytes(mv), len(mv))
        return ctypes.addressof(buf), len(mv), buf
    arr = np.frombuffer(mv, dtype=np.uint8)
    return arr.ctypes.data, arr.nbytes, arr


# ---- drop-in ---------------------------------------------------------------

def rpc_crc32(data, length: Optional[int] = None) -> int:
    """rpc_crc32(data, len) -- reference crc.c:4-9.  ``length`` defaults to len(data)."""
    addr, n, keep = _as_buffer(data)
    if length is None:
        length = n
    r = _lib.rpc_crc32(addr, length)
    del keep
    return int(r)


def rpc_crc32_verify(data, expected_crc: int, length: Optional[int] = None) -> bool:
    """rpc_crc32_verify(data, len, expected) -- reference crc.c:11-14."""
    addr, n, keep = _as_buffer(data)
    if length is None:
        length = n
    r = _lib.rpc_crc32_verify(addr, length, expected_crc & 0xFFFFFFFF)
    del keep
    return bool(r)


def crc32_combine(crc1: int, crc2: int, len2: int) -> int:
    """zlib crc32_combine semantics (zlib.h:1750)."""
    return int(_lib.rpc_crc32_combine(crc1 & 0xFFFFFFFF, crc2 & 0xFFFFFFFF, len2))


# ---- batched, host buffers ---------------------------------------------------

def crc32_batch(buf, offsets: Sequence[int], lengths: Sequence[int]) -> np.ndarray:
    """CRC of every body ``buf[offsets[i] : offsets[i] + lengths[i]]`` (host memory)."""
    addr, _, keep = _as_buffer(buf)
    off = np.ascontiguousarray(offsets, dtype=np.uint64)
    ln = np.ascontiguousarray(lengths, dtype=np.uint32)
    if off.shape != ln.shape:
        raise ValueError("offsets and lengths differ in length")
    out = np.empty(off.shape[0], dtype=np.uint32)
    check(_lib.rpc_crc32_batch(addr, off.ctypes.data, ln.ctypes.data, off.shape[0], out.ctypes.data, 0),
          "rpc_crc32_batch")
    del keep
    return out


def verify_batch(buf, offsets, lengths, expected) -> tuple[int, np.ndarray]:
    """(mismatch count, ok[] uint8) -- batched rpc_crc32_verify."""
    addr, _, keep = _as_buffer(buf)
    off = np.ascontiguousarray(offsets, dtype=np.uint64)
    ln = np.ascontiguousarray(lengths, dtype=np.uint32)
    exp = np.ascontiguousarray(expected, dtype=np.uint32)
    ok = np.empty(off.shape[0], dtype=np.uint8)
    bad = check(_lib.rpc_crc32_verify_batch(addr, off.ctypes.data, ln.ctypes.data, exp.ctypes.data,
                                            off.shape[0], ok.ctypes.data), "rpc_crc32_verify_batch")
    del keep
    return int(bad), ok


# ---- batched, device buffers (torch tensors as HBM plumbing) -----------------

def _torch():
    if _lib.torch is None:
        raise RuntimeError("device-buffer calls need torch (ROCm) for device memory")
    return _lib.torch


def _stream_handle(stream) -> int:
    t = _torch()
    s = stream if stream is not None else t.cuda.current_stream()
    return int(s.cuda_stream)


def _dev_u32_out(n: int, device, out):
    t = _torch()
    if out is None:
        out = t.empty(n, dtype=t.int32, device=device)
    if out.numel() < n or out.element_size() != 4 or not out.is_contiguous():
        raise ValueError("out must be a contiguous 4-byte tensor with >= n elements")
    return out


def device_batch(base, offsets, lengths, out=None, stream=None, max_len: int = 0):
    """Ragged batch over a device byte tensor; offsets int64/uint64, lengths int32/uint32 device tensors.
    ``max_len``: an upper bound on the lengths the caller knows (0 = none); below 256 KiB the
    big-body route's passes are skipped (rpc_crc32_device_batch_bounded; results never depend on it)."""
    n = offsets.numel()
    if lengths.numel() != n:
        raise ValueError("offsets and lengths differ in length")
    out = _dev_u32_out(n, base.device, out)
    if _lib.rpc_crc32_device_batch_bounded is None:  # an older build under A/B (tools/ab_lib.sh)
        check(_lib.rpc_crc32_device_batch(base.data_ptr(), offsets.data_ptr(), lengths.data_ptr(), n,
                                          out.data_ptr(), _stream_handle(stream)), "rpc_crc32_device_batch")
        return out
    check(_lib.rpc_crc32_device_batch_bounded(base.data_ptr(), offsets.data_ptr(), lengths.data_ptr(), n,
                                              int(max_len) & 0xFFFFFFFF, out.data_ptr(), _stream_handle(stream)),
          "rpc_crc32_device_batch_bounded")
    return out


def device_uniform(base, n: int, body_len: int, stride: Optional[int] = None, out=None, stream=None):
    """Equal-length batch: body i = base[i*stride : i*stride + body_len]."""
    if stride is None:
        stride = body_len
    if n and (n - 1) * stride + body_len > base.numel() * base.element_size():
        raise ValueError("bodies exceed the base tensor")
    out = _dev_u32_out(n, base.device, out)
    check(_lib.rpc_crc32_device_uniform(base.data_ptr(), n, body_len, stride, out.data_ptr(),
                                        _stream_handle(stream)), "rpc_crc32_device_uniform")
    return out


def device_large(base, offsets: Iterable[int], lengths: Iterable[int], chunk: int = 0, out=None, stream=None):
    """Large bodies (host-known offsets/lengths, device data), chunked + GF(2)-combined."""
    off = np.ascontiguousarray(list(offsets), dtype=np.uint64)
    ln = np.ascontiguousarray(list(lengths), dtype=np.uint64)
    n = off.shape[0]
    out = _dev_u32_out(n, base.device, out)
    check(_lib.rpc_crc32_device_large(base.data_ptr(), off.ctypes.data, ln.ctypes.data, n, out.data_ptr(),
                                      chunk, _stream_handle(stream)), "rpc_crc32_device_large")
    return out


def _frames_flags(role: str, lift_cap: bool) -> int:
    try:
        f = {"server": FRAMES_SERVER, "client": FRAMES_CLIENT}[role]
    except KeyError:
        raise ValueError("role must be 'server' (PING is control) or 'client' (PONG is control)") from None
    return f | (FRAMES_LIFT_CAP if lift_cap else 0)


def frames_verify(stream_buf, frame_offsets, role: str = "server", lift_cap: bool = False, stream_bytes=None,
                  crc_out=None, stream=None):
    """Verify n wire frames (rpc.h header + body) in a device byte tensor.

    Returns (verdict uint8 tensor of FRAME_*, crc int32 tensor).  ``role`` picks the
    heartbeat that is a control frame: "server" -> PING (rpc_server_main.c:172),
    "client" -> PONG (rpc_async.c:303).  Without ``lift_cap`` a data frame whose
    body_len exceeds MAX_BODY_LEN is FRAME_TOO_LARGE (rpc_server_main.c:189)."""
    t = _torch()
    n = frame_offsets.numel()
    nbytes = stream_buf.numel() * stream_buf.element_size() if stream_bytes is None else int(stream_bytes)
    verdict = t.empty(n, dtype=t.uint8, device=stream_buf.device)
    crc = _dev_u32_out(n, stream_buf.device, crc_out)
    check(_lib.rpc_frames_verify_device(stream_buf.data_ptr(), nbytes, frame_offsets.data_ptr(), n,
                                        _frames_flags(role, lift_cap), verdict.data_ptr(), crc.data_ptr(),
                                        _stream_handle(stream)), "rpc_frames_verify_device")
    return verdict, crc


def frames_stamp(stream_buf, frame_offsets, body_lens, version: int = 1, type_: int = RPC_TYPE_DATA,
                 lift_cap: bool = False, stream_bytes=None, stream=None):
    """Write rpc.h headers (BE version/type/body_len/crc32) in front of device-resident
    bodies; returns the per-frame verdict (FRAME_OK stamped, FRAME_TOO_LARGE /
    FRAME_MALFORMED not stamped)."""
    t = _torch()
    n = frame_offsets.numel()
    nbytes = stream_buf.numel() * stream_buf.element_size() if stream_bytes is None else int(stream_bytes)
    verdict = t.empty(n, dtype=t.uint8, device=stream_buf.device)
    check(_lib.rpc_frames_stamp_device(stream_buf.data_ptr(), nbytes, frame_offsets.data_ptr(), body_lens.data_ptr(),
                                       n, version, type_, FRAMES_LIFT_CAP if lift_cap else 0, verdict.data_ptr(),
                                       _stream_handle(stream)), "rpc_frames_stamp_device")
    return verdict


def fill_random(tensor, seed: int, stream=None):
    """splitmix64 counter stream into a device tensor (nbytes multiple of 8)."""
    nbytes = tensor.numel() * tensor.element_size()
    check(_lib.rpc_crc32_fill_random_device(tensor.data_ptr(), nbytes, seed & (2**64 - 1), _stream_handle(stream)),
          "rpc_crc32_fill_random_device")
    return tensor


def stream_read(tensor, pattern: int = 0, nontemporal: bool = False, nbytes: Optional[int] = None, stream=None):
    """HBM read probe: pattern 0 coalesced 16-B lanes, 1 = 64-B lane segments (grid-stride
    loops), 2 = the rows kernel's own dealing and loads with the CRC work compiled out."""
    if nbytes is None:
        nbytes = (tensor.numel() * tensor.element_size()) // 4096 * 4096
    check(_lib.rpc_crc32_stream_read_device(tensor.data_ptr(), nbytes, pattern, int(nontemporal),
                                            _stream_handle(stream)), "rpc_crc32_stream_read_device")


def set_options(nontemporal: bool = False, max_blocks: int = 0):
    check(_lib.rpc_crc32_set_options(int(nontemporal), max_blocks), "rpc_crc32_set_options")


#: rpc_crc32_set_ragged_path codes (include/rpccrc.h RPCCRC_RAGGED_*)
RAGGED_PATHS = {"auto": 0, "rows": 1, "packed": 2, "split": 3}


def set_ragged_path(path="auto"):
    """Kernel for ragged device batches: "auto" (frames: split, other batches: rows),
    "rows" (one wavefront per body), "packed" (1 KiB chunks of consecutive
    bodies, four per row) or "split" (bodies <= 1 KiB four per row, the rest
    one wavefront per body)."""
    code = RAGGED_PATHS[path] if isinstance(path, str) else int(path)
    check(_lib.rpc_crc32_set_ragged_path(code), "rpc_crc32_set_ragged_path")


def device_status() -> int:
    """0, or -5 (RPCCRC_EIO) once a kernel of an asynchronous call has reported an
    error into the device's error word (until device_clear_status())."""
    return int(_lib.rpc_crc32_device_status())


def device_clear_status() -> int:
    """Clears the device error word; returns the status it held (0 or -5)."""
    return int(_lib.rpc_crc32_device_clear_status())


def service_stop() -> int:
    """Stops the resident drop-in service (the next drop-in call restarts it), so a
    device-wide synchronize does not wait for it; 0, or -5 if it did not leave in time."""
    return int(_lib.rpc_crc32_service_stop())


def service_stats() -> dict:
    """The drop-in service's counters over every device this process used
    (rpccrc_service_stats_t): services, running, launched, answered,
    fallbacks_full, fallbacks_short, bypassed."""
    st = _lib.ServiceStats()
    check(_lib.rpc_crc32_service_stats(ctypes.byref(st)), "rpc_crc32_service_stats")
    return {k: int(getattr(st, k)) for k, _ in st._fields_}


def device_info() -> str:
    buf = ctypes.create_string_buffer(256)
    check(_lib.rpc_crc32_device_info(buf, 256), "rpc_crc32_device_info")
    return buf.value.decode()
