"""ctypes binding of librpccrc.so (include/rpccrc.h).

The shared library is built in-tree by ``__graft_entry__.build()`` /
``make -C rpc_amd/csrc`` into ``rpc_amd/lib/librpccrc.so``.  There is no
fallback: if the library is missing, importing this module raises.

HIP runtime note: PyTorch-ROCm ships its own ``libamdhip64.so.7``.  When torch is
importable we import it *first*, so librpccrc's ``DT_NEEDED libamdhip64.so.7``
binds to the runtime torch already loaded and device pointers / streams from
torch are valid in our calls (one HIP runtime per process).
"""
from __future__ import annotations

import ctypes
import os

try:  # one HIP runtime per process: let torch load it first (see module doc)
    import torch  # noqa: F401
except Exception:  # pragma: no cover - torch is optional for the C-ABI itself
    torch = None

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("RPCCRC_LIB") or os.path.join(HERE, "lib", "librpccrc.so")  # (empty = in-tree)

if not os.path.exists(LIB_PATH):
    raise ImportError(
        f"librpccrc.so not found at {LIB_PATH}; build it with "
        "`python -c 'import __graft_entry__ as g; g.build()'` or `make -C rpc_amd/csrc`"
    )

lib = ctypes.CDLL(LIB_PATH)

_u8p = ctypes.c_void_p
_vp = ctypes.c_void_p
_u32 = ctypes.c_uint32
_u64 = ctypes.c_uint64
_i32 = ctypes.c_int
_sz = ctypes.c_size_t


def _sig(name, restype, *argtypes):
    try:
        f = getattr(lib, name)
    except AttributeError:
        # A/B runs may point RPCCRC_LIB at an older build (tools/ab_lib.sh) that
        # lacks a newer entry point; the in-tree library must export them all
        # (tests/test_abi.py).
        if os.environ.get("RPCCRC_LIB"):
            return None
        raise
    f.restype = restype
    f.argtypes = list(argtypes)
    return f


rpc_crc32 = _sig("rpc_crc32", _u32, _vp, _sz)
rpc_crc32_verify = _sig("rpc_crc32_verify", ctypes.c_bool, _vp, _sz, _u32)
rpc_crc32_batch = _sig("rpc_crc32_batch", _i32, _u8p, _vp, _vp, _sz, _vp, _i32)
rpc_crc32_verify_batch = _sig("rpc_crc32_verify_batch", ctypes.c_int64, _u8p, _vp, _vp, _vp, _sz, _vp)
rpc_crc32_device_batch = _sig("rpc_crc32_device_batch", _i32, _vp, _vp, _vp, _u64, _vp, _vp)
rpc_crc32_device_batch_bounded = _sig("rpc_crc32_device_batch_bounded", _i32, _vp, _vp, _vp, _u64, _u32, _vp, _vp)
rpc_crc32_device_uniform = _sig("rpc_crc32_device_uniform", _i32, _vp, _u64, _u32, _u64, _vp, _vp)
rpc_crc32_device_large = _sig("rpc_crc32_device_large", _i32, _vp, _vp, _vp, _u64, _vp, _u64, _vp)
rpc_frames_verify_device = _sig("rpc_frames_verify_device", _i32, _vp, _u64, _vp, _u64, _i32, _vp, _vp, _vp)
rpc_frames_stamp_device = _sig(
    "rpc_frames_stamp_device", _i32, _vp, _u64, _vp, _vp, _u64, ctypes.c_uint16, ctypes.c_uint16, _i32, _vp, _vp
)
rpc_rx_ring_create = _sig("rpc_rx_ring_create", _i32, ctypes.POINTER(ctypes.c_void_p), _sz, _sz, _i32, _i32)
rpc_rx_ring_destroy = _sig("rpc_rx_ring_destroy", None, _vp)
rpc_rx_ring_reserve = _sig("rpc_rx_ring_reserve", _i32, _vp, _sz, ctypes.POINTER(ctypes.c_void_p))
rpc_rx_ring_commit = _sig("rpc_rx_ring_commit", _i32, _vp, _u64)
rpc_rx_ring_push = _sig("rpc_rx_ring_push", _i32, _vp, _vp, _sz, _u64)
rpc_rx_ring_submit = _sig("rpc_rx_ring_submit", _i32, _vp)
rpc_crc32_combine = _sig("rpc_crc32_combine", _u32, _u32, _u32, _u64)
rpc_crc32_fill_random_device = _sig("rpc_crc32_fill_random_device", _i32, _vp, _u64, _u64, _vp)
rpc_crc32_stream_read_device = _sig("rpc_crc32_stream_read_device", _i32, _vp, _u64, _i32, _i32, _vp)
rpc_crc32_set_options = _sig("rpc_crc32_set_options", _i32, _i32, _i32)
rpc_crc32_set_ragged_path = _sig("rpc_crc32_set_ragged_path", _i32, _i32)
rpc_crc32_strerror = _sig("rpc_crc32_strerror", ctypes.c_char_p, _i32)
rpc_crc32_device_info = _sig("rpc_crc32_device_info", _i32, ctypes.c_char_p, _sz)
rpc_crc32_device_status = _sig("rpc_crc32_device_status", _i32)
rpc_crc32_device_clear_status = _sig("rpc_crc32_device_clear_status", _i32)
rpc_crc32_service_stop = _sig("rpc_crc32_service_stop", _i32)


class ServiceStats(ctypes.Structure):
    """rpccrc_service_stats_t (include/rpccrc.h)."""
    _fields_ = [(k, ctypes.c_uint64) for k in ("services", "running", "launched", "answered", "fallbacks_full",
                                               "fallbacks_short", "bypassed")]


rpc_crc32_service_stats = _sig("rpc_crc32_service_stats", _i32, ctypes.POINTER(ServiceStats))

#: Every symbol include/rpccrc.h declares (checked by tests/test_abi.py).
EXPORTS = (
    "rpc_crc32",
    "rpc_crc32_verify",
    "rpc_crc32_batch",
    "rpc_crc32_verify_batch",
    "rpc_crc32_device_batch",
    "rpc_crc32_device_batch_bounded",
    "rpc_crc32_device_uniform",
    "rpc_crc32_device_large",
    "rpc_frames_verify_device",
    "rpc_frames_stamp_device",
    "rpc_rx_ring_create",
    "rpc_rx_ring_destroy",
    "rpc_rx_ring_reserve",
    "rpc_rx_ring_commit",
    "rpc_rx_ring_push",
    "rpc_rx_ring_submit",
    "rpc_rx_ring_poll",
    "rpc_crc32_combine",
    "rpc_crc32_fill_random_device",
    "rpc_crc32_stream_read_device",
    "rpc_crc32_set_options",
    "rpc_crc32_set_ragged_path",
    "rpc_crc32_strerror",
    "rpc_crc32_device_info",
    "rpc_crc32_device_status",
    "rpc_crc32_device_clear_status",
    "rpc_crc32_service_stop",
    "rpc_crc32_service_stats",
)


class RxFrame(ctypes.Structure):
    """rpc_rx_frame_t (include/rpccrc.h)."""
    _fields_ = [("tag", ctypes.c_uint64), ("frame", ctypes.c_void_p), ("body_len", ctypes.c_uint32),
                ("version", ctypes.c_uint16), ("type", ctypes.c_uint16), ("header_crc", ctypes.c_uint32),
                ("crc", ctypes.c_uint32), ("ok", ctypes.c_uint8), ("verdict", ctypes.c_uint8)]


rpc_rx_ring_poll = _sig("rpc_rx_ring_poll", ctypes.c_int64, _vp, ctypes.POINTER(RxFrame), _sz, _i32)


class RpcCrcError(RuntimeError):
    """A negative return code from librpccrc."""

    def __init__(self, code: int, what: str):
        self.code = code
        msg = rpc_crc32_strerror(code).decode()
        super().__init__(f"{what}: {msg} ({code})")


def check(rc: int, what: str) -> int:
    if rc < 0:
        raise RpcCrcError(rc, what)
    return rc
