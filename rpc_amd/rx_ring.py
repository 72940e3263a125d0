"""Batched server receive ring (include/rpccrc.h ``rpc_rx_ring_*``).

Python mirror of the C-ABI for tests and the bench: frames (12-byte rpc.h header
+ body) are pushed into pinned segments, verified on the GPU a segment at a
time, and polled back in arrival order with their tags.  The reference server
verifies one frame per recv instead (server/rpc_server_main.c:135-238).
"""
from __future__ import annotations

import ctypes
from typing import List, Tuple

from . import _lib
from ._lib import RpcCrcError, check

EAGAIN = -11


class RxRing:
    def __init__(self, segment_bytes: int = 64 << 20, max_frames: int = 1 << 16, nsegments: int = 3,
                 role: str = "server", lift_cap: bool = False):
        self._h = None
        flags = {"server": 0x1, "client": 0x2}.get(role)
        if flags is None:
            raise ValueError("role must be 'server' or 'client'")
        flags |= 0x4 if lift_cap else 0
        h = ctypes.c_void_p()
        check(_lib.rpc_rx_ring_create(ctypes.byref(h), segment_bytes, max_frames, nsegments, flags),
              "rpc_rx_ring_create")
        self._h = h
        self._buf = (_lib.RxFrame * max_frames)()
        self.max_frames = max_frames

    def close(self):
        if getattr(self, "_h", None):
            _lib.rpc_rx_ring_destroy(self._h)
            self._h = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        self.close()

    def push(self, frame: bytes, tag: int) -> int:
        """rpc_rx_ring_push: 0, EAGAIN (-11: poll first) or raises on another error."""
        rc = _lib.rpc_rx_ring_push(self._h, frame, len(frame), tag)
        if rc < 0 and rc != EAGAIN:
            raise RpcCrcError(rc, "rpc_rx_ring_push")
        return rc

    def push_into(self, frame: bytes, tag: int) -> int:
        """reserve + copy + commit, as a recv() loop would land a frame."""
        dst = ctypes.c_void_p()
        rc = _lib.rpc_rx_ring_reserve(self._h, len(frame), ctypes.byref(dst))
        if rc == EAGAIN:
            return rc
        check(rc, "rpc_rx_ring_reserve")
        ctypes.memmove(dst.value, frame, len(frame))
        return check(_lib.rpc_rx_ring_commit(self._h, tag), "rpc_rx_ring_commit")

    def submit(self):
        check(_lib.rpc_rx_ring_submit(self._h), "rpc_rx_ring_submit")

    def poll(self, wait: bool = True) -> List[Tuple[int, int, int, int, bytes, int]]:
        """[(tag, ok, crc, header_crc, body, verdict)] of the oldest submitted segment.
        ``body`` is empty for frames whose body the reference does not read
        (control and over-cap frames land as the 12-byte header alone)."""
        n = check(_lib.rpc_rx_ring_poll(self._h, self._buf, self.max_frames, int(wait)), "rpc_rx_ring_poll")
        res = []
        for i in range(n):
            f = self._buf[i]
            has_body = f.verdict in (0, 1) and f.body_len  # FRAME_BAD_CRC / FRAME_OK
            body = ctypes.string_at(f.frame + 12, f.body_len) if has_body else b""
            res.append((int(f.tag), int(f.ok), int(f.crc), int(f.header_crc), body, int(f.verdict)))
        return res
