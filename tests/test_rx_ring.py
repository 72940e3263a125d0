"""Batched server receive ring (include/rpccrc.h rpc_rx_ring_*).

The reference server verifies each frame as it arrives (server/rpc_server_main.c:227:
rpc_crc32_verify(body, body_len, header crc32)).  The ring must give the same verdict
for every frame -- valid, corrupted body, corrupted CRC field, PING/PONG -- in arrival
order with the caller's tag, across segment rotations and partial polls.  Checked
against the oracle and the captured reference frames (tests/golden)."""
import numpy as np
import pytest

import rpc_amd
from oracle import oracle


def frame(body: bytes, version=1, type_=rpc_amd.RPC_TYPE_DATA, crc=None) -> bytes:
    """rpc.h:3-8 header (big-endian, as rpc_async.c:521-530 stamps it) + body."""
    c = oracle.crc32(body) if crc is None else crc
    return (version.to_bytes(2, "big") + type_.to_bytes(2, "big") + len(body).to_bytes(4, "big")
            + c.to_bytes(4, "big") + body)


def have_gpu():
    try:
        import torch
        return torch.cuda.device_count() > 0
    except Exception:
        return False


@pytest.mark.skipif(have_gpu(), reason="checks the no-device behaviour")
def test_ring_needs_device():
    with pytest.raises(rpc_amd.RpcCrcError) as ei:
        rpc_amd.RxRing(1 << 16, 64, 2)
    assert ei.value.code == -19


def test_ring_rejects_bad_geometry():
    for args in [(8, 64, 2), (1 << 16, 0, 2), (1 << 16, 64, 1), (1 << 16, 64, 65)]:
        with pytest.raises(rpc_amd.RpcCrcError) as ei:
            rpc_amd.RxRing(*args)
        assert ei.value.code == -22
    # exactly one role bit (server: PING is control, client: PONG), LIFT_CAP optional
    import ctypes
    for flags in (0, 3, 4, 8, 1 | 8):
        h = ctypes.c_void_p()
        assert rpc_amd._lib.rpc_rx_ring_create(ctypes.byref(h), 1 << 16, 64, 2, flags) == -22, flags
    with pytest.raises(ValueError):
        rpc_amd.RxRing(1 << 16, 64, 2, role="proxy")


def _workload(n, seed):
    """Frames as a server receives them: JSON-ish bodies up to MAX_BODY_LEN (rpc.h:17),
    some corrupted, PINGs mixed in.  Returns (frames, expected verdicts, expected crcs)."""
    rng = np.random.default_rng(seed)
    frames, ok, crcs = [], [], []
    for i in range(n):
        kind = rng.integers(0, 10)
        if kind == 0:  # PING (rpc_server_main.c:172-187): empty body, crc 0
            frames.append(frame(b"", type_=rpc_amd.RPC_TYPE_PING, crc=0))
            ok.append(1)
            crcs.append(0)
            continue
        body = rng.integers(32, 127, int(rng.integers(1, 1025)), dtype=np.uint8).tobytes()
        f = bytearray(frame(body))
        if kind == 1:  # flipped body bit
            f[12 + int(rng.integers(0, len(body)))] ^= 0x04
        elif kind == 2:  # flipped CRC-field bit
            f[8 + int(rng.integers(0, 4))] ^= 0x80
        frames.append(bytes(f))
        ok.append(int(kind not in (1, 2)))
        crcs.append(oracle.crc32(bytes(f[12:])))
    return frames, ok, crcs


@pytest.mark.gpu
@pytest.mark.parametrize("seg_bytes,max_frames,nseg", [(1 << 20, 4096, 2), (40000, 37, 3), (1 << 16, 1000, 4)])
def test_ring_verdicts_match_reference(seg_bytes, max_frames, nseg):
    frames, ok, crcs = _workload(3000, seg_bytes + nseg)
    got = []
    with rpc_amd.RxRing(seg_bytes, max_frames, nseg) as ring:
        for i, f in enumerate(frames):
            while (ring.push(f, 1000 + i) if i % 2 else ring.push_into(f, 1000 + i)) == rpc_amd.rx_ring.EAGAIN:
                got += ring.poll(wait=True)
        ring.submit()
        while len(got) < len(frames):
            r = ring.poll(wait=True)
            assert r, "ring lost frames"
            got += r
    assert [g[0] for g in got] == [1000 + i for i in range(len(frames))]  # arrival order, tags intact
    assert [g[1] for g in got] == ok
    assert [g[2] for g in got] == crcs
    assert [g[4] for g in got] == [f[12:] for f in frames]
    assert [g[5] for g in got] == [rpc_amd.FRAME_CONTROL if f[2:4] == b"\x00\x01" else
                                   (rpc_amd.FRAME_OK if k else rpc_amd.FRAME_BAD_CRC) for f, k in zip(frames, ok)]


@pytest.mark.gpu
def test_ring_captured_reference_frames(golden):
    """The request/response frames captured from the reference server."""
    with rpc_amd.RxRing(1 << 16, 16, 2) as ring:
        for i, f in enumerate(golden["frames"]):
            hdr = bytes.fromhex(f["header_hex"])
            assert ring.push(hdr + f["body"].encode(), i) == 0
        ring.submit()
        got = ring.poll(wait=True)
    assert [g[1] for g in got] == [1] * len(golden["frames"])
    for g, f in zip(got, golden["frames"]):
        assert g[3] == int(f["header_hex"][16:24], 16)


@pytest.mark.gpu
def test_ring_rejects_inconsistent_length():
    """A header whose body_len disagrees with the landed frame is refused at commit
    (the kernel would otherwise read past the frame)."""
    with rpc_amd.RxRing(1 << 16, 16, 2) as ring:
        f = bytearray(frame(b"abc"))
        f[7] = 9  # body_len 9, only 3 bytes landed
        with pytest.raises(rpc_amd.RpcCrcError) as ei:
            ring.push(bytes(f), 1)
        assert ei.value.code == -22
        assert ring.push(frame(b"abc"), 2) == 0
        ring.submit()
        got = ring.poll(wait=True)
    assert [(g[0], g[1]) for g in got] == [(2, 1)]


@pytest.mark.gpu
def test_ring_partial_polls_and_idle():
    frames, ok, _ = _workload(500, 77)
    with rpc_amd.RxRing(1 << 20, 4096, 2) as ring:
        assert ring.poll(wait=False) == []  # nothing submitted
        for i, f in enumerate(frames):
            assert ring.push(f, i) == 0
        ring.submit()
        ring.submit()  # nothing left to submit: no-op
        got = []
        ring._buf = (rpc_amd._lib.RxFrame * 64)()
        ring.max_frames = 64
        while len(got) < len(frames):
            got += ring.poll(wait=True)
        assert ring.poll(wait=True) == []
    assert [g[1] for g in got] == ok


def _hdr(body_len, crc, type_=rpc_amd.RPC_TYPE_DATA):
    return (1).to_bytes(2, "big") + type_.to_bytes(2, "big") + body_len.to_bytes(4, "big") + crc.to_bytes(4, "big")


@pytest.mark.gpu
@pytest.mark.parametrize("role", ["server", "client"])
def test_ring_control_and_over_cap_frames(role):
    """The reference reads no body for a heartbeat (PING at the server,
    rpc_server_main.c:172-187; PONG at the client, rpc_async.c:303-309) whatever its
    crc32 / body_len fields hold, nor for a data frame over MAX_BODY_LEN
    (rpc_server_main.c:189-195, rpc_async.c:312): such frames land as the 12-byte
    header alone and get FRAME_CONTROL / FRAME_TOO_LARGE."""
    ctl = rpc_amd.RPC_TYPE_PING if role == "server" else rpc_amd.RPC_TYPE_PONG
    other = rpc_amd.RPC_TYPE_PONG if role == "server" else rpc_amd.RPC_TYPE_PING
    body = b'{"jsonrpc":"2.0","id":7,"result":1}'
    frames = [
        (_hdr(500, 0xDEADBEEF, ctl), rpc_amd.FRAME_CONTROL, 1),
        (_hdr(0, 0, ctl), rpc_amd.FRAME_CONTROL, 1),
        (_hdr(2000, 0x1234), rpc_amd.FRAME_TOO_LARGE, 0),
        (_hdr(1025, 0), rpc_amd.FRAME_TOO_LARGE, 0),
        (frame(body), rpc_amd.FRAME_OK, 1),
        (frame(body, type_=other), rpc_amd.FRAME_OK, 1),          # the other heartbeat type is data here
        (frame(body, type_=other, crc=5), rpc_amd.FRAME_BAD_CRC, 0),
        # an empty body: the server verifies it (crc 0), the client drops the
        # connection on its recv of 0 bytes (rpc_async.c:330-349, RPC_RECV_ERR)
        (frame(b"", type_=other), rpc_amd.FRAME_OK if role == "server" else rpc_amd.FRAME_RECV_ERR,
         1 if role == "server" else 0),
        (frame(b""), rpc_amd.FRAME_OK if role == "server" else rpc_amd.FRAME_RECV_ERR, 1 if role == "server" else 0),
    ]
    with rpc_amd.RxRing(1 << 16, 64, 2, role=role) as ring:
        for i, (f, _, _) in enumerate(frames):
            assert ring.push_into(f, i) == 0
        # a data frame landed as a bare header while its body_len is within the cap is refused
        with pytest.raises(rpc_amd.RpcCrcError):
            ring.push(_hdr(100, 0), 99)
        # a control / over-cap header landed together with bytes after it is refused:
        # the reference reads the header alone and takes those bytes for the next frame
        for bad in (_hdr(4, 0, ctl) + b"abcd", _hdr(1025, 0) + bytes(1025)):
            with pytest.raises(rpc_amd.RpcCrcError):
                ring.push(bad, 98)
        ring.submit()
        got = ring.poll(wait=True)
    assert [g[0] for g in got] == list(range(len(frames)))
    assert [g[5] for g in got] == [v for _, v, _ in frames]
    assert [g[1] for g in got] == [ok for _, _, ok in frames]
    assert got[4][4] == body and got[0][4] == b"" and got[2][4] == b""


@pytest.mark.gpu
def test_ring_lifted_cap_large_frames():
    """SURVEY 8f3 through the ring: bodies up to 6 MiB in 16 MiB segments, verified on
    the GPU (the >= 256 KiB ones through the chunk route), one corrupted."""
    rng = np.random.default_rng(5)
    lens = [3000, 1 << 20, (6 << 20) + 5, 17, (256 << 10) + 1, 1024, 70000, (3 << 20) + 11]
    bodies = [rng.integers(0, 256, L, dtype=np.uint8).tobytes() for L in lens]
    frames = [frame(b) for b in bodies]
    bad = bytearray(frames[2])
    bad[12 + 4321] ^= 1
    frames[2] = bytes(bad)
    with rpc_amd.RxRing(16 << 20, 64, 2, lift_cap=True) as ring:
        for i, f in enumerate(frames):
            assert ring.push(f, i) == 0
        ring.submit()
        got = ring.poll(wait=True)
    assert [g[5] for g in got] == [rpc_amd.FRAME_BAD_CRC if i == 2 else rpc_amd.FRAME_OK for i in range(len(lens))]
    assert [g[2] for g in got] == [oracle.crc32(f[12:]) for f in frames]
