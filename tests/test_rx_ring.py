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
