"""Frames on the GPU: batched verify / stamp of rpc.h wire
frames, with the reference's receive-side decisions restated in
``oracle.frame_verdict`` (type first -- PING at the server rpc_server_main.c:172-187,
PONG at the client rpc_async.c:303-309 -- then the MAX_BODY_LEN cap
rpc_server_main.c:189-195 / rpc_async.c:312, then rpc_crc32_verify) and the stream
bound (no read outside the stream).  With the cap lifted (8f3) bodies of any size are
verified, the large ones through the chunk route."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
import rpc_amd  # noqa: E402
from oracle import oracle  # noqa: E402

DEV = "cuda:0"
HDR = 12


def to_dev(a: np.ndarray):
    return torch.from_numpy(np.ascontiguousarray(a)).to(DEV)


def u32(t):
    return t.cpu().numpy().view(np.uint32)


def header(body_len: int, crc: int, type_: int = 0, version: int = 1) -> bytes:
    return (version.to_bytes(2, "big") + type_.to_bytes(2, "big") + (body_len & 0xFFFFFFFF).to_bytes(4, "big")
            + (crc & 0xFFFFFFFF).to_bytes(4, "big"))


def layout(frames, gap=0):
    """Concatenate frames (bytes) with `gap` junk bytes after each; -> (stream, offsets)."""
    offs, blob = [], bytearray()
    for f in frames:
        offs.append(len(blob))
        blob += f + b"\xA5" * gap
    return bytes(blob), np.array(offs, dtype=np.uint64)


def verify(stream: bytes, offs, role="server", lift_cap=False, stream_bytes=None):
    sdev = to_dev(np.frombuffer(stream, dtype=np.uint8).copy())
    v, c = rpc_amd.frames_verify(sdev, to_dev(offs.view(np.int64)), role=role, lift_cap=lift_cap,
                                 stream_bytes=stream_bytes)
    return v.cpu().numpy().tolist(), u32(c).tolist()


def expected(stream: bytes, offs, role="server", lift_cap=False):
    r = [oracle.frame_verdict(stream, int(o), role, lift_cap) for o in offs]
    return [x[0] for x in r], [x[1] for x in r]


def test_frames_verify_and_stamp(golden):
    rng = np.random.default_rng(2)
    bodies = [f["body"].encode() for f in golden["frames"][:2]]
    bodies += [rng.integers(32, 127, int(rng.integers(0, 1025)), dtype=np.uint8).tobytes() for _ in range(300)]
    blob, offs = layout([bytes(HDR) + b for b in bodies], gap=1)
    lens = np.array([len(b) for b in bodies], dtype=np.uint32)
    dblob = to_dev(np.frombuffer(blob, dtype=np.uint8).copy())
    sv = rpc_amd.frames_stamp(dblob, to_dev(offs.view(np.int64)), to_dev(lens.view(np.int32)), version=1,
                              type_=rpc_amd.RPC_TYPE_DATA)
    assert sv.cpu().numpy().tolist() == [rpc_amd.FRAME_OK] * len(bodies)
    stamped = dblob.cpu().numpy().tobytes()
    for i, (o, b) in enumerate(zip(offs, bodies)):
        assert stamped[int(o):int(o) + HDR] == header(len(b), oracle.crc32(b)), i
    # the captured request/response headers are reproduced byte for byte
    assert stamped[:HDR].hex() == golden["frames"][0]["header_hex"]
    assert stamped[int(offs[1]):int(offs[1]) + HDR].hex() == golden["frames"][1]["header_hex"]
    # corrupt some bodies / CRC fields, then verify against the reference's decisions
    arr = np.frombuffer(stamped, dtype=np.uint8).copy()
    for i in range(4, len(bodies), 7):
        if lens[i] > 0:
            arr[int(offs[i]) + HDR + int(lens[i]) // 2] ^= 0x10
        else:
            arr[int(offs[i]) + 11] ^= 1
    got = verify(arr.tobytes(), offs)
    want = expected(arr.tobytes(), offs)
    assert got == want
    assert got[0].count(rpc_amd.FRAME_BAD_CRC) == len(range(4, len(bodies), 7))


def test_captured_ping_pong(golden):
    """The captured PING (client -> server) and PONG (server -> client) headers."""
    ping, pong = (bytes.fromhex(f["header_hex"]) for f in golden["frames"][2:4])
    stream, offs = layout([ping, pong])
    v, _ = verify(stream, offs, role="server")
    assert v == [rpc_amd.FRAME_CONTROL, rpc_amd.FRAME_OK]  # a server reads PONG as an (empty) data frame
    v, _ = verify(stream, offs, role="client")
    # a client reads PING as a data frame with body_len 0: recv(fd, buf, 0) == 0 drops
    # the connection before any verify (rpc_async.c:330-349 -> RPC_RECV_ERR)
    assert v == [rpc_amd.FRAME_RECV_ERR, rpc_amd.FRAME_CONTROL]


@pytest.mark.parametrize("lift_cap", [False, True])
def test_frames_zero_length_bodies(lift_cap):
    """body_len 0 of every type and crc32 field: the server verifies the empty body
    (crc 0 == field? rpc_server_main.c:198-227); the client drops the connection
    unless the frame is a PONG (rpc_async.c:303-309 vs :330-349)."""
    frames = [header(0, c, t) for t in (0, 1, 2, 3, 0xFFFF) for c in (0, 1, 0x80000000, 0xFFFFFFFF)]
    stream, offs = layout(frames, gap=2)
    for role in ("server", "client"):
        got = verify(stream, offs, role, lift_cap)
        assert got == expected(stream, offs, role, lift_cap), role
    v, _ = verify(stream, offs, "client", lift_cap)
    assert v == [rpc_amd.FRAME_CONTROL if t == 2 else rpc_amd.FRAME_RECV_ERR
                 for t in (0, 1, 2, 3, 0xFFFF) for _ in range(4)]
    v, _ = verify(stream, offs, "server", lift_cap)
    assert v == [rpc_amd.FRAME_CONTROL if t == 1 else (rpc_amd.FRAME_OK if c == 0 else rpc_amd.FRAME_BAD_CRC)
                 for t in (0, 1, 2, 3, 0xFFFF) for c in (0, 1, 0x80000000, 0xFFFFFFFF)]


@pytest.fixture(params=["auto", "split"])
def frames_path(request):
    """AUTO frames batches below 16384 frames take the rows kernel; "split" forces the
    split path (small bodies four per row) that large frames batches take."""
    rpc_amd.set_ragged_path(request.param)
    yield request.param
    rpc_amd.set_ragged_path("auto")


@pytest.mark.parametrize("role", ["server", "client"])
@pytest.mark.parametrize("lift_cap", [False, True])
def test_frames_type_rules(role, lift_cap, frames_path):
    """Heartbeats whose crc32 / body_len fields are not zero, unknown types, over-cap
    lengths, empty bodies (one frame in eight): every verdict and CRC equals the
    reference's decision."""
    rng = np.random.default_rng(7 + lift_cap)
    frames = []
    for i in range(600):
        kind = int(rng.integers(0, 8))
        blen = int(rng.integers(0, 1500)) if rng.integers(0, 8) else 0
        body = rng.integers(0, 256, blen, dtype=np.uint8).tobytes()
        crc = oracle.crc32(body)
        if kind == 0:  # PING with junk crc / body_len, landed as the header alone (server reads no body)
            frames.append(header(blen, int(rng.integers(0, 2**32)), rpc_amd.RPC_TYPE_PING))
        elif kind == 1:  # PONG likewise
            frames.append(header(blen, int(rng.integers(0, 2**32)), rpc_amd.RPC_TYPE_PONG))
        elif kind == 2:  # PING / PONG carrying a full, valid body
            frames.append(header(blen, crc, int(rng.integers(1, 3))) + body)
        elif kind == 3:  # unknown type: a data frame for both roles
            frames.append(header(blen, crc, int(rng.integers(3, 65536))) + body)
        elif kind == 4:  # corrupted crc field
            frames.append(header(blen, crc ^ (1 << int(rng.integers(0, 32)))) + body)
        else:
            frames.append(header(blen, crc) + body)
    stream, offs = layout(frames, gap=3)
    assert verify(stream, offs, role, lift_cap) == expected(stream, offs, role, lift_cap)


@pytest.mark.parametrize("lift_cap", [False, True])
def test_frames_bounds_and_oversized_headers(lift_cap):
    """a hostile header must not make the kernels read outside the stream.
    body_len up to 0xFFFFFFFF, frames cut at the stream end, offsets past the end."""
    good = b'{"jsonrpc":"2.0","id":1,"result":30}'
    frames = [header(len(good), oracle.crc32(good)) + good,
              header(0xFFFFFFF0, 0x12345678),           # oversized length, no body
              header(2000, 0) + bytes(100),              # over cap, body cut short
              header(len(good), oracle.crc32(good)) + good,
              header(50, 0) + bytes(10)]                 # body runs past the stream end
    stream, offs = layout(frames)
    offs = np.concatenate([offs, np.array([len(stream) - 5, len(stream) + 100, 2**63], dtype=np.uint64)])
    got = verify(stream, offs, lift_cap=lift_cap)
    assert got == expected(stream, offs, lift_cap=lift_cap)
    v = got[0]
    assert v[0] == v[3] == rpc_amd.FRAME_OK
    assert v[1] == (rpc_amd.FRAME_MALFORMED if lift_cap else rpc_amd.FRAME_TOO_LARGE)
    assert v[4:] == [rpc_amd.FRAME_MALFORMED] * 4
    # stream_bytes bounds the stream below the tensor's size
    sub = int(offs[3])
    v2, _ = verify(stream, offs[:4], lift_cap=lift_cap, stream_bytes=sub + HDR + len(good) - 1)
    assert v2[3] == rpc_amd.FRAME_MALFORMED and v2[0] == rpc_amd.FRAME_OK


def test_frames_stamp_cap_and_bounds():
    """rpc_async.c:499-501: the client refuses to send a body over MAX_BODY_LEN, so
    without LIFT_CAP it is not stamped; bodies past the stream end are not touched."""
    lens = np.array([10, 1024, 1025, 5000, 7], dtype=np.uint32)
    blob, offs = layout([bytes(HDR) + bytes(range(256)) * (int(L) // 256) + bytes(int(L) % 256) for L in lens])
    offs = np.concatenate([offs, np.array([len(blob) - 3], dtype=np.uint64)])
    lens = np.concatenate([lens, np.array([100], dtype=np.uint32)])
    for lift in (False, True):
        d = to_dev(np.frombuffer(blob, dtype=np.uint8).copy())
        v = rpc_amd.frames_stamp(d, to_dev(offs.view(np.int64)), to_dev(lens.view(np.int32)), lift_cap=lift)
        v = v.cpu().numpy().tolist()
        TL = rpc_amd.FRAME_OK if lift else rpc_amd.FRAME_TOO_LARGE
        assert v == [rpc_amd.FRAME_OK, rpc_amd.FRAME_OK, TL, TL, rpc_amd.FRAME_OK, rpc_amd.FRAME_MALFORMED]
        out = d.cpu().numpy().tobytes()
        for i in range(5):
            o, L = int(offs[i]), int(lens[i])
            want = header(L, oracle.crc32(out[o + HDR:o + HDR + L])) if v[i] == rpc_amd.FRAME_OK else bytes(HDR)
            assert out[o:o + HDR] == want, (lift, i)
        assert out[-3:] == blob[-3:]


def test_frames_lifted_cap_large_bodies(frames_path):
    """frames with bodies from 1 B to 64 MiB (MAX_BODY_LEN lifted), stamped
    then verified on the device; the bodies >= 256 KiB go through the chunk route."""
    rng = np.random.default_rng(11)
    lens = [1, 17, 1024, 1025, 4096, 65536, (256 << 10) - 1, 256 << 10, (256 << 10) + 1, (1 << 20) + 13,
            (5 << 20) + 7, 3, (64 << 20) + 5, 0, (17 << 20) + 9, 300, 40000]
    lens += rng.integers(0, 5000, 64).tolist()
    total = sum(HDR + L + 1 for L in lens)
    base = torch.empty((total + 7) // 8 * 8, dtype=torch.uint8, device=DEV)
    rpc_amd.fill_random(base, 0xF8A3E)
    offs = np.cumsum([0] + [HDR + L + 1 for L in lens[:-1]]).astype(np.uint64)
    dl = to_dev(np.array(lens, dtype=np.uint32).view(np.int32))
    do = to_dev(offs.view(np.int64))
    sv = rpc_amd.frames_stamp(base, do, dl, lift_cap=True, stream_bytes=total)
    assert sv.cpu().numpy().tolist() == [rpc_amd.FRAME_OK] * len(lens)
    host = base.cpu().numpy()
    want_crc = [oracle.crc32(host[int(o) + HDR:int(o) + HDR + L]) for o, L in zip(offs, lens)]
    for o, L, c in zip(offs, lens, want_crc):
        assert host[int(o):int(o) + HDR].tobytes() == header(L, c)
    v, c = rpc_amd.frames_verify(base, do, lift_cap=True, stream_bytes=total)
    assert v.cpu().numpy().tolist() == [rpc_amd.FRAME_OK] * len(lens)
    assert u32(c).tolist() == want_crc
    # with the cap in force the same stream is TOO_LARGE above 1 KiB
    v, _ = rpc_amd.frames_verify(base, do, lift_cap=False, stream_bytes=total)
    assert v.cpu().numpy().tolist() == [rpc_amd.FRAME_OK if L <= 1024 else rpc_amd.FRAME_TOO_LARGE for L in lens]
    # flip one byte inside the 64 MiB body and one inside a routed 1 MiB body
    for k in (12, 9):
        pos = int(offs[k]) + HDR + lens[k] // 3
        base[pos] ^= 0x40
    v, _ = rpc_amd.frames_verify(base, do, lift_cap=True, stream_bytes=total)
    v = v.cpu().numpy().tolist()
    assert [i for i, x in enumerate(v) if x != rpc_amd.FRAME_OK] == [9, 12]
    assert v[9] == v[12] == rpc_amd.FRAME_BAD_CRC


@pytest.mark.parametrize("role", ["server", "client"])
def test_frames_lifted_cap_route_all_mixed(role):
    """A small lifted-cap batch (route-all: every body through the chunk route, no
    classify or plain rows pass) with every verdict the parse decides: heartbeats of
    both types, empty bodies, a bad CRC, bodies around the 8176-byte chunk and the
    4096-entry Tq seed table, a header whose body runs past the stream."""
    rng = np.random.default_rng(23 if role == "server" else 24)
    frames = []
    for L in [0, 1, 15, 16, 1024, 1025, 4095, 4096, 4097, 8175, 8176, 8177, 8192, 12289, 16352, 16353, 20000,
              300000, 0, 77]:
        b = rng.integers(0, 256, L, dtype=np.uint8).tobytes()
        frames.append(header(L, oracle.crc32(np.frombuffer(b, dtype=np.uint8)) if L else 0) + b)
    frames.append(header(0, 0, type_=rpc_amd.RPC_TYPE_PING))
    frames.append(header(5, 123, type_=rpc_amd.RPC_TYPE_PONG) + b"abcde")
    b = rng.integers(0, 256, 5000, dtype=np.uint8).tobytes()
    frames.append(header(5000, oracle.crc32(np.frombuffer(b, dtype=np.uint8)) ^ 1) + b)  # bad CRC
    frames.append(header(1 << 20, 7) + b"short")  # runs past the stream
    blob, offs = layout(frames, gap=3)
    got = verify(blob, offs, role=role, lift_cap=True)
    assert got == expected(blob, offs, role=role, lift_cap=True)


@pytest.mark.parametrize("n", [2048, 2049])
def test_frames_lifted_cap_route_modes(n):
    """Lifted-cap batches at the route-all bound (2048 frames: every body through the
    chunk route) and one past it (2049: classify, plain rows pass for bodies under the
    16 KiB small-batch threshold, chunk route for the rest): same verdicts and CRCs."""
    rng = np.random.default_rng(n)
    lens = rng.integers(0, 3000, n)
    lens[::97] = rng.integers(16 << 10, 300 << 10, len(lens[::97]))
    lens[5] = 0
    frames = []
    for i, L in enumerate(lens.tolist()):
        b = rng.integers(0, 256, L, dtype=np.uint8).tobytes()
        c = oracle.crc32(np.frombuffer(b, dtype=np.uint8)) if L else 0
        frames.append(header(L, c ^ (1 if i % 211 == 7 else 0)) + b)
    blob, offs = layout(frames)
    got = verify(blob, offs, lift_cap=True)
    assert got == expected(blob, offs, lift_cap=True)


def aligned_stream(nbytes: int, align: int = 4096):
    """A device byte buffer of nbytes whose first byte is `align`-aligned."""
    t = torch.empty(nbytes + align, dtype=torch.uint8, device=DEV)
    off = (-t.data_ptr()) % align
    return t[off:off + nbytes]


@pytest.mark.parametrize("sparse", [False, True])
def test_frames_lifted_cap_span_mode(sparse):
    """Route-all over a 4 KiB-aligned stream of >= 1 MiB: span mode (the bodies'
    whole interior blocks from one uniform pass over the stream, their first and
    last partial blocks from the fold) when the bodies are dense;
    with 1 MiB gaps between frames the plan falls back to the chunk route.  Bodies
    inside one block, across one boundary, ending on one, starting on one, spanning
    many; every CRC and verdict against the oracle, stamp then verify, a flipped
    byte in an interior block, the head and the tail of a long body."""
    rng = np.random.default_rng(29 + sparse)
    lens = [0, 1, 5, 4083, 4084, 4085, 4096 - HDR, 8192, 8193, 12288 - 7, 3 << 20, (2 << 20) + 4097, 77, 65536 + 3,
            1 << 20, 4096, 4095, 16 << 20, 2, 40000]
    lens += rng.integers(0, 20000, 40).tolist()
    gap = (1 << 20) + 3 if sparse else 0
    sizes = [HDR + L + gap for L in lens]
    total = sum(sizes)
    base = aligned_stream(total)
    fill = torch.empty((total + 7) // 8 * 8, dtype=torch.uint8, device=DEV)
    rpc_amd.fill_random(fill, 0x5BA2)
    base.copy_(fill[:total])
    offs = np.cumsum([0] + sizes[:-1]).astype(np.uint64)
    do = to_dev(offs.view(np.int64))
    dl = to_dev(np.array(lens, dtype=np.uint32).view(np.int32))
    sv = rpc_amd.frames_stamp(base, do, dl, lift_cap=True, stream_bytes=total)
    assert sv.cpu().numpy().tolist() == [rpc_amd.FRAME_OK] * len(lens)
    host = base.cpu().numpy()
    want = [oracle.crc32(host[int(o) + HDR:int(o) + HDR + L]) for o, L in zip(offs, lens)]
    for o, L, c in zip(offs, lens, want):
        assert host[int(o):int(o) + HDR].tobytes() == header(L, c)
    v, c = rpc_amd.frames_verify(base, do, lift_cap=True, stream_bytes=total)
    assert v.cpu().numpy().tolist() == [rpc_amd.FRAME_OK] * len(lens)
    assert u32(c).tolist() == want
    k = lens.index(16 << 20)
    body0 = int(offs[k]) + HDR
    flips = {k: [body0 + (5 << 20) + 123], 10: [int(offs[10]) + HDR + 1], 11: [int(offs[11]) + HDR + lens[11] - 1]}
    for pos in sum(flips.values(), []):
        base[pos] ^= 0x08
    v, _ = rpc_amd.frames_verify(base, do, lift_cap=True, stream_bytes=total)
    v = v.cpu().numpy().tolist()
    assert [i for i, x in enumerate(v) if x != rpc_amd.FRAME_OK] == sorted(flips)
    assert all(v[i] == rpc_amd.FRAME_BAD_CRC for i in flips)


def test_frames_lifted_cap_span_mode_round_values():
    """Span mode over a stream of >= 256 MiB: the span pass deals in DYN rounds and
    also stores each 32-block round's crc0 (BigRoute.rnd), which the fold takes for
    a body's whole rounds; the blocks before and after them come from the block
    table.  Bodies starting and ending on round boundaries (128 KiB), whole rounds
    with no blocks around them, random lengths up to 3 MiB and a 64 MiB body; stamp
    then verify, then flipped bytes inside a whole round, in the blocks before the
    first round and after the last one."""
    R = 128 << 10
    rng = np.random.default_rng(0x20D5)
    lens, pos = [], 0

    def add(L):
        nonlocal pos
        lens.append(L)
        pos += HDR + L

    def align_next_body():  # a filler frame so that the next body starts on a round boundary
        add((-(pos + 2 * HDR)) % R)

    add((64 << 20) + 3 * 4096 + 5)  # blocks 1..31 before its first whole round, 3 after its last
    for k in range(60):
        add(int(rng.integers(0, 3 << 20)))
        if k % 6 == 0:
            align_next_body()
            add([R, 3 * R, 2 * R + 4096, 5 * R - 1, R + 1][k // 6 % 5])
    align_next_body()
    add(40 * R)  # whole rounds only
    while pos < (260 << 20):
        add(int(rng.integers(1 << 20, 4 << 20)))
    total = pos
    offs = np.cumsum([0] + [HDR + L for L in lens[:-1]]).astype(np.uint64)
    base = aligned_stream(total)
    fill = torch.empty((total + 7) // 8 * 8, dtype=torch.uint8, device=DEV)
    rpc_amd.fill_random(fill, 0x20D6)
    base.copy_(fill[:total])
    del fill
    do = to_dev(offs.view(np.int64))
    dl = to_dev(np.array(lens, dtype=np.uint32).view(np.int32))
    sv = rpc_amd.frames_stamp(base, do, dl, lift_cap=True, stream_bytes=total)
    assert sv.cpu().numpy().tolist() == [rpc_amd.FRAME_OK] * len(lens)
    host = base.cpu().numpy()
    want = oracle.crc32_batch_mt(host, offs + np.uint64(HDR), np.array(lens, dtype=np.uint64))
    hdr_crc = [int.from_bytes(host[int(o) + 8:int(o) + 12].tobytes(), "big") for o in offs]
    assert hdr_crc == want.tolist()
    v, c = rpc_amd.frames_verify(base, do, lift_cap=True, stream_bytes=total)
    assert v.cpu().numpy().tolist() == [rpc_amd.FRAME_OK] * len(lens)
    assert u32(c).tolist() == want.tolist()
    # flips: a whole round in the middle of the 64 MiB body, its first interior
    # block (before its first whole round), its last interior block (after the last)
    assert (int(offs[0]) + HDR + lens[0]) // 4096 % 32 == 3
    b0 = int(offs[0]) + HDR
    e0 = b0 + lens[0]
    k_last = len(lens) - 1
    flips = {0: [b0 + (20 << 20) + 77], k_last: [int(offs[k_last]) + HDR + lens[k_last] // 2]}
    first_inner = (b0 + 4095) // 4096 * 4096 + 10
    last_inner = (e0 // 4096 - 1) * 4096 + 4000
    flips[0] += [first_inner, last_inner]
    for p in sum(flips.values(), []):
        base[p] ^= 0x10
    v, _ = rpc_amd.frames_verify(base, do, lift_cap=True, stream_bytes=total)
    v = v.cpu().numpy().tolist()
    assert [i for i, x in enumerate(v) if x != rpc_amd.FRAME_OK] == sorted(flips)
    # each flip alone: one bad frame each time
    for p in sum(flips.values(), []):
        base[p] ^= 0x10
    for p, i in [(first_inner, 0), (last_inner, 0)]:
        base[p] ^= 0x01
        v, _ = rpc_amd.frames_verify(base, do, lift_cap=True, stream_bytes=total)
        assert [j for j, x in enumerate(v.cpu().numpy().tolist()) if x != rpc_amd.FRAME_OK] == [i]
        base[p] ^= 0x01


@pytest.mark.parametrize("role", ["server", "client"])
def test_frames_lifted_cap_span_mode_verdicts(role):
    """Span mode (4 KiB-aligned dense stream of >= 1 MiB) with every verdict the
    parse decides: heartbeats of both types, empty bodies, a bad CRC, a header
    whose length runs past the stream, and the last body ending exactly at a
    stream end that is not a multiple of 4 KiB (its last block is partial, so no
    span-pass block covers it)."""
    rng = np.random.default_rng(41 if role == "server" else 42)
    frames = []
    for L in [300000, 0, 4096 - HDR, 1 << 20, 17, 8192, 0, 65536 + 5]:
        b = rng.integers(0, 256, L, dtype=np.uint8).tobytes()
        frames.append(header(L, oracle.crc32(np.frombuffer(b, dtype=np.uint8)) if L else 0) + b)
    frames.append(header(0, 0, type_=rpc_amd.RPC_TYPE_PING))
    frames.append(header(5, 123, type_=rpc_amd.RPC_TYPE_PONG) + b"abcde")
    b = rng.integers(0, 256, 70000, dtype=np.uint8).tobytes()
    frames.append(header(70000, oracle.crc32(np.frombuffer(b, dtype=np.uint8)) ^ 1) + b)  # bad CRC
    frames.append(header(1 << 22, 7) + b"short")  # runs past the stream
    b = rng.integers(0, 256, 123457, dtype=np.uint8).tobytes()
    frames.append(header(123457, oracle.crc32(np.frombuffer(b, dtype=np.uint8))) + b)  # ends the stream
    blob, offs = layout(frames)  # (the 4 MiB length of the short frame runs past this ~1.7 MiB stream)
    assert len(blob) % 4096 != 0 and len(blob) >= (1 << 20)
    base = aligned_stream(len(blob))
    base.copy_(torch.from_numpy(np.frombuffer(blob, dtype=np.uint8).copy()).to(DEV))
    v, c = rpc_amd.frames_verify(base, to_dev(offs.view(np.int64)), role=role, lift_cap=True, stream_bytes=len(blob))
    want = expected(blob, offs, role=role, lift_cap=True)
    assert (v.cpu().numpy().tolist(), u32(c).tolist()) == want


def test_frames_lifted_cap_stamp_unordered_frames():
    """Lifted-cap stamp over a 4 KiB-aligned dense stream whose frame offsets are
    given in reverse order: the route's span mode is
    for frames in stream order only (its fold reads partial blocks while it
    writes headers), so these take the chunk route -- every header still equals
    the oracle's, computed over the bytes before any header is written."""
    rng = np.random.default_rng(31)
    lens = [5000, 70000, 1 << 20, 3, 4096 - HDR, 200000, 12345, 0, 90000]
    sizes = [HDR + L for L in lens]
    total = sum(sizes)
    base = aligned_stream(total)
    fill = torch.empty((total + 7) // 8 * 8, dtype=torch.uint8, device=DEV)
    rpc_amd.fill_random(fill, 0x77AA)
    base.copy_(fill[:total])
    offs = np.cumsum([0] + sizes[:-1]).astype(np.uint64)
    before = base.cpu().numpy().copy()
    order = np.arange(len(lens))[::-1].copy()
    do = to_dev(offs[order].view(np.int64))
    dl = to_dev(np.array([lens[i] for i in order], dtype=np.uint32).view(np.int32))
    sv = rpc_amd.frames_stamp(base, do, dl, lift_cap=True, stream_bytes=total)
    assert sv.cpu().numpy().tolist() == [rpc_amd.FRAME_OK] * len(lens)
    host = base.cpu().numpy()
    for i, (o, L) in enumerate(zip(offs, lens)):
        o = int(o)
        want = oracle.crc32(before[o + HDR:o + HDR + L])
        assert host[o:o + HDR].tobytes() == header(L, want), i
        assert host[o + HDR:o + HDR + L].tobytes() == before[o + HDR:o + HDR + L].tobytes()


def test_frames_role_flags_rejected():
    d = to_dev(np.zeros(64, dtype=np.uint8))
    o = to_dev(np.zeros(1, dtype=np.int64))
    v = torch.empty(1, dtype=torch.uint8, device=DEV)
    for flags in (0, 3, 8, 1 | 8):
        rc = rpc_amd._lib.rpc_frames_verify_device(d.data_ptr(), 64, o.data_ptr(), 1, flags, v.data_ptr(), None,
                                                   rpc_amd._stream_handle(None))
        assert rc == -22, flags


def test_frames_lifted_cap_end_aligned_route():
    """with RPCCRC_BIG_ALIGNED=0 the route cuts end-aligned chunks
    and its fold (big_combine_kernel) writes CRCs only, so a route-all verify must
    still launch the compare that writes the verdicts.  The lifted-cap verify /
    stamp tests run again in a child process under that setting."""
    import os
    import subprocess
    import sys
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, RPCCRC_BIG_ALIGNED="0")
    p = subprocess.run([sys.executable, "-m", "pytest", "-q", "-m", "gpu", "-p", "no:cacheprovider",
                        os.path.join(repo, "tests", "test_frames.py"), "-k",
                        "lifted_cap_large_bodies or lifted_cap_route_all_mixed or lifted_cap_route_modes"],
                       capture_output=True, text=True, timeout=600, env=env, cwd=repo)
    assert p.returncode == 0, p.stdout[-3000:] + p.stderr[-2000:]
    assert " passed" in p.stdout and "failed" not in p.stdout, p.stdout[-2000:]
