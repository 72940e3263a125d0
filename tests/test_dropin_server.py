"""Drop-in proof (test plan item 4), both halves of the reference.

* Server: the reference's own `server` (built by `make -C oracle dropin` from
  /root/reference/server sources, with crc.c REPLACED by librpccrc.so, nothing
  else changed) answers framed JSON-RPC requests over loopback.  Its verify
  (rpc_server_main.c:227) and stamp (rpc_server_main.c:249) run on the GPU.
* Client: the reference's client library (rpc_async.c, conn_pool.c, pending.c,
  epoll_api.c, rpc_codec.c, gen/rpc_client_gen.c) linked the same way, driven by
  tests/dropin/client_driver.c with 10 user threads (rpc_client_main.c:17):
  stamp at rpc_async.c:525 and receive-thread verify at rpc_async.c:219 on the
  GPU; a corrupted response surfaces RPC_CRC_ERR (rpc_types.h:27).

Frames and CRCs are checked against the captured golden frames and the oracle,
and the batched frames verdicts (rpc_frames_verify_device) against what the
reference server does with the same frames."""
import json
import os
import socket
import struct
import subprocess
import threading
import time

import numpy as np

import pytest

from oracle import oracle

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SERVER = os.path.join(REPO, "oracle", "_ref", "server_rpccrc")
CLIENT = os.path.join(REPO, "oracle", "_ref", "client_rpccrc")
PORT = 8888  # hard-coded in the reference (rpc_server_main.c:65)


def frame(body: bytes, type_=0, crc=None):
    c = oracle.crc32(body) if crc is None else crc
    return struct.pack(">HHII", 1, type_, len(body), c) + body


def recv_exact(s, n):
    buf = b""
    while len(buf) < n:
        chunk = s.recv(n - len(buf))
        if not chunk:
            return buf
        buf += chunk
    return buf


@pytest.fixture(scope="module")
def server(tmp_path_factory):
    if not os.path.exists(SERVER):
        pytest.fail("oracle/_ref/server_rpccrc missing: build it with `make -C oracle dropin` (needs /root/reference)")
    log = open(tmp_path_factory.mktemp("srv") / "server.log", "wb")
    p = subprocess.Popen([SERVER], stdout=log, stderr=subprocess.STDOUT)
    deadline = time.time() + 60
    while time.time() < deadline:
        try:
            socket.create_connection(("127.0.0.1", PORT), timeout=1).close()
            break
        except OSError:
            if p.poll() is not None:
                pytest.fail(f"server exited with {p.returncode}")
            time.sleep(0.2)
    yield p
    p.terminate()
    try:
        p.wait(timeout=10)
    except subprocess.TimeoutExpired:
        p.kill()


def call(body: bytes, crc=None):
    s = socket.create_connection(("127.0.0.1", PORT), timeout=30)
    s.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
    s.sendall(frame(body, crc=crc))
    hdr = recv_exact(s, 12)
    if len(hdr) < 12:
        s.close()
        return None, None
    ver, typ, blen, crc_ = struct.unpack(">HHII", hdr)
    resp = recv_exact(s, blen)
    s.close()
    return (ver, typ, blen, crc_), resp


def test_captured_request_gets_captured_response(server, golden):
    req = golden["frames"][0]
    body = req["body"].encode()
    assert frame(body).hex() [:24] == req["header_hex"]
    hdr, resp = call(body)
    assert resp == golden["frames"][1]["body"].encode()
    assert struct.pack(">HHII", *hdr).hex() == golden["frames"][1]["header_hex"]


def test_many_methods_crc_stamped_by_gpu(server):
    for a, b in [(1, 2), (-5, 7), (123456, 654321)]:
        body = ('{"jsonrpc":"2.0","method":"add_i32","params":{"a":%d,"b":%d},"id":%d}' % (a, b, a & 0xFFFF)).encode()
        hdr, resp = call(body)
        assert hdr is not None and hdr[3] == oracle.crc32(resp), resp
        assert b'"result":%d' % (a + b) in resp


def test_bad_crc_closes_connection(server):
    body = b'{"jsonrpc":"2.0","method":"add_i32","params":{"a":1,"b":2},"id":9}'
    hdr, resp = call(body, crc=oracle.crc32(body) ^ 0x1)
    assert hdr is None  # rpc_server_main.c:227-233: verify fails -> close, no reply


def test_ping_pong(server):
    s = socket.create_connection(("127.0.0.1", PORT), timeout=30)
    s.sendall(struct.pack(">HHII", 1, 1, 0, 0))
    assert recv_exact(s, 12) == struct.pack(">HHII", 1, 2, 0, 0)
    s.close()


def test_ping_with_crc_and_body_len_gets_pong(server):
    """rpc_server_main.c:172-187 answers PING from the header alone: its crc32 and
    body_len fields are never looked at (the batched verdict is FRAME_CONTROL)."""
    s = socket.create_connection(("127.0.0.1", PORT), timeout=30)
    s.sendall(struct.pack(">HHII", 3, 1, 777, 0xDEADBEEF))
    assert recv_exact(s, 12) == struct.pack(">HHII", 3, 2, 0, 0)
    s.close()


def _server_outcome(raw: bytes) -> str:
    """What the reference server does with one frame on a fresh connection."""
    s = socket.create_connection(("127.0.0.1", PORT), timeout=30)
    s.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
    try:
        s.sendall(raw)
        hdr = recv_exact(s, 12)
    except ConnectionResetError:  # closed with our bytes unread: an RST instead of a FIN
        hdr = b""
    s.close()
    if len(hdr) < 12:
        return "closed"
    return "pong" if struct.unpack(">HHII", hdr)[1] == 2 else "reply"


def test_batched_verdicts_match_reference_server(server):
    """The same frames through the reference server (one connection each) and through
    rpc_frames_verify_device(role=server): PONG <-> FRAME_CONTROL, a reply <->
    FRAME_OK, a closed connection <-> FRAME_BAD_CRC / FRAME_TOO_LARGE."""
    torch = pytest.importorskip("torch")
    import rpc_amd
    good = b'{"jsonrpc":"2.0","method":"add_i32","params":{"a":1,"b":2},"id":3}'
    frames = [
        frame(good),
        frame(good, crc=oracle.crc32(good) ^ 0x80000000),
        struct.pack(">HHII", 1, 1, 0, 0),
        struct.pack(">HHII", 1, 1, 64, 0x1234),            # PING with junk fields
        struct.pack(">HHII", 1, 0, 1025, 0) + bytes(1025),  # over MAX_BODY_LEN
        struct.pack(">HHII", 1, 0, 5000, 7),
        frame(good, type_=9),                               # unknown type: data
    ]
    outcome = [_server_outcome(f) for f in frames]
    offs, blob = [], b""
    for f in frames:
        offs.append(len(blob))
        blob += f
    v, _ = rpc_amd.frames_verify(torch.from_numpy(np.frombuffer(blob, np.uint8).copy()).cuda(),
                                 torch.tensor(offs, dtype=torch.int64).cuda(), role="server")
    mapped = {rpc_amd.FRAME_CONTROL: "pong", rpc_amd.FRAME_OK: "reply", rpc_amd.FRAME_BAD_CRC: "closed",
              rpc_amd.FRAME_TOO_LARGE: "closed"}
    assert [mapped[x] for x in v.cpu().tolist()] == outcome
    assert outcome == ["reply", "closed", "pong", "pong", "closed", "closed", "reply"]


def _client(*args, timeout=120):
    if not os.path.exists(CLIENT):
        pytest.fail("oracle/_ref/client_rpccrc missing: build it with `make -C oracle dropin` (needs /root/reference)")
    p = subprocess.run([CLIENT, *map(str, args)], capture_output=True, text=True, timeout=timeout)
    return p.returncode, json.loads(p.stdout.strip().splitlines()[-1]), p.stderr


def test_reference_client_10_threads(server):
    """rpc_client_main.c's shape of work (10 user threads, THREAD_COUNT at :17) through
    the reference client library on librpccrc: every request stamped on the GPU
    (rpc_async.c:525), every response verified on the GPU (rpc_async.c:219), every
    result correct."""
    rc, res, err = _client("stress", PORT, 10, 5)
    assert rc == 0 and res == {"success": 50, "failure": 0}, err[-2000:]


def _bad_crc_reply(req):
    body = json.dumps({"jsonrpc": "2.0", "id": req["id"], "result": 3}, separators=(",", ":")).encode()
    return struct.pack(">HHII", 1, 0, len(body), oracle.crc32(body) ^ 0x00010000) + body


def _bad_crc_server(port_holder, stop, reply=_bad_crc_reply):
    """A server that answers every DATA request with reply(request) -- by default a
    response whose crc32 field is wrong -- and PING with PONG, as the reference
    server would."""
    ls = socket.socket()
    ls.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)
    ls.bind(("127.0.0.1", 0))
    ls.listen(64)
    ls.settimeout(0.5)
    port_holder.append(ls.getsockname()[1])

    def serve(c):
        try:
            while not stop.is_set():
                hdr = recv_exact(c, 12)
                if len(hdr) < 12:
                    return
                ver, typ, blen, _ = struct.unpack(">HHII", hdr)
                if typ == 1:
                    c.sendall(struct.pack(">HHII", ver, 2, 0, 0))
                    continue
                req = json.loads(recv_exact(c, blen))
                r = reply(req)
                if isinstance(r, tuple):  # (bytes, close the connection after them)
                    c.sendall(r[0])
                    if r[1]:
                        return
                else:
                    c.sendall(r)
        except OSError:
            return
        finally:
            c.close()

    while not stop.is_set():
        try:
            c, _ = ls.accept()
        except socket.timeout:
            continue
        threading.Thread(target=serve, args=(c,), daemon=True).start()
    ls.close()


def test_reference_client_flags_corrupted_response():
    """rpc_async.c:219-222: a response whose body fails rpc_crc32_verify (on the GPU)
    completes the call with RPC_CRC_ERR (= 5, rpc_types.h:27)."""
    port, stop = [], threading.Event()
    t = threading.Thread(target=_bad_crc_server, args=(port, stop), daemon=True)
    t.start()
    while not port:
        time.sleep(0.05)
    try:
        rc, res, err = _client("raw", port[0], '{"jsonrpc":"2.0","method":"add_i32","params":{"a":1,"b":2},"id":1}')
    finally:
        stop.set()
        t.join(timeout=5)
    assert res == {"status": 5}, err[-2000:]


def _run_client_against(reply):
    """One `client_rpccrc raw` call against a server answering with reply(request);
    returns the reference client's rpc_error_code."""
    port, stop = [], threading.Event()
    t = threading.Thread(target=_bad_crc_server, args=(port, stop, reply), daemon=True)
    t.start()
    while not port:
        time.sleep(0.05)
    try:
        rc, res, err = _client("raw", port[0], '{"jsonrpc":"2.0","method":"add_i32","params":{"a":1,"b":2},"id":1}',
                               timeout=60)
    finally:
        stop.set()
        t.join(timeout=5)
    return res["status"], err


def test_client_verdicts_match_reference_client():
    """the client-role verdicts pinned against the reference CLIENT itself,
    as test_batched_verdicts_match_reference_server pins the server role.  A scripted
    server answers the request with each response below; the reference client library
    (on librpccrc) completes the call with RPC_OK (0), RPC_RECV_ERR (4) or RPC_CRC_ERR
    (5) (rpc_types.h:22-27), and rpc_frames_verify_device(role=client) must give the
    matching verdict for the same bytes (the first non-heartbeat frame decides):
      * body_len 0, any non-PONG type: the BODY state calls recv(fd, buf, 0), which on
        a non-blocking TCP socket returns 0 once any further byte (or a FIN) is
        pending -- read as a closed peer (rpc_async.c:330-349) -> RPC_RECV_ERR; the
        empty body is never verified <-> FRAME_RECV_ERR.  (With the socket idle it
        returns EAGAIN and the client waits; the call then times out -- nothing is
        verified either way, so the cases below always send something after it.)
      * body_len over MAX_BODY_LEN -> dropped before the body (rpc_async.c:312) -> 4;
      * a PING carrying a valid body is an ordinary data frame at the client -> OK;
      * a PONG (junk crc / body_len fields, no body) is consumed from the header alone
        (rpc_async.c:303-309), then the real response decides."""
    torch = pytest.importorskip("torch")
    import rpc_amd

    def good_body(req):
        return json.dumps({"jsonrpc": "2.0", "id": req["id"], "result": 3}, separators=(",", ":")).encode()

    def good(r):
        return hdr(0, len(good_body(r)), oracle.crc32(good_body(r))) + good_body(r)

    hdr = lambda t, bl, c: struct.pack(">HHII", 1, t, bl, c)  # noqa: E731
    cases = [  # (name, reply(req) -> list of frames, close after them, expected status)
        ("empty data, then a response", lambda r: [hdr(0, 0, 0), good(r)], False, 4),
        ("empty data, crc field set, then a response", lambda r: [hdr(0, 0, 0x1234ABCD), good(r)], False, 4),
        ("empty data, then close", lambda r: [hdr(0, 0, 0)], True, 4),
        ("empty ping, then a response", lambda r: [hdr(1, 0, 0), good(r)], False, 4),
        ("empty unknown type, then a response", lambda r: [hdr(7, 0, 0), good(r)], False, 4),
        ("over cap", lambda r: [hdr(0, 2000, 0)], False, 4),
        ("ping with valid body", lambda r: [hdr(1, len(good_body(r)), oracle.crc32(good_body(r))) + good_body(r)],
         False, 0),
        ("bad crc", lambda r: [hdr(0, len(good_body(r)), oracle.crc32(good_body(r)) ^ 4) + good_body(r)], False, 5),
        ("pong then response", lambda r: [hdr(2, 777, 0xDEADBEEF), good(r)], False, 0),
        ("good", lambda r: [good(r)], False, 0),
    ]
    status_of = {rpc_amd.FRAME_OK: 0, rpc_amd.FRAME_RECV_ERR: 4, rpc_amd.FRAME_TOO_LARGE: 4, rpc_amd.FRAME_BAD_CRC: 5}
    req = {"id": 1}
    for name, reply, close, want in cases:
        status, err = _run_client_against(lambda r, reply=reply, close=close: (b"".join(reply(r)), close))
        assert status == want, (name, status, err[-1500:])
        frames = reply(req)
        offs, blob = [], b""
        for f in frames:
            offs.append(len(blob))
            blob += f
        v, _ = rpc_amd.frames_verify(torch.from_numpy(np.frombuffer(blob, np.uint8).copy()).cuda(),
                                     torch.tensor(offs, dtype=torch.int64).cuda(), role="client")
        v = v.cpu().tolist()
        decisive = next(x for x in v if x != rpc_amd.FRAME_CONTROL)  # heartbeats are consumed first
        assert status_of[decisive] == status, (name, v, status)
        assert v == [oracle.frame_verdict(blob, o, "client")[0] for o in offs], name
