"""Drop-in proof (test plan item 4): the reference's own `server`
(built by `make -C oracle dropin` from /root/reference/server sources, with
crc.c REPLACED by librpccrc.so, nothing else changed) answers framed JSON-RPC
requests over loopback.  Its verify (rpc_server_main.c:227) and stamp
(rpc_server_main.c:249) calls now run on the GPU through rpc_crc32 /
rpc_crc32_verify.  Frames and CRCs are checked against the captured golden
frames and the oracle."""
import os
import socket
import struct
import subprocess
import time

import pytest

from oracle import oracle

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SERVER = os.path.join(REPO, "oracle", "_ref", "server_rpccrc")
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
