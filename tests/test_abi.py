"""C-ABI checks that need no GPU: librpccrc.so loads, exports exactly what
include/rpccrc.h declares (and never zlib's `crc32`), and compute entry points
refuse to run without a HIP device instead of falling back to a CPU path."""
import os
import re
import subprocess
import sys

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(REPO, "rpc_amd", "lib", "librpccrc.so")
HDR = os.path.join(REPO, "include", "rpccrc.h")


def header_symbols():
    txt = open(HDR).read()
    return sorted(set(re.findall(r"RPCCRC_API\s+[\w\s\*]+?\b(\w+)\(", txt)))


def dynamic_symbols():
    out = subprocess.run(["nm", "-D", "--defined-only", LIB], capture_output=True, text=True, check=True).stdout
    return sorted(line.split()[-1] for line in out.splitlines() if line.strip())


def have_gpu():
    try:
        import torch
        return torch.cuda.device_count() > 0
    except Exception:
        return False


def test_library_built():
    assert os.path.exists(LIB), "run __graft_entry__.build()"


def test_exports_match_header():
    hs = header_symbols()
    assert "rpc_crc32" in hs and "rpc_crc32_verify" in hs
    assert dynamic_symbols() == hs


def test_no_zlib_interposition():
    assert "crc32" not in dynamic_symbols()


def test_python_binding_lists_every_export():
    from rpc_amd import _lib
    assert sorted(_lib.EXPORTS) == header_symbols()
    for name in _lib.EXPORTS:
        assert hasattr(_lib.lib, name)


def test_drop_in_signatures_match_reference_header():
    """reference crc.h:8,11 signatures, verbatim."""
    txt = open(HDR).read()
    assert "uint32_t rpc_crc32(const void *data, size_t len);" in txt
    assert "bool rpc_crc32_verify(const void *data, size_t len, uint32_t expected_crc);" in txt


def test_combine_helper_matches_oracle(golden):
    """rpc_crc32_combine is host GF(2) arithmetic (zlib crc32_combine), no device needed."""
    import rpc_amd
    for c in golden["combine"]:
        assert rpc_amd.crc32_combine(c["a_crc"], c["b_crc"], c["len_b"]) == c["crc_ab"]


def test_strerror():
    import rpc_amd
    from rpc_amd import _lib
    assert _lib.rpc_crc32_strerror(-19).decode().startswith("no usable HIP device")
    assert _lib.rpc_crc32_strerror(0).decode() == "ok"


@pytest.mark.skipif(have_gpu(), reason="checks the no-device behaviour")
def test_batch_fails_loudly_without_device():
    import rpc_amd
    buf = np.zeros(64, dtype=np.uint8)
    with pytest.raises(rpc_amd.RpcCrcError) as ei:
        rpc_amd.crc32_batch(buf, [0], [64])
    assert ei.value.code == -19


@pytest.mark.skipif(have_gpu(), reason="checks the no-device behaviour")
def test_drop_in_aborts_without_device():
    code = ("import ctypes; l = ctypes.CDLL(%r); l.rpc_crc32.restype = ctypes.c_uint32; "
            "l.rpc_crc32.argtypes = [ctypes.c_char_p, ctypes.c_size_t]; print(l.rpc_crc32(b'abc', 3))") % LIB
    p = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=120)
    assert p.returncode != 0  # SIGABRT, never a CPU-computed value
    assert "no CPU fallback" in p.stderr


def test_null_and_empty_need_no_device():
    """crc.c:6-7: Z_NULL -> 0 and len 0 -> 0 are decided before any compute."""
    from rpc_amd import _lib
    assert _lib.rpc_crc32(None, 5) == 0
    assert _lib.rpc_crc32(b"abc", 0) == 0
    assert _lib.rpc_crc32(b"abc", 2**32) == 0  # len mod 2^32 == 0


def test_service_stop_without_a_service():
    """rpc_crc32_service_stop with no drop-in service started (no device needed):
    nothing to stop, RPCCRC_OK."""
    import rpc_amd
    assert rpc_amd.service_stop() == 0


def test_test_library_exports_the_same_abi():
    """librpccrc_test.so (fault-injection build for the error-word tests) exports the
    same symbols; only it knows the test switch (the product library must
    not read RPCCRC_TEST_STEAL_GIVEUP)."""
    test_lib = os.path.join(REPO, "rpc_amd", "lib", "librpccrc_test.so")
    assert os.path.exists(test_lib), "run __graft_entry__.build()"
    out = subprocess.run(["nm", "-D", "--defined-only", test_lib], capture_output=True, text=True, check=True).stdout
    assert sorted(line.split()[-1] for line in out.splitlines() if line.strip()) == header_symbols()
    assert b"RPCCRC_TEST_STEAL_GIVEUP" in open(test_lib, "rb").read()
    assert b"RPCCRC_TEST_STEAL_GIVEUP" not in open(LIB, "rb").read()
    assert b"RPCCRC_TEST_DENSE_ONLY" in open(test_lib, "rb").read()
    assert b"RPCCRC_TEST_DENSE_ONLY" not in open(LIB, "rb").read()


def test_service_stats_without_a_service():
    """rpc_crc32_service_stats before any drop-in call (no device needed): every
    counter zero."""
    import rpc_amd
    st = rpc_amd.service_stats()
    assert st == {k: 0 for k in ("services", "running", "launched", "answered", "fallbacks_full",
                                 "fallbacks_short", "bypassed")}, st
