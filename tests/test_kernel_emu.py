"""CPU emulation of the rows and packed kernels' arithmetic (tests/cpu_emu/rows_emu.cpp)
against the oracle: validates the LDS table image, v_perm_b32 address selectors,
permlane transpose, per-lane GF(2) shifts, row Horner, Tq pre-conditioning and the
ZI trailing-pad undo for every body alignment -- without a GPU.  (The GPU parity tests then
check the real kernel.)"""
import os
import subprocess

import numpy as np
import pytest

from oracle import oracle

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

LENS = [0, 1, 2, 3, 4, 5, 15, 16, 17, 31, 63, 64, 65, 127, 1000, 1023, 1024, 1025, 1040, 4080, 4095, 4096,
        4097, 4100, 4111, 8191, 8192, 12345, 65536]


# ---- rows kernel (crc32_rows.h): coalesced pieces + permlane transpose --------------

@pytest.fixture(scope="module")
def rows_emu(tmp_path_factory):
    exe = str(tmp_path_factory.mktemp("emu2") / "rows_emu")
    subprocess.run(["g++", "-O2", "-std=c++17", "-o", exe, os.path.join(REPO, "tests/cpu_emu/rows_emu.cpp"),
                    os.path.join(REPO, "rpc_amd/csrc/crc32_tables.cpp")], check=True)
    return exe


@pytest.mark.parametrize("QB", [1, 5, 6, 4])
@pytest.mark.parametrize("mis", [0, 1, 3, 4, 8, 15])
def test_emulated_rows_kernel_matches_oracle(rows_emu, QB, mis):
    """QB 1: QB = 1 with quarter / half first rows of <= 1 / 2 KiB; QB 6: the same with
    the ragged kernel's per-lane Horner (one merge per body); QB 5: QB = 1 with full
    rows only (uniform batches); QB 4: four bodies per row."""
    rng = np.random.default_rng(QB * 100 + mis)
    if QB in (1, 5, 6):
        lens = (LENS + [1008, 1009, 1010, 1020, 2032, 2033, 2047, 2048, 2049, 2064, 4096 + 1008, 4096 + 2040,
                        8192 + 1500] + rng.integers(0, 20000, 6).tolist() + rng.integers(0, 2100, 12).tolist())
    else:  # QB=4 precondition: len + pad-to-16 <= 1024
        lens = [0, 1, 2, 3, 4, 5, 15, 16, 17, 63, 64, 65, 100, 1000, 1008, 1009] + rng.integers(0, 1010, 12).tolist()
    inp = f"{QB} {mis} {len(lens)}\n" + "\n".join(map(str, lens)) + "\n"
    out = subprocess.run([rows_emu], input=inp.encode(), capture_output=True, check=True).stdout.decode().split()
    assert len(out) == len(lens)
    data = oracle.splitmix_bytes(sum(lens) + mis, 7)
    off = mis
    for L, o in zip(lens, out):
        assert int(o, 16) == oracle.crc32(data[off:off + L]), (QB, mis, L)
        off += L


# ---- packed ragged kernel (crc32_packed.h): chunk stream, slices, runs --------------

@pytest.mark.parametrize("mis", [0, 1, 7, 15])
@pytest.mark.parametrize("nwaves,min_slice,max_slices", [(1, 8, 1 << 20), (3, 1, 1 << 20), (5, 2, 1 << 20),
                                                         (4, 1, 7), (64, 1, 1 << 20)])
def test_emulated_packed_kernel_matches_oracle(rows_emu, mis, nwaves, min_slice, max_slices):
    """Every body written once with the oracle's CRC: empty bodies, bodies of 1..4 chunks
    in every row position, bodies spanning many rows and slices, slices that start
    inside a long body, waves with no work."""
    rng = np.random.default_rng(mis * 131 + nwaves * 7 + min_slice)
    lens = (LENS + [0, 0, 1, 0, 1024, 1023, 1025, 2048, 3072, 4096, 5000] + rng.integers(0, 200, 40).tolist()
            + rng.integers(0, 9000, 12).tolist() + [0, 70000, 2, 0, 17]
            + [0] * 150 + [5] + [0] * 64 + [3000] + [0] * 63 + rng.integers(1, 40, 200).tolist() + [0] * 70)
    inp = f"2 {mis} {len(lens)} {nwaves} {min_slice} {max_slices}\n" + "\n".join(map(str, lens)) + "\n"
    out = subprocess.run([rows_emu], input=inp.encode(), capture_output=True, check=True).stdout.decode().split()
    assert len(out) == len(lens)
    data = oracle.splitmix_bytes(sum(lens) + mis, 7)
    off = mis
    for i, (L, o) in enumerate(zip(lens, out)):
        assert int(o, 16) == oracle.crc32(data[off:off + L]), (i, mis, L)
        off += L


def test_edge_fix_matches_byte_mask(tmp_path):
    """The kernels' edge fix (crc32_edge.h masks on the two edge pieces of a
    window) equals a per-byte mask of the whole window, for every front offset
    and pad z (tests/cpu_emu/edge_emu.cpp)."""
    exe = str(tmp_path / "edge_emu")
    subprocess.run(["g++", "-O2", "-std=c++17", "-o", exe, os.path.join(REPO, "tests/cpu_emu/edge_emu.cpp")],
                   check=True)
    r = subprocess.run([exe], capture_output=True, text=True)
    assert r.returncode == 0, r.stdout + r.stderr
    assert r.stdout.startswith("ok ")


def _mix(z):
    M = (1 << 64) - 1
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & M
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & M
    return z ^ (z >> 31)


def test_service_lane_algebra_matches_zlib(tmp_path):
    """The drop-in service kernel's arithmetic (rpc_amd/csrc/crc32_service_math.h,
    compiled for the host with the gfx950 bitop3 / sbfe immediates emulated bit for
    bit) equals zlib crc32 for every length 1..1024 -- all three size classes, stale
    staging bytes before the body masked (tests/cpu_emu/service_emu.cpp)."""
    import zlib
    exe = str(tmp_path / "service_emu")
    subprocess.run(["g++", "-O2", "-std=c++17", "-o", exe, os.path.join(REPO, "tests/cpu_emu/service_emu.cpp")],
                   check=True)
    lens = list(range(1, 1025))
    out = subprocess.run([exe], input=(f"{len(lens)}\n" + "\n".join(map(str, lens))).encode(), capture_output=True,
                         check=True).stdout.decode().split()
    for k, (ln, got) in enumerate(zip(lens, out)):
        body = bytes(_mix(0x5E17C0DE + k * 4096 + i) & 0xFF for i in range(ln))
        assert int(got, 16) == zlib.crc32(body), ln


def test_service_request_check_rejects_torn_reads(tmp_path):
    """the drop-in service's request check (round 6:
    crc32_service_math.h word_hash sums over the block and, for bodies over 116 B,
    the body's masked words) rejects every mixed stale/current read of consecutive
    JSON-RPC requests on one slot -- pairs of one length whose id and first parameter
    step together (equal XOR deltas in two dwords), inline and body-area pairs
    alternating; every subset of the changed words up to 2^14 reads per request,
    seeded draws beyond.  The same enumeration under round 5's rule (a plain XOR of
    the block, no check over 116 B) finds false accepts of both kinds, so the model
    sees the bug class it is meant to exclude (tests/cpu_emu/svc_check_emu.cpp)."""
    exe = str(tmp_path / "svc_check_emu")
    subprocess.run(["g++", "-O2", "-std=c++17", "-o", exe, os.path.join(REPO, "tests/cpu_emu/svc_check_emu.cpp")],
                   check=True)
    r = subprocess.run([exe, "400"], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    got = dict((k, int(v)) for k, v in (ln.split() for ln in r.stdout.splitlines()))
    assert got["crosschecked"] > 10000
    assert got["r6_reads"] > 1_000_000
    assert got["r6_false_accepts"] == 0
    assert got["r5_inline_false_accepts"] > 0
    assert got["r5_false_accepts"] > got["r5_inline_false_accepts"]
