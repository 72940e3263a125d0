"""CPU emulation of crc32_items_kernel's arithmetic (tests/cpu_emu/kernel_emu.cpp)
against the oracle: validates the LDS table image, v_perm_b32 address selectors,
per-lane GF(2) shifts, row Horner, Tq pre-conditioning and the ZI trailing-pad
undo for every body alignment -- without a GPU.  (The GPU parity tests then
check the real kernel.)"""
import os
import subprocess

import numpy as np
import pytest

from oracle import oracle

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def emu(tmp_path_factory):
    exe = str(tmp_path_factory.mktemp("emu") / "kernel_emu")
    subprocess.run(["g++", "-O2", "-std=c++17", "-o", exe, os.path.join(REPO, "tests/cpu_emu/kernel_emu.cpp"),
                    os.path.join(REPO, "rpc_amd/csrc/crc32_tables.cpp")], check=True)
    return exe


LENS = [0, 1, 2, 3, 4, 5, 15, 16, 17, 31, 63, 64, 65, 127, 1000, 1023, 1024, 1025, 1040, 4080, 4095, 4096,
        4097, 4100, 4111, 8191, 8192, 12345, 65536]


@pytest.mark.parametrize("G", [16, 64])
@pytest.mark.parametrize("mis", [0, 1, 2, 3, 4, 5, 8, 12, 15])
def test_emulated_kernel_matches_oracle(emu, G, mis):
    rng = np.random.default_rng(G * 100 + mis)
    lens = LENS + rng.integers(0, 20000, 8).tolist()
    inp = f"{G} {mis} {len(lens)}\n" + "\n".join(map(str, lens)) + "\n"
    out = subprocess.run([emu], input=inp.encode(), capture_output=True, check=True).stdout.decode().split()
    data = oracle.splitmix_bytes(sum(lens) + mis, 7)
    off = mis
    for L, o in zip(lens, out):
        assert int(o, 16) == oracle.crc32(data[off:off + L]), (G, mis, L)
        off += L


# ---- v2 rows kernel (crc32_rows.h): coalesced pieces + DPP transpose -------------

@pytest.fixture(scope="module")
def rows_emu(tmp_path_factory):
    exe = str(tmp_path_factory.mktemp("emu2") / "rows_emu")
    subprocess.run(["g++", "-O2", "-std=c++17", "-o", exe, os.path.join(REPO, "tests/cpu_emu/rows_emu.cpp"),
                    os.path.join(REPO, "rpc_amd/csrc/crc32_tables.cpp")], check=True)
    return exe


@pytest.mark.parametrize("QB", [1, 4])
@pytest.mark.parametrize("mis", [0, 1, 3, 4, 8, 15])
def test_emulated_rows_kernel_matches_oracle(rows_emu, QB, mis):
    rng = np.random.default_rng(QB * 100 + mis)
    if QB == 1:
        lens = LENS + rng.integers(0, 20000, 6).tolist()
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
