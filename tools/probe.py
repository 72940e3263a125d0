#!/usr/bin/env python3
"""tools/probe.py -- one-process A/B timing of kernel variants on one GPU
(interleaved rounds, median; cdna_hip_programming.md 5.4 rule 24).

  python tools/probe.py [--config ns] [--rounds 5] [--reps 10] [--mode lib|ablate]
mode lib:    stream-read patterns and the product kernel under its runtime options.
mode sustain: each --only variant (ablate names, "product", "stream_nt1")
             launched --launches times back to back with per-launch events,
             while a child process samples power/clocks (DVFS under load).
mode ablate: tools/libprobe.so variants (ABL bits: 1 no-compute, 2 no-combine,
             4 no-load; DEPTH rows in flight; NT loads).  Ablated outputs are
             wrong by construction -- timing only; abl=0 outputs are checked
             against the product kernel.
"""
import argparse
import ctypes
import json
import os
import statistics
import subprocess
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import rpc_amd  # noqa: E402
import bench  # noqa: E402
from bench import Workload  # noqa: E402

# probe-only uniform shapes: bodies shorter than a 4 KiB row (every row partial)
bench.CONFIGS.setdefault("u3k", ("probe: 1M x 3 KiB equal-length bodies", "uniform", 1 << 20, 3072, 0x5EED0103))
bench.CONFIGS.setdefault("u2k", ("probe: 2M x 2 KiB equal-length bodies", "uniform", 1 << 21, 2048, 0x5EED0102))


def timed(fn, reps):
    s = torch.cuda.current_stream()
    fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    for _ in range(reps):
        fn()
    e1.record(s)
    e1.synchronize()
    return e0.elapsed_time(e1) / 1e3 / reps


def lib_variants(w, a):
    nbytes = (w.total // 4096) * 4096
    v = {}
    for pat in (0, 1):
        for nt in (0, 1):
            v[f"stream_read_p{pat}_nt{nt}"] = (lambda pat=pat, nt=nt: rpc_amd.stream_read(
                w.base, pat, bool(nt), nbytes=nbytes), nbytes, None)
    for nt in (0, 1):
        for g in [int(x) for x in a.grids.split(",")]:
            v[f"crc_nt{nt}_grid{g}"] = (w.step, w.algo_bytes, (nt, g))
    return v


def ablate_variants(w, a):
    """Rows-kernel variants: (qb, pair, nt, abl) -- abl bits 1 no-compute,
    2 no-merge, 4 no-load, 8 natural lane->piece load order."""
    so = os.environ.get("RPCCRC_PROBE_LIB", os.path.join(REPO, "tools", "libprobe.so"))
    if not os.path.exists(so):
        subprocess.run(["make", "-C", os.path.join(REPO, "tools")], check=True)
    lib = ctypes.CDLL(so)
    lib.probe_rows.restype = ctypes.c_int
    lib.probe_rows.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint64,
                               ctypes.c_void_p] + [ctypes.c_int] * 6 + [ctypes.c_void_p]
    out = torch.empty(w.n, dtype=torch.int32, device=w.device)
    blocks = 256

    def mk(qb, pair, nt, abl, depth, g=0):
        def f():  # pair's high byte carries the group-dealing shift (a.gshift)
            rc = lib.probe_rows(w.base.data_ptr(), w.n, w.L, w.L, out.data_ptr(), qb, pair | (g << 8), nt, abl, depth,
                                blocks, torch.cuda.current_stream().cuda_stream)
            assert rc == 0, (qb, pair, nt, abl, depth, g, rc)
        return f
    combos = [(1, 1, 1, 0, 1), (1, 1, 0, 0, 1), (1, 1, 1, 1, 1), (1, 1, 1, 2, 1), (1, 1, 1, 3, 1), (1, 1, 1, 4, 1),
              (1, 1, 1, 6, 1), (1, 1, 1, 0, 2), (1, 1, 0, 0, 2), (1, 1, 1, 3, 2),
              (1, 1, 1, 8, 1), (1, 1, 1, 11, 1), (1, 1, 1, 9, 1), (1, 1, 0, 11, 1), (1, 1, 0, 3, 1),
              (1, 1, 1, 16, 1), (1, 1, 1, 19, 1), (1, 1, 1, 32, 1), (1, 1, 1, 35, 1), (1, 1, 1, 51, 1),
              (1, 1, 1, 64, 1), (1, 1, 1, 128, 1), (1, 1, 1, 192, 1), (1, 1, 1, 67, 1), (1, 1, 1, 131, 1), (1, 1, 1, 195, 1),
              (1, 1, 1, 259, 1), (1, 1, 1, 275, 1)]
    combos += [(1, 1, 1, 0, 1, g) for g in (1, 2, 3, 4, 5)] + [(1, 1, 1, 3, 1, 5), (1, 1, 1, 19, 1, 5)]
    combos += [(1, 1, 1, 1024, 1), (1, 1, 1, 1027, 1), (1, 1, 1, 1043, 1)]  # DYN (+ memory only)
    # DYN: merge only / chain only / compute only / no transpose / memory only without transpose
    combos += [(1, 1, 1, 1025, 1), (1, 1, 1, 1026, 1), (1, 1, 1, 1028, 1), (1, 1, 1, 1056, 1), (1, 1, 1, 1059, 1)]
    combos += [(1, 1, 1, 3072, 1), (1, 1, 1, 1040, 1)]  # DYN with NT stores / no stores
    combos += [(1, 1, 1, 9216, 1)]  # DYN, chain of slots 2-3 only: a half-width row's instruction cost
    if w.L <= 1024:  # aligned uniform bodies: z = 0
        combos += [(4, 1, 1, 0, 1), (4, 1, 0, 0, 1), (4, 1, 1, 3, 1), (4, 1, 1, 4, 1), (4, 1, 1, 6, 1),
                   (4, 1, 1, 0, 2), (4, 1, 1, 3, 2)] + [(4, 1, 1, 0, 1, g) for g in (1, 2, 3, 4, 5)] + [(4, 1, 1, 1024, 1), (4, 1, 1, 1027, 1), (4, 1, 1, 1043, 1), (4, 1, 1, 1028, 1), (4, 1, 1, 3072, 1), (4, 1, 1, 1040, 1)]

    def name(c):
        return "qb{}_pair{}_nt{}_abl{}_d{}".format(*c[:5]) + (f"_g{c[5]}" if len(c) > 5 and c[5] else "")
    if a.only:
        keep = set(a.only.split(","))
        combos = [c for c in combos if name(c) in keep]
    v = {name(c): (mk(*c), w.algo_bytes, None) for c in combos}
    # correctness of every non-ablated variant vs the product kernel
    w.step()
    torch.cuda.synchronize()
    ref = w.out.clone()
    for c in combos:
        if c[3] & ~(192 | 512 | 1024) == 0:  # exact variants (seed source / load path / timeline / DYN)
            mk(*c)()
            torch.cuda.synchronize()
            assert torch.equal(out, ref), c
    return v


class WrapWorkload:
    """C3's launch (8M bodies of 4 KiB, 32 GiB read) as a ragged batch over a
    buffer of `gib` GiB: body i at (i * 4096) mod gib GiB."""

    def __init__(self, gib):
        import rpc_amd
        self.kind, self.L, self.n, self.device = "ragged", 4096, 1 << 23, torch.device("cuda", 0)
        span = gib << 30
        self.base = torch.empty(span, dtype=torch.uint8, device=self.device)
        rpc_amd.fill_random(self.base, 0x5EED0005)
        i = torch.arange(self.n, dtype=torch.int64, device=self.device)
        self.offs = (i * 4096) % span
        self.lens = torch.full((self.n,), 4096, dtype=torch.int32, device=self.device)
        self.out = torch.empty(self.n, dtype=torch.int32, device=self.device)
        self.algo_bytes = self.n * (4096 + 16)

    def step(self):
        import rpc_amd
        rpc_amd.device_batch(self.base, self.offs, self.lens, out=self.out)


def timeline(w, a):
    """Per-wave entry / LDS-image-ready / exit times (s_memrealtime, 100 MHz) of the
    product kernel (kRowsAblTimes variant, exact results) after a clock prewarm:
    how much of a launch is fill (launch spread + image copy) and drain (exit spread)."""
    import time
    so = os.environ.get("RPCCRC_PROBE_LIB", os.path.join(REPO, "tools", "libprobe.so"))
    if not os.path.exists(so):
        subprocess.run(["make", "-C", os.path.join(REPO, "tools")], check=True)
    lib = ctypes.CDLL(so)
    lib.probe_rows_times.restype = ctypes.c_int
    lib.probe_rows_times.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint64,
                                     ctypes.c_void_p] + [ctypes.c_int] * 6 + [ctypes.c_void_p, ctypes.c_void_p,
                                                                               ctypes.c_int]
    ragged = w.kind == "ragged"
    qb = 1 if ragged else (4 if w.L <= 1024 else 1)
    nw = 256 * 16
    times = torch.zeros(nw * 4, dtype=torch.int64, device=w.device)
    out = torch.empty(w.n, dtype=torch.int32, device=w.device)
    s = torch.cuda.current_stream()
    if ragged:  # the C2 path: ragged QB = 1, DYN (static rounds, as the product)
        lib.probe_rows_ragged_times.restype = ctypes.c_int
        lib.probe_rows_ragged_times.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64,
                                                ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p,
                                                ctypes.c_int]

    def f():
        if ragged:
            rc = lib.probe_rows_ragged_times(w.base.data_ptr(), w.offs.data_ptr(), w.lens.data_ptr(), w.n,
                                             out.data_ptr(), 256, s.cuda_stream, times.data_ptr(),
                                             a.steal_pct if a.steal else 0)
        else:
            rc = lib.probe_rows_times(w.base.data_ptr(), w.n, w.L, w.L, out.data_ptr(), qb, 1, 1,
                                      512 | (1024 if a.dyn or a.steal else 0) | (4096 if a.steal else 0), 1, 256,
                                      s.cuda_stream, times.data_ptr(), a.gshift)
        assert rc == 0, rc
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < 0.5:
        w.step()
    torch.cuda.synchronize()
    # --surround-ms: each timed launch sits inside that much back-to-back work on
    # either side (steady state), not after the host's pause between reps
    k_around = 1
    if a.surround_ms > 0:
        q0, q1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        q0.record(s)
        for _ in range(3):
            w.step()
        q1.record(s)
        q1.synchronize()
        k_around = max(1, int(a.surround_ms / (q0.elapsed_time(q1) / 3)))
    for rep in range(a.reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        for _ in range(k_around):
            w.step()
        e0.record(s)
        f()
        e1.record(s)
        for _ in range(k_around):
            w.step()
        torch.cuda.synchronize()
        traw = times.view(nw, 4).cpu().numpy()
        t = traw.astype(np.float64)
        live = t[:, 2] > 0
        t = t[live]
        # word 3: tasks (low 24 bits) | shader cycles entry -> exit (s_memtime)
        w3 = traw[live, 3].astype(np.uint64)
        tasks = (w3 & np.uint64(0xFFFFFF)).astype(np.float64)
        cyc = (w3 >> np.uint64(24)).astype(np.float64)
        clk_mhz = cyc / np.maximum(t[:, 2] - t[:, 0], 1.0) * 100.0  # per wave: shader cycles / real 100 MHz ticks
        base = t[:, 0].min()
        ent, img, ext = (t[:, 0] - base) / 100.0, (t[:, 1] - base) / 100.0, (t[:, 2] - base) / 100.0  # us
        pct = lambda x: [round(float(np.percentile(x, q)), 2) for q in (0, 50, 99, 100)]
        # per XCD (workgroup b runs on XCD b % 8; gw = vb * 16 + wave, vb = (b % 8) * 32 + b / 8)
        xcd = (np.arange(nw) // 16 // 32)[live]
        per_xcd = [round(float(np.median(ext[xcd == x])), 1) for x in range(8)]
        wiw = (np.arange(nw) % 16)[live]
        per_wave_slot = [round(float(np.median(ext[wiw == k])), 1) for k in range(16)]
        if a.save:
            np.save(f"{a.save}_rep{rep}.npy", np.stack([ent, img, ext]))
        print(json.dumps({"mode": "timeline", "config": a.config, "wrap_gib": a.wrap_gib, "surround_steps": k_around,
                          "rep": rep, "qb": qb, "waves": int(live.sum()),
                          "gshift": a.gshift, "dyn": a.dyn, "steal": a.steal, "exit_median_per_xcd": per_xcd,
                          "exit_median_per_wave_slot": per_wave_slot,
                          "event_us": round(e0.elapsed_time(e1) * 1e3, 1),
                          "entry_us_p0_50_99_100": pct(ent), "image_ready_us": pct(img),
                          "image_copy_us": pct(img - ent), "exit_us": pct(ext),
                          "tasks_per_wave": pct(tasks),
                          "shader_clock_mhz_p0_50_100": [round(float(np.percentile(clk_mhz, q)), 1) for q in (0, 50, 100)],
                          "shader_clock_mhz_per_xcd": [round(float(np.median(clk_mhz[xcd == x])), 1) for x in range(8)]}),
              flush=True)
    w.step()
    torch.cuda.synchronize()
    ref = w.out.clone()
    f()
    torch.cuda.synchronize()
    assert torch.equal(out, ref), "timeline variant changed the CRCs"


def packed_modes(a):
    """Ragged-batch kernels (rows vs packed) on shapes that isolate their costs:
    uniform 4 KiB / 1 KiB / 3000 B bodies passed as a ragged batch, and C2."""
    dev = torch.device("cuda", 0)
    res = []
    shapes = [("4096x1M", 1 << 20, 4096), ("1024x1M", 1 << 20, 1024), ("3000x1M", 1 << 20, 3000),
              ("frames1M", 1 << 20, None), ("c2", None, None),
              # multi-row ragged items (whole rows only): 4 / 16 rows per body
              ("16384x256K", 1 << 18, 16384), ("65536x64K", 1 << 16, 65536)]
    if a.shapes:
        shapes = [x for x in shapes if x[0] in a.shapes.split(",")]
    for name, n, L in shapes:
        if name == "c2":
            w = Workload("c2", 0, dev)
            base, offs, lens, nbytes = w.base, w.offs, w.lens, w.total
        elif L is None:  # wire frames: 12-B header + body of 1..1024 B (rpc.h:17), back to back
            rng = np.random.default_rng(11)
            ln = rng.integers(1, 1025, n).astype(np.uint32)
            fo = np.concatenate([[0], np.cumsum(ln[:-1].astype(np.uint64) + 12)]).astype(np.uint64)
            nbytes = int(ln.sum())
            base = torch.empty((int(fo[-1]) + 12 + int(ln[-1]) + 64) // 8 * 8, dtype=torch.uint8, device=dev)
            rpc_amd.fill_random(base, 7)
            offs = torch.from_numpy((fo + 12).view(np.int64)).to(dev)
            lens = torch.from_numpy(ln.view(np.int32)).to(dev)
        else:
            nbytes = n * L
            base = torch.empty(nbytes + 64, dtype=torch.uint8, device=dev)
            rpc_amd.fill_random(base, 7)
            offs = (torch.arange(n, dtype=torch.int64, device=dev) * L)
            lens = torch.full((n,), L, dtype=torch.int32, device=dev)
        out = torch.empty(offs.numel(), dtype=torch.int32, device=dev)
        import time
        for path in a.paths.split(","):
            rpc_amd.set_ragged_path(path)
            f = lambda: rpc_amd.device_batch(base, offs, lens, out=out)
            t0 = time.perf_counter()  # clock prewarm (DVFS ramp)
            while time.perf_counter() - t0 < 0.5:
                f()
            torch.cuda.synchronize()
            ts = [timed(f, a.reps) for _ in range(a.rounds)]
            med = statistics.median(ts)
            r = {"mode": "packed", "shape": name, "path": path, "median_us": round(med * 1e6, 1),
                 "min_slice": os.environ.get("RPCCRC_PACKED_MIN_SLICE", "default"),
                 "GiBps": round(nbytes / med / 2**30, 1)}
            res.append(r)
            print(json.dumps(r), flush=True)
        rpc_amd.set_ragged_path("auto")
        del base, offs, lens, out
        torch.cuda.empty_cache()


def ragged_ablate(a):
    """Ragged QB = 1 rows kernel (DYN, the C2 path) under ablation bits on a
    ragged workload (--config c2): what bounds it -- memory, compute, stores,
    the quarter / half first rows.  Interleaved rounds, median; exact variants
    (0, 16384) are checked against the product's CRCs."""
    import time
    so = os.environ.get("RPCCRC_PROBE_LIB", os.path.join(REPO, "tools", "libprobe.so"))
    lib = ctypes.CDLL(so)
    lib.probe_rows_ragged.restype = ctypes.c_int
    lib.probe_rows_ragged.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64,
                                      ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
    w = Workload(a.config, 0, torch.device("cuda", 0))
    assert w.kind == "ragged", "ragged mode needs a ragged config (c2)"
    out = torch.empty(w.n, dtype=torch.int32, device=w.device)
    s = torch.cuda.current_stream()
    names = {0: "product", 16384: "full first rows (no sub-rows)", 3: "memory only", 4: "compute only",
             16: "no stores", 2: "no merge", 19: "memory only, no stores",
             65536: "memory + control of the product's pipeline (XOR fold)"}
    if a.only:
        names = {k: v for k, v in names.items() if str(k) in a.only.split(",")}

    def mk(abl):
        def f():
            rc = lib.probe_rows_ragged(w.base.data_ptr(), w.offs.data_ptr(), w.lens.data_ptr(), w.n, out.data_ptr(),
                                       abl, 256, s.cuda_stream)
            assert rc == 0, (abl, rc)
        return f
    w.step()
    torch.cuda.synchronize()
    ref = w.out.clone()
    for abl in (0, 16384):
        if abl in names:
            mk(abl)()
            torch.cuda.synchronize()
            assert torch.equal(out, ref), f"ragged variant {abl} changed the CRCs"
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < 0.5:
        mk(0)()
    torch.cuda.synchronize()
    res = {k: [] for k in names}
    for _ in range(a.rounds):
        for k in names:
            res[k].append(timed(mk(k), a.reps))
    for k, ts in res.items():
        med = statistics.median(ts)
        print(json.dumps({"mode": "ragged", "config": a.config, "abl": k, "variant": names[k],
                          "median_us": round(med * 1e6, 1), "frac": round(w.algo_bytes / med / 8e12, 4)}), flush=True)


def stream_rows(a):
    """Row-shape stream probes (tools/probe_kernels.hip stream_rows_probe): per
    mode, GB/s and tiles (wave iterations) per us over the north-star buffer,
    after a clock prewarm, interleaved rounds."""
    import time
    so = os.environ.get("RPCCRC_PROBE_LIB", os.path.join(REPO, "tools", "libprobe.so"))
    lib = ctypes.CDLL(so)
    lib.probe_stream_rows.restype = ctypes.c_int
    lib.probe_stream_rows.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_int, ctypes.c_int, ctypes.c_void_p,
                                      ctypes.c_void_p]
    w = Workload("ns", 0, torch.device("cuda", 0))
    out = torch.empty(16, dtype=torch.int32, device=w.device)
    s = torch.cuda.current_stream()
    tb = {0: 4096, 1: 3072, 2: 3072, 3: 8192}
    names = {0: "4 loads / 4 KiB", 1: "3 loads + 1 out-of-range / 3 KiB", 2: "3 loads / 3 KiB", 3: "8 loads / 8 KiB"}

    def mk(m):
        def f():
            assert lib.probe_stream_rows(w.base.data_ptr(), w.total, m, 256, out.data_ptr(), s.cuda_stream) == 0
        return f
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < 0.5:
        mk(0)()
    torch.cuda.synchronize()
    res = {m: [] for m in tb}
    for _ in range(a.rounds):
        for m in tb:
            res[m].append(timed(mk(m), a.reps))
    for m, ts in res.items():
        med = statistics.median(ts)
        tiles = w.total // tb[m]
        nb = tiles * tb[m]
        print(json.dumps({"mode": "streamrows", "variant": m, "shape": names[m], "median_us": round(med * 1e6, 1),
                          "GBps": round(nb / med / 1e9, 1), "tiles_per_us": round(tiles / med / 1e6, 1)}), flush=True)


def sample_smi(stop, log):
    """Child-process power/clock sampler (best effort; rocm-smi or amd-smi)."""
    import threading  # noqa: F401
    import time
    cmds = [["amd-smi", "metric", "-g", "0", "-p", "-c"], ["rocm-smi", "-d", "0", "--showpower", "--showclocks"]]
    cmd = None
    for c in cmds:
        try:
            r = subprocess.run(c, capture_output=True, text=True, timeout=10)
            if r.returncode == 0:
                cmd = c
                break
        except (OSError, subprocess.SubprocessError):
            pass
    if cmd is None:
        return
    t0 = time.perf_counter()
    while not stop.is_set():
        try:
            r = subprocess.run(cmd, capture_output=True, text=True, timeout=10)
            log.append((round(time.perf_counter() - t0, 3), r.stdout))
        except (OSError, subprocess.SubprocessError):
            break
        time.sleep(0.05)


def sustain(w, a):
    import threading
    import time
    names = a.only.split(",") if a.only else ["product", "stream_nt1"]
    abl = ablate_variants(w, argparse.Namespace(only=",".join(n for n in names if n.startswith("qb"))))
    nbytes = (w.total // 4096) * 4096
    fns = {}
    for n in names:
        if n == "product":
            fns[n] = (w.step, w.algo_bytes)
        elif n == "stream_nt1":
            fns[n] = (lambda: rpc_amd.stream_read(w.base, 0, True, nbytes=nbytes), nbytes)
        else:
            fns[n] = (abl[n][0], abl[n][1])
    s = torch.cuda.current_stream()
    smi_log = []
    stop = threading.Event()
    th = threading.Thread(target=sample_smi, args=(stop, smi_log), daemon=True)
    th.start()
    t0 = time.perf_counter()
    for n, (fn, nb) in fns.items():
        time.sleep(2.0)  # let the clocks recover between variants
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(a.launches + 1)]
        tstart = time.perf_counter() - t0
        ev[0].record(s)
        for i in range(a.launches):
            fn()
            ev[i + 1].record(s)
        ev[-1].synchronize()
        d = [ev[i].elapsed_time(ev[i + 1]) * 1e3 for i in range(a.launches)]
        q = len(d) // 4
        print(json.dumps({"variant": n, "config": a.config, "t_start_s": round(tstart, 2),
                          "first10_us": round(statistics.mean(d[:10]), 1),
                          "last_quarter_us": round(statistics.mean(d[-q:]), 1),
                          "min_us": round(min(d), 1), "max_us": round(max(d), 1),
                          "mean_GBps": round(nb / (statistics.mean(d) / 1e6) / 1e9, 1),
                          "per_launch_us": [round(x, 1) for x in d[::max(1, len(d) // 40)]]}), flush=True)
    stop.set()
    th.join(timeout=15)
    import re
    for t, out in smi_log:
        # GFX clocks (per XCD) and socket power, whatever the tool's layout
        gfx = [int(m) for m in re.findall(r"GFX_\d+:\s*\n\s*CLK:\s*(\d+)", out)]
        pw = re.findall(r"(?:SOCKET_POWER|POWER_USAGE|Current Socket Graphics Package Power \(W\)):?\s*([\d.]+)", out)
        print(json.dumps({"smi_t_s": t, "gfx_mhz": gfx, "power_w": pw[:2]}))
    if a.smi_out and smi_log:
        with open(a.smi_out, "w") as f:
            for t, out in smi_log:
                f.write(json.dumps({"t": t, "out": out}) + "\n")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="ns")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--grids", default="0,512,1024")
    ap.add_argument("--shapes", default="", help="packed mode: comma list of shapes (default all)")
    ap.add_argument("--paths", default="rows,packed", help="packed mode: ragged paths to time")
    ap.add_argument("--mode", default="lib", choices=["lib", "ablate", "sustain", "timeline", "packed", "streamrows", "ragged"])
    ap.add_argument("--launches", type=int, default=60)
    ap.add_argument("--smi-out", default="", help="sustain mode: raw SMI samples (jsonl)")
    ap.add_argument("--only", default="", help="comma list of ablate variant names")
    ap.add_argument("--gshift", type=int, default=0, help="timeline: group-dealing shift of the rows kernel")
    ap.add_argument("--dyn", action="store_true", help="timeline: workgroup-dynamic dealing (DYN)")
    ap.add_argument("--steal", action="store_true", help="timeline: DYN with the product's tail stealing")
    ap.add_argument("--steal-pct", type=int, default=3, help="timeline, ragged: pool percent with --steal")
    ap.add_argument("--save", default="", help="timeline: save per-wave times to <save>_rep<k>.npy")
    ap.add_argument("--surround-ms", type=float, default=0.0,
                    help="timeline: this many ms of back-to-back product steps before and after each timed launch")
    ap.add_argument("--wrap-gib", type=int, default=0,
                    help="timeline: C3's 8M x 4 KiB bodies as a ragged batch whose offsets wrap at this many GiB "
                         "(32: C3's own footprint; 4: the north star's) -- the same bytes per launch over a smaller "
                         "address range")
    a = ap.parse_args()
    torch.cuda.set_device(0)
    if a.mode == "packed":
        return packed_modes(a)
    if a.mode == "streamrows":
        return stream_rows(a)
    if a.mode == "ragged":
        return ragged_ablate(a)
    w = Workload(a.config, 0, torch.device("cuda", 0)) if not a.wrap_gib else WrapWorkload(a.wrap_gib)
    if a.mode == "sustain":
        return sustain(w, a)
    if a.mode == "timeline":
        return timeline(w, a)
    variants = lib_variants(w, a) if a.mode == "lib" else ablate_variants(w, a)
    res = {k: [] for k in variants}
    for _ in range(a.rounds):
        for k, (fn, nb, opt) in variants.items():
            if opt is not None:
                rpc_amd.set_options(nontemporal=bool(opt[0]), max_blocks=opt[1])
            res[k].append(timed(fn, a.reps))
            rpc_amd.set_options(False, 0)
    for k, ts in res.items():
        med = statistics.median(ts)
        nb = variants[k][1]
        print(json.dumps({"variant": k, "config": a.config, "median_us": round(med * 1e6, 2),
                          "min_us": round(min(ts) * 1e6, 2), "GBps": round(nb / med / 1e9, 1),
                          "frac_of_8TBps": round(nb / med / 8e12, 4)}), flush=True)


if __name__ == "__main__":
    main()
