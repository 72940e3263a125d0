#!/usr/bin/env python3
"""bench.py -- GiB/s of CRC-32 over device-resident batched bodies on 1..8 MI355X.

Metric (BASELINE.json): "GiB/s CRC32 over device-resident batched bodies;
1/2/4/8 MI355X".  A step = one pass of the batched CRC over the rank's batch
(one launch of the HIP rows kernel; C2: the dense span step's launches,
DESIGN.md 4.9).  Default workload = the north star: 1M x 4 KiB bodies per GPU
(weak scaling), synthetic splitmix64 bytes generated on the device.  Other
BASELINE configs: --config c1 | c2 | c3 | c4.

Launch: python bench.py [--gpus N --steps K --warmup W].  N>1: one process per
GPU under torch.distributed.run -- either the driver's own launch, or, when
WORLD_SIZE is not set, bench.py starts that launcher as a CHILD process itself
(before importing torch or touching a GPU) and exits with its code.  RCCL is
used only as the barrier.  Rank 0 prints ONE JSON line.
"""
from __future__ import annotations

import argparse
import json
import math
import os
import platform
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

# torch and rpc_amd (which loads the HIP runtime) are imported by main() only
# after the N>1 self-launch decision: the launching parent never touches a GPU.
torch = None
rpc_amd = None


def _load_gpu_modules():
    """Import torch and rpc_amd (HIP runtime) on first use."""
    global torch, rpc_amd
    if torch is None:
        import torch as _torch

        torch = _torch
    if rpc_amd is None:
        import rpc_amd as _rpc_amd

        rpc_amd = _rpc_amd

METRIC = "GiB/s CRC32 over device-resident batched bodies; 1/2/4/8 MI355X"
HBM_PEAK_BPS = 8.0e12  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s (spec)
GiB = float(1 << 30)

CONFIGS = {
    # name: (description, kind, bodies per GPU, body length, seed)
    "ns": ("north star: 1M x 4 KiB equal-length bodies per GPU", "uniform", 1 << 20, 4096, 0x5EED0003),
    "c1": ("C1: 1M x 1 KiB equal-length bodies per GPU", "uniform", 1 << 20, 1024, 0x5EED0002),
    "c2": ("C2: 4M ragged bodies per GPU, log-uniform 64 B-64 KiB, offset/length arrays", "ragged", 1 << 22, 0,
           0x5EED0004),
    "c3": ("C3: 8M x 4 KiB bodies per GPU (64M over 8 GPUs)", "uniform", 1 << 23, 4096, 0x5EED0005),
    "c4": ("C4: 16 x 256 MiB large bodies per GPU, chunked CRC + GF(2) combine", "large", 16, 256 << 20,
           0x5EED0006),
}


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warmup", type=int, default=3)
    p.add_argument("--config", default=None, choices=sorted(CONFIGS),
                   help="default: ns (the north star) at --gpus 1, c3 (BASELINE configs[3]: 8M x 4 KiB per GPU, "
                        "64M over 8 GPUs) at --gpus > 1")
    p.add_argument("--nontemporal", type=int, default=-1, help="-1 = library default")
    p.add_argument("--ragged-path", default="auto", choices=["auto", "rows", "packed", "split"],
                   help="ragged-batch kernel (C2): auto = rows for device batches; packed = 1 KiB chunks four per row")
    p.add_argument("--chunk-kib", type=int, default=0, help="C4: chunk size (0 = library default)")
    p.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                   help="N>1 barrier backend: nccl (= RCCL over xGMI, the product); gloo only to rehearse "
                        "several ranks on one GPU")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--no-host-inclusive", action="store_true")
    p.add_argument("--cpu-seconds", type=float, default=10.0, help="target CPU-baseline work (multi-thread leg)")
    p.add_argument("--master-port", type=int, default=0, help="N>1 self-launch: rendezvous port (0 = pick a free one)")
    p.add_argument("--no-scalar-latency", action="store_true")
    p.add_argument("--no-live-traffic", action="store_true",
                   help="skip the two rocprofv3 PMC child passes (roofline.traffic from profiles/traffic.json)")
    p.add_argument("--step-events", type=int, default=0,
                   help="0: events only around the K timed steps (value, mean launch time); the per-launch "
                        "median then comes from a second K-step pass with an event after every step. 1: per-step "
                        "events in the timed pass itself (each event is a marker packet between launches: "
                        "+4 us per C1 step, profiles/r02/r02aj_step_events_ab.txt)")
    p.add_argument("--traffic-child", action="store_true", help=argparse.SUPPRESS)  # live_traffic's PMC child
    p.add_argument("--prewarm-s", type=float, default=0.5,
                   help="untimed steps before the W warmup steps until this much time has passed: the GPU "
                        "clock ramps over the first ~20 launches of sustained load (DESIGN.md 5)")
    args = p.parse_args()
    if args.config is None:
        # BASELINE.json: the north star is quoted at 1 GPU; configs[3] (64M x 4 KiB
        # sharded evenly over 8 GPUs) is the multi-GPU workload -- 8M bodies per
        # rank at every N > 1 (weak scaling).
        world = int(os.environ.get("WORLD_SIZE", "0")) or args.gpus
        args.config = "c3" if max(world, args.gpus) > 1 else "ns"
    return args


class Workload:
    def __init__(self, cfg: str, rank: int, device, chunk: int = 0):
        _load_gpu_modules()
        desc, kind, n, L, seed = CONFIGS[cfg]
        self.name, self.desc, self.kind, self.n, self.L = cfg, desc, kind, n, L
        self.chunk = chunk
        from rpc_amd.shard import rank_seed

        self.seed = rank_seed(seed, rank)
        self.device = device
        if kind == "uniform":
            self.total = n * L
            self.base = torch.empty(self.total, dtype=torch.uint8, device=device)
            self.meta_bytes = 0
        elif kind == "ragged":
            from_oracle_free_lengths = _loguniform_lengths(n, self.seed)
            self.lens_h = from_oracle_free_lengths
            self.offs_h = np.concatenate([[0], np.cumsum(self.lens_h[:-1], dtype=np.uint64)]).astype(np.uint64)
            self.total = int(self.lens_h.sum(dtype=np.uint64))
            self.base = torch.empty((self.total + 15) // 8 * 8, dtype=torch.uint8, device=device)
            self.offs = torch.from_numpy(self.offs_h.view(np.int64)).to(device)
            self.lens = torch.from_numpy(self.lens_h.view(np.int32)).to(device)
            self.meta_bytes = 12 * n
            self.max_len = int(self.lens_h.max())
        else:  # large
            self.total = n * L
            self.base = torch.empty(self.total, dtype=torch.uint8, device=device)
            self.large_offs = [i * L for i in range(n)]
            self.large_lens = [L] * n
            self.meta_bytes = 0
        rpc_amd.fill_random(self.base, self.seed)
        self.out = torch.empty(n, dtype=torch.int32, device=device)
        # algorithmic bytes per launch: body bytes read + metadata read + 4 B/body written
        self.algo_bytes = self.total + self.meta_bytes + 4 * n

    def step(self):
        if self.kind == "uniform":
            rpc_amd.device_uniform(self.base, self.n, self.L, out=self.out)
        elif self.kind == "ragged":
            # the config's own length bound (64 KiB): below the 256 KiB
            # big-body route threshold, so its passes are not launched (the
            # result is the same either way: rpc_crc32_device_batch_bounded)
            rpc_amd.device_batch(self.base, self.offs, self.lens, out=self.out, max_len=self.max_len)
        else:
            rpc_amd.device_large(self.base, self.large_offs, self.large_lens, chunk=self.chunk, out=self.out)


def _loguniform_lengths(n, seed, lo=64, hi=65536):
    """Same formula as oracle.loguniform_lengths (kept here so the timed GPU leg
    does not import the oracle)."""
    k = np.arange(1, n + 1, dtype=np.uint64)
    with np.errstate(over="ignore"):
        z = np.uint64(seed) + k * np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        z = z ^ (z >> np.uint64(31))
    u = (z >> np.uint64(11)).astype(np.float64) * (1.0 / (1 << 53))
    ln = np.floor(lo * np.exp(u * np.log(hi / lo))).astype(np.int64)
    return np.clip(ln, lo, hi).astype(np.uint32)


def log(msg: str):
    """Progress on stderr (a silent minute looks like a hang to the GPU harness)."""
    print(f"bench: {msg}", file=sys.stderr, flush=True)


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.processor() or "unknown"


def cgroup_cpu_quota():
    """CPUs' worth of time the cgroup allows (cpu.max quota / period), or None."""
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        return None if q == "max" else round(int(q) / int(per), 2)
    except (OSError, ValueError):
        return None


def effective_cpus():
    """(CPUs of throughput this process really has, CPUs in its affinity mask): the
    affinity mask capped by the cgroup's cpu.max quota (a 256-thread host that grants
    16 CPUs' worth of time is a 16-CPU baseline)."""
    aff = max(1, len(os.sched_getaffinity(0)))
    q = cgroup_cpu_quota()
    return (max(1, min(aff, int(math.ceil(q)))) if q else aff), aff


# Samples larger than the host's last-level cache (AMD EPYC 9575F: 8 x 32 MiB L3),
# so the baseline streams from DRAM as the GPU streams from HBM.
CPU_SAMPLE_BYTES = 1 << 30


def cpu_baseline(w: Workload, target_s: float):
    """The reference crc.c (+ system libz, built into oracle/_ref) timed on this
    host's cores over a bounded sample of the same workload, at 1 thread and at
    the effective CPU count (affinity mask capped by the cgroup quota)."""
    from oracle import oracle  # cpu_baseline leg only (test/baseline infrastructure)
    import zlib

    ref = oracle.load_ref()
    kind = "reference"
    if ref is None:
        return None
    threads, aff = effective_cpus()
    if w.kind == "uniform":
        nb = min(w.n, CPU_SAMPLE_BYTES // w.L)
        host = w.base[: nb * w.L].cpu().numpy()
        offs = np.arange(nb, dtype=np.uint64) * np.uint64(w.L)
        lens = np.full(nb, w.L, dtype=np.uint32)
        sample = f"{nb} x {w.L} B bodies (first {nb * w.L >> 20} MiB of the same device stream)"
        dev_crc = w.out[:nb].cpu().numpy().view(np.uint32)
    elif w.kind == "ragged":
        nb = int(np.searchsorted(np.cumsum(w.lens_h, dtype=np.uint64), CPU_SAMPLE_BYTES))
        end = int(w.offs_h[nb - 1] + w.lens_h[nb - 1])
        host = w.base[:end].cpu().numpy()
        offs, lens = w.offs_h[:nb], w.lens_h[:nb]
        sample = f"first {nb} ragged bodies ({end >> 20} MiB)"
        dev_crc = w.out[:nb].cpu().numpy().view(np.uint32)
    else:
        host = w.base[: w.L].cpu().numpy()
        offs = np.array([0], dtype=np.uint64)
        lens = np.array([w.L], dtype=np.uint32)
        nb = 1
        sample = f"1 x {w.L >> 20} MiB body (single-threaded by construction)"
        dev_crc = w.out[:1].cpu().numpy().view(np.uint32)
        threads = 1
    nbytes = int(lens.sum(dtype=np.uint64))
    s1, crc1 = ref.batch_timed(host, offs, lens, threads=1, reps=1)
    agree = bool(np.array_equal(crc1, dev_crc))
    reps = 1
    sm, _ = ref.batch_timed(host, offs, lens, threads=threads, reps=1)
    if sm > 0:
        reps = max(1, min(5000, int(math.ceil(target_s / sm))))
    sm, _ = ref.batch_timed(host, offs, lens, threads=threads, reps=reps)
    # Labelled extra only: the same sample on every CPU of the affinity mask
    # (quota bursting; not the baseline).
    all_aff = None
    if aff > threads:
        ta, _ = ref.batch_timed(host, offs, lens, threads=aff, reps=max(1, reps // 4))
        all_aff = {"threads": aff, "GiBps": round(nbytes * max(1, reps // 4) / ta / GiB, 3)}
    # Config C0, the reference's own CPU case: 1024 x 4 KiB
    # JSON-RPC bodies, crc.c at 1 thread and at the effective CPU count; the
    # GPU's CRCs of the same bodies are checked equal.  Timed over the 4 MiB set
    # tiled to 1 GiB, so the sample exceeds the L3 (a 4 MiB set is cache-resident
    # and let 256 threads burst past the quota).
    c0_buf, c0_offs, c0_lens = oracle.json_bodies(1024, 4096, 0x5EED0001)
    c0_bytes = int(c0_lens.sum(dtype=np.uint64))
    _, c0_crc = ref.batch_timed(c0_buf, c0_offs, c0_lens, threads=1, reps=1)
    tiles = max(1, CPU_SAMPLE_BYTES // c0_bytes)
    c0_big = np.tile(c0_buf, tiles)
    c0_boffs = np.arange(1024 * tiles, dtype=np.uint64) * np.uint64(4096)
    c0_blens = np.full(1024 * tiles, 4096, dtype=np.uint32)
    c0 = {"sample": f"1024 x 4096 B JSON-RPC bodies (seed 0x5EED0001), the set tiled {tiles}x "
                    f"({c0_bytes * tiles >> 20} MiB) so it exceeds the L3"}
    for tn in sorted({1, threads}):
        t1, _ = ref.batch_timed(c0_big, c0_boffs, c0_blens, threads=tn, reps=1)
        r = max(1, min(200, int(math.ceil(1.0 / max(t1, 1e-6)))))
        tr, _ = ref.batch_timed(c0_big, c0_boffs, c0_blens, threads=tn, reps=r)
        c0[f"GiBps_{tn}_threads"] = round(c0_bytes * tiles * r / tr / GiB, 3)
    del c0_big
    c0_dev = rpc_amd.device_uniform(torch.from_numpy(c0_buf).to(w.device), 1024, 4096)
    c0["gpu_crcs_match_reference"] = bool(np.array_equal(c0_dev.cpu().numpy().view(np.uint32), c0_crc))
    return {
        "value": round(nbytes * reps / sm / GiB, 3),
        "unit": "GiB/s",
        "cores": threads,
        "cores_source": f"min(affinity mask {aff}, ceil(cgroup cpu.max quota {cgroup_cpu_quota()}))",
        "cgroup_cpu_quota": cgroup_cpu_quota(),
        "all_affinity_threads": all_aff,
        "kind": kind,
        "c0": c0,
        "sample": f"{sample}, {reps} passes on {threads} threads ({sm:.1f} s)",
        "single_thread_value": round(nbytes / s1 / GiB, 3),
        "cpu_model": cpu_model(),
        "libz": zlib.ZLIB_RUNTIME_VERSION,
        "gpu_crcs_match_reference": agree,
    }


# Per-rank correctness at every N: after the timed region each
# rank checks its first RANK_CHECK_BODIES CRCs against the reference crc.c.
RANK_CHECK_BODIES = 1 << 16


def rank_check_sample(w: Workload):
    """(host bytes, offsets, lengths, device CRCs) of this rank's first bodies."""
    nb = min(w.n, RANK_CHECK_BODIES)
    if w.kind == "uniform":
        host = w.base[: nb * w.L].cpu().numpy()
        offs = np.arange(nb, dtype=np.uint64) * np.uint64(w.L)
        lens = np.full(nb, w.L, dtype=np.uint32)
    elif w.kind == "ragged":
        offs, lens = w.offs_h[:nb], w.lens_h[:nb]
        host = w.base[: int(offs[-1] + lens[-1])].cpu().numpy()
    else:  # large: the first body (256 MiB)
        nb = 1
        host = w.base[: w.L].cpu().numpy()
        offs = np.zeros(1, dtype=np.uint64)
        lens = np.full(1, w.L, dtype=np.uint32)
    return host, offs, lens, w.out[:nb].cpu().numpy().view(np.uint32)


def rank_crc_check(host, offs, lens, dev_crc, threads: int) -> dict:
    """This rank's device CRCs against the reference crc.c (oracle/_ref, built from
    /root/reference/crc.c) -- the cpu_baseline leg's checker, outside the timed
    region; the oracle restatement where the reference build is absent."""
    from oracle import oracle  # checker only (test/baseline infrastructure)

    ref = oracle.load_ref()
    if ref is not None:
        _, want = ref.batch_timed(host, offs, lens, threads=threads, reps=1)
        checker = "reference crc.c (oracle/_ref/libref_crc.so)"
    else:
        want = oracle.crc32_batch_mt(host, offs, lens, threads=threads)
        checker = "oracle restatement (oracle/_ref absent)"
    bad = int(np.count_nonzero(np.asarray(dev_crc, dtype=np.uint32) != want))
    return {"bodies": int(len(want)), "mismatches": bad, "checker": checker}


def reduce_crc_check(dist, device, rec: dict, world: int) -> dict:
    """ranks_crc_check over ranks: how many ranks had every sampled CRC right."""
    ok = 1 if rec["mismatches"] == 0 else 0
    if dist is not None:
        from rpc_amd.shard import sum_over_ranks

        ranks_ok = sum_over_ranks(dist, ok, device)
        bodies = sum_over_ranks(dist, rec["bodies"], device)
        mism = sum_over_ranks(dist, rec["mismatches"], device)
    else:
        ranks_ok, bodies, mism = ok, rec["bodies"], rec["mismatches"]
    return {"ranks": world, "ranks_ok": ranks_ok, "bodies_checked": bodies, "mismatches": mism,
            "bodies_per_rank": rec["bodies"], "checker": rec["checker"],
            "of": "each rank's first bodies of its own shard, after the timed region"}


def host_inclusive(w: Workload):
    """Pinned host buffer -> H2D -> kernel -> D2H of CRCs through rpc_crc32_batch."""
    if w.kind != "uniform":
        return None
    nb = min(w.n, (2 << 30) // w.L)
    host = torch.empty(nb * w.L, dtype=torch.uint8, pin_memory=True)
    host.copy_(w.base[: nb * w.L])
    hn = host.numpy()
    offs = np.arange(nb, dtype=np.uint64) * np.uint64(w.L)
    lens = np.full(nb, w.L, dtype=np.uint32)
    best = float("inf")
    for _ in range(3):
        t0 = time.perf_counter()
        out = rpc_amd.crc32_batch(hn, offs, lens)
        best = min(best, time.perf_counter() - t0)
    ok = bool(np.array_equal(out, w.out[:nb].cpu().numpy().view(np.uint32)))
    return {"GiBps": round(nb * w.L / best / GiB, 2), "bytes": nb * w.L, "matches_device_path": ok}


def rx_ring_probe():
    """rpc.h frames (1 KiB bodies, MAX_BODY_LEN) landed in the
    batched receive ring's pinned segments and verified on the GPU segment by
    segment, host-inclusive (tools/rx_bench.c), next to the reference server's
    per-frame rpc_crc32_verify (crc.c, one host core) on the same frames."""
    import subprocess
    exe = os.path.join(REPO, "tools", "rx_bench")
    if not os.path.exists(exe):
        return None
    ref = os.path.join(REPO, "oracle", "_ref", "libref_crc.so")
    cmd = [exe, str(1 << 18), "1024", str(64 << 20), "3"] + ([ref] if os.path.exists(ref) else [])
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=300)
    try:
        r = json.loads(p.stdout.strip().splitlines()[-1])
    except (ValueError, IndexError):
        return {"error": (p.stderr or p.stdout)[-300:], "rc": p.returncode}
    r["rc"] = p.returncode
    return r


def scalar_latency_probe():
    """Per-call latency of the drop-in rpc_crc32 at 12 B, 68 B and 1 KiB on 1 and 10
    threads, beside the reference crc.c on the same host (tools/scalar_bench.c):
    through the resident drop-in service (the default) and, for
    comparison, with a kernel launch per call (RPCCRC_SERVICE=0)."""
    import subprocess
    exe = os.path.join(REPO, "tools", "scalar_bench")
    if not os.path.exists(exe):
        return None
    ref = os.path.join(REPO, "oracle", "_ref", "libref_crc.so")
    out = {}
    for name, env in (("service", {}), ("launch_per_call", {"RPCCRC_SERVICE": "0"})):
        p = subprocess.run([exe] + ([ref] if os.path.exists(ref) else []), capture_output=True, text=True,
                           timeout=300, env=dict(os.environ, **env))
        try:
            r = json.loads(p.stdout.strip().splitlines()[-1])
        except (ValueError, IndexError):
            r = {"error": (p.stderr or p.stdout)[-300:]}
        r["rc"] = p.returncode
        out[name] = r
    return out


def frames_lifted_probe(device, n=1024, reps=5, seed=0x5EED0007):
    """SURVEY.md 8f row 3 (large-body framing): n rpc.h frames back to back in
    HBM, bodies log-uniform 1 B - 64 MiB (MAX_BODY_LEN lifted, RPC_FRAMES_LIFT_CAP),
    stamped and then verified on the device.  Bodies >= 256 KiB take the
    on-device chunk route.  Checks: every frame verifies OK after
    the stamp, and one byte flipped inside the largest body is flagged BAD_CRC
    (the CRCs themselves are checked against the oracle by
    tests/test_frames.py::test_frames_lifted_cap_large_bodies)."""
    lens = _loguniform_lengths(n, seed, lo=1, hi=64 << 20).astype(np.uint64)
    sizes = lens + np.uint64(12)
    offs = np.concatenate([[0], np.cumsum(sizes[:-1], dtype=np.uint64)]).astype(np.uint64)
    total = int(offs[-1] + sizes[-1])
    buf = torch.empty((total + 7) // 8 * 8, dtype=torch.uint8, device=device)
    rpc_amd.fill_random(buf, seed)
    d_offs = torch.from_numpy(offs.view(np.int64)).to(device)
    d_lens = torch.from_numpy(lens.astype(np.uint32).view(np.int32)).to(device)
    stream = torch.cuda.current_stream()

    def timed(fn):
        # clock prewarm as for the main line (the first ~20 launches of sustained
        # load run 15-30 % slower while the clock settles)
        t0 = time.perf_counter()
        while True:
            fn()
            torch.cuda.synchronize()
            if time.perf_counter() - t0 >= 0.3:
                break
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for _ in range(reps):
            fn()
        e1.record(stream)
        e1.synchronize()
        return e0.elapsed_time(e1) / 1e3 / reps

    st = {}
    t_stamp = timed(lambda: st.__setitem__("v", rpc_amd.frames_stamp(buf, d_offs, d_lens, lift_cap=True,
                                                                      stream_bytes=total)))
    stamped = bool((st["v"] == rpc_amd.FRAME_OK).all().item())
    vr = {}
    t_verify = timed(lambda: vr.__setitem__("v", rpc_amd.frames_verify(buf, d_offs, lift_cap=True,
                                                                       stream_bytes=total)[0]))
    all_ok = bool((vr["v"] == rpc_amd.FRAME_OK).all().item())
    big = int(np.argmax(lens))
    pos = int(offs[big]) + 12 + int(lens[big]) // 2
    buf[pos] ^= 0x5A
    v2, _ = rpc_amd.frames_verify(buf, d_offs, lift_cap=True, stream_bytes=total)
    v2 = v2.cpu().numpy()
    buf[pos] ^= 0x5A
    flagged = bool(v2[big] == rpc_amd.FRAME_BAD_CRC and (np.delete(v2, big) == rpc_amd.FRAME_OK).all())
    body = int(lens.sum())
    aligned_4k = buf.data_ptr() % 4096 == 0  # span mode needs a 4 KiB-aligned stream
    del buf
    return {"frames": n, "bodies": "log-uniform 1 B - 64 MiB (LIFT_CAP)", "body_bytes": body,
            "routed_bodies_ge_256KiB": int((lens >= (256 << 10)).sum()),
            "verify_us": round(t_verify * 1e6, 1), "verify_GiBps": round(body / t_verify / GiB, 1),
            "verify_frames_per_s": round(n / t_verify, 1),
            "stamp_us": round(t_stamp * 1e6, 1), "stamp_GiBps": round(body / t_stamp / GiB, 1),
            "all_stamped": stamped, "all_ok_after_stamp": all_ok, "corrupted_frame_flagged": flagged,
            "route_span_mode": aligned_4k and os.environ.get("RPCCRC_BIG_SPAN", "1") != "0"}


def stream_read_probe(w: Workload, steps: int, reps=10, rounds=3):
    """Achievable HBM read rate on the same buffer (SURVEY 8d "a measured
    stream-read kernel"):
      * rows_dealing_GBps -- the ceiling of the product's own memory stream: the
        rows kernel with its CRC work compiled out, same DYN rounds + tail
        stealing, same 4 x 16 B non-temporal loads a row ahead, no stores
        (rpc_crc32_stream_read_device pattern 2).  Timed under the product's
        own protocol: after a re-warm, `rounds` pairs of
        blocks -- K = `steps` probe launches, K product steps -- back to back
        on the product's stream with one event between blocks (order swapped
        every round), so frac_of_stream_read compares the two at one clock.
      * coalesced_nt{1,0}_GBps -- a plain grid-stride loop with coalesced 16-B
        lanes and no tail dealing (rounds 1-3's probe; the product beat it)."""
    nbytes = (w.total // 4096) * 4096
    stream = torch.cuda.current_stream()
    res = {}

    def block(fn, k):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for _ in range(k):
            fn()
        e1.record(stream)
        e1.synchronize()
        return e0.elapsed_time(e1) / 1e3 / k

    def timed(fn):
        fn()
        t0 = time.perf_counter()  # clock prewarm
        while time.perf_counter() - t0 < 0.2:
            fn()
            torch.cuda.synchronize()
        return block(fn, reps)

    nrows = min(nbytes, 1 << 34) // 4096  # <= 16 GiB per launch (C2's 37 GiB: its first 16 GiB)
    if nrows >= (1 << 16):
        try:
            probe = lambda: rpc_amd.stream_read(w.base, 2, nbytes=nrows * 4096)  # noqa: E731
            # re-warm as before the main pass, then every block back to back
            # (one event between blocks, no host sync: the clock stays at its
            # steady state, as in the timed pass)
            t0 = time.perf_counter()
            while time.perf_counter() - t0 < 0.3:
                w.step()
                torch.cuda.synchronize()
            for _ in range(steps):
                w.step()
            seq = []
            for r in range(rounds):
                order = (("probe", probe), ("product", w.step))
                seq += list(order if r % 2 == 0 else order[::-1])
            ev = [torch.cuda.Event(enable_timing=True) for _ in range(len(seq) + 1)]
            ev[0].record(stream)
            for i, (name, fn) in enumerate(seq):
                for _ in range(steps):
                    fn()
                ev[i + 1].record(stream)
            ev[-1].synchronize()
            t = {"probe": [], "product": []}
            for i, (name, _) in enumerate(seq):
                t[name].append(ev[i].elapsed_time(ev[i + 1]) / 1e3 / steps)
            tp, tc = float(np.mean(t["probe"])), float(np.mean(t["product"]))
            res["rows_dealing_GBps"] = round(nrows * 4096 / tp / 1e9, 1)
            res["rows_dealing_us"] = round(tp * 1e6, 2)
            res["product_interleaved_us"] = round(tc * 1e6, 2)
            res["product_interleaved_GBps"] = round(w.algo_bytes / tc / 1e9, 1)
            res["protocol"] = (f"{rounds} x ({steps} probe launches, {steps} product steps), order swapped each "
                               "round, back to back after a 0.3 s re-warm, one event between blocks")
        except rpc_amd.RpcCrcError as e:  # an older library under A/B (tools/ab_lib.sh)
            res["rows_dealing_error"] = str(e)
    for nt in (1, 0):
        t_nt = timed(lambda: rpc_amd.stream_read(w.base, 0, nontemporal=bool(nt), nbytes=nbytes))
        res[f"coalesced_nt{nt}_GBps"] = round(nbytes / t_nt / 1e9, 1)
    return res


def unbounded_ragged_us(w: Workload, steps: int) -> float:
    """Average step of the same ragged batch through rpc_crc32_device_batch (no
    length bound: the big-body route's classify pass and its passes, empty here, run
    too), timed like the main line after a short re-warm."""
    stream = torch.cuda.current_stream()
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < 0.3:
        rpc_amd.device_batch(w.base, w.offs, w.lens, out=w.out)
        torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    for _ in range(steps):
        rpc_amd.device_batch(w.base, w.offs, w.lens, out=w.out)
    e1.record(stream)
    e1.synchronize()
    return round(e0.elapsed_time(e1) * 1e3 / steps, 2)


def load_traffic(cfg: str):
    """HBM bytes per launch from the committed PMC summary (profiles/), or None."""
    p = os.path.join(REPO, "profiles", "traffic.json")
    try:
        with open(p) as f:
            d = json.load(f)
        return d.get(cfg, {}).get("hbm_bytes_per_launch")
    except (OSError, ValueError):
        return None


def pick_launch_traffic(fetch, write):
    """Per-launch (FETCH_SIZE, WRITE_SIZE) from two PMC passes' per-dispatch
    values in launch order.  The big launches are picked on FETCH_SIZE (the
    stream's reads, the same on every launch), within half of the largest, and
    the same positions are read from the WRITE_SIZE pass; medians over them.  A
    few launches that write back dirty lines left by the on-device generator
    (write outliers) then cannot displace the others, as a filter on the write
    values themselves would (profiles/r05final10).  If the passes saw different
    launch counts, the writes are filtered on half their own median."""
    import statistics

    big = [i for i, x in enumerate(fetch) if x >= 0.5 * max(fetch)]
    f = statistics.median([fetch[i] for i in big])
    if len(write) == len(fetch):
        return f, statistics.median([write[i] for i in big])
    w = sorted(write)
    return f, statistics.median([x for x in w if x >= 0.5 * w[len(w) // 2]])


# Kernels of a product step besides the rows kernel (the dense
# span step; 4.3: the large-body combine).  The ragged rows pass that exits at
# once in dense mode is a rows-kernel dispatch: pick_launch_traffic drops it.
AUX_KERNELS = ("dense_plan_kernel", "dense_decide_kernel", "dense_fold_kernel", "crc32_chunk_combine")


def live_traffic(args, algo_bytes: int):
    """HBM bytes per launch of the dominant kernel, measured in this run: two
    rocprofv3 PMC passes (FETCH_SIZE, then WRITE_SIZE -- separate runs, as
    MI355X_MICROARCH.md prescribes) over a short child bench of the same config,
    corrected as that guide says: gfx950 FETCH_SIZE counts half the bytes of a
    wide streaming read (x 2), both are in KiB (x 1024).  The rows kernel also
    runs tiny launches (the big-body route's empty chunk pass): only dispatches
    whose FETCH_SIZE is within half of the largest, the median over them.  Falls
    back to the committed summary."""
    import csv
    import glob
    import shutil
    import subprocess
    import tempfile

    prof = shutil.which("rocprofv3")
    if prof is None:
        return None, "rocprofv3 not found"
    import statistics

    tmp = tempfile.mkdtemp(prefix="rpccrc_pmc_")
    vals = {}
    seq = {}
    aux_med = {}
    try:
        for counter in ("FETCH_SIZE", "WRITE_SIZE"):
            d = os.path.join(tmp, counter)
            cmd = [prof, "--pmc", counter, "-d", d, "-o", "run", "--output-format", "csv", "--",
                   sys.executable, os.path.abspath(__file__), "--config", args.config, "--steps", "3",
                   "--warmup", "1", "--prewarm-s", "0", "--no-cpu-baseline", "--no-host-inclusive",
                   "--no-live-traffic", "--traffic-child"] + (["--ragged-path", args.ragged_path] if args.ragged_path != "auto" else [])
            try:
                # (a one-process group of the parent's launcher would make the child
                # rendezvous on its port: the child runs outside any group)
                env = {k: v for k, v in os.environ.items()
                       if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "LOCAL_WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT")}
                p = subprocess.run(cmd, capture_output=True, text=True, timeout=240, env=env)
            except subprocess.TimeoutExpired:
                return None, f"rocprofv3 --pmc {counter} timed out"
            if p.returncode != 0:
                return None, f"rocprofv3 --pmc {counter} rc={p.returncode}: {(p.stderr or '')[-200:]}"
            per = {}
            aux = {k: {} for k in AUX_KERNELS}
            for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
                for r in csv.DictReader(open(f)):
                    if r["Counter_Name"] != counter:
                        continue
                    key = (f, r["Dispatch_Id"])
                    if "crc32_rows_kernel" in r["Kernel_Name"]:
                        per[key] = per.get(key, 0.0) + float(r["Counter_Value"])
                    for a in AUX_KERNELS:
                        if a in r["Kernel_Name"]:
                            aux[a][key] = aux[a].get(key, 0.0) + float(r["Counter_Value"])
            if not per:
                return None, f"no {counter} rows for crc32_rows_kernel"
            seq[counter] = [per[k] for k in sorted(per, key=lambda k: (k[0], int(k[1])))]
            aux_med[counter] = {a: statistics.median(v.values()) for a, v in aux.items() if v}
        vals["FETCH_SIZE"], vals["WRITE_SIZE"] = pick_launch_traffic(seq["FETCH_SIZE"], seq["WRITE_SIZE"])
    finally:
        shutil.rmtree(tmp, ignore_errors=True)
    rows = 2.0 * vals["FETCH_SIZE"] * 1024 + vals["WRITE_SIZE"] * 1024
    # the step's other kernels (dense plan / decide / fold, the large-body
    # combine): the median per dispatch of each, added to the rows launch
    steps_aux = {a: 2.0 * aux_med["FETCH_SIZE"].get(a, 0.0) * 1024 + aux_med["WRITE_SIZE"].get(a, 0.0) * 1024
                 for a in sorted(set(aux_med["FETCH_SIZE"]) | set(aux_med["WRITE_SIZE"]))}
    hbm = rows + sum(steps_aux.values())
    return {"hbm_bytes_per_launch": hbm, "over_algorithmic": round(hbm / algo_bytes, 4),
            "fetch_size_kib": vals["FETCH_SIZE"], "write_size_kib": vals["WRITE_SIZE"],
            "rows_kernel_bytes": rows, "other_kernels_bytes": {a: round(b) for a, b in steps_aux.items()}}, \
        ("live: rocprofv3 --pmc FETCH_SIZE and WRITE_SIZE passes of this config (2 x FETCH_SIZE + WRITE_SIZE, KiB), "
         "the rows launch plus the median dispatch of each other kernel of the step")


def rank_timing(dist, device, wall: float, kernel_s: float, median_s: float, total: int):
    """Per-launch times over ranks ("over the slowest rank").  N = 1:
    this rank's.  N > 1: the slowest rank's wall time and average / median launch
    (the roofline reports the slowest rank, as `value` does), the fastest rank's
    average launch for the spread, and the bytes of all ranks."""
    if dist is None:
        return {"wall": wall, "kernel_s": kernel_s, "kernel_min_s": kernel_s, "median_s": median_s, "total": total}
    from rpc_amd.shard import max_over_ranks, min_over_ranks, sum_over_ranks

    return {"wall": max_over_ranks(dist, wall, device), "kernel_s": max_over_ranks(dist, kernel_s, device),
            "kernel_min_s": min_over_ranks(dist, kernel_s, device),
            "median_s": max_over_ranks(dist, median_s, device), "total": sum_over_ranks(dist, total, device)}


def roofline_fields(algo_bytes: int, t: dict, world: int) -> dict:
    """The roofline object's timing part: achieved = one rank's algorithmic bytes
    per launch / the slowest rank's average launch (ranks carry equal shards)."""
    achieved = algo_bytes / t["kernel_s"] / 1e9
    return {
        "bound": "hbm",
        "achieved": round(achieved, 1),
        "peak": HBM_PEAK_BPS / 1e9,
        "unit": "GB/s",
        "frac": round(achieved / (HBM_PEAK_BPS / 1e9), 4),
        "avg_launch_us": round(t["kernel_s"] * 1e6, 2),
        "median_launch_us": round(t["median_s"] * 1e6, 2),
        "per_rank": {"ranks": world, "min_us": round(t["kernel_min_s"] * 1e6, 2),
                     "max_us": round(t["kernel_s"] * 1e6, 2),
                     "of": "average launch duration on each rank's kernel stream; achieved/frac use max_us"},
        "algo_bytes_per_launch": algo_bytes,
    }


def reduce_rehearsal(args, world: int, rank: int):
    """RPCCRC_BENCH_REDUCE_ONLY (tests/test_bench_launch.py): the N > 1 reductions and
    the rank-0 roofline fields over gloo on the CPU, with synthetic per-rank launch
    times (rank r: (1 + r / 10) ms per launch) -- no device work."""
    import torch.distributed as dist

    dist.init_process_group("gloo")
    k = 1e-3 * (1.0 + rank / 10.0)
    algo = CONFIGS[args.config][2] * (CONFIGS[args.config][3] + 4)
    t = rank_timing(dist, None, k * args.steps, k, k, algo - 4 * CONFIGS[args.config][2])
    # the per-rank CRC check on a small CPU-made shard (seed of this rank); the
    # "device" CRCs are the oracle's, with body 7 corrupted on RPCCRC_BENCH_BAD_RANK
    from oracle import oracle
    from rpc_amd.shard import rank_seed

    nb, L = 64, 4096
    host = oracle.splitmix_bytes(nb * L, rank_seed(CONFIGS[args.config][4], rank))
    offs = np.arange(nb, dtype=np.uint64) * np.uint64(L)
    lens = np.full(nb, L, dtype=np.uint32)
    dev = oracle.crc32_batch(host, offs, lens)
    if os.environ.get("RPCCRC_BENCH_BAD_RANK") == str(rank):
        dev[7] ^= 1
    chk = reduce_crc_check(dist, None, rank_crc_check(host, offs, lens, dev, 1), world)
    if rank == 0:
        line = {"n_gpus": world, "value": round(t["total"] * args.steps / t["wall"] / GiB, 2),
                "roofline": roofline_fields(algo, t, world),
                "ranks_crc_ok": chk["ranks_ok"] == world, "ranks_crc_check": chk}
        sys.stdout.flush()
        os.write(1, (json.dumps(line) + "\n").encode())
    dist.destroy_process_group()


def free_port() -> int:
    import socket

    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        return so.getsockname()[1]


def self_launch(args) -> int:
    """--gpus N > 1 without a launcher: start torch.distributed.run (one process per
    GPU, 127.0.0.1 rendezvous) as a child with the same arguments and return its exit
    code.  Runs before torch is imported here, so this parent never touches a GPU."""
    import subprocess

    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")  # dmabuf IPC only on these hosts (RCCL)
    rc = 1
    for attempt in range(2):  # a free port can be taken between our probe and the launcher's bind
        port = args.master_port or free_port()
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
               "--master-addr", "127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + sys.argv[1:]
        t0 = time.perf_counter()
        rc = subprocess.call(cmd, env=env)
        if rc == 0 or args.master_port or time.perf_counter() - t0 > 30:
            break
        print(f"bench: launcher exited {rc} within {time.perf_counter() - t0:.1f} s; retrying on a new port",
              file=sys.stderr)
    return rc


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(self_launch(args))
    if os.environ.get("RPCCRC_BENCH_REDUCE_ONLY"):  # CPU rehearsal of the N > 1 reductions (gloo)
        reduce_rehearsal(args, world, rank)
        return
    if os.environ.get("RPCCRC_BENCH_LAUNCH_ONLY"):  # CPU rehearsal of the launch path (tests/test_bench_launch.py)
        line = json.dumps({"rank": rank, "world": world, "local_rank": local_rank, "gpus": args.gpus,
                           "master": os.environ.get("MASTER_ADDR"), "config": args.config}) + "\n"
        sys.stdout.flush()
        os.write(1, line.encode())  # one write(2) < PIPE_BUF: ranks sharing the pipe cannot interleave
        return
    _load_gpu_modules()
    from rpc_amd.shard import barrier

    if world != args.gpus:
        print(f"bench: WORLD_SIZE={world} but --gpus {args.gpus}; using WORLD_SIZE", file=sys.stderr)
    # one process per GPU.  RCCL refuses two ranks on one GPU, so with the nccl
    # backend more local ranks than visible GPUs is an error, stated before any
    # process group exists; ranks beyond the visible GPUs
    # (a gloo rehearsal on a 1-GPU box) share them
    ndev = torch.cuda.device_count()
    local_world = int(os.environ.get("LOCAL_WORLD_SIZE", str(world)))
    if args.dist_backend == "nccl" and local_world > ndev:
        print(f"bench: {local_world} ranks on this node but {ndev} visible GPU(s): the nccl (RCCL) backend needs "
              f"one GPU per rank (use --gpus <= {ndev}, or --dist-backend gloo to share GPUs)", file=sys.stderr)
        sys.exit(2)
    dev_index = local_rank % max(1, ndev)
    torch.cuda.set_device(dev_index)
    device = torch.device("cuda", dev_index)
    dist = None
    # Under torch.distributed.run even one rank joins a process group, so a
    # one-GPU box runs the N > 1 code path (RCCL barrier and reductions) too.
    if world > 1 or "WORLD_SIZE" in os.environ:
        import torch.distributed as dist

        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=device)
        else:
            dist.init_process_group("gloo")
    if args.nontemporal >= 0:
        rpc_amd.set_options(nontemporal=bool(args.nontemporal))
    rpc_amd.set_ragged_path(args.ragged_path)

    w = Workload(args.config, rank, device, chunk=args.chunk_kib * 1024)
    stream = torch.cuda.current_stream()
    prewarm_steps = 0
    t_pw = time.perf_counter()
    while time.perf_counter() - t_pw < args.prewarm_s:
        w.step()
        torch.cuda.synchronize()
        prewarm_steps += 1
    for _ in range(args.warmup):
        w.step()
    torch.cuda.synchronize()
    if dist:
        barrier(dist, device)
    torch.cuda.synchronize()
    # Events on the kernel's stream around the K steps (mean launch time =
    # roofline.achieved).  An event between launches is a marker packet that
    # delays the next launch, so per-step events (for the median)
    # are taken in a second pass below unless --step-events 1.
    evs = [torch.cuda.Event(enable_timing=True) for _ in range(args.steps + 1)]
    t0 = time.perf_counter()
    evs[0].record(stream)
    for k in range(args.steps):
        w.step()
        if args.step_events or k + 1 == args.steps:
            evs[k + 1].record(stream)
    torch.cuda.synchronize()
    if dist:
        barrier(dist, device)
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    if args.step_events:
        step_s = [evs[k].elapsed_time(evs[k + 1]) / 1e3 for k in range(args.steps)]
    else:
        step_s = [evs[0].elapsed_time(evs[args.steps]) / 1e3 / args.steps] * args.steps
    kernel_s = sum(step_s) / args.steps  # avg launch duration on the kernel's stream
    median_s = float(np.median(step_s))
    median_src = "timed pass, an event after every step" if args.step_events else None
    if not args.step_events:
        mev = [torch.cuda.Event(enable_timing=True) for _ in range(args.steps + 1)]
        # The clock drops during the sync above and takes ~20 launches to ramp
        # back (a median over 5 re-warm launches read 16 % slow): ~0.3 s of
        # launches first, enqueued back to back with the measured ones.
        for _ in range(max(args.warmup, int(0.3 / max(kernel_s, 1e-6)))):
            w.step()
        mev[0].record(stream)
        for k in range(args.steps):
            w.step()
            mev[k + 1].record(stream)
        torch.cuda.synchronize()
        median_s = float(np.median([mev[k].elapsed_time(mev[k + 1]) / 1e3 for k in range(args.steps)]))
        median_src = "second K-step pass with an event after every step (each adds a marker between launches)"
    tr = rank_timing(dist, device, wall, kernel_s, median_s, w.total)
    tmax, total_bytes = tr["wall"], tr["total"]
    if args.traffic_child:
        # live_traffic's PMC child: only the product's steps in the trace (no
        # stream probe, unbounded call or CRC check launches to tell apart)
        if dist:
            dist.destroy_process_group()
        return
    # every rank checks its own first bodies (outside the timed region)
    log("per-rank CRC check against the reference crc.c")
    chk = reduce_crc_check(dist, device, rank_crc_check(*rank_check_sample(w),
                                                        threads=max(1, effective_cpus()[0] // max(1, world))), world)

    extra = {}
    cpu = None
    if rank == 0 and world == 1:
        log("stream-read probe")
        extra["stream_read_probe"] = stream_read_probe(w, args.steps)
        if not args.no_host_inclusive:
            log("host-inclusive batch")
            extra["host_inclusive"] = host_inclusive(w)
            if w.kind == "uniform":
                log("receive ring")
                extra["rx_ring"] = rx_ring_probe()
        if w.kind == "ragged":  # the plain (unbounded) entry point beside the bounded one
            extra["unbounded_launch_us"] = unbounded_ragged_us(w, args.steps)
        if w.name == "ns" and not args.no_host_inclusive:
            log("lifted-cap frames (1 B - 64 MiB bodies)")
            extra["frames_lifted"] = frames_lifted_probe(device)
        if not args.no_scalar_latency and not args.no_host_inclusive:
            log("scalar latency")
            extra["scalar_latency"] = scalar_latency_probe()
        if not args.no_cpu_baseline:
            log("CPU baseline (reference crc.c)")
            cpu = cpu_baseline(w, args.cpu_seconds)

    if rank == 0:
        achieved = w.algo_bytes / tr["kernel_s"] / 1e9
        traffic_rec, traffic_src = None, "not measured"
        if world == 1 and not args.no_live_traffic:
            log("measuring HBM traffic (two rocprofv3 PMC passes)")
            traffic_rec, traffic_src = live_traffic(args, w.algo_bytes)
        if traffic_rec is not None:
            traffic = traffic_rec["hbm_bytes_per_launch"]
        else:
            traffic = load_traffic(args.config)
            if traffic is not None:
                traffic_src = f"committed profiles/traffic.json ({traffic_src})"
        line = {
            "metric": METRIC,
            "value": round(total_bytes * args.steps / tmax / GiB, 2),
            "unit": "GiB/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(tmax / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u8",
            "data": "synthetic (counter-based splitmix64 bytes generated on device)",
            "config": {
                "workload": w.desc,
                "bodies_per_gpu": w.n,
                "body_len": w.L if w.kind != "ragged" else "log-uniform 64..65536",
                "ragged_path": args.ragged_path if w.kind == "ragged" else None,
                "entry_point": {"uniform": "rpc_crc32_device_uniform",
                                "ragged": f"rpc_crc32_device_batch_bounded (max_len = {getattr(w, 'max_len', 0)}: "
                                          "no big-body route passes; extra.unbounded_launch_us times "
                                          "rpc_crc32_device_batch)",
                                "large": "rpc_crc32_device_large"}[w.kind],
                "bytes_per_gpu": w.total,
                "parallelism": f"dp{world} (payload-index shards, "
                               + ("RCCL barrier only)" if args.dist_backend == "nccl" or world == 1 else "gloo rehearsal barrier)"),
            },
            "roofline": {
                **roofline_fields(w.algo_bytes, tr, world),
                "traffic": traffic,
                "traffic_source": traffic_src,
                "traffic_detail": traffic_rec,
                "kernel": {"uniform": "crc32_rows_kernel",
                           "ragged": "crc32_packed_kernel (+count/scan/plan)" if args.ragged_path == "packed"
                           else ("the dense span step: dense_plan + dense_decide + crc32_rows_kernel (rows pass, "
                                 "exits at once) + crc32_rows_kernel (span pass) + dense_fold, timed as one step"
                                 if os.environ.get("RPCCRC_DENSE", "1") != "0" and args.ragged_path in ("auto", "rows")
                                 else "crc32_rows_kernel"),
                           "large": "crc32_rows_kernel (+chunk combine)"}[w.kind],
                "median_source": median_src,
                # the achieved rate against a streaming read of the
                # same buffer on the same GPU, measured in this run: the rows
                # kernel's own dealing and loads with no CRC work, in blocks
                # alternating with blocks of product steps (stream_read_probe)
                # (both numerators, named) -- the interleaved
                # product blocks (same protocol and clock as the probe's) and
                # the headline achieved rate of the timed region
                "frac_of_stream_read": (round(extra["stream_read_probe"]["product_interleaved_GBps"]
                                              / extra["stream_read_probe"]["rows_dealing_GBps"], 4)
                                        if "product_interleaved_GBps" in extra.get("stream_read_probe", {}) else None),
                "frac_of_stream_read_numerator": "product_interleaved_GBps",
                "frac_of_stream_read_achieved": (round(w.algo_bytes / tr["kernel_s"] / 1e9
                                                       / extra["stream_read_probe"]["rows_dealing_GBps"], 4)
                                                 if "rows_dealing_GBps" in extra.get("stream_read_probe", {}) else None),
            },
            # the reference crc.c on the host's cores: timed on rank 0 at N = 1 only
            # (an N > 1 run shares the host among N ranks)
            "cpu_baseline": cpu if world == 1 else None,
            # every rank's first bodies against the reference crc.c
            "ranks_crc_ok": chk["ranks_ok"] == world,
            "ranks_crc_check": chk,
            "prewarm": {"seconds": args.prewarm_s, "steps": prewarm_steps},
            "device": rpc_amd.device_info(),
            "extra": extra,
        }
        print(json.dumps(line), flush=True)
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
