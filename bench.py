#!/usr/bin/env python3
"""Headline benchmark: BN256 aggregate-signature verifications/s at batch 4096.

Headline workload (BASELINE.json configs[2]): one
step = 4096 incoming Handel multisignatures verified against a 4000-key
registry resident on the GPU, as processing.go:342-368 verifySignature does
for each of them — the bitset-driven PublicKey.Combine fold over the level's
registry range, then PublicKey.VerifySignature (bn256/go/bn256.go:82-94).
Requests are a random node's random Handel level (partitioner rangeLevel), a
bitset of density U[0.5, 1], the aggregate signature of the set bits, 1/8 of
the aggregates tampered. Inputs (requests, bitset words, signatures) are
resident in HBM; verdict codes are written to HBM, packed into a bitset and
all-gathered over RCCL (the only cross-GPU traffic). The verifier serves a
continuous stream of such batches: four are in flight at a time on the
context's lanes (hg_lane_submit_device: own streams and workspaces over the
one registry and table set, the unpadded pairing kernel), so one batch's
pairing waves share the SIMDs with the next one's and each batch's fold,
comparison and launch gaps hide behind the others' pairing kernels
(--inflight 1: one batch at a time, the `sequential` sub-line).

Sub-lines (never `value`):
  sequential      the headline batch one at a time on the context's stream
  single          config 2: 4096 independent single-signature checks
                  (simul/p2p/aggregator.go:244 verifyPacket)
  full_registry   config 3's VerifyMultiSignature shape: every request spans
                  the whole registry (crypto.go:120-137)
  pipelined       two headline batches in flight on two engine contexts
                  (each with its own tables; the r03 form of the headline)
--committees switches the headline to config 5: each rank is one committee of
4096 signers (its own 4096-key registry) verifying 4096 multisignatures.

Multi-GPU: one process per GPU (torchrun), every rank verifies its own batch
(weak scaling); value = all ranks' checks / max-over-ranks wall time.
Prints ONE JSON line on rank 0.
"""

from __future__ import annotations

import argparse
import json
import os
import platform
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from handel_amd import _lib  # noqa: E402
from handel_amd.distributed import gather_verdicts, pack_verdicts  # noqa: E402
from handel_amd.engine import REQ_DTYPE, DeviceLane, Engine  # noqa: E402

LIB_MESSAGE = b"Everything that is beautiful and noble is the product of reason and calculation."
ORDER = 65000549695646603732796438742359905742570406053903786389881062969044166799969
P = 65000549695646603732796438742359905742825358107623003571877145026864184071783
G1_GEN_BYTES = (1).to_bytes(32, "big") + (P - 2).to_bytes(32, "big")

# Algorithmic work, pinned by tests/test_oracle.py against
# the oracle's op counter (oracle/bn256_ref.c, Karatsuba tower formulas).
# The reference's two-pairing check as one multi-Miller loop over 6u+2 (pk
# lines on the fly, x/crypto's G2Base lines from a table) and x/crypto's final
# exponentiation (fast=2): the work credited by `effective_rate`.
FPMUL_REFERENCE_CHECK = 25271
# The same check as the GPU runs it since r03 (fast=3): the G2Base lines
# normalised (a = 1) and the Fuentes-Castaneda hard part: k_verify's work.
FPMUL_PER_CHECK = 23999
# one G2 mixed addition (madd-2007-bl: 7M2 + 4S2, Fp2 products as 3 Fp products)
FPMUL_PER_G2_ADD = 29
# The GT path (handel_amd/csrc/bn256_gt.hip) runs less than the reference
# algorithm: per check ONE pairing (G2Base at -sig, normalised table lines)
# and its final exponentiation — the oracle's fast=3 count with the pk side
# switched off (tests/test_oracle.py pins it; 19308 with x/crypto's lines and
# chain) — plus one Fp12 product per window-table term of the fold (Karatsuba
# tower: 3 Fp6 x 6 Fp2 x 3 Fp products).
FPMUL_PER_SIG_PAIRING = 18036
FPMUL_PER_GT_MUL = 54
# u32 x u32 multiply-adds per Fp multiplication (8-limb CIOS: 2*8^2 + 8)
MADS_PER_FPMUL = 136
# Peak v_mad_u64_u32 rate, measured by tools/intrate.hip on MI355X with 8
# waves per SIMD (profiles/r01_intrate.jsonl: 34.95 T/s; half the VALU rate:
# 256 CU x 4 SIMD x 32 lanes x 2.4 GHz / 2 = 39.3 T/s spec-derived).
P_MAD_TOPS = 34.95
# HBM3E peak (MI355X_MICROARCH.md: 8.0 TB/s spec, 6.29 measured)
P_HBM_GBS = 8000.0


def seeded_scalars(n: int, seed: int) -> bytes:
    """n secret keys in [1, n) from a seeded generator (RandomG2 rejection rule)."""
    rng = np.random.default_rng(seed)
    out = bytearray()
    while len(out) < 32 * n:
        k = int.from_bytes(rng.bytes(32), "big")
        if 0 < k < ORDER:
            out += k.to_bytes(32, "big")
    return bytes(out)


def _tamper(eng: Engine, sigs: bytearray, n: int) -> np.ndarray:
    """sig + G1 for every 8th signature; expected codes."""
    idx = list(range(0, n, 8))
    bad, codes = eng.combine_g1(b"".join(bytes(sigs[64 * i:64 * i + 64]) for i in idx), G1_GEN_BYTES * len(idx))
    assert not codes.any()
    for j, i in enumerate(idx):
        sigs[64 * i:64 * i + 64] = bad[64 * j:64 * j + 64]
    expect = np.zeros(n, dtype=np.int32)
    expect[idx] = 1
    return expect


def make_batch(eng: Engine, n: int, seed: int):
    """Config 2: n independent (pk, sig) pairs on lib.Message, 1/8 tampered."""
    kb = seeded_scalars(n, seed)
    pks = eng.keygen(kb)
    sigs = bytearray(eng.sign(kb))
    expect = _tamper(eng, sigs, n)
    return pks, bytes(sigs), expect


def make_aggregate_batch(eng: Engine, n_reg: int, n: int, seed: int, full: bool = False):
    """a registry of n_reg keys (loaded into `eng`)
    and n incoming multisignatures as Handel's evaluator receives them: for
    each, a random node's random non-empty level (partitioner rangeLevel,
    partitioner.go:133-178), a bitset of density U[0.5, 1.0] over the level's
    registry range, and the aggregate signature of the set bits (sum of the
    secret keys times H(msg)); 1/8 of the aggregates tampered (+ G1).
    full=True: every request spans the whole registry (crypto.go:120-137)."""
    from handel_amd.partitioner import bits_to_words, level_sizes

    rng = np.random.default_rng(seed)
    kb = seeded_scalars(n_reg, seed)
    reg = eng.keygen(kb)
    assert not eng.registry_load(reg).any()
    limbs = np.frombuffer(kb, dtype=">u4").reshape(n_reg, 8)[:, ::-1].astype(np.int64)  # LE 32-bit limbs
    reqs, words, scalars, signers = [], [], bytearray(), []
    nodes = rng.integers(0, n_reg, size=n)
    for i in range(n):
        if full:
            lo, hi = 0, n_reg
        else:
            levels = level_sizes(int(nodes[i]), n_reg)
            _, lo, hi = levels[rng.integers(len(levels))]
        bits = rng.random(hi - lo) < rng.uniform(0.5, 1.0)
        bits[rng.integers(hi - lo)] = True
        signers.append(int(bits.sum()))
        col = limbs[lo:hi][bits].sum(axis=0)
        k = sum(int(v) << (32 * j) for j, v in enumerate(col)) % ORDER
        w = bits_to_words(bits)
        reqs.append((lo, hi - lo, hi - lo, len(words)))
        words.extend(int(x) for x in w)
        scalars += k.to_bytes(32, "big")
    sigs = bytearray(eng.sign(bytes(scalars)))
    expect = _tamper(eng, sigs, n)
    return (np.array(reqs, dtype=REQ_DTYPE), np.array(words, dtype=np.uint64), bytes(sigs), expect,
            np.array(signers), reg)


def requests_as_packets(reqs, words, sigs: bytes, n_reg: int, seed: int):
    """The wire packets (net.go:34-44) that carry these aggregate requests to
    a receiving instance: for request i, a receiver whose level range is the
    request's (the sibling block of the range), that level, a sender inside
    the range, and the MultiSignature marshal of its bitset and signature
    (crypto.go:65-82). Returns (pool, hg_packet records)."""
    from handel_amd import partitioner as HP
    from handel_amd.packets import Packet, pack_packets

    rng = np.random.default_rng(seed)
    pkts, recv = [], []
    for i, (off, bitlen, size, woff) in enumerate(reqs.tolist()):
        bits = HP.words_to_bits(words[woff:woff + (bitlen + 63) // 64], bitlen)
        for k in range(HP.log2_ceil(n_reg)):
            node = off ^ (1 << k)
            if node < n_reg:
                try:
                    if HP.range_level(node, n_reg, k + 1) == (off, off + size):
                        break
                except HP.PartitionerError:
                    pass
        else:
            raise ValueError(f"request {i} is not a Handel level range")
        pkts.append(Packet(int(rng.integers(off, off + size)), k + 1,
                           HP.multisig_marshal(bits, sigs[64 * i:64 * i + 64])))
        recv.append(node)
    return pack_packets(pkts, recv)


def gt_fold_terms(reqs, words, n_reg: int) -> int:
    """GT-table terms the fold multiplies for this batch (host restatement of
    bn256_gt.hip k_gt_plan: nonzero 16-key windows of the bitset in
    registry-aligned windows, or of its complement inside an aligned Handel
    block when that has fewer, plus the block's own term)."""
    levels = max(1, (n_reg - 1).bit_length())
    total = 0
    for off, bitlen, size, woff in reqs.tolist():
        nw = (bitlen + 63) // 64
        v = 0
        for i, w in enumerate(words[woff:woff + nw].tolist()):
            v |= int(w) << (64 * i)
        v &= (1 << bitlen) - 1
        if v == 0:
            continue
        sh = off & 15

        def nz(x):
            x <<= sh
            return sum(1 for j in range(0, sh + bitlen, 16) if (x >> j) & 0xffff)

        k = (bitlen - 1).bit_length() if bitlen > 1 else 0
        aligned = k <= levels and off % (1 << k) == 0 and (bitlen == 1 << k or off + bitlen == n_reg)
        m_set = nz(v)
        m_unset = nz(((1 << bitlen) - 1) ^ v)
        total += (m_unset + 1) if (aligned and k > 0 and m_unset < m_set) else m_set
    return total


def pmc_traffic(pattern: str):
    """HBM bytes per launch of the kernels matching `pattern`, summed, from the
    committed PMC summaries (profiles/*_pmc.csv, tools/rocpd_summary.py):
    FETCH_SIZE x 2 (gfx950 correction) + WRITE_SIZE per dispatch. Each kernel
    is taken from the newest summary holding nonzero counters for it (a pass
    can come back empty for a kernel; the pairing kernels' counters do not
    depend on the batch's bitsets, so any profile of a 4096-check launch
    serves)."""
    import csv
    import glob
    import re

    # newest = highest round/version in the name (mtimes are not kept by git or the box snapshot)
    def key(path):
        return [int(t) if t.isdigit() else t for t in re.split(r"(\d+)", os.path.basename(path))]

    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "*_pmc.csv")), key=key)

    def read(path):
        vals = {}
        with open(path) as f:
            for row in csv.DictReader(f):
                if re.search(pattern, row["kernel"]) and row["counter"] in ("FETCH_SIZE", "WRITE_SIZE"):
                    vals.setdefault(row["kernel"], {})[row["counter"]] = float(row["avg"])
        return vals

    tables = [(path, read(path)) for path in reversed(files)]
    tables = [(p, v) for p, v in tables if v]
    if not tables:
        return None, None
    # the newest summary names the kernels; each one's bytes from the newest
    # summary with nonzero counters for that kernel
    got, srcs = {}, set()
    for name in tables[0][1]:
        for path, vals in tables:
            v = vals.get(name, {})
            if v.get("FETCH_SIZE", 0) > 0 and "WRITE_SIZE" in v:
                got[name] = int((2 * v["FETCH_SIZE"] + v["WRITE_SIZE"]) * 1024)
                srcs.add(os.path.relpath(path, ROOT))
                break
    if not got:
        return None, None
    return sum(got.values()), ", ".join(sorted(srcs))


def rocprof_kernel_us(pattern: str):
    """Average duration (us) of the kernels matching `pattern` in the newest
    committed kernel-trace summary of the DRIVER's invocation
    (profiles/*_driver_ktrace_stats.csv: rocprofv3 --kernel-trace --stats of
    `bench.py --steps 20 --warmup 5`, tools/gpu_pin.sh), summed over the
    matching kernels; (None, None) if no summary holds them."""
    import csv
    import glob
    import re

    def key(path):
        return [int(t) if t.isdigit() else t for t in re.split(r"(\d+)", os.path.basename(path))]

    for path in sorted(glob.glob(os.path.join(ROOT, "profiles", "*_driver_ktrace_stats.csv")), key=key, reverse=True):
        with open(path) as f:
            rows = [r for r in csv.DictReader(f) if re.search(pattern, r["kernel"])]
        if rows:
            return sum(float(r["avg_us"]) for r in rows), os.path.relpath(path, ROOT)
    return None, None


def rocprof_busy_ms(inflight: int):
    """Per-step device-busy ms of the headline (the union of every kernel
    interval inside the timed region / steps) from the newest committed
    summary of a kernel trace of the driver's invocation with the same batches
    in flight (profiles/*_driver_busy.json, tools/busy_summary.py); (None,
    None) if there is none."""
    import glob
    import re

    def key(path):
        return [int(t) if t.isdigit() else t for t in re.split(r"(\d+)", os.path.basename(path))]

    for path in sorted(glob.glob(os.path.join(ROOT, "profiles", "*_driver_busy.json")), key=key, reverse=True):
        with open(path) as f:
            d = json.load(f)
        if d.get("batches_in_flight") == inflight and d.get("busy_ms_per_step"):
            return float(d["busy_ms_per_step"]), os.path.relpath(path, ROOT)
    return None, None


def _cgroup_quota_cpus():
    """CPUs of CPU time the cgroup grants this process (cgroup v2 cpu.max
    "quota period"), None when unlimited or unreadable."""
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
        return None if q == "max" else int(q) / int(per)
    except (OSError, ValueError):
        return None


def host_cpu():
    """(threads to use, description): every core the process can actually run
    on — the affinity mask, capped by the cgroup's CPU quota when there is one
    (a quota of 16 CPUs lets 256 threads run no faster than 16 cores).
    OMP_NUM_THREADS is reported but not used."""
    try:
        aff = len(os.sched_getaffinity(0))
    except AttributeError:  # pragma: no cover
        aff = os.cpu_count() or 1
    quota = _cgroup_quota_cpus()
    threads = min(aff, max(1, int(quota + 0.999))) if quota else aff
    model = platform.processor() or "unknown"
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:  # pragma: no cover
        pass
    return threads, {"nproc": os.cpu_count(), "affinity": aff, "cgroup_quota_cpus": quota,
                     "omp_num_threads": os.environ.get("OMP_NUM_THREADS"), "model": model}


def _host_scale(per_core: float, info: dict) -> dict:
    """Extrapolations (never the measured value): the whole host's cores at the
    measured per-core rate (the checks are independent), and one GPU's share
    of them (8 GPUs per host)."""
    cores = info.get("affinity") or info.get("nproc") or 1
    return {"host_all_cores_extrapolated": round(per_core * cores, 1),
            "host_share_per_gpu_extrapolated": round(per_core * cores / 8, 1)}


def _timed_repeats(run, min_wall: float):
    """Runs run() until min_wall seconds have passed; (calls, seconds)."""
    calls, t0 = 0, time.perf_counter()
    while True:
        run()
        calls += 1
        dt = time.perf_counter() - t0
        if dt >= min_wall:
            return calls, dt


def cpu_baseline_single(pks: bytes, sigs: bytes, expect: np.ndarray, min_wall: float = 3.0):
    """Config 2 on the reference algorithm restated in C (oracle/bn256_ref.c,
    'port'): two full pairings + GT compare per check."""
    from oracle import ref_lib as R

    threads, info = host_cpu()
    n = len(expect)
    R.set_rehash(True)  # hashedMessage on every check, as VerifySignature does
    try:
        codes = R.verify_batch(LIB_MESSAGE, pks, sigs, nthreads=threads, fast=0)
        assert np.array_equal(codes, expect), "CPU oracle verdicts differ"
        calls, dt = _timed_repeats(lambda: R.verify_batch(LIB_MESSAGE, pks, sigs, nthreads=threads, fast=0),
                                   min_wall)
    finally:
        R.set_rehash(False)
    v = n * calls / dt
    return {"value": round(v, 1), "unit": "verifications/s", "cores": threads, "kind": "port",
            "per_core": round(v / threads, 1), **info, **_host_scale(v / threads, info),
            "sample": f"the same {n} checks (lib.Message, 1/8 tampered) x {calls}, reference algorithm "
                      f"(hashedMessage + 2 pairings + GT compare per check), {threads} threads, {dt:.2f} s wall"}


def cpu_baseline_aggregate(reg: bytes, reqs, words, sigs: bytes, expect: np.ndarray, n_sample: int,
                           min_wall: float = 3.0):
    """Config 3 on the reference algorithm restated in C: per request the
    PublicKey.Combine fold over every set bit (one G2 addition each, as
    processing.go:355-363), then two pairings + GT compare. Measured on every
    usable core for >= min_wall seconds (the sample repeated); when the
    affinity mask holds more threads than the cgroup quota lets run, a second
    measurement with one thread per affinity core shows what the whole mask
    delivers."""
    from oracle import ref_lib as R

    threads, info = host_cpu()
    m = min(n_sample, len(reqs))
    r = reqs[:m]

    def run(nt):
        return R.verify_aggregate(LIB_MESSAGE, reg, r["offset"], r["bitlen"], r["level_size"], words,
                                  r["word_offset"].astype(np.uint64), sigs[:64 * m], nthreads=nt, fast=0)

    R.set_rehash(True)  # hashedMessage on every check, as VerifySignature does
    try:
        assert np.array_equal(run(threads), expect[:m]), "CPU oracle verdicts differ"
        calls, dt = _timed_repeats(lambda: run(threads), min_wall)
        aff_run = None
        if info["affinity"] > threads:
            acalls, adt = _timed_repeats(lambda: run(info["affinity"]), min_wall)
            aff_run = {"threads": info["affinity"], "value": round(m * acalls / adt, 1), "wall_s": round(adt, 2),
                       "note": "one thread per core of the affinity mask; the cgroup quota "
                               f"({info['cgroup_quota_cpus']} CPUs) bounds what they can run"}
    finally:
        R.set_rehash(False)
    v = m * calls / dt
    out = {"value": round(v, 1), "unit": "verifications/s", "cores": threads, "kind": "port",
           "per_core": round(v / threads, 1), **info, **_host_scale(v / threads, info),
           "sample": f"the first {m} requests of the batch x {calls} (same registry, bitsets, signatures), reference "
                     f"algorithm (one G2 addition per set bit + hashedMessage + 2 pairings + GT compare), "
                     f"{threads} threads, {dt:.2f} s wall"}
    if aff_run:
        out["affinity_run"] = aff_run
    return out


def clock_marks() -> dict:
    """Now, in ns, on every host clock a profiler's timestamps may be taken on."""
    return {"monotonic": time.clock_gettime_ns(time.CLOCK_MONOTONIC),
            "boottime": time.clock_gettime_ns(time.CLOCK_BOOTTIME),
            "realtime": time.clock_gettime_ns(time.CLOCK_REALTIME)}


def cpu_baseline_on_rank0(rank: int, dist: bool, args, run):
    """The CPU baseline beside every world size (north_star: the CPU figure
    next to the GPU's, in the same run): rank 0 runs run() after the timed
    regions while the other ranks wait at a barrier, so it never overlaps a
    timed step and every rank leaves together. None when --no-cpu."""
    cpu = None
    if rank == 0 and not args.no_cpu:
        try:
            cpu = run()
        except Exception as e:  # pragma: no cover - reported, not fatal
            cpu = {"error": str(e)}
    if dist:
        import torch.distributed as tdist

        tdist.barrier()
    return cpu


def cpu_probe_workload(n_reg: int = 8, n: int = 4):
    """A tiny config-3-shaped workload made with the CPU oracle (the
    --cpu-probe test hook: no GPU): a registry of n_reg seeded keys, n
    multisignatures over the whole registry, every 2nd tampered."""
    from oracle import ref_lib as R

    rng = np.random.default_rng(5)
    kb = seeded_scalars(n_reg, 5)
    ks = [int.from_bytes(kb[32 * i:32 * i + 32], "big") for i in range(n_reg)]
    reg = R.g2_scalar_base(kb)
    reqs, words, sigs, expect = [], [], b"", []
    for i in range(n):
        bits = rng.random(n_reg) < 0.7
        bits[i % n_reg] = True
        sk = sum(k for k, b in zip(ks, bits) if b) % ORDER
        sig = R.sign(LIB_MESSAGE, sk.to_bytes(32, "big"))
        if i % 2:
            sig = R.g1_add(sig, G1_GEN_BYTES)
        reqs.append((0, n_reg, n_reg, len(words)))
        words.append(int(sum(1 << j for j in range(n_reg) if bits[j])))
        sigs += sig
        expect.append(i % 2)
    from handel_amd.engine import REQ_DTYPE as RD

    return reg, np.array(reqs, dtype=RD), np.array(words, dtype=np.uint64), sigs, np.array(expect, dtype=np.int32)


class Timer:
    """Barrier + synchronize on both sides of the timed region, max over ranks
    (every rank's own time is kept in `rank_times`)."""

    def __init__(self, dev, dist, coll_dev, world: int = 1):
        self.dev, self.dist, self.coll_dev, self.world = dev, dist, coll_dev, world
        self.rank_times = []
        self.marks = {}

    def _sync(self):
        if self.dev.type == "cuda":  # (a CPU device: the gloo test of this class)
            torch.cuda.synchronize(self.dev)

    def prewarm(self, step, seconds: float) -> int:
        """Untimed steps for `seconds` of wall time before the warmup steps, so
        the GPU's clocks have settled whatever the warmup count; returns the
        steps run (reported in the line)."""
        k, t0 = 0, time.perf_counter()
        if self.dist:
            # every rank runs the same number of steps (a step holds a
            # collective): the ranks agree after each step, and stop as soon
            # as one rank's time is up
            import torch.distributed as tdist

            go = torch.ones(1, dtype=torch.int32, device=self.coll_dev)
            while seconds > 0:
                step()
                k += 1
                go.fill_(1 if time.perf_counter() - t0 < seconds else 0)
                tdist.all_reduce(go, op=tdist.ReduceOp.MIN)
                if int(go.item()) == 0:
                    break
            self._sync()
            return k
        while time.perf_counter() - t0 < seconds:
            step()
            k += 1
            if k % 16 == 0:
                self._sync()
        self._sync()
        return k

    def run(self, step, steps: int, warmup: int) -> float:
        for _ in range(warmup):
            step()
        self._sync()
        if self.dist:
            import torch.distributed as tdist
            tdist.barrier()
        self._sync()
        m0 = clock_marks()
        t0 = time.perf_counter()
        for _ in range(steps):
            step()
        self._sync()
        m1 = clock_marks()
        # the timed region on the host clocks a kernel trace may use
        # (tools/busy_summary.py finds the step kernels inside it)
        self.marks = {k: [m0[k], m1[k]] for k in m0}
        if self.dist:
            tdist.barrier()
        dt = time.perf_counter() - t0
        self.rank_times = [dt]
        if self.dist:
            t = torch.tensor([dt], dtype=torch.float64, device=self.coll_dev)
            every = [torch.zeros_like(t) for _ in range(self.world)]
            tdist.all_gather(every, t)
            self.rank_times = [float(x.item()) for x in every]
            dt = max(self.rank_times)
        return dt


def _dev_bytes(b: bytes, dev):
    return torch.frombuffer(bytearray(b), dtype=torch.uint8).to(dev)


class AggregateWorkload:
    """Config 3 (or 5): n multisignatures on an n_reg-key registry per rank."""

    def __init__(self, eng: Engine, n_reg: int, n: int, seed: int, dev, stream, full: bool = False,
                 prepare: bool = True):
        self.eng, self.n, self.stream = eng, n, stream
        (self.reqs, self.words, self.sigs, self.expect, self.signers,
         self.reg) = make_aggregate_batch(eng, n_reg, n, seed, full=full)
        # the per-(message, registry) GT tables, built outside the timed region
        # (once per Handel run: the message and the registry are fixed)
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        if prepare:
            assert eng.prepare_aggregate() == 0
        self.setup_ms = (time.perf_counter() - t0) * 1e3
        self.terms = gt_fold_terms(self.reqs, self.words, n_reg)
        self.d_reqs = _dev_bytes(self.reqs.tobytes(), dev)
        self.d_words = _dev_bytes(self.words.tobytes(), dev)
        self.d_sigs = _dev_bytes(self.sigs, dev)
        self.d_codes = torch.zeros(n, dtype=torch.int32, device=dev)
        self.d_bits = torch.zeros((n + 7) // 8, dtype=torch.uint8, device=dev)
        # algorithmic Fp multiplications of the batch: one G2 addition per set
        # bit (the reference's fold) + one pairing check per request
        self.fpmul = int(self.signers.sum()) * FPMUL_PER_G2_ADD + n * FPMUL_REFERENCE_CHECK

    def submit(self, eng=None, codes=None, stream=None):
        eng = self.eng if eng is None else eng
        codes = self.d_codes if codes is None else codes
        stream = self.stream if stream is None else stream
        eng.verify_aggregate_device(self.d_reqs.data_ptr(), self.n, self.d_words.data_ptr(), self.d_sigs.data_ptr(),
                                    codes.data_ptr(), 0, stream.cuda_stream)

    def pack(self):
        self.eng.pack_verdicts_device(self.d_codes.data_ptr(), self.n, self.d_bits.data_ptr(), self.stream.cuda_stream)

    def submit_bits(self):
        """submit + pack in one submission (hg_verify_aggregate_device_bits)."""
        self.eng.verify_aggregate_device_bits(self.d_reqs.data_ptr(), self.n, self.d_words.data_ptr(),
                                              self.d_sigs.data_ptr(), self.d_codes.data_ptr(), self.d_bits.data_ptr(),
                                              self.stream.cuda_stream)

    def check(self, codes=None):
        got = (codes if codes is not None else self.d_codes).cpu().numpy()
        assert np.array_equal(got, self.expect), \
            f"GPU verdicts differ from the expected pattern at {np.flatnonzero(got != self.expect)[:8]}"


class SingleWorkload:
    """Config 2: n independent single-signature checks per rank."""

    def __init__(self, eng: Engine, n: int, seed: int, dev, stream):
        self.eng, self.n, self.stream = eng, n, stream
        self.pks, self.sigs, self.expect = make_batch(eng, n, seed)
        self.d_pks = _dev_bytes(self.pks, dev)
        self.d_sigs = _dev_bytes(self.sigs, dev)
        self.d_codes = torch.zeros(n, dtype=torch.int32, device=dev)
        self.d_bits = torch.zeros((n + 7) // 8, dtype=torch.uint8, device=dev)
        self.fpmul = n * FPMUL_PER_CHECK

    def submit(self):
        self.eng.verify_batch_device(self.d_pks.data_ptr(), self.d_sigs.data_ptr(), self.n, self.d_codes.data_ptr(),
                                     self.stream.cuda_stream)

    def pack(self):
        self.eng.pack_verdicts_device(self.d_codes.data_ptr(), self.n, self.d_bits.data_ptr(), self.stream.cuda_stream)

    def check(self):
        got = self.d_codes.cpu().numpy()
        assert np.array_equal(got, self.expect), f"GPU verdicts differ at {np.flatnonzero(got != self.expect)[:8]}"


def handel_run_volume(dev, stream, device: int, n_reg: int = 2000, requests: int = 90112, batch: int = 4096,
                      seed: int = 2468):
    """A Handel run's verification volume on a FRESH (message, registry), the
    table builds inside the timed region: config 4 is 2000 nodes x 45.2 checks
    per node ~ 90 k requests of one message (simul/plots/csv/
    handel_0failing_99thr.csv:7; H is fixed per run, bn256/go/bn256.go:210-218).
    'policy': the engine's own volume policy (G2 fold first, the 8-key GT
    tables once 16384 requests have come in); 'prepared': hg_prepare_aggregate
    (the 16-key tables) first. The batch of 4096 config-4-shaped requests is
    resubmitted requests/batch times (the policy counts requests)."""
    out = {"requests": requests, "batch": batch, "registry": n_reg,
           "workload": f"{n_reg}-key registry, random node/level, bitset density U[0.5,1], 1/8 tampered"}
    for mode in ("policy", "prepared"):
        e = Engine(device=device, flavor="go")
        try:
            e.set_aggregate_level(-1)
            assert e.set_message(LIB_MESSAGE) == 0
            wl = AggregateWorkload(e, n_reg, batch, seed=seed, dev=dev, stream=stream, prepare=False)
            torch.cuda.synchronize(dev)
            t0 = time.perf_counter()
            assert not e.registry_load(wl.reg).any()  # a fresh registry: block/window sums, G2 membership
            load_ms = (time.perf_counter() - t0) * 1e3
            torch.cuda.synchronize(dev)
            t0 = time.perf_counter()
            if mode == "prepared":
                assert e.prepare_aggregate() == 0
            for _ in range(requests // batch):
                wl.submit(eng=e)
            torch.cuda.synchronize(dev)
            dt = time.perf_counter() - t0
            wl.check()
            out[mode] = {"ms": round(dt * 1e3, 3), "value": round(requests // batch * batch / dt, 1),
                         "unit": "verifications/s", "tables_at_end": e.aggregate_tables()}
            out["registry_load_ms"] = round(load_ms, 3)
        finally:
            e.close()
    return out


def packet_intake(eng: Engine, head, n_reg: int, dev, stream, timer, args, world: int):
    """Handel.NewPacket's parse step on the device (hg_parse_packets_device):
    the headline's 4096 requests as the wire packets that carry them, in HBM;
    'parse' = packets -> verification requests, 'parse_verify' = packets ->
    verdicts (parse, then the headline's GT submission on the parsed slots)."""
    n = len(head.reqs)
    pool, recs = requests_as_packets(head.reqs, head.words, head.sigs, n_reg, seed=99)
    stride = eng.packet_stride_words()
    d_pool = _dev_bytes(pool, dev)
    d_pkts = _dev_bytes(recs.tobytes(), dev)
    d_reqs = torch.zeros(2 * n * REQ_DTYPE.itemsize, dtype=torch.uint8, device=dev)
    d_words = torch.zeros(2 * n * stride, dtype=torch.int64, device=dev)
    d_sigs = torch.zeros(2 * n * 64, dtype=torch.uint8, device=dev)
    d_pcodes = torch.zeros(2 * n, dtype=torch.int32, device=dev)
    codes = torch.zeros(n, dtype=torch.int32, device=dev)
    s = stream.cuda_stream

    def parse():
        eng.parse_packets_device(d_pool.data_ptr(), len(pool), d_pkts.data_ptr(), n, stride, d_reqs.data_ptr(),
                                 d_words.data_ptr(), d_sigs.data_ptr(), d_pcodes.data_ptr(), s)

    def parse_verify():
        parse()
        eng.verify_aggregate_device(d_reqs.data_ptr(), n, d_words.data_ptr(), d_sigs.data_ptr(), codes.data_ptr(), 0,
                                    s)

    pdt = timer.run(parse, args.steps, args.warmup)
    assert (d_pcodes[:n] == 0).all().item(), "every headline packet parses"
    vdt = timer.run(parse_verify, args.steps, args.warmup)
    assert np.array_equal(codes.cpu().numpy(), head.expect), "verdicts from parsed packets"
    # the parse kernel alone, HIP events on its stream
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    reps = 20
    ev[0].record(stream)
    for _ in range(reps):
        parse()
    ev[1].record(stream)
    torch.cuda.synchronize(dev)
    k_ms = ev[0].elapsed_time(ev[1]) / reps
    moved = len(pool) + recs.nbytes + 2 * n * (REQ_DTYPE.itemsize + 8 * stride + 64 + 4)
    achieved = moved / (k_ms * 1e-3) / 1e9
    return {"metric": "Handel packets parsed/sec (batch 4096)", "value": round(n * args.steps * world / pdt, 1),
            "unit": "packets/s", "ms_per_step": round(pdt / args.steps * 1e3, 4),
            "parse_verify": {"value": round(n * args.steps * world / vdt, 1), "unit": "verifications/s",
                             "ms_per_step": round(vdt / args.steps * 1e3, 4),
                             "what": "wire packets in HBM -> parse -> GT submission -> verdicts"},
            "workload": f"the headline's {n} requests as wire packets ({len(pool)} B), receiver and level per packet",
            "roofline": {"bound": "hbm", "achieved": round(achieved, 2), "peak": P_HBM_GBS, "unit": "GB/s",
                         "frac": round(achieved / P_HBM_GBS, 4), "traffic": None, "kernel": "k_parse_packets",
                         "kernel_ms": round(k_ms, 4),
                         "work": f"bytes per launch: pool {len(pool)} + records {recs.nbytes} + 2 slots x "
                                 f"(request 16 + {stride} words x 8 + signature 64 + code 4) per packet",
                         "note": "a 4096-packet launch is launch/latency bound; the fraction says so"}}


def batch_latency(eng: Engine, head, dev, sizes=(32, 128, 512, 4096), reps: int = 15):
    """The small-batch floor: wall time of ONE batch of n requests, submitted
    alone and waited for (the first n requests of the headline batch). 'device':
    inputs resident in HBM (hg_verify_aggregate_device + synchronize); 'host':
    host buffers in and codes out (hg_verify_aggregate: what a batcher or the
    verifier service pays per batch). Median over reps. A batch of n <= 4096
    checks holds one pairing wave per SIMD at most, so its latency is one
    pairing kernel whatever n is."""
    out = {}
    s = torch.cuda.Stream(dev)
    for m in sizes:
        m = min(m, head.n)
        codes = torch.zeros(m, dtype=torch.int32, device=dev)
        dev_t, host_t = [], []
        r = head.reqs[:m]
        for _ in range(reps):
            t0 = time.perf_counter()
            eng.verify_aggregate_device(head.d_reqs.data_ptr(), m, head.d_words.data_ptr(), head.d_sigs.data_ptr(),
                                        codes.data_ptr(), 0, s.cuda_stream)
            s.synchronize()
            dev_t.append(time.perf_counter() - t0)
        assert np.array_equal(codes.cpu().numpy(), head.expect[:m])
        for _ in range(reps):
            t0 = time.perf_counter()
            got = eng.verify_aggregate(r, head.words, head.sigs[:64 * m])
            host_t.append(time.perf_counter() - t0)
        assert np.array_equal(got, head.expect[:m])
        d, h = float(np.median(dev_t)) * 1e3, float(np.median(host_t)) * 1e3
        out[str(m)] = {"device_ms": round(d, 4), "host_ms": round(h, 4),
                       "verif_per_s_device": round(m / d * 1e3, 1), "verif_per_s_host": round(m / h * 1e3, 1)}
    return out


def under_profiler() -> bool:
    """A rocprofv3 run: its tool library is preloaded into this process and
    every process started from it."""
    return "rocprofiler" in os.environ.get("LD_PRELOAD", "") or any(k.startswith("ROCPROF") for k in os.environ)


def config4_proxy(model: str, timeout: int = 180, extra=()):
    """Config 4's verification load in simul's single-host process layout
    (tests/native/handel_proxy.c): 8 processes x 250 Handel instances x 45
    checks on a 2000-key registry, one check in flight per instance, every
    verdict checked against the expected one. model 'service': one GPU-owning
    verifier process (hg_service_*, 8 lanes) and 8 client processes that load
    only libhandel_client.so; 'contexts': every process its own context, GT
    tables and batcher (the r03 layout). Not Handel completion time.

    The proxy runs in a session of its own: on a timeout the whole process
    group (the proxy and the processes it forked) is killed, and the line
    keeps the tail of what they printed (each process reports its phases on
    stderr), so a stall names the phase it stalled in."""
    import signal
    import subprocess

    from handel_amd import build as B

    args = ["-D", "1", "-P", "1", "-l", "8"] if model == "service" else ["-D", "0", "-P", "1"]
    try:
        pr = subprocess.Popen([B.HANDEL_PROXY, B.LIB, *args, *extra], stdout=subprocess.PIPE, stderr=subprocess.PIPE,
                              text=True, start_new_session=True)
    except OSError as e:  # pragma: no cover - reported, not fatal
        return {"error": str(e)}
    try:
        out, err = pr.communicate(timeout=timeout)
    except subprocess.TimeoutExpired:
        try:
            os.killpg(pr.pid, signal.SIGKILL)  # the group this call started (its own session)
        except ProcessLookupError:  # pragma: no cover
            pass
        out, err = pr.communicate()
        return {"error": f"timed out after {timeout} s (process group killed)", "under_profiler": under_profiler(),
                "stderr_tail": err[-2500:], "stdout_tail": out[-500:]}
    if pr.returncode != 0:
        return {"error": f"rc {pr.returncode}", "stderr_tail": err[-2500:]}
    d = json.loads(out.strip().splitlines()[-1])
    keep = ("model", "procs", "instances_per_proc", "registry", "checks_per_instance", "lanes", "hw_queues",
            "requests", "batches", "mean_batch", "wall_ms", "throughput", "latency_us", "hbm_total_bytes",
            "contexts", "mismatches")
    return {k: d[k] for k in keep if k in d}


def want_config4_proxy(rank: int, world: int, args) -> bool:
    """The config-4 proxy line runs on a one-rank run only (rank 0, world 1),
    and never with --no-service or --no-extra."""
    return rank == 0 and world == 1 and not args.no_service and not args.no_extra


def timed_phases(eng: Engine, run):
    """Runs run() with the engine's HIP-event timing on; returns per-phase
    (mean ms per interval) for verify / aggregate fold / whole submission."""
    eng.timing_enable(True)
    for ph in (_lib.HG_PHASE_VERIFY, _lib.HG_PHASE_AGGREGATE, _lib.HG_PHASE_SUBMIT):
        eng.timing_read_phase(ph)
    run()
    out = {}
    for name, ph in (("verify", _lib.HG_PHASE_VERIFY), ("fold", _lib.HG_PHASE_AGGREGATE),
                     ("submit", _lib.HG_PHASE_SUBMIT)):
        ms, k = eng.timing_read_phase(ph)
        out[name] = ms / k if k else None
    eng.timing_enable(False)
    return out


def roofline(fpmul: int, ms: float, kernel: str, traffic_pattern: str, work: str, rocprof_pattern: str = None):
    """VALU roofline of `fpmul` Fp multiplications over `ms` (HIP events on the
    launch stream). rocprof_pattern: the kernels whose summed rocprof average
    (the driver-invocation profile) gives the same work's `frac_rocprof`."""
    achieved = fpmul * MADS_PER_FPMUL / (ms * 1e-3) / 1e12
    traffic, src = pmc_traffic(traffic_pattern)
    out = {"bound": "valu", "achieved": round(achieved, 3), "peak": P_MAD_TOPS, "unit": "Tmad/s",
           "frac": round(achieved / P_MAD_TOPS, 4), "traffic": traffic, "traffic_unit": "bytes/launch",
           "traffic_source": src, "kernel": kernel, "kernel_ms": round(ms, 4), "work": work}
    if rocprof_pattern:
        us, rsrc = rocprof_kernel_us(rocprof_pattern)
        if us:
            out["rocprof_kernel_ms"] = round(us / 1e3, 4)
            out["frac_rocprof"] = round(fpmul * MADS_PER_FPMUL / (us * 1e-6) / 1e12 / P_MAD_TOPS, 4)
            out["rocprof_source"] = rsrc
    return out


def progress(what: str):
    """One line per phase on stderr (the JSON line stays alone on stdout): a
    long run under a profiler shows it is alive."""
    print(f"[bench {time.strftime('%H:%M:%S')}] {what}", file=sys.stderr, flush=True)


def lanes_rate(eng: Engine, wl, inflight: int, timer, steps: int, warmup: int, dev) -> float:
    """wl's batch with `inflight` batches in flight on the context's lanes, as
    the headline runs (unpadded pairing kernel, each lane ordered on its own
    stream); every lane's last verdicts are checked. Returns the timed seconds."""
    lanes = [DeviceLane(eng, wl.n, pad=False) for _ in range(inflight)]
    codes = [torch.zeros(wl.n, dtype=torch.int32, device=dev) for _ in lanes]
    turn = [0]

    def st():
        i = turn[0] % inflight
        turn[0] += 1
        lanes[i].submit_device(wl.d_reqs.data_ptr(), wl.n, wl.d_words.data_ptr(), wl.d_sigs.data_ptr(),
                               codes[i].data_ptr(), 0, lanes[i].stream)

    try:
        for _ in range(inflight):
            st()
        torch.cuda.synchronize(dev)
        dt = timer.run(st, steps, warmup)
        for c in codes:
            wl.check(c)
    finally:
        for ln in lanes:
            ln.close()
    return dt


def single_stream_rate(single: "SingleWorkload", inflight: int, timer, steps: int, warmup: int, dev, device: int,
                       world: int, coll_dev, dist: bool):
    """Config 2 as a stream, the way the headline runs: `inflight` batches in
    flight, each on a verification context of its own (its stream and
    workspace) in the split form (hg_set_verify_split: the Miller loop on a
    compact team region, so two batches' waves share the SIMDs, then the
    12-lane final exponentiation); each step is one whole batch — verdicts,
    bitset, gather — on its context's stream. Every context's last verdicts
    are checked. Returns the timed seconds."""
    n = single.n
    ctxs = []
    try:
        for _ in range(inflight):
            e = Engine(device=device, flavor="go")
            assert e.set_message(LIB_MESSAGE) == 0
            e.set_verify_split(True)
            ctxs.append((e, torch.cuda.Stream(dev), torch.zeros(n, dtype=torch.int32, device=dev),
                         torch.zeros((n + 7) // 8, dtype=torch.uint8, device=dev),
                         [torch.zeros((n + 7) // 8, dtype=torch.uint8, device=coll_dev) for _ in range(world)]))
        turn = [0]

        def st():
            e, s, codes, bits, gath = ctxs[turn[0] % inflight]
            turn[0] += 1
            with torch.cuda.stream(s):
                e.verify_batch_device(single.d_pks.data_ptr(), single.d_sigs.data_ptr(), n, codes.data_ptr(),
                                      s.cuda_stream)
                e.pack_verdicts_device(codes.data_ptr(), n, bits.data_ptr(), s.cuda_stream)
                gather_verdicts(bits.to(coll_dev) if dist else bits, world, gath)

        torch.cuda.synchronize(dev)
        for _ in range(inflight):
            st()
        torch.cuda.synchronize(dev)
        dt = timer.run(st, steps, warmup)
        for _, _, codes, bits, _ in ctxs:
            got = codes.cpu().numpy()
            assert np.array_equal(got, single.expect), f"config-2 stream verdicts differ at {np.flatnonzero(got != single.expect)[:8]}"
            assert torch.equal(bits, pack_verdicts(codes)), "config-2 stream bitset differs from the codes"
    finally:
        for c in ctxs:
            c[0].close()
    return dt


def _free_port() -> int:
    import socket

    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as so:
        so.bind(("127.0.0.1", 0))
        return so.getsockname()[1]


def launch_ranks(n: int, argv) -> int:
    """`python bench.py --gpus N` outside torchrun: start N rank processes (one
    per GPU) as a CHILD torch.distributed.run on 127.0.0.1 with the same
    arguments, and return its exit code. Called before any HIP call of this
    process (nothing here touches the device), and the ranks are fresh
    processes, never an exec of this one."""
    import subprocess

    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.abspath(__file__), *argv]
    progress(f"launching {n} ranks: {' '.join(cmd[1:6])} ...")
    return subprocess.call(cmd, env=dict(os.environ, HG_BENCH_LAUNCHED="1"))


def world_from_env(gpus):
    """(world, rank, local rank) of this process; SystemExit(2) when --gpus
    names a different world size than the launcher started (the line's n_gpus
    would otherwise not be what was asked for)."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if gpus is not None and gpus != world:
        print(f"bench.py: --gpus {gpus} but the launcher started a world of {world} rank(s)", file=sys.stderr)
        raise SystemExit(2)
    return world, rank, local


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None,
                    help="GPUs (ranks) of this node; outside torchrun N > 1 starts N ranks itself")
    ap.add_argument("--launch-probe", action="store_true",
                    help="test hook: start the ranks, join the process group (gloo, no device), print the "
                         "world each rank saw, exit")
    ap.add_argument("--cpu-probe", action="store_true",
                    help="test hook: start the ranks (gloo, no device), run the CPU baseline's rank-0 leg on a tiny "
                         "oracle-made workload exactly as the bench does after its timed regions, print rank 0's line")
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--batch", type=int, default=4096)
    ap.add_argument("--committees", action="store_true",
                    help="config 5: each rank is one committee of 4096 signers (own 4096-key registry)")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-extra", action="store_true", help="headline only (no single / full / pipelined lines)")
    ap.add_argument("--inflight", type=int, default=None,
                    help="headline: batches in flight on the context's lanes (1: one batch at a time on the "
                         "context's stream; default 4; 1 in the gloo rehearsal)")
    ap.add_argument("--pipeline", type=int, default=2, help="batches in flight for the 'pipelined' line (1: skip)")
    ap.add_argument("--pipeline-overlap", type=int, default=1,
                    help="the pipelined line's contexts run their fold beside the pairing kernel (1) or before it (0)")
    ap.add_argument("--cpu-sample", type=int, default=4096, help="requests in the CPU baseline's sample")
    ap.add_argument("--no-service", action="store_true", help="skip the config-4 process-model lines")
    ap.add_argument("--prewarm", type=float, default=0.3,
                    help="seconds of untimed headline steps before the warmup steps (GPU clocks settle)")
    args = ap.parse_args()
    if "WORLD_SIZE" not in os.environ and (args.gpus or 1) > 1:
        # the driver's `python bench.py --gpus N`: one rank per GPU, started here
        raise SystemExit(launch_ranks(args.gpus, sys.argv[1:]))
    world, rank, local = world_from_env(args.gpus)
    if args.cpu_probe:
        import torch.distributed as tdist

        if world > 1:
            tdist.init_process_group("gloo")
        reg, reqs, words, sigs, expect = cpu_probe_workload()
        cpu = cpu_baseline_on_rank0(rank, world > 1, args, lambda: cpu_baseline_aggregate(
            reg, reqs, words, sigs, expect, len(reqs), min_wall=0.2))
        if rank == 0:
            print(json.dumps({"n_gpus": world, "cpu_baseline": cpu}))
        if world > 1:
            tdist.destroy_process_group()
        return
    if args.launch_probe:
        import torch.distributed as tdist

        if world > 1:
            tdist.init_process_group("gloo")
        seen = tdist.get_world_size() if world > 1 else 1
        ranks = [None] * world
        if world > 1:
            tdist.all_gather_object(ranks, rank)
            tdist.destroy_process_group()
        if rank == 0:
            print(json.dumps({"n_gpus": world, "world_size_seen": seen, "ranks": ranks if world > 1 else [0],
                              "launched": os.environ.get("HG_BENCH_LAUNCHED") == "1"}))
        return
    if args.inflight is None:
        # the gloo rehearsal (ranks sharing a GPU) runs one batch at a time per
        # rank, so the processes on one device stay within 16 queues together
        args.inflight = 1 if os.environ.get("HG_BENCH_BACKEND", "nccl") == "gloo" else 4
    # every HIP stream on a hardware queue of its own (the lanes' pairing and
    # fold streams, the per-lane torch streams, the context's and the pipelined
    # line's): sharing queues serialises one lane's kernels behind another's.
    # Read when the HIP runtime starts (the first device call below).
    # (the box presets 4: raised, never lowered; HG_BENCH_HW_QUEUES forces a value)
    # (per lane: its pairing and fold streams; the gather runs on the lane's
    # own stream; + the context's, torch's and RCCL's)
    want_q = int(os.environ.get("HG_BENCH_HW_QUEUES", "0")) or (min(16, 2 * args.inflight + 4)
                                                                 if args.inflight > 1 else 0)
    if want_q and (os.environ.get("HG_BENCH_HW_QUEUES") or int(os.environ.get("GPU_MAX_HW_QUEUES", "0")) < want_q):
        os.environ["GPU_MAX_HW_QUEUES"] = str(want_q)

    # HG_BENCH_FORCE_PG=1 (a test hook: tests/test_gpu_rccl.py): the process
    # group and every collective of the N-rank path even with one rank, so
    # the RCCL branch runs on a one-GPU box exactly as each rank of N runs it
    dist = world > 1 or os.environ.get("HG_BENCH_FORCE_PG") == "1"
    # HG_BENCH_BACKEND=gloo is a rehearsal mode for boxes with fewer GPUs than
    # ranks (ranks share devices round-robin, collectives on host copies); the
    # production path is one rank per GPU over RCCL ("nccl").
    backend = os.environ.get("HG_BENCH_BACKEND", "nccl")
    ndev = torch.cuda.device_count()
    local_dev = local % ndev if backend == "gloo" else local
    if dist:
        import torch.distributed as tdist

        torch.cuda.set_device(local_dev)
        if backend == "nccl":
            tdist.init_process_group("nccl", device_id=torch.device("cuda", local_dev))
        else:
            tdist.init_process_group("gloo")
    else:
        torch.cuda.set_device(0)
    dev = torch.device("cuda", local_dev)
    coll_dev = dev if backend == "nccl" else torch.device("cpu")
    timer = Timer(dev, dist, coll_dev, world)
    stream = torch.cuda.current_stream(dev)
    n = args.batch

    eng = Engine(device=local_dev, flavor="go")
    assert eng.set_message(LIB_MESSAGE) == 0
    n_reg = 4096 if args.committees else 4000
    head = AggregateWorkload(eng, n_reg, n, seed=4321 + rank, dev=dev, stream=stream)
    gathered = [torch.zeros((n + 7) // 8, dtype=torch.uint8, device=coll_dev) for _ in range(world)]

    def seq_step():
        # one batch at a time on the context's stream: the batch's verdicts and
        # their bitset (bit i = check i valid), then the bitsets gathered over
        # RCCL: the only cross-GPU traffic
        head.submit_bits()
        gather_verdicts(head.d_bits.to(coll_dev), world, gathered)

    # the headline: a verifier fed a continuous stream of 4096-request batches
    # keeps `inflight` of them in flight on the context's lanes (hg_lane_*:
    # own streams and workspaces, the one registry and table set, the unpadded
    # pairing kernel so two batches' waves share the SIMDs); each step is one
    # whole batch — its verdicts, bitset and gather — on the lane's stream
    inflight = max(1, args.inflight)
    lanes, lane_out = [], []
    if inflight > 1:
        for i in range(inflight):
            lanes.append(DeviceLane(eng, n, pad=False))
            codes_i = head.d_codes if i == 0 else torch.zeros(n, dtype=torch.int32, device=dev)
            bits_i = head.d_bits if i == 0 else torch.zeros((n + 7) // 8, dtype=torch.uint8, device=dev)
            gath_i = gathered if i == 0 else [torch.zeros((n + 7) // 8, dtype=torch.uint8, device=coll_dev)
                                              for _ in range(world)]
            # the gather runs on the lane's own stream (wrapped for torch), right
            # after the lane's verdicts; the lane's next batch follows it there
            lane_out.append((torch.cuda.ExternalStream(lanes[-1].stream, device=dev) if dist else None,
                             codes_i, bits_i, gath_i))
    turn = [0]

    def lane_step():
        i = turn[0] % inflight
        turn[0] += 1
        st, codes_i, bits_i, gath_i = lane_out[i]
        if not dist:
            # nothing reads the verdicts between steps (the gather is the
            # identity): the lane orders each batch after its own previous one
            lanes[i].submit_device(head.d_reqs.data_ptr(), n, head.d_words.data_ptr(), head.d_sigs.data_ptr(),
                                   codes_i.data_ptr(), bits_i.data_ptr(), lanes[i].stream)
            gather_verdicts(bits_i, world, gath_i)
            return
        with torch.cuda.stream(st):
            lanes[i].submit_device(head.d_reqs.data_ptr(), n, head.d_words.data_ptr(), head.d_sigs.data_ptr(),
                                   codes_i.data_ptr(), bits_i.data_ptr(), lanes[i].stream)
            gather_verdicts(bits_i.to(coll_dev), world, gath_i)

    step = lane_step if inflight > 1 else seq_step
    for _ in range(inflight):
        step()
    torch.cuda.synchronize(dev)
    for codes_i in ([o[1] for o in lane_out] if lanes else [head.d_codes]):
        head.check(codes_i)
    assert torch.equal(head.d_bits, pack_verdicts(head.d_codes)), "HIP verdict bitset differs from the codes"
    progress(f"headline: {inflight} in flight, prewarm / warmup / {args.steps} timed steps")
    prewarm_steps = timer.prewarm(step, args.prewarm)
    dt = timer.run(step, args.steps, args.warmup)
    head_marks = dict(timer.marks)
    rank_ms = [round(t / args.steps * 1e3, 4) for t in timer.rank_times]
    # every rank's gathered bitsets: each rank tampers every 8th aggregate of
    # its own batch, so all world bitsets equal this rank's expected one
    want = pack_verdicts(torch.from_numpy(head.expect))
    gather_check = {"world_size_seen": tdist.get_world_size() if dist else 1, "backend": backend if dist else None,
                    "ranks_checked": world, "lanes_checked": max(1, len(lanes))}
    for codes_i, bits_i, gath_i in ([(o[1], o[2], o[3]) for o in lane_out] if lanes
                                    else [(head.d_codes, head.d_bits, gathered)]):
        head.check(codes_i)
        for r in range(world):
            g = gath_i[r] if dist else bits_i
            assert torch.equal(g.cpu(), want), f"gathered bitset of rank {r} differs"
    for ln in lanes:
        ln.close()
    sequential = None
    progress("headline done; sequential, per-kernel phases")
    if inflight > 1 and not args.no_extra:
        sdt_seq = timer.run(seq_step, args.steps, args.warmup)
        head.check()
        sequential = {"value": round(n * args.steps * world / sdt_seq, 1), "unit": "verifications/s",
                      "ms_per_step": round(sdt_seq / args.steps * 1e3, 4),
                      "what": "the headline batch one at a time on the context's stream (the next batch starts "
                              "after the previous one's verdicts): the latency-bound rate, padded pairing kernel"}
    ph = timed_phases(eng, lambda: [head.submit() for _ in range(5)])
    # the kernels on their own (fold, then the pairing kernel: no overlap),
    # for the per-kernel rooflines
    eng.set_fold_overlap(False)
    ph_seq = timed_phases(eng, lambda: [head.submit() for _ in range(5)])
    eng.set_fold_overlap(True)
    value = n * args.steps * world / dt
    # the dominant kernels of the step: the GT fold (plan, chunks, combine) and
    # the pairing check, on the work they implement (the primary roofline).
    # Time base: with batches in flight the kernels of different batches
    # overlap (two pairing waves per SIMD), so the step's device time is the
    # timed region per step; one batch at a time it is the submission's kernel
    # time, prologue to comparison (HIP events on the launch stream)
    agg_ms = dt / args.steps * 1e3 if inflight > 1 else ph["submit"]
    impl_fpmul = head.terms * FPMUL_PER_GT_MUL + n * FPMUL_PER_SIG_PAIRING
    # batches in flight run on unpadded lanes: the 12-lane pairing kernel with
    # its line kernels (bn256_sig12.hip); one batch at a time, the padded
    # 16-lane k_verify_sig (hg_api.cpp: sig12_for)
    # (the 12-lane pairing runs split around its norm inversion since r06:
    # k_sig12_miller, k_sig12_ninv, k_sig12_fe; k_verify_sig12 with
    # HG_SIG12_SPLIT=0)
    sig_kernel = (r"(k_verify_sig12|k_sig12_miller|k_sig12_fe)<false>|k_sig12_ninv|k_sig_(lines|scalars)"
                  if inflight > 1 else r"k_verify_sig<4, true(, true)?>")
    roof = roofline(impl_fpmul, agg_ms,
                    (f"the GT submission, {inflight} batches in flight (timed region per step): k_agg_prologue, "
                     "k_sig_scalars + k_sig_lines + k_sig12_miller + k_sig12_ninv + k_sig12_fe (12-lane teams)"
                     if inflight > 1
                     else "the GT submission: k_agg_prologue, k_verify_sig") + " beside the GT fold (k_gt_plan, "
                    "k_gt_chunks, k_gt_combine), k_gt_compare_bits",
                    r"k_agg_prologue|k_gt_(plan<16>|chunks|combine|compare_bits)|" + sig_kernel,
                    f"implemented work: {head.terms} window-table terms x {FPMUL_PER_GT_MUL} Fp-mul (one Fp12 "
                    f"product each) + {n} x {FPMUL_PER_SIG_PAIRING} Fp-mul (one pairing + final exponentiation "
                    f"per check), x {MADS_PER_FPMUL} u32 mads",
                    rocprof_pattern=sig_kernel + r"|k_gt_compare_bits")
    # frac_rocprof: the same work over the device-busy time per step of a
    # committed kernel trace of this invocation (the union of the timed
    # region's kernel intervals / steps, tools/busy_summary.py); the older
    # per-launch form stays as frac_rocprof_per_launch (with batches in
    # flight a launch lasts longer than a step, so that form is low)
    if "frac_rocprof" in roof:
        roof["frac_rocprof_per_launch"] = roof.pop("frac_rocprof")
        roof["rocprof_kernel_ms_per_launch"] = roof.pop("rocprof_kernel_ms")
    busy_ms, busy_src = rocprof_busy_ms(inflight)
    if busy_ms:
        roof["frac_rocprof"] = round(impl_fpmul * MADS_PER_FPMUL / (busy_ms * 1e-3) / 1e12 / P_MAD_TOPS, 4)
        roof["rocprof_busy_ms_per_step"] = busy_ms
        roof["rocprof_busy_source"] = busy_src
    roof["frac_rocprof_note"] = (
        "the same implemented work over the device-busy time per timed step in a kernel trace of the driver's "
        "invocation (every kernel interval inside the timed region merged, / steps; the trace's own line records "
        "the region): reproduces `frac` from a committed profile. frac_rocprof_per_launch: over the rocprof average "
        "launch duration of the step's pairing kernels and comparison" + (
            f" — with {inflight} batches in flight two launches share the SIMDs, so a launch lasts longer than a "
            "step and that fraction is below `frac`" if inflight > 1 else ""))
    if inflight > 1:
        roof["sequential_submit_ms"] = round(ph["submit"], 4)
        roof["sequential_frac"] = round(impl_fpmul * MADS_PER_FPMUL / (ph["submit"] * 1e-3) / 1e12 / P_MAD_TOPS, 4)
    roof["kernels_ms"] = {"fold": round(ph["fold"], 4), "k_verify": round(ph["verify"], 4),
                          "submit": round(ph["submit"], 4)}
    # the reference algorithm's work over the same time: a rate, not a
    # utilisation (the GT path skips the G2 fold and the pk-side pairing)
    effective = {"value": round(head.fpmul * MADS_PER_FPMUL / (agg_ms * 1e-3) / 1e12, 3),
                 "unit": "Tmad/s of reference-algorithm work",
                 "work": f"the REFERENCE algorithm per check (SURVEY.md 8(d)): {FPMUL_PER_G2_ADD} Fp-mul per set bit "
                         f"(G2 addition) + {FPMUL_REFERENCE_CHECK} (two-pairing check), x {MADS_PER_FPMUL} u32 mads; mean "
                         f"{head.signers.mean():.1f} set bits",
                 "note": "work the GT path does not run is credited here; not a fraction of any peak"}
    roof_verify = roofline(n * FPMUL_PER_SIG_PAIRING, ph_seq["verify"], "k_verify_sig", r"k_verify_sig<4, false(, true)?>",
                           f"{FPMUL_PER_SIG_PAIRING} Fp-mul x {MADS_PER_FPMUL} u32 mads per check (one pairing "
                           "+ final exponentiation, oracle op count); kernel alone (fold not beside it)",
                           rocprof_pattern=r"k_verify_sig<4, true(, (true|false))?>")
    # the headline's pairing kernel alone: k_sig_scalars + k_sig_lines +
    # k_verify_sig12 on one stream, HIP events around 5 launches. Its padded
    # form (hg_sig_pairing_device kernel 2): one batch alone occupies 820 of
    # the 1024 SIMDs with one wave each — the unpadded form alone would let
    # the dispatcher stack two waves on some SIMDs and leave others empty —
    # so this is the kernel's latency-bound rate (in flight, two batches'
    # waves share every SIMD: the primary roofline's time base)
    sig_stream = torch.cuda.Stream(dev)
    d_fe = torch.empty(n * 480, dtype=torch.uint8, device=dev)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    with torch.cuda.stream(sig_stream):
        eng.sig_pairing_device(head.d_sigs.data_ptr(), n, d_fe.data_ptr(), Engine.SIG_K12_PAD, sig_stream.cuda_stream)
        ev[0].record(sig_stream)
        for _ in range(5):
            eng.sig_pairing_device(head.d_sigs.data_ptr(), n, d_fe.data_ptr(), Engine.SIG_K12_PAD,
                                   sig_stream.cuda_stream)
        ev[1].record(sig_stream)
    torch.cuda.synchronize(dev)
    sig12_ms = ev[0].elapsed_time(ev[1]) / 5
    del d_fe
    # (padded launches keep the single kernel: the split form is the
    # throughput form of batches in flight)
    sig12_pad = r"k_verify_sig12<true>|k_sig_(lines|scalars)"
    roof_sig12 = roofline(n * FPMUL_PER_SIG_PAIRING, sig12_ms,
                          "k_sig_scalars + k_sig_lines + k_verify_sig12<true>",
                          sig12_pad,
                          f"{FPMUL_PER_SIG_PAIRING} Fp-mul x {MADS_PER_FPMUL} u32 mads per check (the line "
                          "evaluations included); one launch alone, one wave per SIMD",
                          rocprof_pattern=sig12_pad)
    roof_fold = roofline(head.terms * FPMUL_PER_GT_MUL, ph_seq["fold"], "k_gt_plan + k_gt_chunks + k_gt_combine",
                         r"k_gt_(plan<16>|chunks|combine)",
                         f"{head.terms} window-table terms x {FPMUL_PER_GT_MUL} Fp-mul (one Fp12 product each); "
                         "kernels alone (not beside the pairing kernel)")
    roof["kernels_alone_ms"] = {"fold": round(ph_seq["fold"], 4), "k_verify": round(ph_seq["verify"], 4),
                                "submit": round(ph_seq["submit"], 4)}

    extra = {}
    progress("sub-lines")
    if not args.no_extra:
        # config 2: independent single-signature checks
        single = SingleWorkload(eng, n, seed=1234 + rank, dev=dev, stream=stream)

        def sstep():
            single.submit()
            single.pack()
            gather_verdicts(single.d_bits.to(coll_dev), world, gathered)

        sdt = timer.run(sstep, args.steps, args.warmup)
        single.check()
        sph = timed_phases(eng, lambda: [single.submit() for _ in range(5)])
        # the same batches as a stream, `inflight` in flight (the headline's
        # form): the line's value; one batch at a time is `sequential`
        s_inflight = max(1, args.inflight)
        progress(f"single: {s_inflight} in flight")
        idt = single_stream_rate(single, s_inflight, timer, args.steps, args.warmup, dev, local_dev, world, coll_dev,
                                 dist)
        extra["single"] = {
            "metric": "BN254 single-sig verifications/sec (batch 4096)",
            "value": round(n * args.steps * world / idt, 1), "unit": "verifications/s",
            "ms_per_step": round(idt / args.steps * 1e3, 4), "batches_in_flight": s_inflight,
            "form": "split (k_verify_ml + k_sig12_norm / ninv / fe + k_fe_verdicts), one context per batch in flight",
            "workload": f"config 2: {n} independent BLS pairing checks per GPU (lib.Message, 1/8 tampered)",
            "roofline": roofline(single.fpmul, idt / args.steps * 1e3, "k_verify_ml + k_sig12_* (in flight)",
                                 r"k_verify_ml", f"{FPMUL_PER_CHECK} Fp-mul x {MADS_PER_FPMUL} u32 mads per check, "
                                 "over the stream's step time"),
            "sequential": {"value": round(n * args.steps * world / sdt, 1),
                           "ms_per_step": round(sdt / args.steps * 1e3, 4), "form": "k_verify (one kernel)",
                           "roofline": roofline(single.fpmul, sph["verify"], "k_verify", r"k_verify(?!_)",
                                                f"{FPMUL_PER_CHECK} Fp-mul x {MADS_PER_FPMUL} u32 mads per check")}}
        # at every world size: rank 0 after this line's timed region, the
        # other ranks at a barrier
        extra["single"]["cpu_baseline"] = cpu_baseline_on_rank0(
            rank, dist, args, lambda: cpu_baseline_single(single.pks, single.sigs, single.expect))
        del single
        # config 2 with registry keys (the p2p aggregator's verifyPacket,
        # simul/p2p/aggregator.go:244): one-key aggregate requests on the head
        # registry, so each check is the GT path's single pairing
        rng = np.random.default_rng(4242 + rank)
        idx = rng.integers(0, n_reg, size=n)
        kb = np.frombuffer(seeded_scalars(n_reg, 4321 + rank), dtype=np.uint8).reshape(n_reg, 32)
        rsigs = bytearray(eng.sign(kb[idx].tobytes()))
        rexpect = _tamper(eng, rsigs, n)
        rreqs = np.array([(int(i), 1, 1, j) for j, i in enumerate(idx)], dtype=REQ_DTYPE)
        rwords = np.ones(n, dtype=np.uint64)
        d_rreqs, d_rwords = _dev_bytes(rreqs.tobytes(), dev), _dev_bytes(rwords.tobytes(), dev)
        d_rsigs = _dev_bytes(bytes(rsigs), dev)
        rcodes = torch.zeros(n, dtype=torch.int32, device=dev)

        def rstep():
            eng.verify_aggregate_device(d_rreqs.data_ptr(), n, d_rwords.data_ptr(), d_rsigs.data_ptr(),
                                        rcodes.data_ptr(), 0, stream.cuda_stream)

        rdt = timer.run(rstep, args.steps, args.warmup)
        assert np.array_equal(rcodes.cpu().numpy(), rexpect), "registry single-signature verdicts"

        class _RegSingles:  # the batch in lanes_rate's shape
            d_reqs, d_words, d_sigs = d_rreqs, d_rwords, d_rsigs

            def check(self, codes):
                assert np.array_equal(codes.cpu().numpy(), rexpect), "registry single-signature verdicts (lanes)"
        _RegSingles.n = n
        reg_inflight = None
        if inflight > 1:
            ridt = lanes_rate(eng, _RegSingles(), inflight, timer, args.steps, args.warmup, dev)
            reg_inflight = {"value": round(n * args.steps * world / ridt, 1), "unit": "verifications/s",
                            "ms_per_step": round(ridt / args.steps * 1e3, 4), "batches_in_flight": inflight,
                            "what": "the same batches in flight on the context's lanes, as the headline runs"}
        progress("single_registry")
        extra["single_registry"] = {
            "metric": "BN254 single-sig verifications/sec, registry keys (batch 4096)",
            "value": round(n * args.steps * world / rdt, 1), "unit": "verifications/s",
            "ms_per_step": round(rdt / args.steps * 1e3, 4), "inflight": reg_inflight,
            "workload": f"{n} single signatures from random nodes of the {n_reg}-key registry (one-key aggregate "
                        "requests: the GT path), lib.Message, 1/8 tampered"}
        # VerifyMultiSignature shape: every request spans the whole registry
        full = AggregateWorkload(eng, n_reg, n, seed=8765 + rank, dev=dev, stream=stream, full=True)
        fdt = timer.run(full.submit, args.steps, args.warmup)
        full.check()
        fph = timed_phases(eng, lambda: [full.submit() for _ in range(5)])
        full_inflight = None
        if inflight > 1:
            idt = lanes_rate(eng, full, inflight, timer, args.steps, args.warmup, dev)
            full_inflight = {"value": round(n * args.steps * world / idt, 1), "unit": "verifications/s",
                             "ms_per_step": round(idt / args.steps * 1e3, 4), "batches_in_flight": inflight,
                             "what": "the same batches in flight on the context's lanes, as the headline runs"}
        progress("full_registry")
        extra["full_registry"] = {
            "metric": "BN254 aggregate-sig verifications/sec (VerifyMultiSignature over the registry)",
            "value": round(n * args.steps * world / fdt, 1), "unit": "verifications/s",
            "ms_per_step": round(fdt / args.steps * 1e3, 4),
            "workload": f"{n} multisigs per GPU, every request spans the whole {n_reg}-key registry "
                        "(crypto.go:120-137), bitset density U[0.5,1], 1/8 tampered",
            "signers_per_check_mean": round(float(full.signers.mean()), 1),
            "inflight": full_inflight,
            "kernels_ms": {k: round(v, 4) for k, v in fph.items() if v is not None},
            "roofline": roofline(full.terms * FPMUL_PER_GT_MUL + n * FPMUL_PER_SIG_PAIRING, fph["submit"],
                                 "the GT submission (as the headline)",
                                 r"k_agg_prologue|k_gt_(plan<16>|chunks|combine|compare(?!_))|k_verify_sig<4, true(, (true|false))?>",
                                 f"implemented work: {full.terms} window-table terms x {FPMUL_PER_GT_MUL} Fp-mul + "
                                 f"{n} x {FPMUL_PER_SIG_PAIRING} Fp-mul, x {MADS_PER_FPMUL} u32 mads")}
        del full
        # reload the headline registry (the full-registry workload replaced it)
        assert not eng.registry_load(head.reg).any()
        assert eng.prepare_aggregate() == 0
        if args.pipeline > 1:
            # a verifier serving a continuous stream: batches in flight on several
            # HIP streams, one engine context (own workspaces) per stream
            engs = [eng] + [Engine(device=local_dev, flavor="go") for _ in range(args.pipeline - 1)]
            for e in engs:
                e.set_fold_overlap(bool(args.pipeline_overlap))
            for e in engs[1:]:
                assert e.set_message(LIB_MESSAGE) == 0
                assert not e.registry_load(head.reg).any()
                assert e.prepare_aggregate() == 0
            streams = [stream] + [torch.cuda.Stream(dev) for _ in engs[1:]]
            codes_p = [head.d_codes] + [torch.zeros(n, dtype=torch.int32, device=dev) for _ in engs[1:]]

            def pstep():
                for e, st, cd in zip(engs, streams, codes_p):
                    head.submit(eng=e, codes=cd, stream=st)

            pdt = timer.run(pstep, args.steps, args.warmup)
            for cd in codes_p:
                head.check(cd)
            progress("pipelined")
            extra["pipelined"] = {"value": round(n * len(engs) * args.steps * world / pdt, 1),
                                  "unit": "verifications/s", "batches_in_flight": len(engs), "batch": n,
                                  "ms_per_step": round(pdt / args.steps * 1e3, 4),
                                  "note": "headline batch on each of the streams; throughput with batches overlapped"}
            for e in engs[1:]:
                e.close()
            eng.set_fold_overlap(True)

        progress("packet_intake")
        extra["packet_intake"] = packet_intake(eng, head, n_reg, dev, stream, timer, args, world)
        progress("batch_latency")
        extra["batch_latency"] = {
            "what": "one batch submitted alone and waited for (median of 15), first n headline requests: the "
                    "per-check latency floor a one-check-at-a-time evaluator (processing.go:228-287) sees",
            "pairing_kernel": "k_verify_sig_split<2> (two waves per check, DESIGN.md 3e) for n <= 2048, "
                              "k_verify_sig<4, true> above",
            **batch_latency(eng, head, dev)}
        progress("handel_run_volume")
        extra["handel_run_volume"] = handel_run_volume(dev, stream, local_dev)
        if want_config4_proxy(rank, world, args):
            # one GPU's line: the proxy's processes open device 0 (single-host
            # simul on one GPU), so it never runs beside other ranks
            progress("config4_proxy")
            extra["config4_proxy"] = {
                "what": "simul's 2000-node single-host verification load (8 processes x 250 instances x 45 checks, "
                        "one check in flight per instance) on this GPU; checks/s, per-check latency, HBM",
                "service": config4_proxy("service"), "contexts": config4_proxy("contexts")}

    progress("CPU baseline" if rank == 0 and not args.no_cpu else "done")
    # at every world size (north_star: the CPU figure beside each N): rank 0,
    # after every timed region, the other ranks waiting at a barrier
    cpu = cpu_baseline_on_rank0(rank, dist, args, lambda: cpu_baseline_aggregate(
        head.reg, head.reqs, head.words, head.sigs, head.expect, args.cpu_sample))
    if rank == 0:
        workload = (f"config 5: one committee of {n_reg} signers per GPU, {n} multisigs at random Handel levels"
                    if args.committees else
                    f"config 3: {n} Handel multisigs per GPU on a {n_reg}-key registry, random node/level")
        line = {
            "metric": "BN254 aggregate-sig verifications/sec (batch 4096)",
            "value": round(value, 1),
            "unit": "verifications/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(dt / args.steps * 1e3, 4),
            "batches_in_flight": inflight,
            "hw_queues": os.environ.get("GPU_MAX_HW_QUEUES"),
            "rank_ms_per_step": {"min": min(rank_ms), "max": max(rank_ms), "per_rank": rank_ms},
            "timed_region_ns": head_marks,
            "prewarm": {"seconds": args.prewarm, "steps": prewarm_steps, "what": "untimed headline steps before the "
                        "warmup steps (GPU clocks settled whatever the warmup count)"},
            "gather": {**gather_check, "what": "every rank's all-gathered verdict bitset checked against the expected "
                       "one (world 1: the gather is the identity, the rank's own bitset is checked)"},
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u32 (26-bit-limb Fp, 64-bit accumulators)",
            "data": "synthetic (seeded keys, lib.Message, bitset density U[0.5,1], 1/8 tampered aggregates)",
            "config": {"workload": workload + ", bitset density U[0.5,1], 1/8 tampered",
                       "batch_per_gpu": n, "registry": n_reg, "message": "lib.Message (81 B)",
                       "signers_per_check_mean": round(float(head.signers.mean()), 1),
                       "signers_per_check_max": int(head.signers.max()),
                       "parallelism": f"dp{world} (batches per GPU, {inflight} in flight on the context's lanes; RCCL "
                                      "all_gather of verdict bitsets)"},
            "roofline": roof,
            "effective_rate": effective,
            "roofline_k_verify": roof_verify,
            "roofline_k_verify_sig12": roof_sig12,
            "roofline_gt_fold": roof_fold,
            "setup": {"ms": round(head.setup_ms, 2), "what": "per (message, registry), outside the timed "
                      f"region: e(H, pk_i) for {n_reg} keys + GT products of every 16-key window subset and aligned "
                      "block (hg_prepare_aggregate)",
                      "cold_value": round(n / ((head.setup_ms + dt / args.steps * 1e3) * 1e-3), 1)},
            "cpu_baseline": cpu,
            "gpu_over_cpu": (round(value / cpu["value"], 1) if cpu and cpu.get("value") else None),
            "sequential": sequential,
            **extra,
        }
        print(json.dumps(line))
    eng.close()
    if dist:
        tdist.destroy_process_group()


if __name__ == "__main__":
    main()
