#!/usr/bin/env python3
"""Headline benchmark: BN256 BLS verifications/s at batch 4096 on MI355X.

Workload (BASELINE.json configs[1]): one step =
4096 independent PublicKey.VerifySignature(lib.Message, sig) checks
(bn256/go/bn256.go:82-94) with 1/8 of the signatures tampered, inputs
(marshalled pks and sigs) already resident in HBM, verdict codes written
back to HBM, then the verdict bitset gathered to rank 0 over RCCL.
Keys/signatures are synthetic (seeded scalars, keygen/sign on the GPU).

Multi-GPU: one process per GPU (torchrun), every rank verifies its own batch
of 4096 (weak scaling, no data-path collective); the only exchange is the
all_gather of 512-byte verdict bitsets.

Prints ONE JSON line on rank 0.
"""

from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from handel_amd.distributed import gather_verdicts, pack_verdicts  # noqa: E402
from handel_amd.engine import Engine  # noqa: E402

LIB_MESSAGE = b"Everything that is beautiful and noble is the product of reason and calculation."
ORDER = 65000549695646603732796438742359905742570406053903786389881062969044166799969
P = 65000549695646603732796438742359905742825358107623003571877145026864184071783
G1_GEN_BYTES = (1).to_bytes(32, "big") + (P - 2).to_bytes(32, "big")

# Algorithmic work per check, fixed before tuning by the oracle's op counter
# (oracle/bn256_ref.c, fast=2: one multi-Miller loop over 6u+2 with the pk
# lines on the fly and the G2Base lines from a table, one final
# exponentiation, Karatsuba tower formulas): Fp multiplications per check.
# tests/test_oracle.py pins this number.
FPMUL_PER_CHECK = 25271
# u32 x u32 multiply-adds per Fp multiplication (8-limb CIOS: 2*8^2 + 8)
MADS_PER_FPMUL = 136
# Peak v_mad_u64_u32 rate, measured by tools/intrate.hip on MI355X with 8
# waves per SIMD (profiles/r01_intrate.jsonl: 34.95 T/s, the highest of the
# round's runs; half the VALU rate: 256 CU x 4 SIMD x 32 lanes x 2.4 GHz / 2 =
# 39.3 T/s spec-derived).
P_MAD_TOPS = 34.95


def seeded_scalars(n: int, seed: int) -> bytes:
    """n secret keys in [1, n) from a seeded generator (RandomG2 rejection rule)."""
    rng = np.random.default_rng(seed)
    out = bytearray()
    while len(out) < 32 * n:
        k = int.from_bytes(rng.bytes(32), "big")
        if 0 < k < ORDER:
            out += k.to_bytes(32, "big")
    return bytes(out)


def make_batch(eng: Engine, n: int, seed: int):
    kb = seeded_scalars(n, seed)
    pks = eng.keygen(kb)
    sigs = bytearray(eng.sign(kb))
    # tamper 1/8 of the signatures: sig + G1
    idx = list(range(0, n, 8))
    a = b"".join(bytes(sigs[64 * i:64 * i + 64]) for i in idx)
    bad, codes = eng.combine_g1(a, G1_GEN_BYTES * len(idx))
    assert not codes.any()
    for j, i in enumerate(idx):
        sigs[64 * i:64 * i + 64] = bad[64 * j:64 * j + 64]
    expect = np.zeros(n, dtype=np.int32)
    expect[idx] = 1
    return pks, bytes(sigs), expect


def make_aggregate_batch(eng: Engine, n_reg: int, n: int, seed: int, full: bool = False):
    """a registry of n_reg keys and n incoming
    multisignatures as Handel's evaluator receives them: for each, a random
    node's random non-empty level (partitioner rangeLevel, partitioner.go:133-178),
    a bitset of density U[0.5, 1.0] over the level's registry range, and the
    aggregate signature of the set bits (sum of the secret keys times H(msg));
    1/8 of the aggregates tampered (+ G1). full=True: every request spans the
    whole registry (crypto.go:120-137 VerifyMultiSignature, config 3's second
    workload)."""
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
    idx = list(range(0, n, 8))
    bad, codes = eng.combine_g1(b"".join(bytes(sigs[64 * i:64 * i + 64]) for i in idx), G1_GEN_BYTES * len(idx))
    assert not codes.any()
    for j, i in enumerate(idx):
        sigs[64 * i:64 * i + 64] = bad[64 * j:64 * j + 64]
    expect = np.zeros(n, dtype=np.int32)
    expect[idx] = 1
    from handel_amd.engine import REQ_DTYPE

    return np.array(reqs, dtype=REQ_DTYPE), np.array(words, dtype=np.uint64), bytes(sigs), expect, np.array(signers)


def pmc_traffic():
    """HBM bytes per k_verify launch from the newest committed PMC summary
    (profiles/*_pmc.csv, written by tools/profile_round.sh +
    tools/rocpd_summary.py): FETCH_SIZE x 2 (gfx950 correction) + WRITE_SIZE."""
    import csv
    import glob

    import re

    # newest = highest round/version in the name (mtimes are not kept by git or the box snapshot)
    def key(path):
        return [int(t) if t.isdigit() else t for t in re.split(r"(\d+)", os.path.basename(path))]

    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "*_pmc.csv")), key=key)
    for path in reversed(files):
        vals = {}
        with open(path) as f:
            for row in csv.DictReader(f):
                if "k_verify" in row["kernel"]:
                    vals[row["counter"]] = float(row["avg"])
        if "FETCH_SIZE" in vals and "WRITE_SIZE" in vals:
            return int((2 * vals["FETCH_SIZE"] + vals["WRITE_SIZE"]) * 1024), os.path.relpath(path, ROOT)
    return None, None


def cpu_baseline(n_sample: int, pks: bytes, sigs: bytes, expect: np.ndarray):
    """The reference algorithm restated in C (oracle/bn256_ref.c, 'port'):
    two full pairings + GT compare per check, timed on this host's cores."""
    from oracle import ref_lib as R

    threads = min(16, os.cpu_count() or 1)
    reps = 3  # ~25 s of CPU work on 16 threads at the measured ~8k checks/s
    t0 = time.perf_counter()
    for _ in range(reps):
        codes = R.verify_batch(LIB_MESSAGE, pks[:128 * n_sample], sigs[:64 * n_sample], nthreads=threads, fast=0)
        assert np.array_equal(codes, expect[:n_sample]), "CPU oracle verdicts differ"
    dt = time.perf_counter() - t0
    return {"value": round(reps * n_sample / dt, 1), "unit": "verifications/s", "cores": threads, "kind": "port",
            "sample": f"{reps} passes over {n_sample} checks of the same batch (lib.Message, 1/8 tampered), "
                      f"reference algorithm (2 pairings + GT compare), {threads} threads, {dt:.2f} s wall"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=4096)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-aggregate", action="store_true", help="skip the config-3 aggregate-verify line")
    ap.add_argument("--pipeline", type=int, default=2,
                    help="batches in flight for the extra 'pipelined' report (1: skip)")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = world > 1
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

    eng = Engine(device=local_dev, flavor="go")
    assert eng.set_message(LIB_MESSAGE) == 0
    n = args.batch
    pks, sigs, expect = make_batch(eng, n, seed=1234 + rank)
    d_pks = torch.frombuffer(bytearray(pks), dtype=torch.uint8).to(dev)
    d_sigs = torch.frombuffer(bytearray(sigs), dtype=torch.uint8).to(dev)
    d_codes = torch.zeros(n, dtype=torch.int32, device=dev)
    gathered = [torch.zeros((n + 7) // 8, dtype=torch.uint8, device=coll_dev) for _ in range(world)]
    d_bits = torch.zeros((n + 7) // 8, dtype=torch.uint8, device=dev)
    stream = torch.cuda.current_stream(dev)

    def step():
        eng.verify_batch_device(d_pks.data_ptr(), d_sigs.data_ptr(), n, d_codes.data_ptr(), stream.cuda_stream)
        # verdict bitset (bit i = check i valid), gathered over RCCL: the only cross-GPU traffic
        eng.pack_verdicts_device(d_codes.data_ptr(), n, d_bits.data_ptr(), stream.cuda_stream)
        gather_verdicts(d_bits.to(coll_dev), world, gathered)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(dev)
    got = d_codes.cpu().numpy()
    assert np.array_equal(got, expect), f"GPU verdicts differ from the expected pattern: {np.flatnonzero(got != expect)[:8]}"
    assert torch.equal(d_bits, pack_verdicts(d_codes)), "HIP verdict bitset differs from the codes"

    eng.timing_enable(True)
    eng.timing_read()
    if dist:
        tdist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize(dev)
    if dist:
        tdist.barrier()
    dt = time.perf_counter() - t0
    kern_ms, launches = eng.timing_read()
    eng.timing_enable(False)
    if dist:
        t = torch.tensor([dt], dtype=torch.float64, device=coll_dev)
        tdist.all_reduce(t, op=tdist.ReduceOp.MAX)
        dt = float(t.item())
    got = d_codes.cpu().numpy()
    assert np.array_equal(got, expect)

    total = n * args.steps * world
    value = total / dt
    avg_kernel_ms = kern_ms / max(launches, 1)
    achieved = n * FPMUL_PER_CHECK * MADS_PER_FPMUL / (avg_kernel_ms * 1e-3) / 1e12
    traffic, traffic_src = pmc_traffic()
    roofline = {"bound": "valu", "achieved": round(achieved, 3), "peak": P_MAD_TOPS, "unit": "Tmad/s",
                "frac": round(achieved / P_MAD_TOPS, 4), "traffic": traffic, "traffic_unit": "bytes/launch",
                "traffic_source": traffic_src,
                "kernel": "k_verify", "kernel_ms": round(avg_kernel_ms, 4),
                "work_per_check": f"{FPMUL_PER_CHECK} Fp-mul x {MADS_PER_FPMUL} u32 mads"}
    # config 3: aggregate verification of Handel multisignatures on a
    # 4000-key registry — bitset-driven G2 Combine + pairing check, inputs resident
    def time_aggregate(full: bool):
        reqs, words, asigs, aexpect, sizes = make_aggregate_batch(eng, 4000, n, seed=4321 + rank, full=full)
        d_reqs = torch.frombuffer(bytearray(reqs.tobytes()), dtype=torch.uint8).to(dev)
        d_words = torch.frombuffer(bytearray(words.tobytes()), dtype=torch.uint8).to(dev)
        d_asigs = torch.frombuffer(bytearray(asigs), dtype=torch.uint8).to(dev)
        d_acodes = torch.zeros(n, dtype=torch.int32, device=dev)

        def astep():
            eng.verify_aggregate_device(d_reqs.data_ptr(), n, d_words.data_ptr(), d_asigs.data_ptr(),
                                        d_acodes.data_ptr(), 0, stream.cuda_stream)

        for _ in range(args.warmup):
            astep()
        torch.cuda.synchronize(dev)
        assert np.array_equal(d_acodes.cpu().numpy(), aexpect), "aggregate verdicts differ from the expected pattern"
        if dist:
            tdist.barrier()
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        for _ in range(args.steps):
            astep()
        torch.cuda.synchronize(dev)
        if dist:
            tdist.barrier()
        adt = time.perf_counter() - t0
        if dist:
            t = torch.tensor([adt], dtype=torch.float64, device=coll_dev)
            tdist.all_reduce(t, op=tdist.ReduceOp.MAX)
            adt = float(t.item())
        assert np.array_equal(d_acodes.cpu().numpy(), aexpect)
        scope = ("every request spans the whole 4000-key registry (VerifyMultiSignature)" if full else
                 "random node/level of a 4000-node Handel registry")
        return {"metric": "BN254 aggregate-sig verifications/sec (Handel multisigs, 4000-key registry)",
                "value": round(n * args.steps * world / adt, 1), "unit": "verifications/s",
                "ms_per_step": round(adt / args.steps * 1e3, 4),
                "workload": f"config 3: {n} multisigs per GPU, {scope}, bitset density U[0.5,1], 1/8 tampered",
                "signers_per_check_mean": round(float(sizes.mean()), 1),
                "signers_per_check_max": int(sizes.max())}

    aggregate = aggregate_full = None
    if not args.no_aggregate:
        aggregate = time_aggregate(False)
        aggregate_full = time_aggregate(True)

    # Pipelined batches (reported beside the headline, never as `value`): a
    # Handel node verifies a continuous stream of batches, and two 4096-check
    # batches in flight on two HIP streams (two engine contexts, each with its
    # own scratch) put two k_verify waves on every SIMD instead of one.
    pipelined = None
    if args.pipeline > 1:
        engs = [eng] + [Engine(device=local_dev, flavor="go") for _ in range(args.pipeline - 1)]
        for e in engs[1:]:
            assert e.set_message(LIB_MESSAGE) == 0
        streams = [torch.cuda.Stream(dev) for _ in engs]
        codes_p = [torch.zeros(n, dtype=torch.int32, device=dev) for _ in engs]

        def pstep():
            for e, st, cd in zip(engs, streams, codes_p):
                e.verify_batch_device(d_pks.data_ptr(), d_sigs.data_ptr(), n, cd.data_ptr(), st.cuda_stream)

        for _ in range(args.warmup):
            pstep()
        torch.cuda.synchronize(dev)
        for cd in codes_p:
            assert np.array_equal(cd.cpu().numpy(), expect), "pipelined verdicts differ"
        if dist:
            tdist.barrier()
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        for _ in range(args.steps):
            pstep()
        torch.cuda.synchronize(dev)
        if dist:
            tdist.barrier()
        pdt = time.perf_counter() - t0
        if dist:
            t = torch.tensor([pdt], dtype=torch.float64, device=coll_dev)
            tdist.all_reduce(t, op=tdist.ReduceOp.MAX)
            pdt = float(t.item())
        for cd in codes_p:
            assert np.array_equal(cd.cpu().numpy(), expect)
        pipelined = {"value": round(n * len(engs) * args.steps * world / pdt, 1), "unit": "verifications/s",
                     "batches_in_flight": len(engs), "batch": n,
                     "ms_per_step": round(pdt / args.steps * 1e3, 4),
                     "note": "same batch of 4096 on each of the streams; throughput with batches overlapped"}
        for e in engs[1:]:
            e.close()

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu:
        try:
            cpu = cpu_baseline(min(n, 4096), pks, sigs, expect)
        except Exception as e:  # pragma: no cover - reported, not fatal
            cpu = {"error": str(e)}
    if rank == 0:
        line = {
            "metric": "BN254 aggregate-sig verifications/sec (batch 4096)",
            "value": round(value, 1),
            "unit": "verifications/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(dt / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u32 (26-bit-limb Fp, 64-bit accumulators)",
            "data": "synthetic (seeded keys, lib.Message, 1/8 tampered signatures)",
            "config": {"workload": "config 2: 4096 independent BLS pairing checks per GPU (bn256, dclxvi curve)",
                       "batch_per_gpu": n, "message": "lib.Message (81 B)", "parallelism": f"dp{world} (replicated registry, sharded batches)"},
            "roofline": roofline,
            "cpu_baseline": cpu,
            "aggregate": aggregate,
            "aggregate_full_registry": aggregate_full,
            "pipelined": pipelined,
        }
        print(json.dumps(line))
    eng.close()
    if dist:
        tdist.destroy_process_group()


if __name__ == "__main__":
    main()
