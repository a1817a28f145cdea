"""Multi-GPU sharding of independent verification batches.

One process per GPU. Checks are independent, so the batch is split into
contiguous slices (or, for N committees, one committee per GPU) with the
registry and H(m) replicated; the only exchange is a gather of the per-rank
verdict bitsets (bit i = check i valid, willf layout: byte j holds checks
8j..8j+7, LSB first) over RCCL (backend "nccl") — or gloo on CPU tests.
"""

from __future__ import annotations

from typing import List, Tuple

import torch


def shard_range(n: int, rank: int, world: int) -> Tuple[int, int]:
    """Contiguous slice [lo, hi) of n checks for `rank` (sizes differ by <= 1)."""
    lo = n * rank // world
    hi = n * (rank + 1) // world
    return lo, hi


def pack_verdicts(codes: torch.Tensor) -> torch.Tensor:
    """int32 verdict codes -> uint8 bitset of valid checks (code == 0)."""
    n = codes.numel()
    nbits = (n + 7) // 8 * 8
    ok = torch.zeros(nbits, dtype=torch.int32, device=codes.device)
    ok[:n] = (codes == 0).to(torch.int32)
    weights = (2 ** torch.arange(8, device=codes.device, dtype=torch.int32)).view(1, 8)
    return (ok.view(-1, 8) * weights).sum(dim=1).to(torch.uint8)


def unpack_verdicts(bits: torch.Tensor, n: int) -> torch.Tensor:
    b = bits.to(torch.int32).view(-1, 1)
    shifts = torch.arange(8, device=bits.device, dtype=torch.int32).view(1, 8)
    return ((b >> shifts) & 1).view(-1)[:n].to(torch.bool)


def gather_verdicts(bits: torch.Tensor, world: int, out: List[torch.Tensor] = None) -> List[torch.Tensor]:
    """all_gather of equal-size bitsets (every rank gets every rank's verdicts).
    With one rank and no process group the gather is the identity and copies
    nothing: the result (and out[0], when `out` is given) IS `bits`, so it
    changes when the caller rewrites `bits` (bench.py's world-1 step gathers
    nothing, and says so). With a process group of one rank (bench.py's
    HG_BENCH_FORCE_PG test hook) the collective runs."""
    import torch.distributed as dist

    if world == 1 and not (dist.is_available() and dist.is_initialized()):  # the gather is the identity
        if out is None:
            return [bits]
        out[0] = bits
        return out
    if out is None:
        out = [torch.empty_like(bits) for _ in range(world)]
    dist.all_gather(out, bits)
    return out


def verify_sharded(verify_fn, n: int, rank: int, world: int, device=None) -> torch.Tensor:
    """Sharded verification of one batch of n independent checks: this rank
    verifies the contiguous slice shard_range(n, rank, world) with
    verify_fn(lo, hi) -> int32 codes (on `device`), packs its verdicts and
    all-gathers every rank's bitset (slices differ by at most one check, so
    bitsets are padded to the largest). Returns the n verdicts of the whole
    batch (bool, check i valid), in batch order, on every rank."""
    lo, hi = shard_range(n, rank, world)
    codes = verify_fn(lo, hi)
    if device is None:
        device = codes.device
    width = (-(-n // world) + 7) // 8
    bits = torch.zeros(width, dtype=torch.uint8, device=device)
    if hi > lo:
        mine = pack_verdicts(codes.to(device))
        bits[:mine.numel()] = mine
    got = gather_verdicts(bits, world)
    parts = []
    for r in range(world):
        a, b = shard_range(n, r, world)
        parts.append(unpack_verdicts(got[r], b - a))
    return torch.cat(parts) if parts else torch.zeros(0, dtype=torch.bool)
