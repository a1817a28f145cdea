"""GPU parity: the HIP path (through the C-ABI) against the CPU oracle.

Integer/byte work, so the bar is bit-exact: field products, GT marshals
(bn256.Pair(...).Marshal(), bn256/go/bn256.go:88-89), verdict codes, and
marshalled aggregate keys / combined signatures.
"""

import numpy as np
import pytest

from oracle import bn256_oracle as O
from oracle import ref_lib as R
from tests import _fixtures as F

pytestmark = pytest.mark.gpu


def test_fp_mul_matches_bigint(engine):
    rng = np.random.default_rng(1)
    n = 257
    vals = [0, 1, 2, O.P - 1, O.P - 2, (1 << 255), O.P // 2]
    a_int = vals + [int.from_bytes(rng.bytes(32), "little") % O.P for _ in range(n - len(vals))]
    b_int = list(reversed(vals)) + [int.from_bytes(rng.bytes(32), "little") % O.P for _ in range(n - len(vals))]

    def words(xs):
        return np.array([[(x >> (32 * i)) & 0xFFFFFFFF for i in range(8)] for x in xs], dtype=np.uint32)

    # products whose canonical REDC output has the top 26-bit limb of p (the
    # guarded conditional subtraction's branch is taken and must keep them)
    top = (O.P >> 234) << 234
    edge = [O.P - 1, O.P - 2, O.P - 12345, top, top + 1, top + (1 << 233), O.P - (1 << 200)]
    a_int += edge + [(c * pow(3, -1, O.P)) % O.P for c in edge]
    b_int += [1] * len(edge) + [3] * len(edge)
    out = engine.fp_mul(words(a_int), words(b_int))
    got = [sum(int(w) << (32 * i) for i, w in enumerate(row)) for row in out]
    want = [(x * y) % O.P for x, y in zip(a_int, b_int)]
    assert got == want


def _gt_from_marshal(b):
    order = [5, 3, 1, 4, 2, 0]
    c = [None] * 6
    for i, k in enumerate(order):
        c[k] = (int.from_bytes(b[64 * i:64 * i + 32], "big"), int.from_bytes(b[64 * i + 32:64 * i + 64], "big"))
    return c


@pytest.mark.parametrize("op", range(11))
def test_team_fp12_ops_match_oracle(engine, op):
    rng = np.random.default_rng(100 + op)
    n = 6
    elems, others = [], []
    for _ in range(n):
        f = [(int(rng.integers(0, 2 ** 62)) * (O.P // 2 ** 62) % O.P, int.from_bytes(rng.bytes(32), "big") % O.P)
             for _ in range(6)]
        g = [(int.from_bytes(rng.bytes(32), "big") % O.P, int.from_bytes(rng.bytes(32), "big") % O.P)
             for _ in range(6)]
        if op in (2, 7, 10):  # cyclotomic-subgroup inputs
            f = O.f12_mul(O.f12_conj(f), O.f12_inv(f))
            f = O.f12_mul(f, O.f12_frob2(f))
        elems.append(f)
        others.append(g)
    a = b"".join(O.f12_marshal(f) for f in elems)
    b = b"".join(O.f12_marshal(g) for g in others)
    out = engine.fp12_op(op, a, b)
    ref = {0: lambda f, g: O.f12_mul(f, g), 1: lambda f, g: O.f12_sqr(f), 2: lambda f, g: O.f12_sqr(f),
           3: lambda f, g: O.f12_frob(f), 4: lambda f, g: O.f12_frob2(f), 5: lambda f, g: O.f12_inv(f),
           6: lambda f, g: O.f12_conj(f), 7: lambda f, g: O.f12_pow(f, O.U),
           8: lambda f, g: O.final_exponentiation(f), 9: lambda f, g: O.f12_sqr(f),
           10: lambda f, g: O.f12_sqr(f)}[op]
    for i in range(n):
        assert out[384 * i:384 * (i + 1)] == O.f12_marshal(ref(elems[i], others[i])), f"op {op} elem {i}"


def test_pair_matches_oracle_gt_bytes(engine):
    cases = [(O.G1_GEN, O.G2_GEN), (O.g1_mul(O.G1_GEN, 7), O.G2_GEN), (O.G1_GEN, O.g2_mul(O.G2_GEN, 11)),
             (O.g1_mul(O.G1_GEN, 123456789), O.g2_mul(O.G2_GEN, 987654321)), (None, O.G2_GEN), (O.G1_GEN, None)]
    g1 = b"".join(O.g1_marshal(p) for p, _ in cases)
    g2 = b"".join(O.g2_marshal(q) for _, q in cases)
    gt, codes = engine.pair(g1, g2)
    assert list(codes) == [0] * len(cases)
    for i, (p, q) in enumerate(cases):
        want = O.f12_marshal(O.pair(p, q))
        assert gt[384 * i:384 * (i + 1)] == want, f"pair case {i}"


def test_keygen_and_sign_match_oracle(engine):
    ks = F.scalars(40, b"keygen")
    kb = F.scalar_bytes(ks)
    assert engine.keygen(kb) == R.g2_scalar_base(kb)
    assert engine.set_message(F.LIB_MESSAGE) == 0
    assert engine.sign(kb) == R.sign(F.LIB_MESSAGE, kb)


def test_verify_batch_matches_oracle(engine):
    _, pks, sigs = F.keys_and_sigs(64, seed=b"vb")
    sigs = F.tamper(sigs, every=8)
    assert engine.set_message(F.LIB_MESSAGE) == 0
    got = engine.verify_batch(pks, sigs)
    want = R.verify_batch(F.LIB_MESSAGE, pks, sigs, nthreads=8)
    assert list(got) == list(want)
    assert (got == 1).sum() == 8 and (got == 0).sum() == 56


def test_verify_batch_edge_cases(engine):
    msg = F.TEST_MESSAGES[0]
    ks, pks, sigs = F.keys_and_sigs(4, msg=msg, seed=b"edge")
    z128, z64 = bytes(128), bytes(64)
    off_curve_g1 = (1).to_bytes(32, "big") + (1).to_bytes(32, "big")
    off_curve_g2 = bytes(127) + b"\x01"
    cases_pk = [pks[0:128], z128, z128, pks[128:256], off_curve_g2, pks[384:512]]
    cases_sig = [sigs[0:64], z64, sigs[64:128], z64, sigs[192:256], off_curve_g1]
    pk_b, sig_b = b"".join(cases_pk), b"".join(cases_sig)
    assert engine.set_message(msg) == 0
    got = list(engine.verify_batch(pk_b, sig_b))
    # oracle verdicts
    want = []
    for p, s in zip(cases_pk, cases_sig):
        P, e1 = O.g2_unmarshal(p, "go")
        S, e2 = O.g1_unmarshal(s, "go")
        if e1:
            want.append(R.RC_PK_UNMARSHAL)
        elif e2:
            want.append(R.RC_SIG_UNMARSHAL)
        else:
            want.append(0 if O.verify_signature(P, msg, S) is None else 1)
    assert got == want
    assert got[1] == 0  # infinity pk with infinity sig verifies (e(H,inf) = 1 = e(inf,G2))


def test_hash_reject_message(engine):
    _, pks, sigs = F.keys_and_sigs(2, msg=F.TEST_MESSAGES[1], seed=b"rej")
    assert engine.set_message(F.REJECT_MESSAGES[0]) == 2
    assert list(engine.verify_batch(pks, sigs)) == [2, 2]


def test_combine_g1_matches_oracle(engine):
    _, _, sigs = F.keys_and_sigs(9, seed=b"comb")
    a = sigs[:4 * 64] + sigs[0:64] + bytes(64)
    b = sigs[4 * 64:8 * 64] + O.g1_marshal(O.g1_neg(O.g1_unmarshal(sigs[0:64])[0])) + sigs[64:128]
    out, codes = engine.combine_g1(a, b)
    assert list(codes) == [0] * 6
    for i in range(6):
        assert out[64 * i:64 * i + 64] == R.g1_add(a[64 * i:64 * i + 64], b[64 * i:64 * i + 64])
    assert out[4 * 64:5 * 64] == bytes(64)  # sig + (-sig) = infinity


def test_verify_aggregate_matches_oracle(engine, agg_level):
    n_reg = 50
    ks, reg, _ = F.keys_and_sigs(n_reg, seed=b"agg")
    msg = F.LIB_MESSAGE
    assert list(engine.registry_load(reg)) == [0] * n_reg
    assert engine.set_message(msg) == 0
    rng = np.random.default_rng(7)
    # level ranges of a 50-node Handel registry seen from node 3 (partitioner rangeLevel)
    ranges = []
    for lvl in range(1, O.log2_ceil(n_reg) + 1):
        rl, err = O.range_level(3, n_reg, lvl)
        if err is None:
            ranges.append((rl[0], rl[1] - rl[0]))
    ranges.append((0, n_reg))  # full registry (VerifyMultiSignature)
    bitsets = F.random_bitsets(rng, [s for _, s in ranges])
    bitsets[0] = [True] * ranges[0][1]
    sigs = b""
    for (off, size), bits in zip(ranges, bitsets):
        agg = None
        for i, b in enumerate(bits):
            if b:
                s = O.g1_mul(O.hashed_message(msg)[0], ks[off + i])
                agg = s if agg is None else O.g1_add(agg, s)
        sigs += O.g1_marshal(agg)
    sigs = bytearray(sigs)
    sigs[64:128] = F.tamper(bytes(sigs[64:128]), every=1)  # one bad aggregate
    reqs, words = F.pack_requests(ranges, bitsets)
    reqs.append((0, 3, 4, 0))  # bitlen != level size
    bitsets.append([True] * 3)
    sigs += bytes(sigs[0:64])
    codes, agg = engine.verify_aggregate(np.array(reqs, dtype=engine_req_dtype()), words, bytes(sigs), want_agg=True)
    woff = np.array([r[3] for r in reqs], dtype=np.uint64)
    want, want_agg = R.verify_aggregate(msg, reg, [r[0] for r in reqs], [r[1] for r in reqs],
                                        [r[2] for r in reqs], words, woff, bytes(sigs), nthreads=4,
                                        want_agg=True)
    assert list(codes) == list(want)
    for i in range(len(reqs)):
        if want[i] in (0, 1):
            assert agg[128 * i:128 * (i + 1)] == want_agg[128 * i:128 * (i + 1)], f"agg {i}"
    assert codes[1] == 1 and codes[-1] == 3 and codes[0] == 0


def engine_req_dtype():
    from handel_amd.engine import REQ_DTYPE
    return REQ_DTYPE


def test_aggregate_block_complement_matches_oracle(engine, agg_level):
    """Level ranges of a 300-key registry (aligned blocks, clipped last blocks,
    multi-word bitsets) at densities that take the block-sum complement path
    (all set, all but one, just over half) and the direct path (half, one bit),
    with a duplicated key (doubling inside the fold) and an infinity key."""
    n_reg = 300
    ks = F.scalars(n_reg, seed=b"agg-blocks")
    ks[17] = ks[16]                        # duplicate registry key
    reg = bytearray(R.g2_scalar_base(F.scalar_bytes(ks)))
    reg[128 * 40:128 * 41] = bytes(128)    # infinity key (all-zero marshal)
    reg = bytes(reg)
    assert list(engine.registry_load(reg)) == [0] * n_reg
    msg = F.LIB_MESSAGE
    assert engine.set_message(msg) == 0
    ranges = []
    for node in (0, 5, 77, 150, 299):
        for lvl in range(1, O.log2_ceil(n_reg) + 1):
            rl, err = O.range_level(node, n_reg, lvl)
            if err is None:
                ranges.append((rl[0], rl[1] - rl[0]))
    ranges.append((0, n_reg))
    ranges = sorted(set(ranges))
    rng = np.random.default_rng(11)
    bitsets = []
    for i, (off, size) in enumerate(ranges):
        kind = i % 5
        if kind == 0:
            bits = [True] * size
        elif kind == 1:
            bits = [True] * size
            bits[int(rng.integers(size))] = False
        elif kind == 2:
            bits = list(rng.permutation([True] * (size // 2 + 1) + [False] * (size - size // 2 - 1)))
        elif kind == 3:
            bits = list(rng.permutation([True] * (size // 2) + [False] * (size - size // 2)))
        else:
            bits = [False] * size
            bits[int(rng.integers(size))] = True
        bitsets.append([bool(b) for b in bits])
    reqs, words = F.pack_requests(ranges, bitsets)
    sigs = O.g1_marshal(O.G1_GEN) * len(reqs)
    codes, agg = engine.verify_aggregate(np.array(reqs, dtype=engine_req_dtype()), words, sigs, want_agg=True)
    woff = np.array([r[3] for r in reqs], dtype=np.uint64)
    want, want_agg = R.verify_aggregate(msg, reg, [r[0] for r in reqs], [r[1] for r in reqs],
                                        [r[2] for r in reqs], words, woff, sigs, nthreads=4, want_agg=True)
    assert list(codes) == list(want)
    for i in range(len(reqs)):
        assert agg[128 * i:128 * (i + 1)] == want_agg[128 * i:128 * (i + 1)], f"agg {i} {ranges[i]}"


def test_aggregate_unaligned_ranges_match_oracle(engine, agg_level):
    """Ranges that are not Handel level blocks (offsets off the 8-key window
    grid, lengths that straddle windows and words): the window subset-sum fold
    must shift the bitset into registry-aligned windows and never take the
    block complement."""
    n_reg = 200
    ks = F.scalars(n_reg, seed=b"agg-unaligned")
    reg = R.g2_scalar_base(F.scalar_bytes(ks))
    assert list(engine.registry_load(reg)) == [0] * n_reg
    msg = F.LIB_MESSAGE
    assert engine.set_message(msg) == 0
    ranges = [(3, 70), (13, 5), (101, 99), (7, 1), (63, 66), (1, 128), (129, 64), (0, 200), (190, 10)]
    rng = np.random.default_rng(5)
    bitsets = []
    for i, (off, size) in enumerate(ranges):
        p = [0.9, 0.5, 0.1][i % 3]
        bits = [bool(b) for b in rng.random(size) < p]
        if not any(bits):
            bits[0] = True
        bitsets.append(bits)
    bitsets[2] = [True] * ranges[2][1]
    reqs, words = F.pack_requests(ranges, bitsets)
    sigs = O.g1_marshal(O.G1_GEN) * len(reqs)
    codes, agg = engine.verify_aggregate(np.array(reqs, dtype=engine_req_dtype()), words, sigs, want_agg=True)
    woff = np.array([r[3] for r in reqs], dtype=np.uint64)
    want, want_agg = R.verify_aggregate(msg, reg, [r[0] for r in reqs], [r[1] for r in reqs],
                                        [r[2] for r in reqs], words, woff, sigs, nthreads=4, want_agg=True)
    assert list(codes) == list(want)
    for i in range(len(reqs)):
        assert agg[128 * i:128 * (i + 1)] == want_agg[128 * i:128 * (i + 1)], f"agg {i} {ranges[i]}"


def test_empty_batches(engine):
    """n = 0 on every batched entry point: no launch, no error, empty results."""
    assert engine.set_message(F.LIB_MESSAGE) == 0
    assert len(engine.verify_batch(b"", b"")) == 0
    assert len(engine.verify_aggregate(np.zeros(0, dtype=engine_req_dtype()), np.zeros(0, dtype=np.uint64), b"")) == 0
    out, codes = engine.combine_g1(b"", b"")
    assert out == b"" and len(codes) == 0
    assert engine.keygen(b"") == b"" and engine.sign(b"") == b""


@pytest.mark.parametrize("flavor", ["go", "cf"])
def test_full_size_ragged_batch_matches_oracle(request, flavor):
    """BASELINE config 2 at full size plus a ragged tail (4100 checks: more
    teams than one wave per SIMD holds, last workgroup partly filled), every
    verdict against the C restatement of the reference algorithm, under both
    upstream flavors' decode rules (cf: the default curve of every shipped
    simul config)."""
    import bench

    engine = request.getfixturevalue("engine" if flavor == "go" else "engine_cf")
    n = 4100
    assert engine.set_message(F.LIB_MESSAGE) == 0  # make_batch signs with the context's message
    pks, sigs, expect = bench.make_batch(engine, n, seed=99)
    got = engine.verify_batch(pks, sigs)
    want = R.verify_batch(F.LIB_MESSAGE, pks, sigs, nthreads=16, flavor=0 if flavor == "go" else 1)
    assert np.array_equal(got, want)
    assert np.array_equal(got, expect)  # exactly the tampered 1/8 fail


@pytest.mark.parametrize("flavor", ["go", "cf"])
@pytest.mark.parametrize("full", [False, True], ids=["levels", "full_registry"])
def test_full_size_aggregate_matches_oracle(request, full, flavor, agg_level):
    """BASELINE config 3 at full size: 4096 multisigs on a 4000-key registry
    (random Handel levels, or VerifyMultiSignature over the whole registry),
    verdicts and aggregate-key marshals byte-exact against the C restatement,
    under both upstream flavors (cf decodes the registry with its subgroup
    check)."""
    import bench

    engine = request.getfixturevalue("engine" if flavor == "go" else "engine_cf")
    n, n_reg = 4096, 4000
    assert engine.set_message(F.LIB_MESSAGE) == 0
    reqs, words, sigs, expect, _, reg = bench.make_aggregate_batch(engine, n_reg, n, seed=77, full=full)
    codes = engine.verify_aggregate(reqs, words, sigs)  # verdicts only: the GT path alone at level 2
    codes_a, agg = engine.verify_aggregate(reqs, words, sigs, want_agg=True)  # + the G2 fold for the keys
    assert np.array_equal(codes, expect)  # exactly the tampered 1/8 fail
    assert np.array_equal(codes_a, expect)
    want, want_agg = R.verify_aggregate(F.LIB_MESSAGE, reg, reqs["offset"], reqs["bitlen"], reqs["level_size"],
                                        words, reqs["word_offset"].astype(np.uint64), sigs, nthreads=16,
                                        want_agg=True)
    assert np.array_equal(codes, want)
    assert agg == want_agg


@pytest.mark.parametrize("n", [1, 7, 8, 4100])
def test_pack_verdicts_matches_codes(engine, n):
    """hg_pack_verdicts_device: bit j of byte b = (code[8b+j] == 0), tail bits 0;
    the same bytes as the torch restatement in handel_amd/distributed.py."""
    import torch

    from handel_amd.distributed import pack_verdicts

    rng = np.random.default_rng(n)
    codes = rng.choice(np.array([0, 0, 0, 1, 2, 3, 6], dtype=np.int32), size=n)
    d_codes = torch.from_numpy(codes).cuda()
    d_bits = torch.full(((n + 7) // 8,), 0xA5, dtype=torch.uint8, device="cuda")
    engine.pack_verdicts_device(d_codes.data_ptr(), n, d_bits.data_ptr(), torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    want = np.packbits(np.concatenate([codes == 0, np.zeros((-n) % 8, bool)]), bitorder="little")
    assert np.array_equal(d_bits.cpu().numpy(), want)
    assert torch.equal(d_bits, pack_verdicts(d_codes))


@pytest.mark.parametrize("flavor", ["go", "cf"])
def test_verify_split_form_matches_oracle(flavor):
    """Config 2's split form (hg_set_verify_split: k_verify_ml on the compact
    team region, the 12-lane final exponentiation with batched inversions,
    k_fe_verdicts): 4100 ragged checks plus the edge cases of
    test_verify_batch_edge_cases (infinity pk and/or sig, off-curve points)
    against the C restatement, and two contexts with a batch in flight each on
    their own streams give the same codes as the one-kernel form."""
    import torch

    import bench
    from handel_amd.engine import Engine

    dev = torch.device("cuda:0")
    n = 4100
    one = Engine(device=0, flavor=flavor)
    split = [Engine(device=0, flavor=flavor) for _ in range(2)]
    try:
        for e in [one] + split:
            assert e.set_message(F.LIB_MESSAGE) == 0
        for e in split:
            e.set_verify_split(True)
        pks, sigs, expect = bench.make_batch(one, n, seed=77)
        # edge cases in the tail: infinity pk / sig, off-curve points
        z128, z64 = bytes(128), bytes(64)
        off_g1 = (1).to_bytes(32, "big") + (1).to_bytes(32, "big")
        off_g2 = bytes(127) + b"\x01"
        pks = pks + z128 + z128 + pks[:128] + off_g2 + pks[128:256]
        sigs = sigs + z64 + sigs[:64] + z64 + sigs[64:128] + off_g1
        m = n + 5
        # the one-kernel form against the oracle on the batch (its edge cases:
        # test_verify_batch_edge_cases, test_cf_signature_decode_edge_cases),
        # the split form against the one-kernel form on everything
        want = one.verify_batch(pks, sigs)
        assert np.array_equal(want[:n], R.verify_batch(F.LIB_MESSAGE, pks[:128 * n], sigs[:64 * n], nthreads=16,
                                                       flavor=0 if flavor == "go" else 1))
        if flavor == "go":
            assert np.array_equal(want, R.verify_batch(F.LIB_MESSAGE, pks, sigs, nthreads=16, flavor=0))
        assert np.array_equal(split[0].verify_batch(pks, sigs), want)
        # both split contexts in flight at once on their own streams
        d_pks = torch.frombuffer(bytearray(pks), dtype=torch.uint8).to(dev)
        d_sigs = torch.frombuffer(bytearray(sigs), dtype=torch.uint8).to(dev)
        codes = [torch.full((m,), -1, dtype=torch.int32, device=dev) for _ in split]
        streams = [torch.cuda.Stream(dev) for _ in split]
        torch.cuda.synchronize(dev)
        for rep in range(3):
            for e, c, s in zip(split, codes, streams):
                e.verify_batch_device(d_pks.data_ptr(), d_sigs.data_ptr(), m, c.data_ptr(), s.cuda_stream)
        torch.cuda.synchronize(dev)
        for c in codes:
            assert np.array_equal(c.cpu().numpy(), want)
        assert np.array_equal(want[:n], expect)
    finally:
        for e in [one] + split:
            e.close()


def test_verify_split_form_small_batches(engine):
    """The split form on batches smaller than one workgroup of either half
    (1 and 7 checks: one partly filled 4-team Miller wave, one partly filled
    5-team final-exponentiation wave, one inversion block) gives the one-kernel
    form's codes."""
    from handel_amd.engine import Engine

    split = Engine(device=0, flavor="go")
    try:
        assert engine.set_message(F.LIB_MESSAGE) == 0
        assert split.set_message(F.LIB_MESSAGE) == 0
        split.set_verify_split(True)
        _, pks, sigs = F.keys_and_sigs(7, seed=b"split-small")
        sigs = F.tamper(sigs, every=3)
        for n in (1, 7):
            want = engine.verify_batch(pks[:128 * n], sigs[:64 * n])
            assert list(split.verify_batch(pks[:128 * n], sigs[:64 * n])) == list(want)
        assert list(want) == list(R.verify_batch(F.LIB_MESSAGE, pks, sigs, nthreads=4))
    finally:
        split.close()
