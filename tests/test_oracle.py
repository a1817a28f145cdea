"""CPU suite: the oracle is pinned against everything the reference and its
upstream define, and the C restatement against the Python
one. The reference's own bn256 tests are property tests (no known-answer
vectors), so those properties are re-run here: TestSign, TestCombine,
TestMarshalling (bn256/go/bn256_test.go:39-103)."""

import ctypes
import hashlib

import numpy as np
import pytest

from oracle import bn256_oracle as O
from oracle import ref_lib as R
from tests import _fixtures as F


# ------------------------------------------------------------------ constants
def test_curve_constants():
    assert O.P.bit_length() == 256 and O.P > 2 ** 255
    assert O.P % 4 == 3
    assert O.g1_on_curve(*O.G1_GEN) and O.g2_on_curve(*O.G2_GEN)
    assert O.g1_mul(O.G1_GEN, O.ORDER) is None
    assert O.g2_mul(O.G2_GEN, O.ORDER) is None
    # twist b' = 3/xi
    assert O.f2_mul(O.TWIST_B, O.XI) == (0, 3)


def test_xcrypto_frobenius_constants():
    """x/crypto/bn256 constants.go values (decimal, i-coefficient first)."""
    assert O.GAMMA1[1] == (8669379979083712429711189836753509758585994370025260553045152614783263110636,
                           19998038925833620163537568958541907098007303196759855091367510456613536016040)
    assert O.XI_TO_P_MINUS_1_OVER_3 == (
        26098034838977895781559542626833399156321265654106457577426020397262786167059,
        15931493369629630809226283458085260090334794394361662678240713231519278691715)
    assert O.XI_TO_P_MINUS_1_OVER_2 == (
        50997318142241922852281555961173165965672272825141804376761836765206060036244,
        38665955945962842195025998234511023902832543644254935982879660597356748036009)
    assert O.XI_TO_PSQ_MINUS_1_OVER_3 == \
        65000549695646603727810655408050771481677621702948236658134783353303381437752


def test_naf_is_six_u_plus_two():
    assert sum(d << i for i, d in enumerate(O.SIX_U_PLUS_2_NAF)) == 6 * O.U + 2
    assert len(O.SIX_U_PLUS_2_NAF) == 66
    assert sum(1 for d in O.SIX_U_PLUS_2_NAF if d) == 19


# ------------------------------------------------------------------ pairing
def test_final_exponentiation_is_exact_power():
    f = O.miller(O.G2_GEN, O.G1_GEN)
    assert O.final_exponentiation(f) == O.f12_pow(f, (O.P ** 12 - 1) // O.ORDER)


def test_pairing_independent_of_addition_chain():
    """Plain binary expansion of 6u+2 gives the same reduced pairing as the NAF."""
    binary = [int(b) for b in reversed(bin(6 * O.U + 2)[2:])]
    P1 = O.g1_mul(O.G1_GEN, 5)
    Q1 = O.g2_mul(O.G2_GEN, 9)
    a = O.final_exponentiation(O.miller(Q1, P1))
    b = O.final_exponentiation(O.miller(Q1, P1, naf=binary))
    assert a == b


def _g2base_lines_normalised(p, unit=False):
    """The G2Base Miller loop of O.miller with every line divided by its
    constant coefficient a (k_g2_lines' table, the LINE_FIX / LFEV programs):
    yields (a, line) per step; unit: the signature at infinity (SX = NSY = 0,
    every line w^3)."""
    def norm(a, b, c):
        ai = O.f2_inv(a)
        b, c = O.f2_mul(b, ai), O.f2_mul(c, ai)
        return a, ((O.F2_ZERO, O.F2_ZERO) if unit else (b, c))

    q = O.G2_GEN
    px, py = p
    r, r2, nq = (q[0], q[1], O.F2_ONE, O.F2_ONE), O.f2_sqr(q[1]), (q[0], O.f2_neg(q[1]))
    naf = O.SIX_U_PLUS_2_NAF
    out = []
    for i in range(len(naf) - 1, 0, -1):
        a, b, c, r = O._line_double(r, px, py)
        out.append(("dbl", norm(a, b, c)))
        if naf[i - 1]:
            a, b, c, r = O._line_add(r, q if naf[i - 1] > 0 else nq, px, py, r2)
            out.append(("add", norm(a, b, c)))
    q1 = (O.f2_mul(O.f2_conj(q[0]), O.XI_TO_P_MINUS_1_OVER_3), O.f2_mul(O.f2_conj(q[1]), O.XI_TO_P_MINUS_1_OVER_2))
    mq2 = (O.f2_muls(q[0], O.XI_TO_PSQ_MINUS_1_OVER_3), q[1])
    for pt in (q1, mq2):
        a, b, c, r = O._line_add(r, pt, px, py, O.f2_sqr(pt[1]))
        out.append(("add", norm(a, b, c)))
    return out


def _miller_normalised(p, unit=False):
    f, first = O.F12_ONE, True
    for kind, (a, (b, c)) in _g2base_lines_normalised(p, unit):
        assert a != O.F2_ZERO  # the normalisation divides by every line's a
        if kind == "dbl" and not first:
            f = O.f12_sqr(f)
        first = False
        f = O._mul_line(f, O.F2_ONE, b, c)
    return f


def test_normalised_g2base_lines_give_the_same_pairing():
    """The kernels' G2Base lines (a = 1): same reduced pairing at -sig as
    x/crypto's, and the all-w^3 lines of a signature at infinity reduce to 1."""
    assert len(_g2base_lines_normalised(O.G1_GEN)) == 85  # kNumLines
    for k in (1, 77):
        p = O.g1_neg(O.g1_mul(O.G1_GEN, k))
        assert O.final_exponentiation(_miller_normalised(p)) == O.pair(p, O.G2_GEN)
    assert O.final_exponentiation(_miller_normalised(O.G1_GEN, unit=True)) == O.F12_ONE


def test_final_exponentiation_fc_is_a_fixed_power():
    """The GPU's hard part (Fuentes-Castaneda et al.): FE^m with m coprime to
    the group order, so x -> x^m is a bijection of GT and equality tests agree
    with the reference's chain, for pairing values and arbitrary elements."""
    import math
    import random
    m = O.FC_EXPONENT
    assert math.gcd(m, O.ORDER) == 1
    rng = random.Random(11)
    f1 = O.miller(O.g2_mul(O.G2_GEN, 5), O.g1_mul(O.G1_GEN, 7))
    f2 = [(rng.randrange(O.P), rng.randrange(O.P)) for _ in range(6)]
    for f in (f1, f2):
        assert O.final_exponentiation_fc(f) == O.f12_pow(O.final_exponentiation(f), m)
    assert O.final_exponentiation_fc(O.F12_ONE) == O.F12_ONE


def test_bilinearity_and_nondegeneracy():
    e = O.pair(O.G1_GEN, O.G2_GEN)
    assert not O.f12_is_one(e)
    assert O.f12_is_one(O.f12_pow(e, O.ORDER))
    a, b = 1234567, 7654321
    assert O.pair(O.g1_mul(O.G1_GEN, a), O.g2_mul(O.G2_GEN, b)) == O.f12_pow(e, a * b)
    assert O.pair(None, O.G2_GEN) == O.F12_ONE and O.pair(O.G1_GEN, None) == O.F12_ONE


def test_c_restatement_matches_python_pair():
    for k1, k2 in ((1, 1), (3, 17), (2 ** 200 + 5, 99)):
        p, q = O.g1_mul(O.G1_GEN, k1), O.g2_mul(O.G2_GEN, k2)
        assert R.pair(O.g1_marshal(p), O.g2_marshal(q)) == O.f12_marshal(O.pair(p, q))
    assert R.pair(bytes(64), O.g2_marshal(O.G2_GEN)) == O.f12_marshal(O.F12_ONE)


# ------------------------------------------------------------------ hashing
def test_hash_admissibility_of_reference_messages():
    for m in [F.LIB_MESSAGE] + F.TEST_MESSAGES:
        k, err = O.hash_scalar(m)
        assert err is None and 0 < k < O.ORDER
        assert k == int.from_bytes(hashlib.sha256(m).digest(), "big")
    for m in F.REJECT_MESSAGES:
        assert O.hash_scalar(m) == (None, "EOF")


def test_rand_int_rejection_reads_next_block():
    # crypto/rand.Int with a reader holding two 32-byte blocks: first >= n is rejected
    big = (O.ORDER + 5).to_bytes(32, "big")
    k, err = O.rand_int(O.ByteReader(big + (7).to_bytes(32, "big")), O.ORDER)
    assert (k, err) == (7, None)
    assert O.rand_int(O.ByteReader(big), O.ORDER) == (None, "EOF")


# ------------------------------------------------------------------ reference property tests
def test_sign_verify_roundtrip():  # bn256_test.go TestSign
    msg = b"Get Funky Tonight"
    sk, pk = O.new_key_pair(O.SeededReader(b"sign"))
    sig, err = O.sign(sk, msg)
    assert err is None
    assert len(O.g1_marshal(sig)) == 64 and len(O.g2_marshal(pk)) == 128
    assert O.verify_signature(pk, msg, sig) is None
    assert O.verify_signature(pk, b"other message", sig) is not None


def test_combine():  # bn256_test.go TestCombine
    msg = b"Get Funky Tonight"
    r = O.SeededReader(b"combine")
    sk1, pk1 = O.new_key_pair(r)
    sk2, pk2 = O.new_key_pair(r)
    assert O.g2_marshal(pk1) != O.g2_marshal(pk2)
    s1, _ = O.sign(sk1, msg)
    s2, _ = O.sign(sk2, msg)
    assert O.verify_signature(O.g2_add(pk1, pk2), msg, O.g1_add(s1, s2)) is None
    assert O.verify_signature_fast(O.g2_add(pk1, pk2), msg, O.g1_add(s1, s2)) is None


def test_marshalling_roundtrip():  # bn256_test.go TestMarshalling
    sk, pk = O.new_key_pair(O.SeededReader(b"marshal"))
    skb = O.sk_marshal(sk)
    assert int.from_bytes(skb, "big") == sk and (len(skb) == 0 or skb[0] != 0)
    for flavor in ("go", "cf"):
        pt, err = O.g2_unmarshal(O.g2_marshal(pk), flavor)
        assert err is None and pt == pk


def test_unmarshal_flavors():
    g1 = O.g1_marshal(O.G1_GEN)
    # x/crypto accepts coordinates >= p (taken mod p); cloudflare rejects them
    x = (1 + O.P).to_bytes(32, "big")
    assert O.g1_unmarshal(x + g1[32:], "go") == (O.G1_GEN, None)
    assert O.g1_unmarshal(x + g1[32:], "cf") == (None, O.ERR_CF_EXCEEDS)
    assert O.g1_unmarshal(g1[:63], "go")[1] == O.ERR_GO_SIG_UNMARSHAL
    assert O.g1_unmarshal(g1[:63], "cf")[1] == O.ERR_CF_NOT_ENOUGH
    assert O.g1_unmarshal(g1 + b"\x00", "cf") == (O.G1_GEN, None)
    assert O.g1_unmarshal(bytes(64), "go") == (None, None)
    assert O.g2_unmarshal(bytes(128), "go") == (None, None)
    bad = bytes(63) + b"\x05" + bytes(32)
    assert O.g1_unmarshal(bad, "go")[1] == O.ERR_GO_SIG_UNMARSHAL
    assert O.g1_unmarshal(bad, "cf")[1] == O.ERR_CF_MALFORMED


def test_product_form_matches_reference_verdicts():
    msg = F.TEST_MESSAGES[0]
    ks, pks, sigs = F.keys_and_sigs(6, msg=msg, seed=b"prod")
    sigs = F.tamper(sigs, every=3)
    a = R.verify_batch(msg, pks, sigs, fast=0)
    b = R.verify_batch(msg, pks, sigs, fast=1)
    c = R.verify_batch(msg, pks, sigs, fast=2)
    assert list(a) == list(b) == list(c) == [1, 0, 0, 1, 0, 0]
    py = [0 if O.verify_signature(O.g2_unmarshal(pks[128 * i:128 * i + 128])[0], msg,
                                  O.g1_unmarshal(sigs[64 * i:64 * i + 64])[0]) is None else 1 for i in range(6)]
    assert list(a) == py


def test_rehash_per_check_matches_batch_hash():
    """bench.py's CPU baseline hashes the message on every check, as the
    reference's VerifySignature does (bn256/go/bn256.go:82-94): same verdicts."""
    msg = F.TEST_MESSAGES[0]
    ks, pks, sigs = F.keys_and_sigs(4, msg=msg, seed=b"rehash")
    sigs = F.tamper(sigs, every=2)
    once = R.verify_batch(msg, pks, sigs, nthreads=2, fast=2)
    R.set_rehash(True)
    try:
        each = R.verify_batch(msg, pks, sigs, nthreads=2, fast=2)
    finally:
        R.set_rehash(False)
    assert list(once) == list(each) == [1, 0, 1, 0]


def test_algorithmic_work_per_check_is_pinned():
    """bench.py's work figures = the oracle's op counter for one check: the
    reference's product-form check (fast=2, effective_rate) and the algorithm
    k_verify runs (fast=3: normalised G2Base lines, Fuentes-Castaneda hard
    part)."""
    import bench

    L = R.lib()
    L.ref_fp_mul_count.restype = ctypes.c_uint64
    _, pks, sigs = F.keys_and_sigs(3, seed=b"cnt")
    for fast, want in ((2, bench.FPMUL_REFERENCE_CHECK), (3, bench.FPMUL_PER_CHECK)):
        counts = []
        for n in (1, 3):
            L.ref_reset_count(1)
            R.verify_batch(F.LIB_MESSAGE, pks[:128 * n], sigs[:64 * n], nthreads=1, fast=fast)
            counts.append(L.ref_fp_mul_count())
        L.ref_reset_count(0)
        assert (counts[1] - counts[0]) // 2 == want


def test_sig_pairing_work_is_pinned():
    """The GT path's check kernel (k_verify_sig) runs one pairing, G2Base at
    -sig, and its final exponentiation: the oracle's count of the same check
    with the pk side off (pk = infinity, fast=3) is bench.FPMUL_PER_SIG_PAIRING."""
    import bench

    L = R.lib()
    L.ref_fp_mul_count.restype = ctypes.c_uint64
    _, _, sigs = F.keys_and_sigs(3, seed=b"cnt")
    inf = bytes(128 * 3)
    counts = []
    for n in (1, 3):
        L.ref_reset_count(1)
        R.verify_batch(F.LIB_MESSAGE, inf[:128 * n], sigs[:64 * n], nthreads=1, fast=3)
        counts.append(L.ref_fp_mul_count())
    L.ref_reset_count(0)
    assert (counts[1] - counts[0]) // 2 == bench.FPMUL_PER_SIG_PAIRING


# ------------------------------------------------------------------ Handel-level helpers
def test_range_level_matches_partitioner_table():
    """The reference's own table: partitioner_test.go:296-343 TestPartitionerBinTreeRangeAt (n = 17)."""
    table = [(1, 0, False, 1, 2), (1, 1, False, 0, 1), (1, 2, False, 2, 4), (1, 3, False, 4, 8),
             (1, 4, False, 8, 16), (1, 5, False, 16, 17), (16, 0, False, 16, 17), (16, 1, True, 0, 0),
             (16, 2, True, 0, 0), (16, 3, True, 0, 0), (16, 4, True, 0, 0), (16, 5, False, 0, 16),
             (1, 7, True, 0, 0)]
    for node, lvl, is_err, lo, hi in table:
        rng_, err = O.range_level(node, 17, lvl)
        if is_err:
            assert err is not None, (node, lvl)
        else:
            assert err is None and rng_ == (lo, hi), (node, lvl, rng_)


def test_bitset_marshal_roundtrip():
    rng = np.random.default_rng(3)
    for n in (1, 63, 64, 65, 2048):
        bits = [bool(b) for b in rng.random(n) < 0.7]
        assert O.bitset_unmarshal(O.bitset_marshal(bits)) == bits
        blob = O.multisig_marshal(bits, O.G1_GEN)
        assert int.from_bytes(blob[:2], "big") == 2 + 8 + 8 * ((n + 63) // 64)


def test_aggregate_c_matches_python():
    n = 12
    ks, reg, _ = F.keys_and_sigs(n, seed=b"aggc")
    rng = np.random.default_rng(5)
    bitsets = F.random_bitsets(rng, [n, 8, 4])
    ranges = [(0, n), (8, 8)[:2], (4, 4)]
    ranges = [(0, n), (0, 8), (8, 4)]
    msg = F.LIB_MESSAGE
    h, _ = O.hashed_message(msg)
    sigs = b""
    pks = [O.g2_unmarshal(reg[128 * i:128 * i + 128])[0] for i in range(n)]
    for (off, size), bits in zip(ranges, bitsets):
        agg = None
        for i, b in enumerate(bits):
            if b:
                s = O.g1_mul(h, ks[off + i])
                agg = s if agg is None else O.g1_add(agg, s)
        sigs += O.g1_marshal(agg)
    reqs, words = F.pack_requests(ranges, bitsets)
    codes, agg_b = R.verify_aggregate(msg, reg, [r[0] for r in reqs], [r[1] for r in reqs], [r[2] for r in reqs],
                                      words, [r[3] for r in reqs], sigs, want_agg=True)
    assert list(codes) == [0, 0, 0]
    for j, ((off, size), bits) in enumerate(zip(ranges, bitsets)):
        st, agg = O.aggregate_pk(pks[off:off + size], bits)
        assert agg_b[128 * j:128 * j + 128] == O.g2_marshal(agg)
        assert O.verify_request(pks, off, off + size, bits, O.g1_unmarshal(sigs[64 * j:64 * j + 64])[0],
                                msg) is None


def test_aggregate_error_precedence_follows_the_reference_flow():
    """When several errors apply to one request, the oracle reports the one
    the reference meets first: the signature's unmarshal in
    Handel.parseSignatures (handel.go:390-395) before the bit length
    (handel.go:399-402, processing.go:350-352); hashedMessage inside
    VerifySignature (bn256/go/bn256.go:84-88) before the nil aggregate's
    pairing (the panic, HG_ERR_EMPTY_AGG)."""
    import numpy as np

    from oracle import bn256_oracle as O
    from oracle import ref_lib as R
    from tests import _fixtures as F

    ks, reg, _ = F.keys_and_sigs(8, seed=b"precedence")
    good = R.sign(F.LIB_MESSAGE, F.scalar_bytes(ks[:1]))
    bad = b"\xff" * 32 + good[32:]  # x >= p: no point
    #            (off, bitlen, level, word)  words
    cases = [((0, 8, 8, 0), 0xFF, bad, 5),    # bad signature only
             ((0, 7, 8, 0), 0x7F, bad, 5),    # bad signature + bit length off its level
             ((0, 8, 8, 0), 0x00, bad, 5),    # bad signature + empty bitset
             ((0, 7, 8, 0), 0x00, good, 3),   # level + empty
             ((0, 8, 8, 0), 0x00, good, 6),   # empty only
             ((0, 1, 1, 0), 0x01, good, 0)]   # key 0's own signature
    reqs = [c[0] for c in cases]
    words = np.array([c[1] for c in cases], dtype=np.uint64)
    woff = np.arange(len(cases), dtype=np.uint64)
    sigs = b"".join(c[2] for c in cases)
    got = R.verify_aggregate(F.LIB_MESSAGE, reg, [r[0] for r in reqs], [r[1] for r in reqs], [r[2] for r in reqs],
                             words, woff, sigs, nthreads=1)
    assert got.tolist() == [c[3] for c in cases]
    # an unhashable message: EOF before the nil aggregate, the level error first
    msg = F.REJECT_MESSAGES[0]
    assert O.hash_scalar(msg)[1] is not None
    got = R.verify_aggregate(msg, reg, [r[0] for r in reqs], [r[1] for r in reqs], [r[2] for r in reqs],
                             words, woff, sigs, nthreads=1)
    assert got.tolist() == [5, 5, 5, 3, 2, 2]
    pks = [O.g2_unmarshal(reg[128 * i:128 * i + 128], "go")[0] for i in range(8)]
    assert O.verify_request(pks, 0, 8, [False] * 8, O.G1_GEN, msg) == "handel: EOF"
    assert O.verify_request(pks, 0, 8, [False] * 8, O.G1_GEN, F.LIB_MESSAGE) == O.ERR_EMPTY_AGGREGATE
