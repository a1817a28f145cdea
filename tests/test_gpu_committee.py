"""GPU suite: BASELINE config 5's unit of work at full size.

One committee = a 4096-key registry (an exact power of two: the top Handel
block is the whole registry and the last 16-key window is full, edges the
4000-key tests never reach) verifying 4096 incoming multisignatures at random
Handel levels (partitioner rangeLevel) plus VerifyMultiSignature requests over
the whole registry (crypto.go:120-137, processing.go:342-368). Verdicts and
marshalled aggregate keys are checked against the C restatement of the
reference algorithm.
"""

import numpy as np
import pytest

from oracle import ref_lib as R
from tests import _fixtures as F

pytestmark = pytest.mark.gpu


def committee_batch(engine, n_reg=4096, n_levels=3584, n_full=512, seed=55):
    """n_levels multisigs at random levels + n_full full-registry ones, all on
    the same seeded registry (bench.make_aggregate_batch draws the keys from
    the seed, so both halves see identical keys)."""
    import bench

    a = bench.make_aggregate_batch(engine, n_reg, n_levels, seed=seed)
    b = bench.make_aggregate_batch(engine, n_reg, n_full, seed=seed, full=True)
    assert a[5] == b[5]
    reqs_b = b[0].copy()
    reqs_b["word_offset"] += len(a[1])
    reqs = np.concatenate([a[0], reqs_b])
    words = np.concatenate([a[1], b[1]])
    return reqs, words, a[2] + b[2], np.concatenate([a[3], b[3]]), a[5]


@pytest.mark.parametrize("flavor", ["go", "cf"])
def test_full_size_committee_matches_oracle(request, flavor):
    engine = request.getfixturevalue("engine" if flavor == "go" else "engine_cf")
    assert engine.set_message(F.LIB_MESSAGE) == 0
    reqs, words, sigs, expect, reg = committee_batch(engine)
    assert engine.registry_non_g2() == 0
    assert engine.prepare_aggregate() == 0
    assert engine.aggregate_tables() == 2
    assert len(reqs) == 4096 and int((reqs["bitlen"] == 4096).sum()) == 512
    codes = engine.verify_aggregate(reqs, words, sigs)
    assert np.array_equal(codes, expect)
    codes_a, agg = engine.verify_aggregate(reqs, words, sigs, want_agg=True)
    assert np.array_equal(codes_a, expect)
    want, want_agg = R.verify_aggregate(F.LIB_MESSAGE, reg, reqs["offset"], reqs["bitlen"], reqs["level_size"],
                                        words, reqs["word_offset"].astype(np.uint64), sigs, nthreads=16,
                                        want_agg=True)
    assert np.array_equal(codes, want)
    assert agg == want_agg
    # the top level of node ids >= 2048 is the aligned half [0, 2048) and vice
    # versa; full-size blocks of 2048 are present at every level size
    assert int((reqs["bitlen"] == 2048).sum()) > 0
    full = reqs["bitlen"] == 4096
    assert engine.verify_multisig(reqs["bitlen"][full], reqs["word_offset"][full], words,
                                  b"".join(sigs[64 * i:64 * i + 64] for i in np.flatnonzero(full))).tolist() \
        == expect[full].tolist()
