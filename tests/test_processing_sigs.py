"""CPU suite: BatchVerifier refuses signatures the reference cannot unmarshal
instead of padding them.

x/crypto's G1.Unmarshal wants exactly 64 bytes (SigBLS.UnmarshalBinary,
bn256/go/bn256.go:182-190: "bn256: multisig can't unmarshal"); cloudflare's
wants at least 64 and ignores what follows (bn256/cf/bn256.go:183-190:
"bn256: multisig can't unmarshal: bn256: not enough data"). A stub engine
records what reaches the GPU; the texts come from the C library's
hg_code_string (no GPU needed).
"""

import numpy as np
import pytest

from handel_amd import _lib
from handel_amd.processing import BatchVerifier, sig_length_code
from handel_amd.sigprocessing import IncomingSig, MultiSig

GO_TEXT = "bn256: multisig can't unmarshal"
CF_TEXT = "bn256: multisig can't unmarshal: bn256: not enough data"


class StubEngine:
    """The Engine surface BatchVerifier uses; every submitted request passes."""

    def __init__(self, flavor):
        self.flavor_name = flavor
        self.flavor = _lib.HG_FLAVOR_CF if flavor == "cf" else _lib.HG_FLAVOR_GO
        self.L = _lib.load(build_if_missing=False)
        self.submitted = []

    def registry_load(self, pks):
        return np.zeros(len(pks) // 128, dtype=np.int32)

    def set_message(self, msg):
        return 0

    def prepare_aggregate(self):
        return 0

    def verify_aggregate(self, reqs, words, sigs):
        assert len(sigs) == 64 * len(reqs)
        self.submitted.append(sigs)
        return np.zeros(len(reqs), dtype=np.int32)

    def verify_multisig(self, bitlens, woffs, words, sigs):
        assert len(sigs) == 64 * len(bitlens)
        self.submitted.append(sigs)
        return np.zeros(len(bitlens), dtype=np.int32)

    def code_string(self, c):
        return self.L.hg_code_string(int(c), self.flavor).decode()

    def processing_error_string(self, c):
        return self.L.hg_processing_error_string(int(c), self.flavor).decode()


@pytest.mark.parametrize("flavor", ["go", "cf"])
def test_bad_signature_lengths_get_the_reference_errors(flavor):
    eng = StubEngine(flavor)
    bv = BatchVerifier(eng, bytes(128 * 16), b"msg", node_id=3)
    lengths = [0, 32, 63, 64, 65, 128]
    sigs = [bytes([7]) * n for n in lengths]
    items = [IncomingSig(origin=0, level=1, ms=MultiSig(1, 1, s)) for s in sigs]
    out = bv.verify_levels(items)
    for n, o in zip(lengths, out):
        if n < 64:
            assert o == (CF_TEXT if flavor == "cf" else GO_TEXT), (n, o)
        elif n == 64 or flavor == "cf":
            assert o is None, (n, o)  # cloudflare reads the first 64 bytes
        else:
            assert o == GO_TEXT, (n, o)
    # only the parseable ones reached the GPU, each as exactly 64 bytes
    sent = b"".join(eng.submitted)
    ok = [s for s in sigs if sig_length_code(flavor, s) == 0]
    assert sent == b"".join(s[:64] for s in ok)
    # raw codes and VerifyMultiSignature follow the same rule
    codes = bv.verify_ranges([(0, 2, [True, False], s) for s in sigs])
    want = [(_lib.HG_ERR_SIG_CF_SHORT if flavor == "cf" else _lib.HG_ERR_SIG_UNMARSHAL)
            if (len(s) < 64 or (flavor == "go" and len(s) != 64)) else 0 for s in sigs]
    assert list(codes) == want
    txt = bv.verify_multisignatures([([True] * 16, s) for s in sigs])
    assert [t is None for t in txt] == [w == 0 for w in want]


def test_batcher_submit_checks_the_word_count():
    """hg_batcher_submit copies ceil(bitlen/64) words: a shorter array is refused
    before the native call."""
    from handel_amd.engine import Batcher

    b = Batcher.__new__(Batcher)  # no context needed: the check precedes the call
    with pytest.raises(ValueError):
        Batcher.submit(b, b"m", 0, 65, 65, np.zeros(1, dtype=np.uint64), bytes(64))
