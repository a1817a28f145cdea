"""CPU suite: the C-ABI library loads and exports every symbol
include/handel_gpu.h declares (no compute calls without a GPU), and the
Python binding declares exactly that set."""

import ctypes
import os
import re

from handel_amd import _lib
from handel_amd import build as B

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_symbols(header="handel_gpu.h"):
    text = open(os.path.join(ROOT, "include", header)).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return set(re.findall(r"^\s*(?:const\s+)?[A-Za-z_]\w*\s*\**\s*(hg_\w+)\s*\(", text, flags=re.M))


def test_header_declares_expected_entry_points():
    syms = declared_symbols()
    for s in ("hg_create", "hg_verify_batch", "hg_verify_aggregate", "hg_pair", "hg_registry_load",
              "hg_set_message", "hg_combine_g1", "hg_aggregate_pk", "hg_keygen", "hg_sign"):
        assert s in syms


def test_library_exports_every_declared_symbol():
    path = B.build_library()
    lib = ctypes.CDLL(path)
    for s in declared_symbols():
        assert hasattr(lib, s), s
    assert set(_lib.SIGNATURES) == declared_symbols()


def test_version_and_code_strings_without_gpu():
    L = _lib.load(build_if_missing=False)
    assert L.hg_version() >= 1
    assert L.hg_code_string(1, 0) == b"bn256: signature invalid"
    assert L.hg_code_string(3, 0) == b"handel: inconsistent bitset with given level"
    assert L.hg_code_string(2, 0) == b"EOF"
    assert L.hg_code_string(7, 1) == b"bn256: coordinate exceeds modulus"


def test_exact_error_strings_without_gpu():
    """Every code's text (hg_code_string) and the verifySignature wrapping
    (hg_processing_error_string), against the reference's error values."""
    L = _lib.load(build_if_missing=False)
    go, cf = _lib.HG_FLAVOR_GO, _lib.HG_FLAVOR_CF
    code = lambda c, f=go: L.hg_code_string(c, f).decode()  # noqa: E731
    proc = lambda c, f=go: L.hg_processing_error_string(c, f).decode()  # noqa: E731
    assert code(_lib.HG_OK) == "" and proc(_lib.HG_OK) == ""
    # bn256/go/bn256.go:91,117,186; processing.go:351; crypto.go:123
    assert code(_lib.HG_ERR_PK_UNMARSHAL) == "unable to unmarshal"
    assert code(_lib.HG_ERR_SIG_UNMARSHAL) == "bn256: multisig can't unmarshal"
    assert code(_lib.HG_ERR_MULTI_SIZES) == "verify multisignature: inconsistent sizes"
    # cloudflare wraps the G1 error in SigBLS.UnmarshalBinary (bn256/cf/bn256.go:183-190)
    assert code(_lib.HG_ERR_SIG_CF_EXCEEDS, cf) == "bn256: multisig can't unmarshal: bn256: coordinate exceeds modulus"
    assert code(_lib.HG_ERR_SIG_CF_MALFORMED, cf) == "bn256: multisig can't unmarshal: bn256: malformed point"
    assert code(_lib.HG_ERR_SIG_CF_SHORT, cf) == "bn256: multisig can't unmarshal: bn256: not enough data"
    assert code(_lib.HG_ERR_CF_MALFORMED, cf) == "bn256: malformed point"
    # processing.go:361-365 wraps VerifySignature's errors; the level error is returned as is (:350-352)
    assert proc(_lib.HG_ERR_SIG_INVALID) == "handel: bn256: signature invalid"
    assert proc(_lib.HG_ERR_HASH_EOF) == "handel: EOF"
    assert proc(_lib.HG_ERR_LEVEL) == "handel: inconsistent bitset with given level"
    assert "handel: handel:" not in "".join(proc(c) for c in range(14))


def test_null_handles_are_refused_without_gpu():
    """Entry points that take a context or lane refuse NULL before touching
    the device (no GPU here: nothing else may run)."""
    L = _lib.load(build_if_missing=False)
    assert L.hg_context_simds(None) == 0
    assert L.hg_lane_set_latency_form(None, 2048) == _lib.HG_ERR_ARG
    assert L.hg_lane_set_pairing_padding(None, 1) == _lib.HG_ERR_ARG
    assert L.hg_sig_pairing_device(None, None, 0, None, 0, None) == _lib.HG_ERR_ARG
    assert L.hg_set_verify_split(None, 1) == _lib.HG_ERR_ARG
    assert L.hg_set_fold_overlap(None, 1) == _lib.HG_ERR_ARG
