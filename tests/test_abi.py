"""CPU suite: the C-ABI library loads and exports every symbol
include/handel_gpu.h declares (no compute calls without a GPU), and the
Python binding declares exactly that set."""

import ctypes
import os
import re

from handel_amd import _lib
from handel_amd import build as B

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_symbols():
    text = open(os.path.join(ROOT, "include", "handel_gpu.h")).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return set(re.findall(r"^\s*(?:int|void|size_t|const char\*)\s+(hg_\w+)\s*\(", text, flags=re.M))


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
