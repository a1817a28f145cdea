"""CPU suite: consistency of the Go drop-in source under go/ with the C ABI.

There is no Go toolchain here, so the Go files are never compiled. What can be
checked without one: every C identifier the cgo code uses is declared in
include/handel_gpu.h (and exported by the built library), the error texts the
Go tests expect are the ones hg_code_string returns, and the Handel config
hook patch applies to the reference's config.go / handel.go.
"""

import ctypes
import os
import re
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GO = os.path.join(ROOT, "go")
HEADER = (open(os.path.join(ROOT, "include", "handel_gpu.h")).read() +
          open(os.path.join(ROOT, "include", "handel_client.h")).read())


def _go_sources():
    out = {}
    for d, _, files in os.walk(GO):
        for f in files:
            if f.endswith(".go"):
                out[os.path.relpath(os.path.join(d, f), GO)] = open(os.path.join(d, f)).read()
    return out


def test_go_files_present():
    src = _go_sources()
    for f in ("bn256/hip/engine.go", "bn256/hip/bn256.go", "bn256/hip/batcher.go", "bn256/hip/registry.go",
              "bn256/hip/bn256_test.go", "handel/batched_processing.go", "bn256/hipsvc/client.go"):
        assert f in src, f
    assert os.path.exists(os.path.join(GO, "handel", "config_hook.patch"))


def test_cgo_identifiers_declared_in_header():
    used = set()
    for text in _go_sources().values():
        used |= set(re.findall(r"\bC\.(hg_\w+|HG_\w+)", text))
    assert used, "the cgo binding uses the C ABI"
    for name in sorted(used):
        assert re.search(r"\b%s\b" % name, HEADER), f"{name} not declared in include/handel_gpu.h or handel_client.h"


def test_cgo_functions_exported_by_library():
    from handel_amd import build as B

    if not os.path.exists(B.LIB):
        pytest.skip("library not built")
    lib = ctypes.CDLL(B.LIB)
    client = ctypes.CDLL(B.build_client(verbose=False))
    for name, text in _go_sources().items():
        funcs = set(re.findall(r"\bC\.(hg_[a-z0-9_]+)\(", text))
        funcs.discard("hg_request")
        # the service client package links libhandel_client.so only (no GPU runtime)
        target = client if name.startswith("bn256/hipsvc/") else lib
        for f in sorted(funcs):
            assert hasattr(target, f), (name, f)


def test_go_expected_error_texts_match_abi():
    """Every error text the Go tests assert is one hg_code_string /
    hg_processing_error_string produces (or a Go-side length check's text
    mirroring the reference wrappers)."""
    from handel_amd import build as B

    if not os.path.exists(B.LIB):
        pytest.skip("library not built")
    lib = ctypes.CDLL(B.LIB)
    lib.hg_code_string.restype = ctypes.c_char_p
    lib.hg_processing_error_string.restype = ctypes.c_char_p
    abi = set()
    for code in list(range(0, 14)) + [100, 101]:
        for flavor in (0, 1):
            abi.add(lib.hg_code_string(code, flavor).decode())
            abi.add(lib.hg_processing_error_string(code, flavor).decode())
    go_side = {"EOF", "unable to unmarshal", "bn256: multisig can't unmarshal",
               "bn256: multisig can't unmarshal: bn256: not enough data", "bn256: not enough data"}
    texts = set()
    for text in _go_sources().values():
        for call in re.findall(r"EqualError\((.*?)\)\n", text, flags=re.S):
            lits = re.findall(r'"([^"]*)"', call)
            texts.add(lits[-1])
    assert texts
    # the shim's own errors ("hip: ..."), raised by errors.New in its sources
    own = set()
    for name, text in _go_sources().items():
        if not name.endswith("_test.go"):
            own.update(t for t in re.findall(r'errors\.New\("([^"]*)"\)', text) if t.startswith("hip: "))
    for t in texts:
        assert t in abi or t in go_side or t in own, t
    # the Go-side texts are the reference wrappers' own
    assert "verify multisignature: inconsistent sizes" in abi
    assert "handel: bn256: signature invalid" in abi


@pytest.mark.skipif(not os.path.isdir("/root/reference") or shutil.which("patch") is None,
                    reason="reference tree or patch(1) absent")
def test_config_hook_patch_applies(tmp_path):
    for f in ("config.go", "handel.go"):
        shutil.copy(os.path.join("/root/reference", f), tmp_path / f)
    r = subprocess.run(["patch", "-p1", "--dry-run", "-i", os.path.join(GO, "handel", "config_hook.patch")],
                       cwd=tmp_path, capture_output=True, text=True)
    assert r.returncode == 0, r.stdout + r.stderr


def test_batched_processing_uses_reference_internals():
    """batched_processing.go relies only on package-handel names that exist in
    the reference (read as text when the tree is present)."""
    if not os.path.isdir("/root/reference"):
        pytest.skip("reference tree absent")
    src = open(os.path.join(GO, "handel", "batched_processing.go")).read()
    ref = "".join(open(os.path.join("/root/reference", f)).read()
                  for f in os.listdir("/root/reference") if f.endswith(".go"))
    for name in ("incomingSig", "deathPillPair", "newIndividualSigFilter", "signatureProcessing", "SigEvaluator",
                 "Partitioner", "IdentitiesAt", "Logger", "Filter", "MultiSignature", "Identity"):
        assert name in src
        assert re.search(r"\b%s\b" % name, ref), name
