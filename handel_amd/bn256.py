"""Mirror of the reference's bn256 plugin (bn256/go/bn256.go, bn256/cf/bn256.go)
backed by the MI355X engine: same names, argument meaning and error
behaviour, so code written against Handel's crypto.go interfaces ports over.

Single calls go to the GPU one at a time (correct but latency-bound); the
throughput path is `handel_amd.processing.BatchVerifier`, which submits many
`VerifySignature` requests per launch. There is no CPU fallback.
"""

from __future__ import annotations

import hashlib
import os
import threading
from typing import Optional

from ._lib import HG_ERR_HASH_EOF, HG_OK, HandelGPUError
from .engine import Engine

ORDER = 65000549695646603732796438742359905742570406053903786389881062969044166799969

_engines = {}
_eng_lock = threading.Lock()


def engine(flavor: str = "go", device: Optional[int] = None) -> Engine:
    """Process-wide engine per (flavor, device) (the package-level state of
    bn256/go: G2Base, Hash)."""
    dev = int(os.environ.get("HG_DEVICE", "0")) if device is None else device
    with _eng_lock:
        key = (flavor, dev)
        if key not in _engines:
            _engines[key] = Engine(device=dev, flavor=flavor)
        return _engines[key]


class BN256Error(Exception):
    pass


class _Base:
    flavor = "go"

    @classmethod
    def _eng(cls) -> Engine:
        return engine(cls.flavor)


class PublicKey(_Base):
    """bn256/go/bn256.go:69-121: a G2 point (marshalled form cached)."""

    def __init__(self, marshalled: Optional[bytes] = None):
        self.p = marshalled  # None = the Constructor's empty key (nil *G2)

    def String(self) -> str:
        if self.flavor == "cf":  # bn256/cf/bn256.go:75-80: hex(sha256(marshal))
            return hashlib.sha256(self.MarshalBinary()).hexdigest()
        return self.MarshalBinary().hex()

    def MarshalBinary(self) -> bytes:
        if self.p is None:
            raise BN256Error("nil public key")
        return self.p

    def UnmarshalBinary(self, buff: bytes) -> None:
        """PublicKey.UnmarshalBinary: raises BN256Error with the reference text."""
        e = self._eng()
        if self.flavor == "go" and len(buff) != 128:
            raise BN256Error("unable to unmarshal")
        if self.flavor == "cf" and len(buff) < 128:
            raise BN256Error("bn256: not enough data")
        out, codes = e.combine_g2(bytes(buff[:128]), bytes(128))
        if codes[0] != HG_OK:
            raise BN256Error(e.code_string(int(codes[0])))
        # keep the GPU's re-encoding of the decoded point: x/crypto takes
        # coordinates mod p and its Marshal writes them reduced
        self.p = out

    def Combine(self, other: "PublicKey") -> "PublicKey":
        """bn256/go/bn256.go:97-105: nil receiver returns the argument."""
        if self.p is None:
            return other
        out, codes = self._eng().combine_g2(self.p, other.MarshalBinary())
        if codes[0] != HG_OK:
            raise BN256Error(self._eng().code_string(int(codes[0])))
        return type(self)(out)

    def VerifySignature(self, msg: bytes, sig: "SigBLS") -> Optional[BN256Error]:
        """Returns None on success, a BN256Error otherwise (Go's error return)."""
        e = self._eng()
        if self.p is None:
            raise BN256Error("runtime error: invalid memory address or nil pointer dereference")
        # hashing and the check under one lock hold of the shared context, so
        # concurrent callers with different messages cannot interleave
        codes = e.verify_batch_msg(msg, self.p, sig.MarshalBinary())
        if codes[0] == HG_OK:
            return None
        return BN256Error(e.code_string(int(codes[0])))


class SigBLS(_Base):
    """bn256/go/bn256.go:168-204: a G1 point."""

    def __init__(self, marshalled: Optional[bytes] = None):
        self.e = marshalled

    def MarshalBinary(self) -> bytes:
        if self.e is None:
            raise BN256Error("bn256: multisig can't marshal if nil")
        return self.e

    def UnmarshalBinary(self, b: bytes) -> None:
        e = self._eng()
        if self.flavor == "go" and len(b) != 64:
            raise BN256Error("bn256: multisig can't unmarshal")
        if self.flavor == "cf" and len(b) < 64:
            raise BN256Error("bn256: multisig can't unmarshal: bn256: not enough data")
        out, codes = e.combine_g1(bytes(b[:64]), bytes(64))
        if codes[0] != HG_OK:
            # go: "bn256: multisig can't unmarshal"; cf: the G1 error wrapped (bn256/cf/bn256.go:183-190)
            raise BN256Error(e.code_string(int(codes[0])))
        self.e = out  # re-encoded (reduced) like the upstream Marshal

    def Combine(self, other: "SigBLS") -> "SigBLS":
        if self.e is None:
            return other
        out, codes = self._eng().combine_g1(self.e, other.MarshalBinary())
        if codes[0] != HG_OK:
            raise BN256Error(self._eng().code_string(int(codes[0])))
        return type(self)(out)


class SecretKey(_Base):
    """bn256/go/bn256.go:122-166."""

    def __init__(self, s: Optional[int] = None):
        self.s = s

    def Sign(self, msg: bytes, reader=None) -> SigBLS:
        e = self._eng()
        try:
            return _flavored(SigBLS, self.flavor)(e.sign_msg(msg, self.s.to_bytes(32, "big")))
        except HandelGPUError as err:
            if f"code {HG_ERR_HASH_EOF}:" in str(err):
                raise BN256Error("EOF") from None
            raise

    def MarshalBinary(self) -> bytes:
        return self.s.to_bytes((self.s.bit_length() + 7) // 8, "big")

    def UnmarshalBinary(self, buff: bytes) -> None:
        self.s = int.from_bytes(buff, "big")


def rand_scalar(read) -> int:
    """RandomG2's scalar: crypto/rand.Int(r, Order) until > 0 (32 bytes per try)."""
    while True:
        b = read(32)
        if len(b) < 32:
            raise BN256Error("EOF")
        k = int.from_bytes(b, "big")
        if 0 < k < ORDER:
            return k


def NewKeyPair(reader=None):
    """bn256/go/bn256.go:129-142 (reader: callable n -> bytes, default os.urandom)."""
    read = reader or os.urandom
    k = rand_scalar(read)
    pk = engine().keygen(k.to_bytes(32, "big"))
    return SecretKey(k), PublicKey(pk)


_classes = {}


def _flavored(base, flavor: str):
    """The subclass of base bound to one upstream flavor (one per (base, flavor))."""
    if base.flavor == flavor:
        return base
    with _eng_lock:
        key = (base, flavor)
        if key not in _classes:
            _classes[key] = type(base.__name__, (base,), {"flavor": flavor})
        return _classes[key]


class Constructor:
    """bn256/go/bn256.go:34-67 / cf: the handel.Constructor + simul extension."""

    def __init__(self, flavor: str = "go"):
        self.flavor = flavor
        self._pk = _flavored(PublicKey, flavor)
        self._sig = _flavored(SigBLS, flavor)
        self._sk = _flavored(SecretKey, flavor)

    def Signature(self) -> SigBLS:
        return self._sig()

    def PublicKey(self) -> PublicKey:
        return self._pk()

    def SecretKey(self) -> SecretKey:
        return self._sk()

    def KeyPair(self, reader=None):
        sk, pk = NewKeyPair(reader)
        return self._sk(sk.s), self._pk(pk.p)


def NewConstructor(flavor: str = "go") -> Constructor:
    return Constructor(flavor)
