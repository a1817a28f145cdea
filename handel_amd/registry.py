"""GPU-resident Handel registry from the simulator's node files.

The simulator keeps every node as a CSV record ``id,address,private_hex,public_hex``
(simul/lib/parser.go:105-155 csvParser, records built by nodes.go:24-64:
Private = SecretKey.MarshalBinary = big.Int.Bytes, Public =
PublicKey.MarshalBinary = 128-byte G2 marshal). The reference decodes each
public key with one ``PublicKey.UnmarshalBinary`` per node at start-up
(nodes.go:57-60); here the whole column goes to the GPU in one
``hg_registry_load`` (batched G2 unmarshal + on-curve check + the aligned block
sums the aggregation kernels use).

``generate_records`` is GenerateNodes (generator.go:11-24) with the key pairs
computed by one batched ``hg_keygen``: secret keys from a caller-supplied
reader under NewKeyPair's rejection rule (bn256/go/bn256.go:129-142), public
keys k * G2 on the GPU.
"""

from __future__ import annotations

import csv
import io
from dataclasses import dataclass
from typing import Callable, List, Sequence

from .engine import Engine

ORDER = 65000549695646603732796438742359905742570406053903786389881062969044166799969


@dataclass
class NodeRecord:
    """simul/lib/nodes.go:9-15 NodeRecord (hex-encoded keys)."""
    id: int
    addr: str
    private: str
    public: str


class RegistryError(ValueError):
    pass


def read_records(path_or_text: str, is_text: bool = False) -> List[NodeRecord]:
    """csvParser.Read (parser.go:105-137): exactly 4 fields per record, the id
    parsed as a base-10 int32; stops at EOF."""
    f = io.StringIO(path_or_text) if is_text else open(path_or_text, newline="")
    try:
        out = []
        for line in csv.reader(f):
            if len(line) != 4:
                raise RegistryError("record on line %d: wrong number of fields" % (len(out) + 1))
            try:
                i = int(line[0], 10)
            except ValueError as e:
                raise RegistryError(f'strconv.ParseInt: parsing "{line[0]}": invalid syntax') from e
            if not -(1 << 31) <= i < (1 << 31):
                raise RegistryError(f'strconv.ParseInt: parsing "{line[0]}": value out of range')
            out.append(NodeRecord(i, line[1], line[2], line[3]))
        return out
    finally:
        f.close()


def write_records(path: str, records: Sequence[NodeRecord]) -> None:
    """csvParser.Write (parser.go:139-155)."""
    with open(path, "w", newline="") as f:
        w = csv.writer(f, lineterminator="\n")
        for r in records:
            w.writerow([str(r.id), r.addr, r.private, r.public])


def registry_bytes(records: Sequence[NodeRecord]) -> bytes:
    """The public keys in registry order (record i is identity i), 128 B each."""
    out = bytearray()
    for i, r in enumerate(records):
        if r.id != i:
            raise RegistryError(f"record {i} has id {r.id}: the array registry needs ids 0..N-1 in order")
        pk = bytes.fromhex(r.public)
        if len(pk) != 128:
            raise RegistryError(f"node {r.id}: public key of {len(pk)} bytes")
        out += pk
    return bytes(out)


def load_registry(eng: Engine, records: Sequence[NodeRecord]) -> int:
    """Decodes the registry on the GPU; returns its size or raises with the
    first failing node (the reference fails start-up on the first bad key)."""
    pks = registry_bytes(records)
    codes = eng.registry_load(pks)
    bad = [i for i, c in enumerate(codes) if c]
    if bad:
        raise RegistryError(f"node {bad[0]}: " + eng.code_string(int(codes[bad[0]])))
    return len(records)


def secret_marshal(k: int) -> bytes:
    """SecretKey.MarshalBinary = big.Int.Bytes: minimal big-endian."""
    return k.to_bytes((k.bit_length() + 7) // 8, "big")


def random_scalars(n: int, read: Callable[[int], bytes]) -> List[int]:
    """NewKeyPair's secret keys: rand.Int(r, Order) draws 32 bytes and retries
    until k < n, and RandomG2 retries on k == 0 (bn256/go/bn256.go:129-142)."""
    out = []
    while len(out) < n:
        k = int.from_bytes(read(32), "big")
        if 0 < k < ORDER:
            out.append(k)
    return out


def generate_records(eng: Engine, addresses: Sequence[str], read: Callable[[int], bytes]) -> List[NodeRecord]:
    """GenerateNodes (generator.go:11-24): ids 0..N-1 in address order."""
    ks = random_scalars(len(addresses), read)
    pks = eng.keygen(b"".join(k.to_bytes(32, "big") for k in ks))
    return [NodeRecord(i, a, secret_marshal(k).hex(), pks[128 * i:128 * (i + 1)].hex())
            for i, (a, k) in enumerate(zip(addresses, ks))]
