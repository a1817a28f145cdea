#!/usr/bin/env python3
"""Code size of every device function in a hipcc object or shared library:
extracts the gfx950 code object from the offload bundle in .hip_fatbin and
lists symbol sizes (llvm-readelf). Build tooling (I-cache footprint check).

  python tools/kernel_sizes.py handel_amd/_build/bn256_verify.o
"""

import struct
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin/"


def bundles(path):
    data = open(path, "rb").read()
    magic = b"__CLANG_OFFLOAD_BUNDLE__"
    pos = 0
    while True:
        i = data.find(magic, pos)
        if i < 0:
            return
        n = struct.unpack_from("<Q", data, i + 24)[0]
        off = i + 32
        for _ in range(n):
            o, sz, tl = struct.unpack_from("<QQQ", data, off)
            triple = data[off + 24:off + 24 + tl].decode()
            off += 24 + tl
            if "gfx" in triple and sz:
                yield triple, data[i + o:i + o + sz]
        pos = i + 1


def resources(path):
    """{kernel symbol: {"vgpr", "vgpr_spill", "sgpr_spill", "lds", "scratch"}} from
    the gfx950 code objects' metadata notes (llvm-readelf --notes)."""
    import re

    out = {}
    for triple, blob in bundles(path):
        if "gfx950" not in triple:
            continue
        with tempfile.NamedTemporaryFile(suffix=".co") as f:
            f.write(blob)
            f.flush()
            notes = subprocess.run([LLVM + "llvm-readelf", "--notes", f.name], capture_output=True, text=True).stdout
        for b in notes.split("- .agpr_count")[1:]:
            def g(k):
                m = re.search(r"\." + k + r":\s+(\S+)", b)
                return int(m.group(1)) if m else None
            name = re.search(r"\.name:\s+(\S+)", b).group(1)
            out[name] = {"vgpr": g("vgpr_count"), "vgpr_spill": g("vgpr_spill_count"),
                         "sgpr_spill": g("sgpr_spill_count"), "lds": g("group_segment_fixed_size"),
                         "scratch": g("private_segment_fixed_size")}
    return out


def main():
    for triple, blob in bundles(sys.argv[1]):
        with tempfile.NamedTemporaryFile(suffix=".co") as f:
            f.write(blob)
            f.flush()
            out = subprocess.run([LLVM + "llvm-readelf", "-sW", f.name], capture_output=True, text=True).stdout
        rows = []
        for line in out.splitlines():
            p = line.split()
            if len(p) >= 8 and p[3] == "FUNC":
                rows.append((int(p[2]), p[7]))
        print(triple, "total FUNC bytes:", sum(r[0] for r in rows))
        for sz, name in sorted(rows, reverse=True)[:12]:
            print(f"{sz:10d}  {name[:100]}")


if __name__ == "__main__":
    main()
