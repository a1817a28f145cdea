#!/usr/bin/env python3
"""Static instruction mix of the kernels in a hipcc object: extracts the gfx950
code object (tools/kernel_sizes.py), disassembles it and counts instructions
per kernel by class (VALU, v_mad_u64_u32, SALU, LDS, VMEM, branch). A build-time
proxy for instruction-count changes (dynamic counts come from the SQ_INSTS_*
PMC passes on the GPU box).

  python tools/isa_count.py handel_amd/_build/bn256_gt.o [name-regex]
"""

import re
import subprocess
import sys
import tempfile

from kernel_sizes import LLVM, bundles


def classify(op: str) -> str:
    if op.startswith("v_mad_u64_u32"):
        return "mad64"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith(("global_", "buffer_", "flat_", "scratch_")):
        return "vmem"
    if op.startswith("s_cbranch") or op.startswith("s_branch"):
        return "branch"
    if op.startswith("s_"):
        return "salu"
    if op.startswith("v_"):
        return "valu"
    return "other"


def main():
    pat = re.compile(sys.argv[2] if len(sys.argv) > 2 else ".")
    for triple, blob in bundles(sys.argv[1]):
        with tempfile.NamedTemporaryFile(suffix=".co") as f:
            f.write(blob)
            f.flush()
            out = subprocess.run([LLVM + "llvm-objdump", "-d", "--no-show-raw-insn", "-C", f.name],
                                 capture_output=True, text=True).stdout
        cur, counts = None, {}
        for line in out.splitlines():
            m = re.match(r"^[0-9a-f]+ <(.+)>:$", line)
            if m:
                cur = m.group(1)
                continue
            if cur is None or not line.startswith("\t"):
                continue
            op = line.split()[0]
            c = counts.setdefault(cur, {})
            k = classify(op)
            c[k] = c.get(k, 0) + 1
        for name, c in counts.items():
            if pat.search(name):
                tot = sum(c.values())
                print(f"{tot:7d}  " + " ".join(f"{k}={v}" for k, v in sorted(c.items())) + f"  {name[:90]}")


if __name__ == "__main__":
    main()
