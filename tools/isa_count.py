#!/usr/bin/env python3
"""Instruction mix of the gfx950 kernels in a host object or library (static counts).

    python tools/isa_count.py <lib.so | obj.o> <kernel-name regex> [top]

Prints, per matching kernel, the static count of VALU / LDS / SALU instructions and the most
frequent opcodes -- the per-node accounting of DESIGN.md's AES sections comes from this on
straight-line code (the tree kernels' loops run every instruction of a body once per node).
"""
import collections
import re
import sys

sys.path.insert(0, __import__("os").path.dirname(__file__))
from check_plane_asm import disassemble  # noqa: E402


def kernels(asm_text):
    name, body = None, []
    for ln in asm_text.splitlines():
        m = re.match(r"^[0-9a-f]+ <(\S+)>:", ln)
        if m:
            if name:
                yield name, body
            name, body = m.group(1), []
        elif name:
            body.append(ln)
    if name:
        yield name, body


def main():
    path, pat = sys.argv[1], re.compile(sys.argv[2])
    top = int(sys.argv[3]) if len(sys.argv) > 3 else 20
    for name, body in kernels(disassemble(path)):
        if not pat.search(name):
            continue
        ops = collections.Counter()
        for ln in body:
            m = re.match(r"^\s+([a-z_0-9]+)\b", ln)
            if m:
                ops[m.group(1)] += 1
        valu = sum(v for k, v in ops.items() if k.startswith("v_"))
        lds = sum(v for k, v in ops.items() if k.startswith("ds_"))
        salu = sum(v for k, v in ops.items() if k.startswith("s_"))
        print(f"{name}: valu {valu}  lds {lds}  salu {salu}")
        for k, v in ops.most_common(top):
            print(f"    {k:28s} {v}")


if __name__ == "__main__":
    main()
