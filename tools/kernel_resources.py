#!/usr/bin/env python3
"""Register, LDS and scratch use of the gfx950 kernels in a library (code-object metadata).

    python tools/kernel_resources.py <lib.so> [kernel-name regex]

Prints, per matching kernel: VGPRs, AGPRs, SGPRs, spilled VGPRs/SGPRs, scratch bytes per lane
and static LDS -- the check that a kernel change did not push a hot loop into scratch.
"""
import os
import re
import subprocess
import sys
import tempfile

sys.path.insert(0, os.path.dirname(__file__))
from check_plane_asm import LLVM, code_objects  # noqa: E402


def metadata(lib):
    with tempfile.TemporaryDirectory() as td:
        return "\n".join(subprocess.check_output([os.path.join(LLVM, "llvm-readelf"), "--notes", co],
                                                 text=True) for co in code_objects(lib, td))


def main():
    lib = sys.argv[1]
    pat = re.compile(sys.argv[2] if len(sys.argv) > 2 else ".")
    text = metadata(lib)
    fields = (".vgpr_count", ".agpr_count", ".sgpr_count", ".vgpr_spill_count",
              ".sgpr_spill_count", ".private_segment_fixed_size", ".group_segment_fixed_size")
    for blk in re.split(r"\n\s*- \.", text):
        m = re.search(r"\.name:\s+(\S+)", blk)
        if not m or not pat.search(m.group(1)):
            continue
        vals = []
        for f in fields:
            mm = re.search(re.escape(f) + r":\s+(\d+)", blk)
            vals.append(mm.group(1) if mm else "?")
        print(m.group(1)[:110], dict(zip([f.strip(".") for f in fields], vals)))


if __name__ == "__main__":
    main()
