#!/usr/bin/env python3
"""Build-time ISA check of the many-round scan's inline-asm mask loads (csrc/pir_kernels.hip,
plane_masks_issue / planes_fold2_next).

Those statements issue `s_load_dwordx8 s[a:a+7], s[base], s_off` from inline asm, so the
compiler does not know the destination SGPRs arrive late: the code relies on every consumer of
the tuple being the next fold statement, which opens with `s_waitcnt lgkmcnt(0)`.  A copy,
spill or any other use of the tuple that the register allocator places between the load and
that wait would read stale SGPRs and give silently wrong answers.  This script disassembles the
gfx950 code object inside libpir_engine.so and checks, for every such load, that no
instruction between it and the next `lgkmcnt(0)` wait reads or writes a destination SGPR and
that no branch intervenes.

    python tools/check_plane_asm.py [path/to/libpir_engine.so]

Exit status 0 when clean; prints the offending instructions otherwise.
"""
import os
import re
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"
TARGET = "hipv4-amdgcn-amd-amdhsa--gfx950"
HERE = os.path.dirname(os.path.abspath(__file__))
DEFAULT_LIB = os.path.join(HERE, "..", "erasurecodedpir_amd", "libpir_engine.so")

# the asm form: 8-dword scalar load with an SGPR offset (the compiler's own loads of kernel
# arguments and constants use immediate offsets)
LOAD_RE = re.compile(r"^\s*s_load_dwordx8\s+s\[(\d+):(\d+)\],\s*s\[\d+:\d+\],\s*s(\d+)\s*(//.*)?$")
SREG_RE = re.compile(r"\bs\[(\d+):(\d+)\]|\bs(\d+)\b")
BRANCH_RE = re.compile(r"^\s*s_(cbranch\w*|branch|setpc_b64|swappc_b64|endpgm)\b")
FWD_RE = re.compile(r"^\s*s_(cbranch\w*|branch)\s+(-?\d+)\s*//\s*([0-9A-Fa-f]+):")
ADDR_RE = re.compile(r"//\s*([0-9A-Fa-f]+):")


def code_objects(lib, td):
    """Paths (under td) of every gfx950 code object in lib's .hip_fatbin section (one offload
    bundle per translation unit, concatenated: pir_kernels.o, the pir_query_<k>.o parts, ...)."""
    magic = b"__CLANG_OFFLOAD_BUNDLE__"
    fat = os.path.join(td, "fatbin.bin")
    subprocess.check_call([os.path.join(LLVM, "llvm-objcopy"), "--dump-section",
                           f".hip_fatbin={fat}", lib, os.path.join(td, "stripped.so")])
    data = open(fat, "rb").read()
    starts = [m.start() for m in re.finditer(re.escape(magic), data)] + [len(data)]
    cos = []
    for i in range(len(starts) - 1):
        part = os.path.join(td, f"bundle{i}.bin")
        with open(part, "wb") as f:
            f.write(data[starts[i]:starts[i + 1]])
        co = os.path.join(td, f"gfx950_{i}.co")
        r = subprocess.run([os.path.join(LLVM, "clang-offload-bundler"), "--unbundle",
                            "--type=o", f"--input={part}", f"--targets={TARGET}",
                            f"--output={co}"], capture_output=True)
        if r.returncode != 0 or not os.path.getsize(co):
            continue  # a bundle without device code for this target
        cos.append(co)
    return cos


def disassemble(lib):
    """Text disassembly of every gfx950 code object in lib (code_objects)."""
    with tempfile.TemporaryDirectory() as td:
        return "\n".join(subprocess.check_output([os.path.join(LLVM, "llvm-objdump"), "-d",
                                                  "--no-show-raw-insn", co], text=True)
                         for co in code_objects(lib, td))


def sregs(text):
    """SGPR numbers an instruction names (operands only; the trailing // comment dropped)."""
    regs = set()
    for m in SREG_RE.finditer(text.split("//", 1)[0]):
        if m.group(3) is not None:
            regs.add(int(m.group(3)))
        else:
            regs.update(range(int(m.group(1)), int(m.group(2)) + 1))
    return regs


def check(asm_text):
    """[(function, load line, offending line)], number of asm loads checked."""
    lines = asm_text.splitlines()
    func = "?"
    bad, nloads = [], 0
    for i, ln in enumerate(lines):
        if ln.endswith(">:"):
            func = ln
            continue
        m = LOAD_RE.match(ln)
        if not m:
            continue
        nloads += 1
        dst = set(range(int(m.group(1)), int(m.group(2)) + 1))
        window, wait_addr = [], None
        for ln2 in lines[i + 1:]:
            op = ln2.strip()
            if not op or op.endswith(">:"):
                bad.append((func, ln.strip(), "<end of function before the wait>"))
                break
            if op.startswith("s_waitcnt") and "lgkmcnt(0)" in op:
                a = ADDR_RE.search(op)
                wait_addr = int(a.group(1), 16) if a else None
                break
            window.append(op)
        else:
            continue
        if wait_addr is None:
            continue
        for op in window:
            fwd = FWD_RE.match(op)
            if fwd:
                # a forward branch whose target lies inside the window (at or before the wait)
                # is fine: the target's path is the rest of this linear window, checked here
                tgt = int(fwd.group(3), 16) + 4 + 4 * int(fwd.group(2))
                if int(fwd.group(2)) >= 0 and tgt <= wait_addr:
                    continue
            if BRANCH_RE.match(op) or dst & sregs(op):
                bad.append((func, ln.strip(), op))
                break
    return bad, nloads


def main(argv):
    lib = os.path.abspath(argv[1] if len(argv) > 1 else DEFAULT_LIB)
    bad, nloads = check(disassemble(lib))
    if nloads == 0:
        print("no asm mask loads found (many-round k_query instances missing?)")
        return 2
    for func, load, op in bad:
        print(f"{func}\n  load: {load}\n  uses the tuple before its wait: {op}")
    print(f"{nloads} asm mask loads checked, {len(bad)} hazards")
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main(sys.argv))
