#!/usr/bin/env python3
"""Build-time ISA check of the four-Russians folds (csrc/pir_m4r.h) in libpir_engine.so.

Inside every GPR-index window (s_set_gpr_idx_on ... s_set_gpr_idx_off) only the fold's own
instructions may appear: index changes, their wait state, the packed fold's SGPR-only
s_bfe_u32 index extracts, and v_xor_b32 whose src0 (the indexed operand) is a combination
register (v96-v127).  Every index change is followed directly by an s_nop or an s_bfe_u32 (the
stale-index hazard, tools/micro/scan_m4r.hip).  In the functions that fold, no SGPR
spill lane (v_writelane_b32) lands in the combination registers.  The windows leave M0 holding
the index (s_set_gpr_idx_off does not restore it), so every fold tools/gen_m4r.py emits saves
M0 into an SGPR before its first window and restores it after its last: the compiler's M0
survives the fold, across loop back-edges too.  The linear-order check below (after a window,
no instruction reads M0 before something writes it again -- the restore is such a write) is a
backstop that catches a fold emitted without the save/restore.

    python tools/check_m4r_asm.py [lib]
"""
import os
import re
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from check_plane_asm import disassemble  # noqa: E402

PINNED = range(96, 128)
XOR_RE = re.compile(r"^\s*v_xor_b32(?:_e32)?\s+v(\d+),\s*v(\d+),\s*v(\d+)")
WL_RE = re.compile(r"^\s*v_writelane_b32\s+v(\d+),")
# the packed fold's next-index extract (m4r_fold4p): SGPRs only, so the index mode leaves it alone
# and it is the wait state of the index change before it
SBFE_RE = re.compile(r"^s_bfe_u32\s+(?:s\d+|vcc_lo|vcc_hi),\s*s\d+,\s*0x400[01][0-9a-f]$")
# s_set_gpr_idx_* reading an SGPR an s_bfe_u32 wrote 2 instructions before took a stale index
# (tests/test_gpu_encode.py::test_configs4_pipeline_end_to_end, 4 rounds): keep them apart
MIN_EXTRACT_DIST = 6
M0_TOKEN = re.compile(r"\bm0\b")
# instructions that read M0 implicitly (LDS-DMA buffer loads, s_movrel, messages, GWS)
M0_IMPLICIT = re.compile(r"^(s_movrel|s_sendmsg|ds_gws|s_ttracedata)|^(buffer|global)_load\S*.*\blds\b")


def m0_access(o):
    """'w' if the instruction writes M0, 'r' if it reads it, None otherwise."""
    mnem, _, rest = o.partition(" ")
    ops = [x.strip() for x in rest.split(",")] if rest else []
    if mnem.startswith("s_set_gpr_idx_on") or (ops and ops[0] == "m0"):
        return "w"
    if any(M0_TOKEN.search(x) for x in ops[1:]) or M0_IMPLICIT.search(o):
        return "r"
    return None


def op(ln):
    return ln.strip().split("//", 1)[0].strip()


def check(asm_text):
    """[(function, problem)], number of index windows checked."""
    lines = [ln for ln in asm_text.splitlines()]
    bad, windows = [], 0
    func, folds, inside = "?", False, False
    spills = []
    prev = ""
    m0_stale = False
    n_ins, bfe_at = 0, {}
    for ln in lines:
        if ln.endswith(">:"):
            if folds:
                bad += [(func, s) for s in spills]
            func, folds, inside, spills, prev, m0_stale = ln, False, False, [], "", False
            bfe_at = {}
            continue
        o = op(ln)
        if not o:
            continue
        n_ins += 1
        if o.startswith("v_readlane_b32") and prev.startswith("v_or_b32_dpp") and \
                o.split(",")[1].strip() == prev.split()[1].rstrip(","):
            bad.append((func, f"v_readlane right after the DPP write of its source: {o}"))
        sb = SBFE_RE.match(o)
        if sb:
            bfe_at[o.split()[1].rstrip(",")] = n_ins
        if o.startswith(("s_set_gpr_idx_on", "s_set_gpr_idx_idx")):
            src = o.split()[1].rstrip(",")
            if src in bfe_at and n_ins - bfe_at[src] < MIN_EXTRACT_DIST:
                bad.append((func, f"index SGPR extracted {n_ins - bfe_at[src]} instructions "
                                  f"before its index change: {o}"))
        m = WL_RE.match(o)
        if m and int(m.group(1)) in PINNED:
            spills.append(f"spill lane in a combination register: {o}")
        if prev.startswith(("s_set_gpr_idx_on", "s_set_gpr_idx_idx")) and not (
                o.startswith("s_nop") or SBFE_RE.match(o)):
            bad.append((func, f"no wait state after '{prev}': {o}"))
        if not inside and not o.startswith("s_set_gpr_idx_off"):
            acc = m0_access(o)
            if acc == "w":
                m0_stale = False
            elif acc == "r" and m0_stale:
                bad.append((func, f"M0 read after an index window before it is rewritten: {o}"))
        if o.startswith("s_set_gpr_idx_on"):
            if inside:
                bad.append((func, "nested index window"))
            inside, folds = True, True
            windows += 1
        elif o.startswith("s_set_gpr_idx_off"):
            inside, m0_stale = False, True
        elif inside and not (o.startswith(("s_set_gpr_idx_idx", "s_nop")) or SBFE_RE.match(o)):
            x = XOR_RE.match(o)
            if not x or int(x.group(2)) not in PINNED:
                bad.append((func, f"foreign instruction in an index window: {o}"))
        prev = o
    if folds:
        bad += [(func, s) for s in spills]
    return bad, windows


def main(argv):
    lib = argv[1] if len(argv) > 1 else os.path.join(
        os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "erasurecodedpir_amd",
        "libpir_engine.so")
    bad, n = check(disassemble(lib))
    print(f"{n} index windows checked, {len(bad)} problems")
    for f, p in bad[:20]:
        print(f, p)
    return 1 if bad or not n else 0


if __name__ == "__main__":
    sys.exit(main(sys.argv))
