"""Build-time ISA check (CPU): the many-round scan's inline-asm mask loads are consumed only
after their wait (tools/check_plane_asm.py; csrc/pir_kernels.hip plane_masks_issue)."""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "erasurecodedpir_amd", "libpir_engine.so")
sys.path.insert(0, os.path.join(ROOT, "tools"))


@pytest.mark.skipif(not os.path.exists(LIB), reason="libpir_engine.so not built")
def test_plane_mask_loads_have_no_early_readers():
    import check_plane_asm as C
    bad, nloads = C.check(C.disassemble(LIB))
    assert nloads > 0, "no asm mask loads found: the many-round k_query instances are missing"
    assert not bad, "\n".join(f"{f}: {ld} -> {op}" for f, ld, op in bad)


def test_checker_flags_an_early_reader():
    import check_plane_asm as C
    asm = "\n".join([
        "0000 <k>:",
        "\ts_load_dwordx8 s[36:43], s[12:13], s30  // 000000000010: C00C",
        "\ts_mov_b32 s50, s37  // 000000000018: BE",
        "\ts_waitcnt lgkmcnt(0)  // 00000000001C: BF8C",
        "\tv_bitop3_b32 v1, v1, v4, s36 bitop3:0x78  // 000000000020: D234",
        "",
    ])
    bad, n = C.check(asm)
    assert n == 1 and len(bad) == 1 and "s_mov_b32" in bad[0][2]
    clean = asm.replace("s_mov_b32 s50, s37", "s_mov_b32 s50, s51")
    assert C.check(clean) == ([], 1)


@pytest.mark.skipif(not os.path.exists(LIB), reason="libpir_engine.so not built")
def test_four_russians_index_windows_are_clean():
    """Every GPR-index window of the four-Russians folds (csrc/pir_m4r.h) holds only the fold's
    instructions, each index change has its wait state, and no spill lane sits in v96-v127."""
    import check_m4r_asm as M
    bad, n = M.check(M.disassemble(LIB))
    assert n > 0, "no index windows: the four-Russians k_query / k_scan_uni instances are missing"
    assert not bad, "\n".join(f"{f}: {p}" for f, p in bad)


def test_four_russians_checker_flags_problems():
    import check_m4r_asm as M
    good = ["0000 <k>:", "\tv_readlane_b32 s6, v62, 0", "\ts_set_gpr_idx_on s6, gpr_idx(SRC0)",
            "\ts_nop 0", "\tv_xor_b32 v45, v112, v45", "\ts_set_gpr_idx_idx s7", "\ts_nop 0",
            "\tv_xor_b32 v44, v112, v44", "\ts_set_gpr_idx_off", ""]
    assert M.check("\n".join(good)) == ([], 1)
    no_nop = [ln for ln in good if ln != "\ts_nop 0"]
    assert len(M.check("\n".join(no_nop))[0]) == 2
    foreign = good[:4] + ["\tv_mov_b32 v3, v4"] + good[4:]
    assert any("foreign" in p for _, p in M.check("\n".join(foreign))[0])
    spill = good[:1] + ["\tv_writelane_b32 v100, s5, 3"] + good[1:]
    assert any("spill" in p for _, p in M.check("\n".join(spill))[0])


def _aes_round_groups(asm):
    """For every column-shape AES round in k_query (its key-schedule broadcast `quad_perm:
    [3,3,3,3]`), the number of ds_read_b32 issued between that round's first lookup and the
    s_waitcnt that ends them (pir_aes.h aes_col: all 8 as one group)."""
    import re
    out = []
    fn = None
    lines = asm.split("\n")
    for i, ln in enumerate(lines):
        m = re.match(r"[0-9a-f]{16} <(\S+)>:", ln)
        if m:
            fn = m.group(1)
            continue
        if fn is None or "k_query" not in fn or "quad_perm:[3,3,3,3]" not in ln:
            continue
        n, seen = 0, False
        for ln2 in lines[i + 1:i + 80]:
            s = ln2.strip()
            if s.startswith("ds_read_b32"):
                n += 1
                seen = True
            elif seen and s.startswith("s_waitcnt") and "lgkmcnt" in s:
                break
        out.append((fn, n))
    return out


@pytest.mark.skipif(not os.path.exists(LIB), reason="libpir_engine.so not built")
def test_column_aes_rounds_issue_one_lookup_group():
    """k_query's column-shape AES (tile-root descent, narrow tile levels) issues each round's 8
    LDS lookups -- the key schedule's 4 and the state's 4 -- as ONE group before a single wait
    (round 5: the compiler had split them into 3 dependent batches at 128 VGPRs)."""
    import check_plane_asm as C
    groups = _aes_round_groups(C.disassemble(LIB))
    assert len(groups) > 100, "no column-shape AES rounds found in k_query"
    bad = [(f, n) for f, n in groups if n != 8]
    assert not bad, f"{len(bad)} of {len(groups)} rounds split: {bad[:5]}"


def _fused_reduce_handoffs(asm):
    """Per k_query instance with the in-kernel slab reduce (pir_kernels.hip, `if (out)`): the
    returning counter add (global_atomic_add ... sc0) and what precedes / follows it."""
    import re
    out = []
    fn, body = None, []

    def flush():
        if fn and "k_query" in fn:
            ins = [ln.split("//")[0].strip() for ln in body]
            for i, s in enumerate(ins):
                if s.startswith("global_atomic_add ") and " sc0" in s:
                    before = ins[:i]
                    sc1 = any(t.startswith("global_store_dword") and " sc1" in t for t in before)
                    # the last vector store of any kind (the non-fused branch's plain slab store
                    # is laid out after the sc1 one) must be waited for before the add
                    vst = [j for j, t in enumerate(before)
                           if t.startswith(("global_store", "buffer_store", "flat_store", "scratch_store"))]
                    between = before[vst[-1] + 1:] if vst else []
                    waited = any(t.startswith("s_waitcnt") and "vmcnt(0)" in t for t in between)
                    reloads = any(t.startswith("global_load_dword") and " sc1" in t for t in ins[i + 1:])
                    out.append((fn, sc1, waited, reloads))
    for ln in asm.split("\n"):
        m = re.match(r"[0-9a-f]{16} <(\S+)>:", ln)
        if m:
            flush()
            fn, body = m.group(1), []
        elif fn:
            body.append(ln)
    flush()
    return out


@pytest.mark.skipif(not os.path.exists(LIB), reason="libpir_engine.so not built")
def test_fused_reduce_handoff_is_write_through():
    """The in-kernel slab reduce ($PIR_FUSED_REDUCE, off by default) hands the slabs to the last
    workgroup WITHOUT release / acquire fences (round 5: each was an XCD-wide L2 write-back or
    invalidate).  What makes it correct is gfx950-specific and is pinned here on the built
    library: every k_query instance's slab stores are write-through (sc1), an s_waitcnt vmcnt(0)
    separates the last vector store from the counter's returning atomic add, and the last
    workgroup's slab reloads bypass the non-coherent caches (sc1).  A
    compiler or ISA change that breaks this fails here instead of silently."""
    import check_plane_asm as C
    hs = _fused_reduce_handoffs(C.disassemble(LIB))
    assert len(hs) >= 8, f"only {len(hs)} fused-reduce hand-offs found in k_query"
    bad = [h for h in hs if not all(h[1:])]
    assert not bad, bad[:4]
