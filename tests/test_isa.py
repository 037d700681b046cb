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
