#!/usr/bin/env python3
"""Generate erasurecodedpir_amd/csrc/pir_m4r.h: the four-Russians GF(2^8) plane folds.

The many-round scan keeps, per round a and coefficient bit b, a bit-plane accumulator
Z[a][b] ^= x for every row whose round-a coefficient has bit b set.  Four Russians over rows:
for a group of 4 rows the 16 XOR combinations of the rows are built once (11 v_xor per dword)
into 16 consecutive VGPRs, and each plane then takes ONE v_xor whose source register is
selected by the plane's 4-bit index (bit b of the 4 rows' round-a coefficients) through
GPR-index mode (s_set_gpr_idx_on/idx, src0 indexed).  The indices are computed lane-parallel
(lane 8a + b holds plane (a, b)'s) and moved to SGPRs by v_readlane, 8 at a time, outside the
indexing mode (it indexes every VALU src0).  Per plane: 1 v_readlane + 1 SALU + VEC v_xor,
against VEC v_bitop3 with an SGPR mask (that form issues at about half the rate;
profiles/r02_micro/valu_rate.log, scan_4r2.log).

Everything of one group is ONE asm statement: the combination registers (pinned to
v[128 - 16 VEC, 128)) hold nothing the compiler knows about, so no compiler code may run
between building them and the last plane.  Operand numbering: Z[a][b][v] = (a * VEC + v) * 8 + b.

usage: python3 tools/gen_m4r.py > erasurecodedpir_amd/csrc/pir_m4r.h
"""

VARIANTS = [(1, n) for n in range(1, 9)] + [(2, n) for n in range(1, 6)]


def combos(base, xs):
    r = [f"v{base + i}" for i in range(16)]
    a, b, c, d = xs
    return [
        f"v_mov_b32 {r[0]}, 0", f"v_mov_b32 {r[1]}, {a}", f"v_mov_b32 {r[2]}, {b}",
        f"v_xor_b32 {r[3]}, {a}, {b}", f"v_mov_b32 {r[4]}, {c}", f"v_xor_b32 {r[5]}, {a}, {c}",
        f"v_xor_b32 {r[6]}, {b}, {c}", f"v_xor_b32 {r[7]}, {r[3]}, {c}", f"v_mov_b32 {r[8]}, {d}",
        f"v_xor_b32 {r[9]}, {a}, {d}", f"v_xor_b32 {r[10]}, {b}, {d}",
        f"v_xor_b32 {r[11]}, {r[3]}, {d}", f"v_xor_b32 {r[12]}, {c}, {d}",
        f"v_xor_b32 {r[13]}, {r[5]}, {d}", f"v_xor_b32 {r[14]}, {r[6]}, {d}",
        f"v_xor_b32 {r[15]}, {r[7]}, {d}",
    ]


def fold(vec, na):
    base = 128 - 16 * vec
    # GPR-index mode lives in M0 (s_set_gpr_idx_on/idx write it, _off does not restore it), and
    # M0 is a reserved register the compiler does not let an asm statement clobber: save it on
    # entry and restore it on exit, so whatever the compiler keeps in M0 survives the fold.
    lines = ["s_mov_b32 %[m0s], m0"]
    for v in range(vec):
        lines += combos(base + 16 * v, [f"%[x{i}{v}]" for i in range(4)])
    for a in range(na):
        for b in range(8):
            lines.append(f"v_readlane_b32 %[s{b}], %[vi], {8 * a + b}")
        lines.append("@NOP_RL")
        for b in range(8):
            lines.append(f"s_set_gpr_idx_on %[s0], gpr_idx(SRC0)" if b == 0
                         else f"s_set_gpr_idx_idx %[s{b}]")
            lines.append("@NOP_IDX")
            for v in range(vec):
                z = (a * vec + v) * 8 + b
                lines.append(f"v_xor_b32 %{z}, v{base + 16 * v}, %{z}")
        lines.append("s_set_gpr_idx_off")
    lines.append("s_mov_b32 m0, %[m0s]")
    def emit(ln):
        if ln == "@NOP_RL":
            return "      PIR_M4R_NOP_RL"
        if ln == "@NOP_IDX":
            return "      PIR_M4R_NOP_IDX"
        return f'      "{ln}\\n\\t"'
    body = "\n".join(emit(ln) for ln in lines)
    zops = ", ".join(f'"+v"(Z[{a}][{b}][{v}])' for a in range(na) for v in range(vec)
                     for b in range(8))
    sops = ", ".join([f'[s{b}] "=&s"(s{b})' for b in range(8)] + ['[m0s] "=&s"(m0s)'])
    xins = ", ".join(f'[x{i}{v}] "v"(x{i}[{v}])' for i in range(4) for v in range(vec))
    clob = ", ".join(f'"v{r}"' for r in range(base, 128))
    return f"""template <>
__device__ __forceinline__ void m4r_fold4<{vec}, {na}>(uint32_t (&Z)[{na}][8][{vec}], const uint32_t* x0,
                                           const uint32_t* x1, const uint32_t* x2,
                                           const uint32_t* x3, uint32_t vi) {{
  uint32_t s0, s1, s2, s3, s4, s5, s6, s7, m0s;
  asm volatile(
{body}
      : {zops},
        {sops}
      : {xins}, [vi] "v"(vi)
      : {clob});
}}
"""


def fold_packed(vec, na):
    """The same fold with the plane indices packed 8 to a dword (lane 8a + 7 of vp holds round a's:
    bits [4b, 4b + 4) = plane (a, b)'s index): NA v_readlane per group instead of 8 NA, each index
    extracted by s_bfe_u32 -- placed between s_set_gpr_idx_idx and the plane's v_xor, so it is
    that index change's wait state too (no s_nop)."""
    base = 128 - 16 * vec
    # vp comes straight from m4r_pack's last DPP v_or: a v_readlane of it right behind that
    # write read the value before it (round 0's indices of planes 0-3 lost, the readlanes one
    # instruction later right: 4-round 768-thread k_scan_uni, tools/diag/m4r_rounds.py) -- the
    # compiler's hazard recognizer does not see into this statement, so wait here
    lines = ["s_nop 4"]
    lines += [f"v_readlane_b32 %[p{a}], %[vp], {8 * a + 7}" for a in range(na)]
    lines.append("s_mov_b32 %[m0s], m0")
    n = 8 * na
    # an index change reads an SGPR the SALU wrote: keep every extract >= 6 instructions before
    # its s_set_gpr_idx_* (3 planes ahead, 4 SGPRs in rotation; the first 3 sit amid the
    # combinations, >= 8 instructions after the readlanes and before the window opens)
    ahead = 3
    def reg(k):
        return f"s{k % (ahead + 1)}"
    def bfe(k):
        return f"s_bfe_u32 %[{reg(k)}], %[p{k // 8}], {hex((4 << 16) | (4 * (k % 8)))}"
    comb = []
    for v in range(vec):
        comb += combos(base + 16 * v, [f"%[x{i}{v}]" for i in range(4)])
    lines += comb[:8] + [bfe(k) for k in range(min(ahead, n))] + comb[8:]
    lines.append("s_set_gpr_idx_on %[s0], gpr_idx(SRC0)")
    for k in range(n):
        if k + ahead < n:
            lines.append(bfe(k + ahead))
        lines.append("@PACK_WAIT" if k + ahead < n else "@NOP_IDX")
        a, b = divmod(k, 8)
        for v in range(vec):
            z = (a * vec + v) * 8 + b
            lines.append(f"v_xor_b32 %{z}, v{base + 16 * v}, %{z}")
        if k + 1 < n:
            lines.append(f"s_set_gpr_idx_idx %[{reg(k + 1)}]")
    lines.append("s_set_gpr_idx_off")
    lines.append("s_mov_b32 m0, %[m0s]")
    def emit(ln):
        if ln == "@NOP_IDX":
            return "      PIR_M4R_NOP_IDX"
        if ln == "@PACK_WAIT":
            return "      PIR_M4R_PACK_NOP"
        return f'      "{ln}\\n\\t"'
    body = "\n".join(emit(ln) for ln in lines)
    zops = ", ".join(f'"+v"(Z[{a}][{b}][{v}])' for a in range(na) for v in range(vec)
                     for b in range(8))
    sops = ", ".join([f'[p{a}] "=&s"(p{a})' for a in range(na)] +
                     [f'[s{i}] "=&s"(s{i})' for i in range(ahead + 1)] + ['[m0s] "=&s"(m0s)'])
    xins = ", ".join(f'[x{i}{v}] "v"(x{i}[{v}])' for i in range(4) for v in range(vec))
    clob = ", ".join([f'"v{r}"' for r in range(base, 128)] + ['"scc"'])
    pdecl = ", ".join(f"p{a}" for a in range(na))
    return f"""template <>
__device__ __forceinline__ void m4r_fold4p<{vec}, {na}>(uint32_t (&Z)[{na}][8][{vec}], const uint32_t* x0,
                                            const uint32_t* x1, const uint32_t* x2,
                                            const uint32_t* x3, uint32_t vp) {{
  uint32_t {pdecl}, {", ".join(f"s{i}" for i in range(ahead + 1))}, m0s;
  asm volatile(
{body}
      : {zops},
        {sops}
      : {xins}, [vp] "v"(vp)
      : {clob});
}}
"""


def fold_sgpr(vec, na):
    """m4r_fold4p with round a's packed plane indices already in an SGPR (p[a], bits [4b, 4b + 4)
    = plane (a, b)'s index): the k_query scan waves build the packed words of all 64 groups of a
    tile at once, one group per lane (m4r_tile_index), and read group G's with v_readlane before
    the statement -- no readlane, DPP pack or wait state inside it."""
    base = 128 - 16 * vec
    lines = ["s_mov_b32 %[m0s], m0"]
    n = 8 * na
    ahead = 3
    def reg(k):
        return f"s{k % (ahead + 1)}"
    def bfe(k):
        return f"s_bfe_u32 %[{reg(k)}], %[p{k // 8}], {hex((4 << 16) | (4 * (k % 8)))}"
    comb = []
    for v in range(vec):
        comb += combos(base + 16 * v, [f"%[x{i}{v}]" for i in range(4)])
    lines += comb[:8] + [bfe(k) for k in range(min(ahead, n))] + comb[8:]
    lines.append("s_set_gpr_idx_on %[s0], gpr_idx(SRC0)")
    for k in range(n):
        if k + ahead < n:
            lines.append(bfe(k + ahead))
        lines.append("@PACK_WAIT" if k + ahead < n else "@NOP_IDX")
        a, b = divmod(k, 8)
        for v in range(vec):
            z = (a * vec + v) * 8 + b
            lines.append(f"v_xor_b32 %{z}, v{base + 16 * v}, %{z}")
        if k + 1 < n:
            lines.append(f"s_set_gpr_idx_idx %[{reg(k + 1)}]")
    lines.append("s_set_gpr_idx_off")
    lines.append("s_mov_b32 m0, %[m0s]")
    def emit(ln):
        if ln == "@NOP_IDX":
            return "      PIR_M4R_NOP_IDX"
        if ln == "@PACK_WAIT":
            return "      PIR_M4R_PACK_NOP"
        return f'      "{ln}\\n\\t"'
    body = "\n".join(emit(ln) for ln in lines)
    zops = ", ".join(f'"+v"(Z[{a}][{b}][{v}])' for a in range(na) for v in range(vec)
                     for b in range(8))
    sops = ", ".join([f'[s{i}] "=&s"(s{i})' for i in range(ahead + 1)] + ['[m0s] "=&s"(m0s)'])
    xins = ", ".join(f'[x{i}{v}] "v"(x{i}[{v}])' for i in range(4) for v in range(vec))
    pins = ", ".join(f'[p{a}] "s"(p[{a}])' for a in range(na))
    clob = ", ".join([f'"v{r}"' for r in range(base, 128)] + ['"scc"'])
    return f"""template <>
__device__ __forceinline__ void m4r_fold4s<{vec}, {na}>(uint32_t (&Z)[{na}][8][{vec}], const uint32_t* x0,
                                            const uint32_t* x1, const uint32_t* x2,
                                            const uint32_t* x3, const uint32_t* p) {{
  uint32_t {", ".join(f"s{i}" for i in range(ahead + 1))}, m0s;
  asm volatile(
{body}
      : {zops},
        {sops}
      : {xins}, {pins}
      : {clob});
}}
"""


def main():
    out = ['// GENERATED by tools/gen_m4r.py -- do not edit.  Four-Russians plane folds (see there).',
           '#pragma once', '#include <hip/hip_runtime.h>', '#include <stdint.h>', '',
           '// wait states after the readlanes (none needed: 8 instructions apart) / after each index change',
           '#ifndef PIR_M4R_NOP_RL', '#define PIR_M4R_NOP_RL ""', '#endif',
           '// s_set_gpr_idx_idx -> the VALU that reads through the new index: without a wait state',
           '// the indexed read is sometimes stale (tools/micro/scan_m4r.hip: wrong planes at 16',
           '// waves per CU, VEC 1 and split; right with s_nop 1 or s_nop 0, s_nop 0 4-7 % faster;',
           '// profiles/r02_micro/scan_m4r_nop.log, scan_m4r_nop0.log).  The 12-wave VEC 2 row that',
           '// differs in every variant of scan_m4r_nop.log is the micro\'s own tail: 2^22 rows over',
           '// 1536 row-waves is 2730-2731 rows per wave, not a multiple of the 4-row group, and its',
           '// last partial group re-read row r0 with the next wave\'s coefficients (708a01d: 3 x 2^20',
           '// rows, 2048 per wave, every variant right).  The engine\'s scans fold whole 4-row groups',
           '// whose rows past the end have zero coefficients.',
           '#ifndef PIR_M4R_NOP_IDX', '#define PIR_M4R_NOP_IDX "s_nop 0\\n\\t"', '#endif',
           '// m4r_fold4p: wait state after each index change besides the next extract',
           '#if PIR_M4R_PACK_WAIT', '#define PIR_M4R_PACK_NOP "s_nop 0\\n\\t"', '#else',
           '#define PIR_M4R_PACK_NOP ""', '#endif', '',
           'namespace pir {', '',
           '// Fold 4 rows (x0..x3: VEC dwords each) into NA rounds x 8 bit planes; vi = the plane',
           '// indices, lane 8a + b = bits b of the 4 rows\' round-a coefficients (row i -> bit i).',
           'template <int VEC, int NA>',
           '__device__ __forceinline__ void m4r_fold4(uint32_t (&Z)[NA][8][VEC], const uint32_t* x0,',
           '                                          const uint32_t* x1, const uint32_t* x2,',
           '                                          const uint32_t* x3, uint32_t vi);', '',
           '// The same fold from packed indices: lane 8a + 7 of vp = round a\'s 8 plane indices,',
           '// plane (a, b) in bits [4b, 4b + 4) (m4r_pack of the per-lane indices).',
           'template <int VEC, int NA>',
           '__device__ __forceinline__ void m4r_fold4p(uint32_t (&Z)[NA][8][VEC], const uint32_t* x0,',
           '                                           const uint32_t* x1, const uint32_t* x2,',
           '                                           const uint32_t* x3, uint32_t vp);', '',
           '// The same fold from packed indices already in SGPRs: p[a] = round a\'s 8 plane indices.',
           'template <int VEC, int NA>',
           '__device__ __forceinline__ void m4r_fold4s(uint32_t (&Z)[NA][8][VEC], const uint32_t* x0,',
           '                                           const uint32_t* x1, const uint32_t* x2,',
           '                                           const uint32_t* x3, const uint32_t* p);', '']
    for vec, na in VARIANTS:
        out.append(fold(vec, na))
        out.append(fold_packed(vec, na))
        if vec == 2 and na >= 3:  # k_query's four-Russians scan waves (3-5 rounds)
            out.append(fold_sgpr(vec, na))
    out.append('}  // namespace pir')
    print("\n".join(out))


if __name__ == "__main__":
    main()
