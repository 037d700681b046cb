// Micro-benchmark (not part of the product): the many-round GF(2^8) scan of configs[4] (5 rounds,
// wave-uniform coefficients, 1 KiB records) -- four Russians over rows at TWO dwords per lane.
//   MODE 2: the product's form -- 8 masks per (row, round) from a 256 x 8-dword table
//           (s_load_dwordx8), one v_bitop3 per (plane, dword)
//   MODE 3: HBM only (one XOR per dword)
//   MODE 8: four Russians: per group of 4 rows the 16 XOR combinations of each of the lane's two
//           dwords (v96-v111, v112-v127); per plane one s_bfe_u32 (its 4-bit index from the
//           spread word) + s_set_gpr_idx_idx, then TWO v_xor whose src0 is indexed
//   MODE 9: as 8, but the 40 plane indices of a group are computed lane-parallel on the VALU
//           (lane k = plane k) and moved to SGPRs by v_readlane, 8 per round outside the
//           indexing mode: per plane 1 SALU (s_set_gpr_idx_idx) + 1 v_readlane + 2 v_xor
// Checksum: XOR over all plane words x their plane number (independent of the wave split only
// within one WAVES value: compare modes at equal WAVES).
// Build: hipcc -O3 --offload-arch=gfx950 -o scan_4r2 scan_4r2.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)

typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
typedef uint32_t u32x8 __attribute__((ext_vector_type(8)));

constexpr int NQ = 5;

__constant__ uint32_t c_spread[256];  // nibble k = bit k of c

__device__ __forceinline__ uint32_t mxor(uint32_t z, uint32_t x, uint32_t m) {
  return __builtin_amdgcn_bitop3_b32(z, x, m, 0x78);
}

#define ZR(a) "+v"(Z[a][0][0]), "+v"(Z[a][1][0]), "+v"(Z[a][2][0]), "+v"(Z[a][3][0]), \
              "+v"(Z[a][4][0]), "+v"(Z[a][5][0]), "+v"(Z[a][6][0]), "+v"(Z[a][7][0]), \
              "+v"(Z[a][0][1]), "+v"(Z[a][1][1]), "+v"(Z[a][2][1]), "+v"(Z[a][3][1]), \
              "+v"(Z[a][4][1]), "+v"(Z[a][5][1]), "+v"(Z[a][6][1]), "+v"(Z[a][7][1])

// combos of 4 rows (a, b, c, d) for one dword into v[B .. B+15]: v[B+i] = XOR of rows whose bit
// is set in i
// (written out per base register: the assembler has no arithmetic on register names)
#define COMBO16(r0, r1, r2, r3, r4, r5, r6, r7, r8, r9, r10, r11, r12, r13, r14, r15, a, b, c, d) \
  "v_mov_b32 " r0 ", 0\n\t"                                                                     \
  "v_mov_b32 " r1 ", %[" a "]\n\t"                                                              \
  "v_mov_b32 " r2 ", %[" b "]\n\t"                                                              \
  "v_xor_b32 " r3 ", %[" a "], %[" b "]\n\t"                                                    \
  "v_mov_b32 " r4 ", %[" c "]\n\t"                                                              \
  "v_xor_b32 " r5 ", %[" a "], %[" c "]\n\t"                                                    \
  "v_xor_b32 " r6 ", %[" b "], %[" c "]\n\t"                                                    \
  "v_xor_b32 " r7 ", " r3 ", %[" c "]\n\t"                                                      \
  "v_mov_b32 " r8 ", %[" d "]\n\t"                                                              \
  "v_xor_b32 " r9 ", %[" a "], %[" d "]\n\t"                                                    \
  "v_xor_b32 " r10 ", %[" b "], %[" d "]\n\t"                                                   \
  "v_xor_b32 " r11 ", " r3 ", %[" d "]\n\t"                                                     \
  "v_xor_b32 " r12 ", %[" c "], %[" d "]\n\t"                                                   \
  "v_xor_b32 " r13 ", " r5 ", %[" d "]\n\t"                                                     \
  "v_xor_b32 " r14 ", " r6 ", %[" d "]\n\t"                                                     \
  "v_xor_b32 " r15 ", " r7 ", %[" d "]\n\t"
#define COMBO_LO(a, b, c, d) COMBO16("v96", "v97", "v98", "v99", "v100", "v101", "v102", "v103", \
  "v104", "v105", "v106", "v107", "v108", "v109", "v110", "v111", a, b, c, d)
#define COMBO_HI(a, b, c, d) COMBO16("v112", "v113", "v114", "v115", "v116", "v117", "v118", \
  "v119", "v120", "v121", "v122", "v123", "v124", "v125", "v126", "v127", a, b, c, d)

// one group of 4 rows x 2 dwords per lane into the 80 plane words, everything in ONE asm
// statement (the combos in v96-v127 must not be touched by compiler code between the planes).
// Operand numbers: Z[a][b][v] = 16a + 8v + b.
__device__ __forceinline__ void fold4_bfe(uint32_t (&Z)[NQ][8][2], const uint32_t* x0,
                                          const uint32_t* x1, const uint32_t* x2,
                                          const uint32_t* x3, const uint32_t* w) {
  uint32_t t;
  asm volatile(
      COMBO_LO("a", "b", "c", "d") COMBO_HI("e", "f", "g", "h")
      "s_set_gpr_idx_on 0, gpr_idx(SRC0)\n\t"
      "s_bfe_u32 %[t], %[w0], 0x40000\n\t"
      "s_set_gpr_idx_idx %[t]\n\t"
      "v_xor_b32 %0, v96, %0\n\t"
      "v_xor_b32 %8, v112, %8\n\t"
      "s_bfe_u32 %[t], %[w0], 0x40004\n\t"
      "s_set_gpr_idx_idx %[t]\n\t"
      "v_xor_b32 %1, v96, %1\n\t"
      "v_xor_b32 %9, v112, %9\n\t"
      "s_bfe_u32 %[t], %[w0], 0x40008\n\t"
      "s_set_gpr_idx_idx %[t]\n\t"
      "v_xor_b32 %2, v96, %2\n\t"
      "v_xor_b32 %10, v112, %10\n\t"
      "s_bfe_u32 %[t], %[w0], 0x4000c\n\t"
      "s_set_gpr_idx_idx %[t]\n\t"
      "v_xor_b32 %3, v96, %3\n\t"
      "v_xor_b32 %11, v112, %11\n\t"
      "s_bfe_u32 %[t], %[w0], 0x40010\n\t"
      "s_set_gpr_idx_idx %[t]\n\t"
      "v_xor_b32 %4, v96, %4\n\t"
      "v_xor_b32 %12, v112, %12\n\t"
      "s_bfe_u32 %[t], %[w0], 0x40014\n\t"
      "s_set_gpr_idx_idx %[t]\n\t"
      "v_xor_b32 %5, v96, %5\n\t"
      "v_xor_b32 %13, v112, %13\n\t"
      "s_bfe_u32 %[t], %[w0], 0x40018\n\t"
      "s_set_gpr_idx_idx %[t]\n\t"
      "v_xor_b32 %6, v96, %6\n\t"
      "v_xor_b32 %14, v112, %14\n\t"
      "s_bfe_u32 %[t], %[w0], 0x4001c\n\t"
      "s_set_gpr_idx_idx %[t]\n\t"
      "v_xor_b32 %7, v96, %7\n\t"
      "v_xor_b32 %15, v112, %15\n\t"
      "s_bfe_u32 %[t], %[w1], 0x40000\n\t"
      "s_set_gpr_idx_idx %[t]\n\t"
      "v_xor_b32 %16, v96, %16\n\t"
      "v_xor_b32 %24, v112, %24\n\t"
      "s_bfe_u32 %[t], %[w1], 0x40004\n\t"
      "s_set_gpr_idx_idx %[t]\n\t"
      "v_xor_b32 %17, v96, %17\n\t"
      "v_xor_b32 %25, v112, %25\n\t"
      "s_bfe_u32 %[t], %[w1], 0x40008\n\t"
      "s_set_gpr_idx_idx %[t]\n\t"
      "v_xor_b32 %18, v96, %18\n\t"
      "v_xor_b32 %26, v112, %26\n\t"
      "s_bfe_u32 %[t], %[w1], 0x4000c\n\t"
      "s_set_gpr_idx_idx %[t]\n\t"
      "v_xor_b32 %19, v96, %19\n\t"
      "v_xor_b32 %27, v112, %27\n\t"
      "s_bfe_u32 %[t], %[w1], 0x40010\n\t"
      "s_set_gpr_idx_idx %[t]\n\t"
      "v_xor_b32 %20, v96, %20\n\t"
      "v_xor_b32 %28, v112, %28\n\t"
      "s_bfe_u32 %[t], %[w1], 0x40014\n\t"
      "s_set_gpr_idx_idx %[t]\n\t"
      "v_xor_b32 %21, v96, %21\n\t"
      "v_xor_b32 %29, v112, %29\n\t"
      "s_bfe_u32 %[t], %[w1], 0x40018\n\t"
      "s_set_gpr_idx_idx %[t]\n\t"
      "v_xor_b32 %22, v96, %22\n\t"
      "v_xor_b32 %30, v112, %30\n\t"
      "s_bfe_u32 %[t], %[w1], 0x4001c\n\t"
      "s_set_gpr_idx_idx %[t]\n\t"
      "v_xor_b32 %23, v96, %23\n\t"
      "v_xor_b32 %31, v112, %31\n\t"
      "s_bfe_u32 %[t], %[w2], 0x40000\n\t"
      "s_set_gpr_idx_idx %[t]\n\t"
      "v_xor_b32 %32, v96, %32\n\t"
      "v_xor_b32 %40, v112, %40\n\t"
      "s_bfe_u32 %[t], %[w2], 0x40004\n\t"
      "s_set_gpr_idx_idx %[t]\n\t"
      "v_xor_b32 %33, v96, %33\n\t"
      "v_xor_b32 %41, v112, %41\n\t"
      "s_bfe_u32 %[t], %[w2], 0x40008\n\t"
      "s_set_gpr_idx_idx %[t]\n\t"
      "v_xor_b32 %34, v96, %34\n\t"
      "v_xor_b32 %42, v112, %42\n\t"
      "s_bfe_u32 %[t], %[w2], 0x4000c\n\t"
      "s_set_gpr_idx_idx %[t]\n\t"
      "v_xor_b32 %35, v96, %35\n\t"
      "v_xor_b32 %43, v112, %43\n\t"
      "s_bfe_u32 %[t], %[w2], 0x40010\n\t"
      "s_set_gpr_idx_idx %[t]\n\t"
      "v_xor_b32 %36, v96, %36\n\t"
      "v_xor_b32 %44, v112, %44\n\t"
      "s_bfe_u32 %[t], %[w2], 0x40014\n\t"
      "s_set_gpr_idx_idx %[t]\n\t"
      "v_xor_b32 %37, v96, %37\n\t"
      "v_xor_b32 %45, v112, %45\n\t"
      "s_bfe_u32 %[t], %[w2], 0x40018\n\t"
      "s_set_gpr_idx_idx %[t]\n\t"
      "v_xor_b32 %38, v96, %38\n\t"
      "v_xor_b32 %46, v112, %46\n\t"
      "s_bfe_u32 %[t], %[w2], 0x4001c\n\t"
      "s_set_gpr_idx_idx %[t]\n\t"
      "v_xor_b32 %39, v96, %39\n\t"
      "v_xor_b32 %47, v112, %47\n\t"
      "s_bfe_u32 %[t], %[w3], 0x40000\n\t"
      "s_set_gpr_idx_idx %[t]\n\t"
      "v_xor_b32 %48, v96, %48\n\t"
      "v_xor_b32 %56, v112, %56\n\t"
      "s_bfe_u32 %[t], %[w3], 0x40004\n\t"
      "s_set_gpr_idx_idx %[t]\n\t"
      "v_xor_b32 %49, v96, %49\n\t"
      "v_xor_b32 %57, v112, %57\n\t"
      "s_bfe_u32 %[t], %[w3], 0x40008\n\t"
      "s_set_gpr_idx_idx %[t]\n\t"
      "v_xor_b32 %50, v96, %50\n\t"
      "v_xor_b32 %58, v112, %58\n\t"
      "s_bfe_u32 %[t], %[w3], 0x4000c\n\t"
      "s_set_gpr_idx_idx %[t]\n\t"
      "v_xor_b32 %51, v96, %51\n\t"
      "v_xor_b32 %59, v112, %59\n\t"
      "s_bfe_u32 %[t], %[w3], 0x40010\n\t"
      "s_set_gpr_idx_idx %[t]\n\t"
      "v_xor_b32 %52, v96, %52\n\t"
      "v_xor_b32 %60, v112, %60\n\t"
      "s_bfe_u32 %[t], %[w3], 0x40014\n\t"
      "s_set_gpr_idx_idx %[t]\n\t"
      "v_xor_b32 %53, v96, %53\n\t"
      "v_xor_b32 %61, v112, %61\n\t"
      "s_bfe_u32 %[t], %[w3], 0x40018\n\t"
      "s_set_gpr_idx_idx %[t]\n\t"
      "v_xor_b32 %54, v96, %54\n\t"
      "v_xor_b32 %62, v112, %62\n\t"
      "s_bfe_u32 %[t], %[w3], 0x4001c\n\t"
      "s_set_gpr_idx_idx %[t]\n\t"
      "v_xor_b32 %55, v96, %55\n\t"
      "v_xor_b32 %63, v112, %63\n\t"
      "s_bfe_u32 %[t], %[w4], 0x40000\n\t"
      "s_set_gpr_idx_idx %[t]\n\t"
      "v_xor_b32 %64, v96, %64\n\t"
      "v_xor_b32 %72, v112, %72\n\t"
      "s_bfe_u32 %[t], %[w4], 0x40004\n\t"
      "s_set_gpr_idx_idx %[t]\n\t"
      "v_xor_b32 %65, v96, %65\n\t"
      "v_xor_b32 %73, v112, %73\n\t"
      "s_bfe_u32 %[t], %[w4], 0x40008\n\t"
      "s_set_gpr_idx_idx %[t]\n\t"
      "v_xor_b32 %66, v96, %66\n\t"
      "v_xor_b32 %74, v112, %74\n\t"
      "s_bfe_u32 %[t], %[w4], 0x4000c\n\t"
      "s_set_gpr_idx_idx %[t]\n\t"
      "v_xor_b32 %67, v96, %67\n\t"
      "v_xor_b32 %75, v112, %75\n\t"
      "s_bfe_u32 %[t], %[w4], 0x40010\n\t"
      "s_set_gpr_idx_idx %[t]\n\t"
      "v_xor_b32 %68, v96, %68\n\t"
      "v_xor_b32 %76, v112, %76\n\t"
      "s_bfe_u32 %[t], %[w4], 0x40014\n\t"
      "s_set_gpr_idx_idx %[t]\n\t"
      "v_xor_b32 %69, v96, %69\n\t"
      "v_xor_b32 %77, v112, %77\n\t"
      "s_bfe_u32 %[t], %[w4], 0x40018\n\t"
      "s_set_gpr_idx_idx %[t]\n\t"
      "v_xor_b32 %70, v96, %70\n\t"
      "v_xor_b32 %78, v112, %78\n\t"
      "s_bfe_u32 %[t], %[w4], 0x4001c\n\t"
      "s_set_gpr_idx_idx %[t]\n\t"
      "v_xor_b32 %71, v96, %71\n\t"
      "v_xor_b32 %79, v112, %79\n\t"
      "s_set_gpr_idx_off"
      : ZR(0), ZR(1), ZR(2), ZR(3), ZR(4), [t] "=&s"(t)
      : [a] "v"(x0[0]), [b] "v"(x1[0]), [c] "v"(x2[0]), [d] "v"(x3[0]), [e] "v"(x0[1]),
        [f] "v"(x1[1]), [g] "v"(x2[1]), [h] "v"(x3[1]), [w0] "s"(w[0]), [w1] "s"(w[1]), [w2] "s"(w[2]),
        [w3] "s"(w[3]), [w4] "s"(w[4])
      : "v96", "v97", "v98", "v99", "v100", "v101", "v102", "v103", "v104",
        "v105", "v106", "v107", "v108", "v109", "v110", "v111", "v112", "v113", "v114", "v115",
        "v116", "v117", "v118", "v119", "v120", "v121", "v122", "v123", "v124", "v125", "v126",
        "v127", "m0");
}

// the same with the plane indices from lanes 0-39 of vidx (lane 8a + b = plane (a, b)), moved to
// SGPRs by v_readlane 8 at a time outside the indexing mode (it indexes every VALU src0)
__device__ __forceinline__ void fold4_rl(uint32_t (&Z)[NQ][8][2], const uint32_t* x0,
                                         const uint32_t* x1, const uint32_t* x2,
                                         const uint32_t* x3, uint32_t vidx) {
  uint32_t s0, s1, s2, s3, s4, s5, s6, s7;
  asm volatile(
      COMBO_LO("a", "b", "c", "d") COMBO_HI("e", "f", "g", "h")
      "v_readlane_b32 %[s0], %[v], 0\n\t"
      "v_readlane_b32 %[s1], %[v], 1\n\t"
      "v_readlane_b32 %[s2], %[v], 2\n\t"
      "v_readlane_b32 %[s3], %[v], 3\n\t"
      "v_readlane_b32 %[s4], %[v], 4\n\t"
      "v_readlane_b32 %[s5], %[v], 5\n\t"
      "v_readlane_b32 %[s6], %[v], 6\n\t"
      "v_readlane_b32 %[s7], %[v], 7\n\t"
      "s_set_gpr_idx_on %[s0], gpr_idx(SRC0)\n\t"
      "v_xor_b32 %0, v96, %0\n\t"
      "v_xor_b32 %8, v112, %8\n\t"
      "s_set_gpr_idx_idx %[s1]\n\t"
      "v_xor_b32 %1, v96, %1\n\t"
      "v_xor_b32 %9, v112, %9\n\t"
      "s_set_gpr_idx_idx %[s2]\n\t"
      "v_xor_b32 %2, v96, %2\n\t"
      "v_xor_b32 %10, v112, %10\n\t"
      "s_set_gpr_idx_idx %[s3]\n\t"
      "v_xor_b32 %3, v96, %3\n\t"
      "v_xor_b32 %11, v112, %11\n\t"
      "s_set_gpr_idx_idx %[s4]\n\t"
      "v_xor_b32 %4, v96, %4\n\t"
      "v_xor_b32 %12, v112, %12\n\t"
      "s_set_gpr_idx_idx %[s5]\n\t"
      "v_xor_b32 %5, v96, %5\n\t"
      "v_xor_b32 %13, v112, %13\n\t"
      "s_set_gpr_idx_idx %[s6]\n\t"
      "v_xor_b32 %6, v96, %6\n\t"
      "v_xor_b32 %14, v112, %14\n\t"
      "s_set_gpr_idx_idx %[s7]\n\t"
      "v_xor_b32 %7, v96, %7\n\t"
      "v_xor_b32 %15, v112, %15\n\t"
      "s_set_gpr_idx_off\n\t"
      "v_readlane_b32 %[s0], %[v], 8\n\t"
      "v_readlane_b32 %[s1], %[v], 9\n\t"
      "v_readlane_b32 %[s2], %[v], 10\n\t"
      "v_readlane_b32 %[s3], %[v], 11\n\t"
      "v_readlane_b32 %[s4], %[v], 12\n\t"
      "v_readlane_b32 %[s5], %[v], 13\n\t"
      "v_readlane_b32 %[s6], %[v], 14\n\t"
      "v_readlane_b32 %[s7], %[v], 15\n\t"
      "s_set_gpr_idx_on %[s0], gpr_idx(SRC0)\n\t"
      "v_xor_b32 %16, v96, %16\n\t"
      "v_xor_b32 %24, v112, %24\n\t"
      "s_set_gpr_idx_idx %[s1]\n\t"
      "v_xor_b32 %17, v96, %17\n\t"
      "v_xor_b32 %25, v112, %25\n\t"
      "s_set_gpr_idx_idx %[s2]\n\t"
      "v_xor_b32 %18, v96, %18\n\t"
      "v_xor_b32 %26, v112, %26\n\t"
      "s_set_gpr_idx_idx %[s3]\n\t"
      "v_xor_b32 %19, v96, %19\n\t"
      "v_xor_b32 %27, v112, %27\n\t"
      "s_set_gpr_idx_idx %[s4]\n\t"
      "v_xor_b32 %20, v96, %20\n\t"
      "v_xor_b32 %28, v112, %28\n\t"
      "s_set_gpr_idx_idx %[s5]\n\t"
      "v_xor_b32 %21, v96, %21\n\t"
      "v_xor_b32 %29, v112, %29\n\t"
      "s_set_gpr_idx_idx %[s6]\n\t"
      "v_xor_b32 %22, v96, %22\n\t"
      "v_xor_b32 %30, v112, %30\n\t"
      "s_set_gpr_idx_idx %[s7]\n\t"
      "v_xor_b32 %23, v96, %23\n\t"
      "v_xor_b32 %31, v112, %31\n\t"
      "s_set_gpr_idx_off\n\t"
      "v_readlane_b32 %[s0], %[v], 16\n\t"
      "v_readlane_b32 %[s1], %[v], 17\n\t"
      "v_readlane_b32 %[s2], %[v], 18\n\t"
      "v_readlane_b32 %[s3], %[v], 19\n\t"
      "v_readlane_b32 %[s4], %[v], 20\n\t"
      "v_readlane_b32 %[s5], %[v], 21\n\t"
      "v_readlane_b32 %[s6], %[v], 22\n\t"
      "v_readlane_b32 %[s7], %[v], 23\n\t"
      "s_set_gpr_idx_on %[s0], gpr_idx(SRC0)\n\t"
      "v_xor_b32 %32, v96, %32\n\t"
      "v_xor_b32 %40, v112, %40\n\t"
      "s_set_gpr_idx_idx %[s1]\n\t"
      "v_xor_b32 %33, v96, %33\n\t"
      "v_xor_b32 %41, v112, %41\n\t"
      "s_set_gpr_idx_idx %[s2]\n\t"
      "v_xor_b32 %34, v96, %34\n\t"
      "v_xor_b32 %42, v112, %42\n\t"
      "s_set_gpr_idx_idx %[s3]\n\t"
      "v_xor_b32 %35, v96, %35\n\t"
      "v_xor_b32 %43, v112, %43\n\t"
      "s_set_gpr_idx_idx %[s4]\n\t"
      "v_xor_b32 %36, v96, %36\n\t"
      "v_xor_b32 %44, v112, %44\n\t"
      "s_set_gpr_idx_idx %[s5]\n\t"
      "v_xor_b32 %37, v96, %37\n\t"
      "v_xor_b32 %45, v112, %45\n\t"
      "s_set_gpr_idx_idx %[s6]\n\t"
      "v_xor_b32 %38, v96, %38\n\t"
      "v_xor_b32 %46, v112, %46\n\t"
      "s_set_gpr_idx_idx %[s7]\n\t"
      "v_xor_b32 %39, v96, %39\n\t"
      "v_xor_b32 %47, v112, %47\n\t"
      "s_set_gpr_idx_off\n\t"
      "v_readlane_b32 %[s0], %[v], 24\n\t"
      "v_readlane_b32 %[s1], %[v], 25\n\t"
      "v_readlane_b32 %[s2], %[v], 26\n\t"
      "v_readlane_b32 %[s3], %[v], 27\n\t"
      "v_readlane_b32 %[s4], %[v], 28\n\t"
      "v_readlane_b32 %[s5], %[v], 29\n\t"
      "v_readlane_b32 %[s6], %[v], 30\n\t"
      "v_readlane_b32 %[s7], %[v], 31\n\t"
      "s_set_gpr_idx_on %[s0], gpr_idx(SRC0)\n\t"
      "v_xor_b32 %48, v96, %48\n\t"
      "v_xor_b32 %56, v112, %56\n\t"
      "s_set_gpr_idx_idx %[s1]\n\t"
      "v_xor_b32 %49, v96, %49\n\t"
      "v_xor_b32 %57, v112, %57\n\t"
      "s_set_gpr_idx_idx %[s2]\n\t"
      "v_xor_b32 %50, v96, %50\n\t"
      "v_xor_b32 %58, v112, %58\n\t"
      "s_set_gpr_idx_idx %[s3]\n\t"
      "v_xor_b32 %51, v96, %51\n\t"
      "v_xor_b32 %59, v112, %59\n\t"
      "s_set_gpr_idx_idx %[s4]\n\t"
      "v_xor_b32 %52, v96, %52\n\t"
      "v_xor_b32 %60, v112, %60\n\t"
      "s_set_gpr_idx_idx %[s5]\n\t"
      "v_xor_b32 %53, v96, %53\n\t"
      "v_xor_b32 %61, v112, %61\n\t"
      "s_set_gpr_idx_idx %[s6]\n\t"
      "v_xor_b32 %54, v96, %54\n\t"
      "v_xor_b32 %62, v112, %62\n\t"
      "s_set_gpr_idx_idx %[s7]\n\t"
      "v_xor_b32 %55, v96, %55\n\t"
      "v_xor_b32 %63, v112, %63\n\t"
      "s_set_gpr_idx_off\n\t"
      "v_readlane_b32 %[s0], %[v], 32\n\t"
      "v_readlane_b32 %[s1], %[v], 33\n\t"
      "v_readlane_b32 %[s2], %[v], 34\n\t"
      "v_readlane_b32 %[s3], %[v], 35\n\t"
      "v_readlane_b32 %[s4], %[v], 36\n\t"
      "v_readlane_b32 %[s5], %[v], 37\n\t"
      "v_readlane_b32 %[s6], %[v], 38\n\t"
      "v_readlane_b32 %[s7], %[v], 39\n\t"
      "s_set_gpr_idx_on %[s0], gpr_idx(SRC0)\n\t"
      "v_xor_b32 %64, v96, %64\n\t"
      "v_xor_b32 %72, v112, %72\n\t"
      "s_set_gpr_idx_idx %[s1]\n\t"
      "v_xor_b32 %65, v96, %65\n\t"
      "v_xor_b32 %73, v112, %73\n\t"
      "s_set_gpr_idx_idx %[s2]\n\t"
      "v_xor_b32 %66, v96, %66\n\t"
      "v_xor_b32 %74, v112, %74\n\t"
      "s_set_gpr_idx_idx %[s3]\n\t"
      "v_xor_b32 %67, v96, %67\n\t"
      "v_xor_b32 %75, v112, %75\n\t"
      "s_set_gpr_idx_idx %[s4]\n\t"
      "v_xor_b32 %68, v96, %68\n\t"
      "v_xor_b32 %76, v112, %76\n\t"
      "s_set_gpr_idx_idx %[s5]\n\t"
      "v_xor_b32 %69, v96, %69\n\t"
      "v_xor_b32 %77, v112, %77\n\t"
      "s_set_gpr_idx_idx %[s6]\n\t"
      "v_xor_b32 %70, v96, %70\n\t"
      "v_xor_b32 %78, v112, %78\n\t"
      "s_set_gpr_idx_idx %[s7]\n\t"
      "v_xor_b32 %71, v96, %71\n\t"
      "v_xor_b32 %79, v112, %79\n\t"
      "s_set_gpr_idx_off\n\t"
      : ZR(0), ZR(1), ZR(2), ZR(3), ZR(4), [s0] "=&s"(s0), [s1] "=&s"(s1), [s2] "=&s"(s2),
        [s3] "=&s"(s3), [s4] "=&s"(s4), [s5] "=&s"(s5), [s6] "=&s"(s6), [s7] "=&s"(s7)
      : [a] "v"(x0[0]), [b] "v"(x1[0]), [c] "v"(x2[0]), [d] "v"(x3[0]), [e] "v"(x0[1]),
        [f] "v"(x1[1]), [g] "v"(x2[1]), [h] "v"(x3[1]), [v] "v"(vidx)
      : "v96", "v97", "v98", "v99", "v100", "v101", "v102", "v103", "v104",
        "v105", "v106", "v107", "v108", "v109", "v110", "v111", "v112", "v113", "v114", "v115",
        "v116", "v117", "v118", "v119", "v120", "v121", "v122", "v123", "v124", "v125", "v126",
        "v127", "m0");
}

template <int MODE, int WAVES>
__global__ __launch_bounds__(WAVES * 64) void k(const uint8_t* __restrict__ shard, uint64_t nrec,
                                                const uint2* __restrict__ coef,
                                                const u32x8* __restrict__ mtab,
                                                uint32_t* __restrict__ out) {
  constexpr int VEC = 2;
  constexpr int GROUPS = 1024 / (64 * VEC * 4);  // column groups of a 1 KiB record
  constexpr int U = 8;
  const int lane = threadIdx.x & 63;
  const uint32_t wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t grp = wv % GROUPS;
  const uint64_t wave = (uint64_t)blockIdx.x * (WAVES / GROUPS) + wv / GROUPS;
  const uint64_t nw = (uint64_t)gridDim.x * (WAVES / GROUPS);
  const uint64_t r0 = wave * nrec / nw, r1 = (wave + 1) * nrec / nw;
  const uint8_t* base = shard + grp * (64 * VEC * 4) + lane * VEC * 4;
  // MODE 9: lane k (< 40) = plane k = (round k / 8, bit k % 8)
  const uint32_t la = (uint32_t)lane >> 3, lb = (uint32_t)lane & 7u;
  const uint32_t lsh = 8u * (la & 3u) + lb;
  const bool lhi = la >= 4;
  uint32_t Z[NQ][8][VEC];
#pragma unroll
  for (int a = 0; a < NQ; ++a)
#pragma unroll
    for (int b = 0; b < 8; ++b)
#pragma unroll
      for (int v = 0; v < VEC; ++v) Z[a][b][v] = 0;
  uint32_t xn[U][VEC];
  uint2 cn[U];
  auto load_batch = [&](uint64_t r) __attribute__((always_inline)) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint64_t rr = r + u < r1 ? r + u : r0;
      const u32x2 q = __builtin_nontemporal_load(reinterpret_cast<const u32x2*>(base + rr * 1024));
      xn[u][0] = q.x;
      xn[u][1] = q.y;
      cn[u] = coef[rr];
    }
  };
  if (r0 + U <= r1) load_batch(r0);
  for (uint64_t r = r0; r + U <= r1; r += U) {
    uint32_t x[U][VEC];
    uint32_t c0[U], c1[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
#pragma unroll
      for (int v = 0; v < VEC; ++v) x[u][v] = xn[u][v];
      c0[u] = __builtin_amdgcn_readfirstlane(cn[u].x);
      c1[u] = __builtin_amdgcn_readfirstlane(cn[u].y);
    }
    load_batch(r + U);
    if constexpr (MODE == 3) {
#pragma unroll
      for (int u = 0; u < U; ++u) Z[0][0][0] ^= x[u][0];
    } else if constexpr (MODE == 2) {
#pragma unroll
      for (int u = 0; u < U; ++u)
#pragma unroll
        for (int a = 0; a < NQ; ++a) {
          const uint32_t ca = ((a < 4 ? c0[u] : c1[u]) >> (8 * (a & 3))) & 0xffu;
          const u32x8 t = mtab[ca];
#pragma unroll
          for (int b = 0; b < 8; ++b)
#pragma unroll
            for (int v = 0; v < VEC; ++v) Z[a][b][v] = mxor(Z[a][b][v], x[u][v], t[b]);
        }
    } else {
#pragma unroll
      for (int g = 0; g < U; g += 4) {
        if constexpr (MODE == 8) {
          uint32_t w[NQ];
#pragma unroll
          for (int a = 0; a < NQ; ++a) {
            uint32_t acc = 0;
#pragma unroll
            for (int i = 0; i < 4; ++i) {
              const uint32_t ca = ((a < 4 ? c0[g + i] : c1[g + i]) >> (8 * (a & 3))) & 0xffu;
              acc |= c_spread[ca] << i;
            }
            w[a] = acc;
          }
          fold4_bfe(Z, x[g], x[g + 1], x[g + 2], x[g + 3], w);
        } else {
          uint32_t vidx = 0;
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const uint32_t cw = lhi ? c1[g + i] : c0[g + i];
            vidx |= ((cw >> lsh) & 1u) << i;
          }
          fold4_rl(Z, x[g], x[g + 1], x[g + 2], x[g + 3], vidx);
        }
      }
    }
  }
  uint32_t acc = 0;
#pragma unroll
  for (int a = 0; a < NQ; ++a)
#pragma unroll
    for (int b = 0; b < 8; ++b)
#pragma unroll
      for (int v = 0; v < VEC; ++v) acc ^= Z[a][b][v] * (2 * (8 * a + b) + 1);
  atomicXor(out, acc);
}

__global__ void fill(uint8_t* d, size_t n, uint64_t seed) {
  size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  for (; i < n / 8; i += (size_t)gridDim.x * blockDim.x) {
    uint64_t z = seed + i * 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    reinterpret_cast<uint64_t*>(d)[i] = z ^ (z >> 31);
  }
}

template <int MODE, int WAVES>
static int run(const uint8_t* shard, uint64_t nrec, const uint2* coef, const u32x8* mtab,
               uint32_t* out, int cus) {
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  CK(hipMemset(out, 0, 4));
  hipLaunchKernelGGL((k<MODE, WAVES>), dim3(cus), dim3(WAVES * 64), 0, 0, shard, nrec, coef, mtab, out);
  uint32_t sum = 0;
  CK(hipMemcpy(&sum, out, 4, hipMemcpyDeviceToHost));
  CK(hipEventRecord(e0));
  const int iters = 5;
  for (int it = 0; it < iters; ++it)
    hipLaunchKernelGGL((k<MODE, WAVES>), dim3(cus), dim3(WAVES * 64), 0, 0, shard, nrec, coef, mtab, out);
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  float ms;
  CK(hipEventElapsedTime(&ms, e0, e1));
  ms /= iters;
  printf("MODE=%d WAVES=%2d  %.3f ms  %.1f GB/s  checksum %08x\n", MODE, WAVES, ms,
         nrec * 1024.0 / ms / 1e6, sum);
  return 0;
}

int main() {
  int cus;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  const uint64_t nrec = 1ull << 22;  // 4 GiB
  uint8_t* shard;
  uint2* coef;
  u32x8* mtab;
  uint32_t* out;
  CK(hipMalloc(&shard, nrec * 1024));
  CK(hipMalloc(&coef, nrec * 8));
  CK(hipMalloc(&mtab, 256 * 32));
  CK(hipMalloc(&out, 256));
  uint32_t h[256 * 8], sp[256];
  for (int c = 0; c < 256; ++c) {
    sp[c] = 0;
    for (int b = 0; b < 8; ++b) {
      h[c * 8 + b] = ((c >> b) & 1) ? 0xffffffffu : 0u;
      sp[c] |= (uint32_t)((c >> b) & 1) << (4 * b);
    }
  }
  CK(hipMemcpy(mtab, h, sizeof(h), hipMemcpyHostToDevice));
  CK(hipMemcpyToSymbol(HIP_SYMBOL(c_spread), sp, sizeof(sp)));
  hipLaunchKernelGGL(fill, dim3(4096), dim3(256), 0, 0, shard, nrec * 1024, 1);
  hipLaunchKernelGGL(fill, dim3(4096), dim3(256), 0, 0, (uint8_t*)coef, nrec * 8, 2);
  CK(hipDeviceSynchronize());
  run<3, 8>(shard, nrec, coef, mtab, out, cus);
  run<2, 8>(shard, nrec, coef, mtab, out, cus);
  run<8, 8>(shard, nrec, coef, mtab, out, cus);
  run<9, 8>(shard, nrec, coef, mtab, out, cus);
  run<2, 16>(shard, nrec, coef, mtab, out, cus);
  run<8, 16>(shard, nrec, coef, mtab, out, cus);
  run<9, 16>(shard, nrec, coef, mtab, out, cus);
  return hipDeviceSynchronize() == hipSuccess ? 0 : 1;
}
