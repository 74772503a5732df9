// valu_ceiling.hip — issue cost of one wave64 VALU instruction per class on gfx950, measured.
//
// Measurement infrastructure (VERDICT r4 "Next round" 1), not product code.  The persistent
// render kernel's roofline (bench.py `valu_roofline`) prices its VALU instructions by class;
// this program measures what one instruction of each class holds a SIMD for, at 1, 2 and 4
// waves per SIMD, so that price is measured here rather than read off a table.
//
// Each wave runs a loop of `iters` x 128 instructions of one class: 8 independent chains (the
// dependent-issue latency of every class measured here is covered 8 deep), 16 asm statements
// per iteration, one instruction per chain per statement.  Workgroups of 256 x W threads
// (W waves on each of the CU's 4 SIMDs) declare 96 KiB of dynamic LDS, so at most one
// workgroup fits a CU (160 KiB), and the grid is one workgroup per CU.  Every wave stamps the
// shader clock (s_memtime) and the 100 MHz reference clock (s_memrealtime) around its loop
// after a workgroup barrier; the stamps go to a buffer of their own (nothing else reads them).
//
// Reported per (class, W), medians over 5 launches:
//   cyc_per_inst   = SIMD cycles one wave64 instruction of the class holds the SIMD for:
//                    (latest end - earliest start of the workgroup's waves, in shader cycles)
//                    / (W x 128 x iters), median over workgroups;
//   clock_ghz      = shader cycles / reference ticks x 0.1 GHz over the same span;
//   event_cyc      = the same figure from the launch's HIP-event time x that clock x CUs
//                    (whole-launch, includes launch overhead; a cross-check).
// One JSON line per (class, W) on stdout.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <algorithm>
#include <array>
#include <utility>
#include <vector>

#define CK(x)                                                                                   \
  do {                                                                                          \
    hipError_t e_ = (x);                                                                        \
    if (e_ != hipSuccess) {                                                                     \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_));       \
      exit(1);                                                                                  \
    }                                                                                           \
  } while (0)

typedef float f2 __attribute__((ext_vector_type(2)));

enum Op {
  OP_FMA_F32, OP_ADD_F32, OP_ADD_U32, OP_CNDMASK, OP_MUL_LO_U32, OP_MAD_U64_U32, OP_PK_FMA_F32,
  OP_FMA_F64, OP_MUL_F64, OP_ADD_F64, OP_RCP_F32, OP_RCP_F64, OP_MIX_F32_F64,
  // 32-bit classes the render kernel issues most (generic 32-bit body, GEN32 below)
  OP_CNDMASK_VCC, OP_AND_B32, OP_MOV_B32, OP_CMP_F32_VCC, OP_CMP_F32_SGPR, OP_FMA_F32_SGPR, OP_MUL_F32,
  OP_MAX_F32, OP_MED3_F32, OP_ADD_CO_U32, OP_LSHL_ADD_U32, OP_BFE_U32, OP_MUL_U32_U24, OP_CVT_F32_U32,
  // f64 results from 32-bit inputs and back
  OP_CVT_F64_F32, OP_CVT_F32_F64,
  OP_MIX3_F32_F64,  // 3 f32 FMAs per f64 FMA (the render kernel's f64 share is 21-25 %)
  OP_COUNT
};
static const char* kOpName[OP_COUNT] = {
    "v_fma_f32", "v_add_f32", "v_add_u32", "v_cndmask_b32_e64(sgpr)", "v_mul_lo_u32", "v_mad_u64_u32",
    "v_pk_fma_f32", "v_fma_f64", "v_mul_f64", "v_add_f64", "v_rcp_f32", "v_rcp_f64",
    "mix_fma_f32_f64_1to1", "v_cndmask_b32_e32(vcc)", "v_and_b32", "v_mov_b32", "v_cmp_lt_f32_e32(vcc)",
    "v_cmp_lt_f32_e64(sgpr)", "v_fma_f32(sgpr operand)", "v_mul_f32", "v_max_f32", "v_med3_f32",
    "v_add_co_u32", "v_lshl_add_u32", "v_bfe_u32", "v_mul_u32_u24", "v_cvt_f32_u32", "v_cvt_f64_f32",
    "v_cvt_f32_f64", "mix_fma_f32_f64_3to1"};

// one statement: one instruction on each of the 8 chains
#define CH8(INS) INS(0) INS(1) INS(2) INS(3) INS(4) INS(5) INS(6) INS(7)
#define S16(X) X X X X X X X X X X X X X X X X  /* 16 statements: 128 instructions per iteration */

// Generic 32-bit class: chains %0..%7 (32-bit VGPRs), inputs %8 / %9 (VGPRs), %10 (an SGPR
// pair), %11 (an SGPR).  INS(n) is one instruction on chain n, as a string literal.
#define R8(INS) INS("0") INS("1") INS("2") INS("3") INS("4") INS("5") INS("6") INS("7")
#define I_CNDMASK_VCC(n) "v_cndmask_b32_e32 %" n ", %" n ", %8, vcc\n"
#define I_AND(n) "v_and_b32 %" n ", %" n ", %8\n"
#define I_MOV(n) "v_mov_b32 %" n ", %8\n"
#define I_CMP_VCC(n) "v_cmp_lt_f32_e32 vcc, %" n ", %8\n"
#define I_CMP_SGPR(n) "v_cmp_lt_f32_e64 s[0:1], %" n ", %8\n"
#define I_FMA_SGPR(n) "v_fma_f32 %" n ", %" n ", %11, %9\n"
#define I_MUL_F32(n) "v_mul_f32 %" n ", %" n ", %8\n"
#define I_MAX_F32(n) "v_max_f32 %" n ", %" n ", %8\n"
#define I_MED3(n) "v_med3_f32 %" n ", %" n ", %8, %9\n"
#define I_ADD_CO(n) "v_add_co_u32 %" n ", vcc, %" n ", %8\n"
#define I_LSHL_ADD(n) "v_lshl_add_u32 %" n ", %" n ", 1, %8\n"
#define I_BFE(n) "v_bfe_u32 %" n ", %" n ", 3, 17\n"
#define I_MUL24(n) "v_mul_u32_u24 %" n ", %" n ", %8\n"
#define I_CVT_F32_U32(n) "v_cvt_f32_u32 %" n ", %" n "\n"
#define GEN32_STMT(INS, PRE)                                                                     \
  asm volatile(PRE R8(INS)                                                                     \
               : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) \
               : "v"(m), "v"(c), "s"(mask), "s"(sm)                                            \
               : "vcc", "s0", "s1");

template <int OP>
__device__ __forceinline__ void gen32(uint32_t iters, uint32_t* ii, uint64_t mask) {
  uint32_t a0 = ii[0], a1 = ii[1], a2 = ii[2], a3 = ii[3], a4 = ii[4], a5 = ii[5], a6 = ii[6], a7 = ii[7];
  const uint32_t m = ii[8], c = ii[9], sm = __builtin_amdgcn_readfirstlane(ii[8]);
  for (uint32_t it = 0; it < iters; ++it) {
    // the vcc-reading class sets vcc once per statement (one scalar move per 8 VALU instructions)
    if constexpr (OP == OP_CNDMASK_VCC) { S16(GEN32_STMT(I_CNDMASK_VCC, "s_mov_b64 vcc, %10\n")) }
    else if constexpr (OP == OP_AND_B32) { S16(GEN32_STMT(I_AND, "")) }
    else if constexpr (OP == OP_MOV_B32) { S16(GEN32_STMT(I_MOV, "")) }
    else if constexpr (OP == OP_CMP_F32_VCC) { S16(GEN32_STMT(I_CMP_VCC, "")) }
    else if constexpr (OP == OP_CMP_F32_SGPR) { S16(GEN32_STMT(I_CMP_SGPR, "")) }
    else if constexpr (OP == OP_FMA_F32_SGPR) { S16(GEN32_STMT(I_FMA_SGPR, "")) }
    else if constexpr (OP == OP_MUL_F32) { S16(GEN32_STMT(I_MUL_F32, "")) }
    else if constexpr (OP == OP_MAX_F32) { S16(GEN32_STMT(I_MAX_F32, "")) }
    else if constexpr (OP == OP_MED3_F32) { S16(GEN32_STMT(I_MED3, "")) }
    else if constexpr (OP == OP_ADD_CO_U32) { S16(GEN32_STMT(I_ADD_CO, "")) }
    else if constexpr (OP == OP_LSHL_ADD_U32) { S16(GEN32_STMT(I_LSHL_ADD, "")) }
    else if constexpr (OP == OP_BFE_U32) { S16(GEN32_STMT(I_BFE, "")) }
    else if constexpr (OP == OP_MUL_U32_U24) { S16(GEN32_STMT(I_MUL24, "")) }
    else { S16(GEN32_STMT(I_CVT_F32_U32, "")) }
  }
  ii[0] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}

template <int OP>
__device__ __forceinline__ void body(uint32_t iters, float* fo, double* dd, uint64_t* uu, uint32_t* ii, f2* pp) {
  if constexpr (OP >= OP_CNDMASK_VCC && OP <= OP_CVT_F32_U32) {
    gen32<OP>(iters, ii, uu[0]);
  } else if constexpr (OP == OP_CVT_F64_F32 || OP == OP_CVT_F32_F64) {
    // 4 f32 and 4 f64 values, converted back and forth: each statement converts every chain
    // one way (the two directions alternate by statement, so both stay live; each is timed
    // as the pair's mean), 8 instructions per statement
    float a0 = fo[0], a1 = fo[1], a2 = fo[2], a3 = fo[3];
    double b0 = dd[0], b1 = dd[1], b2 = dd[2], b3 = dd[3];
    for (uint32_t it = 0; it < iters; ++it) {
      if constexpr (OP == OP_CVT_F64_F32) {
        S16(asm volatile("v_cvt_f64_f32 %4, %0\n v_cvt_f64_f32 %5, %1\n v_cvt_f64_f32 %6, %2\n v_cvt_f64_f32 %7, %3\n"
                         "v_cvt_f64_f32 %4, %1\n v_cvt_f64_f32 %5, %2\n v_cvt_f64_f32 %6, %3\n v_cvt_f64_f32 %7, %0"
                         : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(b0), "+v"(b1), "+v"(b2), "+v"(b3));)
      } else {
        S16(asm volatile("v_cvt_f32_f64 %0, %4\n v_cvt_f32_f64 %1, %5\n v_cvt_f32_f64 %2, %6\n v_cvt_f32_f64 %3, %7\n"
                         "v_cvt_f32_f64 %0, %5\n v_cvt_f32_f64 %1, %6\n v_cvt_f32_f64 %2, %7\n v_cvt_f32_f64 %3, %4"
                         : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(b0), "+v"(b1), "+v"(b2), "+v"(b3));)
      }
    }
    fo[0] = a0 + a1 + a2 + a3;
    dd[0] = b0 + b1 + b2 + b3;
  } else if constexpr (OP == OP_MIX3_F32_F64) {
    float a0 = fo[0], a1 = fo[1], a2 = fo[2], a3 = fo[3], a4 = fo[4], a5 = fo[5];
    double b0 = dd[0], b1 = dd[1];
    const float m = fo[8], c = fo[9];
    const double dm = dd[8], dc = dd[9];
    for (uint32_t it = 0; it < iters; ++it) {
      S16(asm volatile(
              "v_fma_f32 %0, %0, %8, %9\n v_fma_f32 %1, %1, %8, %9\n v_fma_f32 %2, %2, %8, %9\n v_fma_f64 %6, %6, %10, %11\n"
              "v_fma_f32 %3, %3, %8, %9\n v_fma_f32 %4, %4, %8, %9\n v_fma_f32 %5, %5, %8, %9\n v_fma_f64 %7, %7, %10, %11"
              : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(b0), "+v"(b1)
              : "v"(m), "v"(c), "v"(dm), "v"(dc));)
    }
    fo[0] = a0 + a1 + a2 + a3 + a4 + a5;
    dd[0] = b0 + b1;
  } else if constexpr (OP == OP_FMA_F32 || OP == OP_ADD_F32 || OP == OP_RCP_F32) {
    float a0 = fo[0], a1 = fo[1], a2 = fo[2], a3 = fo[3], a4 = fo[4], a5 = fo[5], a6 = fo[6], a7 = fo[7];
    const float m = fo[8], c = fo[9];
    for (uint32_t it = 0; it < iters; ++it) {
      if constexpr (OP == OP_FMA_F32) {
        S16(asm volatile(
               "v_fma_f32 %0, %0, %8, %9\n v_fma_f32 %1, %1, %8, %9\n v_fma_f32 %2, %2, %8, %9\n"
               "v_fma_f32 %3, %3, %8, %9\n v_fma_f32 %4, %4, %8, %9\n v_fma_f32 %5, %5, %8, %9\n"
               "v_fma_f32 %6, %6, %8, %9\n v_fma_f32 %7, %7, %8, %9"
               : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)
               : "v"(m), "v"(c));)
      } else if constexpr (OP == OP_ADD_F32) {
        S16(asm volatile(
               "v_add_f32 %0, %0, %8\n v_add_f32 %1, %1, %8\n v_add_f32 %2, %2, %8\n v_add_f32 %3, %3, %8\n"
               "v_add_f32 %4, %4, %8\n v_add_f32 %5, %5, %8\n v_add_f32 %6, %6, %8\n v_add_f32 %7, %7, %8"
               : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)
               : "v"(c));)
      } else {
        S16(asm volatile(
               "v_rcp_f32 %0, %0\n v_rcp_f32 %1, %1\n v_rcp_f32 %2, %2\n v_rcp_f32 %3, %3\n"
               "v_rcp_f32 %4, %4\n v_rcp_f32 %5, %5\n v_rcp_f32 %6, %6\n v_rcp_f32 %7, %7"
               : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7));)
      }
    }
    fo[0] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7;
  } else if constexpr (OP == OP_ADD_U32 || OP == OP_CNDMASK || OP == OP_MUL_LO_U32) {
    uint32_t a0 = ii[0], a1 = ii[1], a2 = ii[2], a3 = ii[3], a4 = ii[4], a5 = ii[5], a6 = ii[6], a7 = ii[7];
    const uint32_t m = ii[8];
    const uint64_t mask = uu[0];
    for (uint32_t it = 0; it < iters; ++it) {
      if constexpr (OP == OP_ADD_U32) {
        S16(asm volatile(
               "v_add_u32 %0, %0, %8\n v_add_u32 %1, %1, %8\n v_add_u32 %2, %2, %8\n v_add_u32 %3, %3, %8\n"
               "v_add_u32 %4, %4, %8\n v_add_u32 %5, %5, %8\n v_add_u32 %6, %6, %8\n v_add_u32 %7, %7, %8"
               : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)
               : "v"(m));)
      } else if constexpr (OP == OP_CNDMASK) {
        S16(asm volatile(
               "v_cndmask_b32_e64 %0, %0, %8, %9\n v_cndmask_b32_e64 %1, %1, %8, %9\n"
               "v_cndmask_b32_e64 %2, %2, %8, %9\n v_cndmask_b32_e64 %3, %3, %8, %9\n"
               "v_cndmask_b32_e64 %4, %4, %8, %9\n v_cndmask_b32_e64 %5, %5, %8, %9\n"
               "v_cndmask_b32_e64 %6, %6, %8, %9\n v_cndmask_b32_e64 %7, %7, %8, %9"
               : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)
               : "v"(m), "s"(mask));)
      } else {
        S16(asm volatile(
               "v_mul_lo_u32 %0, %0, %8\n v_mul_lo_u32 %1, %1, %8\n v_mul_lo_u32 %2, %2, %8\n"
               "v_mul_lo_u32 %3, %3, %8\n v_mul_lo_u32 %4, %4, %8\n v_mul_lo_u32 %5, %5, %8\n"
               "v_mul_lo_u32 %6, %6, %8\n v_mul_lo_u32 %7, %7, %8"
               : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)
               : "v"(m));)
      }
    }
    ii[0] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
  } else if constexpr (OP == OP_MAD_U64_U32) {
    uint64_t a0 = uu[0], a1 = uu[1], a2 = uu[2], a3 = uu[3], a4 = uu[4], a5 = uu[5], a6 = uu[6], a7 = uu[7];
    const uint32_t m = ii[8], n = ii[9];
    for (uint32_t it = 0; it < iters; ++it) {
      S16(asm volatile(
             "v_mad_u64_u32 %0, vcc, %8, %9, %0\n v_mad_u64_u32 %1, vcc, %8, %9, %1\n"
             "v_mad_u64_u32 %2, vcc, %8, %9, %2\n v_mad_u64_u32 %3, vcc, %8, %9, %3\n"
             "v_mad_u64_u32 %4, vcc, %8, %9, %4\n v_mad_u64_u32 %5, vcc, %8, %9, %5\n"
             "v_mad_u64_u32 %6, vcc, %8, %9, %6\n v_mad_u64_u32 %7, vcc, %8, %9, %7"
             : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)
             : "v"(m), "v"(n)
             : "vcc");)
    }
    uu[0] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
  } else if constexpr (OP == OP_PK_FMA_F32) {
    f2 a0 = pp[0], a1 = pp[1], a2 = pp[2], a3 = pp[3], a4 = pp[4], a5 = pp[5], a6 = pp[6], a7 = pp[7];
    const f2 m = pp[8], c = pp[9];
    for (uint32_t it = 0; it < iters; ++it) {
      S16(asm volatile(
             "v_pk_fma_f32 %0, %0, %8, %9\n v_pk_fma_f32 %1, %1, %8, %9\n v_pk_fma_f32 %2, %2, %8, %9\n"
             "v_pk_fma_f32 %3, %3, %8, %9\n v_pk_fma_f32 %4, %4, %8, %9\n v_pk_fma_f32 %5, %5, %8, %9\n"
             "v_pk_fma_f32 %6, %6, %8, %9\n v_pk_fma_f32 %7, %7, %8, %9"
             : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)
             : "v"(m), "v"(c));)
    }
    pp[0] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7;
  } else if constexpr (OP == OP_FMA_F64 || OP == OP_MUL_F64 || OP == OP_ADD_F64 || OP == OP_RCP_F64) {
    double a0 = dd[0], a1 = dd[1], a2 = dd[2], a3 = dd[3], a4 = dd[4], a5 = dd[5], a6 = dd[6], a7 = dd[7];
    const double m = dd[8], c = dd[9];
    for (uint32_t it = 0; it < iters; ++it) {
      if constexpr (OP == OP_FMA_F64) {
        S16(asm volatile(
               "v_fma_f64 %0, %0, %8, %9\n v_fma_f64 %1, %1, %8, %9\n v_fma_f64 %2, %2, %8, %9\n"
               "v_fma_f64 %3, %3, %8, %9\n v_fma_f64 %4, %4, %8, %9\n v_fma_f64 %5, %5, %8, %9\n"
               "v_fma_f64 %6, %6, %8, %9\n v_fma_f64 %7, %7, %8, %9"
               : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)
               : "v"(m), "v"(c));)
      } else if constexpr (OP == OP_MUL_F64) {
        S16(asm volatile(
               "v_mul_f64 %0, %0, %8\n v_mul_f64 %1, %1, %8\n v_mul_f64 %2, %2, %8\n v_mul_f64 %3, %3, %8\n"
               "v_mul_f64 %4, %4, %8\n v_mul_f64 %5, %5, %8\n v_mul_f64 %6, %6, %8\n v_mul_f64 %7, %7, %8"
               : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)
               : "v"(m));)
      } else if constexpr (OP == OP_ADD_F64) {
        S16(asm volatile(
               "v_add_f64 %0, %0, %8\n v_add_f64 %1, %1, %8\n v_add_f64 %2, %2, %8\n v_add_f64 %3, %3, %8\n"
               "v_add_f64 %4, %4, %8\n v_add_f64 %5, %5, %8\n v_add_f64 %6, %6, %8\n v_add_f64 %7, %7, %8"
               : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)
               : "v"(c));)
      } else {
        S16(asm volatile(
               "v_rcp_f64 %0, %0\n v_rcp_f64 %1, %1\n v_rcp_f64 %2, %2\n v_rcp_f64 %3, %3\n"
               "v_rcp_f64 %4, %4\n v_rcp_f64 %5, %5\n v_rcp_f64 %6, %6\n v_rcp_f64 %7, %7"
               : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7));)
      }
    }
    dd[0] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7;
  } else {  // OP_MIX_F32_F64: 4 f32 and 4 f64 chains, alternating
    float a0 = fo[0], a1 = fo[1], a2 = fo[2], a3 = fo[3];
    double b0 = dd[0], b1 = dd[1], b2 = dd[2], b3 = dd[3];
    const float m = fo[8], c = fo[9];
    const double dm = dd[8], dc = dd[9];
    for (uint32_t it = 0; it < iters; ++it) {
      S16(asm volatile(
             "v_fma_f32 %0, %0, %8, %9\n v_fma_f64 %4, %4, %10, %11\n v_fma_f32 %1, %1, %8, %9\n"
             "v_fma_f64 %5, %5, %10, %11\n v_fma_f32 %2, %2, %8, %9\n v_fma_f64 %6, %6, %10, %11\n"
             "v_fma_f32 %3, %3, %8, %9\n v_fma_f64 %7, %7, %10, %11"
             : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(b0), "+v"(b1), "+v"(b2), "+v"(b3)
             : "v"(m), "v"(c), "v"(dm), "v"(dc));)
    }
    fo[0] = a0 + a1 + a2 + a3;
    dd[0] = b0 + b1 + b2 + b3;
  }
}

struct Stamp {
  unsigned long long t0, t1, r0, r1;
};

template <int OP>
__global__ void k_valu(uint32_t iters, float* sink, Stamp* stamps, uint32_t seed) {
  extern __shared__ char lds_pad[];  // only to hold the CU: one workgroup per CU
  const uint32_t tid = threadIdx.x + blockIdx.x * blockDim.x;
  // operands: ordinary values near 1 (no denormals, no infinities), per lane
  float fo[10];
  double dd[10];
  uint64_t uu[8];
  uint32_t ii[10];
  f2 pp[10];
  for (int i = 0; i < 10; ++i) {
    const uint32_t h = (tid * 2654435761u) ^ (seed + 97u * i);
    fo[i] = 1.0f + (h & 0xffff) * 1e-9f;
    dd[i] = 1.0 + (h & 0xffff) * 1e-12;
    ii[i] = h | 1u;
    pp[i] = f2{fo[i], fo[i] * 0.5f + 0.5f};
    if (i < 8) uu[i] = ((uint64_t)h << 32) | (h ^ 0x9e3779b9u);
  }
  fo[8] = 0.99999994f;
  fo[9] = 1e-7f;
  dd[8] = 0.9999999999;
  dd[9] = 1e-10;
  pp[8] = f2{0.99999994f, 0.99999994f};
  pp[9] = f2{1e-7f, 1e-7f};
  uu[0] = (seed & 1) ? ~0ull : 0x5555555555555555ull;  // the cndmask's selector
  __syncthreads();
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  const unsigned long long r0 = __builtin_amdgcn_s_memrealtime();
  __builtin_amdgcn_s_waitcnt(0xC07F);
  body<OP>(iters, fo, dd, uu, ii, pp);
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  const unsigned long long r1 = __builtin_amdgcn_s_memrealtime();
  __builtin_amdgcn_s_waitcnt(0xC07F);
  const uint32_t wave = tid >> 6;
  if ((threadIdx.x & 63) == 0) stamps[wave] = Stamp{t0, t1, r0, r1};
  // keep every chain live: the sum only reaches memory under a condition no lane meets
  const float v = fo[0] + (float)dd[0] + (float)(ii[0] & 1) + (float)(uu[0] & 1) + pp[0].x + pp[0].y;
  if (v == -1.2345f) sink[tid] = v + lds_pad[tid & 7];
}

typedef void (*KFn)(uint32_t, float*, Stamp*, uint32_t);
template <int... I>
static constexpr auto make_table(std::integer_sequence<int, I...>) {
  return std::array<KFn, sizeof...(I)>{k_valu<I>...};
}
static const auto kFn = make_table(std::make_integer_sequence<int, OP_COUNT>{});

static double median(std::vector<double> v) {
  std::sort(v.begin(), v.end());
  return v.empty() ? 0.0 : v[v.size() / 2];
}

int main(int argc, char** argv) {
  const int reps = 5;
  const uint32_t base_iters = argc > 1 ? (uint32_t)atoi(argv[1]) : 2048;
  int dev = 0;
  CK(hipSetDevice(dev));
  hipDeviceProp_t prop;
  CK(hipGetDeviceProperties(&prop, dev));
  const int cus = prop.multiProcessorCount;
  const size_t lds = 96 * 1024;  // > 80 KiB: one workgroup per CU
  float* sink;
  Stamp* stamps;
  CK(hipMalloc(&sink, (size_t)cus * 1024 * sizeof(float)));
  CK(hipMalloc(&stamps, (size_t)cus * 16 * sizeof(Stamp)));
  for (int op = 0; op < OP_COUNT; ++op)
    CK(hipFuncSetAttribute((const void*)kFn[op], hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  // warm the clock: ~1 s of launches before the first measured one (MI355X_MICROARCH.md DVFS (6))
  for (int i = 0; i < 60; ++i) hipLaunchKernelGGL(kFn[OP_FMA_F32], dim3(cus), dim3(1024), lds, 0, 8 * base_iters, sink, stamps, 1u);
  CK(hipDeviceSynchronize());
  fprintf(stderr, "device %s, %d CUs, iters %u\n", prop.name, cus, base_iters);
  const int op_from = argc > 2 ? atoi(argv[2]) : 0;
  for (int op = op_from; op < OP_COUNT; ++op) {
    for (int w : {1, 2, 4}) {
      const int threads = 256 * w, waves = cus * 4 * w;
      const uint32_t iters = base_iters * 4 / w;  // about the same launch time for every W
      std::vector<double> cyc, clk, ev_cyc;
      std::vector<Stamp> h(waves);
      for (int r = 0; r < reps; ++r) {
        CK(hipEventRecord(e0, 0));
        hipLaunchKernelGGL(kFn[op], dim3(cus), dim3(threads), lds, 0, iters, sink, stamps, (uint32_t)(r + 1));
        CK(hipGetLastError());
        CK(hipEventRecord(e1, 0));
        CK(hipEventSynchronize(e1));
        float ms = 0.f;
        CK(hipEventElapsedTime(&ms, e0, e1));
        CK(hipMemcpy(h.data(), stamps, waves * sizeof(Stamp), hipMemcpyDeviceToHost));
        std::vector<double> per_wg, per_wg_clk;
        for (int b = 0; b < cus; ++b) {
          unsigned long long t0 = ~0ull, t1 = 0, r0 = ~0ull, r1 = 0;
          for (int k = 0; k < 4 * w; ++k) {
            const Stamp& s = h[b * 4 * w + k];
            t0 = std::min(t0, s.t0);
            t1 = std::max(t1, s.t1);
            r0 = std::min(r0, s.r0);
            r1 = std::max(r1, s.r1);
          }
          per_wg.push_back((double)(t1 - t0) / ((double)w * 128.0 * iters));
          per_wg_clk.push_back((double)(t1 - t0) / (double)(r1 - r0) * 0.1);
        }
        const double c = median(per_wg), g = median(per_wg_clk);
        cyc.push_back(c);
        clk.push_back(g);
        ev_cyc.push_back(ms * 1e-3 * g * 1e9 / ((double)w * 128.0 * iters));
      }
      printf("{\"class\": \"%s\", \"waves_per_simd\": %d, \"insts_per_wave\": %llu, \"cyc_per_inst\": %.4f, "
             "\"clock_ghz\": %.4f, \"event_cyc_per_inst\": %.4f, \"cus\": %d}\n",
             kOpName[op], w, (unsigned long long)iters * 128ull, median(cyc), median(clk), median(ev_cyc), cus);
      fflush(stdout);
    }
  }
  CK(hipFree(sink));
  CK(hipFree(stamps));
  return 0;
}
