// Issue cost (independent stream) and latency (dependent chain) of the
// instructions in the Cholesky pivot on gfx950, alone (one wave per SIMD) and
// beside a partner wave issuing back-to-back v_mfma_f64_16x16x4_f64 (two
// waves per SIMD: waves 0-3 of each 512-thread workgroup run op A, waves 4-7
// op B).  Cycles per instruction = s_memtime delta / (ITERS * 16), median
// over waves.  Every stream is hand-written asm, so nothing is reordered.
//   hipcc --offload-arch=gfx950 -O3 -o fp64_issue_probe fp64_issue_probe.hip && ./fp64_issue_probe
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <vector>

constexpr int ITERS = 256;

enum Op {
  NONE, MFMA, MFMA1, MFMA2, MFMA8, FMA_IND, FMA_DEP, FMACDPP_IND, FMACDPP_DEP, MOVDPP_IND, RLANE_IND, BPERM_IND, BPERM_DEP,
  RCP_IND, RCP_DEP, CND_IND, NOP0, MUL_IND, FMAC_IND, NOP1, MFMA_ASM4, MFMA_ASM8, IADD_IND, SALU_IND, MOVB32_IND, MFMA_PAD, MFMA_PAD_FMA
};
static const char* NAMES[] = {"none", "mfma_f64_16x16x4 x4 chains", "mfma x1 chain", "mfma x2 chains", "mfma x8 chains", "v_fma_f64 indep", "v_fma_f64 dep chain",
                              "v_fmac_f64_dpp indep", "v_fmac_f64_dpp+s_nop1 dep", "v_mov_b64_dpp indep",
                              "v_readlane_b32 indep", "ds_bpermute_b32 indep", "ds_bpermute+wait dep",
                              "v_rcp_f64 indep", "v_rcp_f64 dep chain", "v_cndmask_b32 indep", "s_nop 0",
                              "v_mul_f64 indep", "v_fmac_f64_e32 indep", "s_nop 1",
                              "asm mfma x4 acc (16/blk)", "asm mfma x8 acc (16/blk)",
                              "v_add_u32 indep", "s_add_u32 indep", "v_mov_b32 indep",
                              "mfma + s_nop 7,6 (60 cyc)", "8 mfma + 8 own fma (per mfma)"};

#define R16(x) x x x x x x x x x x x x x x x x

template <int OP>
__device__ __forceinline__ void body(double* v, double w) {
  // v[0..7]: 8 independent 64-bit registers; every stream issues 16 instructions
  if constexpr (OP == MFMA || OP == MFMA1 || OP == MFMA2 || OP == MFMA8) {
    // NC distinct accumulation chains (distinct initial values: no CSE), 16 MFMAs
    typedef double v4d __attribute__((ext_vector_type(4)));
    constexpr int NC = OP == MFMA1 ? 1 : OP == MFMA2 ? 2 : OP == MFMA8 ? 8 : 4;
    v4d a[NC];
    for (int j = 0; j < NC; ++j) a[j] = v4d{v[j % 8] + j, v[(j + 1) % 8] - j, v[(j + 2) % 8] * (j + 1), v[(j + 3) % 8]};
    for (int i = 0; i < 16 / NC; ++i)
      for (int j = 0; j < NC; ++j) a[j] = __builtin_amdgcn_mfma_f64_16x16x4f64(w, v[j % 8], a[j], 0, 0, 0);
    double t = 0;
    for (int j = 0; j < NC; ++j) t += a[j][0] + a[j][3];
    v[0] += t;
  } else if constexpr (OP == FMA_IND) {
    asm volatile(R16("v_fma_f64 %0, %8, %8, %0\n v_fma_f64 %1, %8, %8, %1\n v_fma_f64 %2, %8, %8, %2\n v_fma_f64 %3, %8, %8, %3\n"
                     "v_fma_f64 %4, %8, %8, %4\n v_fma_f64 %5, %8, %8, %5\n v_fma_f64 %6, %8, %8, %6\n v_fma_f64 %7, %8, %8, %7\n")
                 : "+v"(v[0]), "+v"(v[1]), "+v"(v[2]), "+v"(v[3]), "+v"(v[4]), "+v"(v[5]), "+v"(v[6]), "+v"(v[7]) : "v"(w));
  } else if constexpr (OP == FMA_DEP) {
    asm volatile(R16("v_fma_f64 %0, %1, %1, %0\n") : "+v"(v[0]) : "v"(w));
  } else if constexpr (OP == FMACDPP_IND) {
    asm volatile(R16("v_fmac_f64_dpp %0, %0, %8 row_newbcast:3 row_mask:0xf bank_mask:0xf\n v_fmac_f64_dpp %1, %1, %8 row_newbcast:3 row_mask:0xf bank_mask:0xf\n"
                     "v_fmac_f64_dpp %2, %2, %8 row_newbcast:3 row_mask:0xf bank_mask:0xf\n v_fmac_f64_dpp %3, %3, %8 row_newbcast:3 row_mask:0xf bank_mask:0xf\n"
                     "v_fmac_f64_dpp %4, %4, %8 row_newbcast:3 row_mask:0xf bank_mask:0xf\n v_fmac_f64_dpp %5, %5, %8 row_newbcast:3 row_mask:0xf bank_mask:0xf\n"
                     "v_fmac_f64_dpp %6, %6, %8 row_newbcast:3 row_mask:0xf bank_mask:0xf\n v_fmac_f64_dpp %7, %7, %8 row_newbcast:3 row_mask:0xf bank_mask:0xf\n")
                 : "+v"(v[0]), "+v"(v[1]), "+v"(v[2]), "+v"(v[3]), "+v"(v[4]), "+v"(v[5]), "+v"(v[6]), "+v"(v[7]) : "v"(w));
  } else if constexpr (OP == FMACDPP_DEP) {
    asm volatile(R16("s_nop 1\n v_fmac_f64_dpp %0, %0, %1 row_newbcast:3 row_mask:0xf bank_mask:0xf\n") : "+v"(v[0]) : "v"(w));
  } else if constexpr (OP == MOVDPP_IND) {
    asm volatile(R16("v_mov_b64_dpp %0, %8 row_newbcast:3 row_mask:0xf bank_mask:0xf bound_ctrl:1\n v_mov_b64_dpp %1, %8 row_newbcast:3 row_mask:0xf bank_mask:0xf bound_ctrl:1\n"
                     "v_mov_b64_dpp %2, %8 row_newbcast:3 row_mask:0xf bank_mask:0xf bound_ctrl:1\n v_mov_b64_dpp %3, %8 row_newbcast:3 row_mask:0xf bank_mask:0xf bound_ctrl:1\n"
                     "v_mov_b64_dpp %4, %8 row_newbcast:3 row_mask:0xf bank_mask:0xf bound_ctrl:1\n v_mov_b64_dpp %5, %8 row_newbcast:3 row_mask:0xf bank_mask:0xf bound_ctrl:1\n"
                     "v_mov_b64_dpp %6, %8 row_newbcast:3 row_mask:0xf bank_mask:0xf bound_ctrl:1\n v_mov_b64_dpp %7, %8 row_newbcast:3 row_mask:0xf bank_mask:0xf bound_ctrl:1\n")
                 : "=&v"(v[0]), "=&v"(v[1]), "=&v"(v[2]), "=&v"(v[3]), "=&v"(v[4]), "=&v"(v[5]), "=&v"(v[6]), "=&v"(v[7]) : "v"(w));
  } else if constexpr (OP == RLANE_IND) {
    int s0, s1, s2, s3;
    asm volatile(R16("v_readlane_b32 %0, %4, 3\n v_readlane_b32 %1, %4, 7\n v_readlane_b32 %2, %4, 11\n v_readlane_b32 %3, %4, 13\n")
                 : "=s"(s0), "=s"(s1), "=s"(s2), "=s"(s3) : "v"(__double2loint(w)));
    v[0] += s0 + s1 + s2 + s3;
  } else if constexpr (OP == BPERM_IND) {
    int r[8];
    asm volatile(R16("ds_bpermute_b32 %0, %8, %9\n ds_bpermute_b32 %1, %8, %9 offset:4\n ds_bpermute_b32 %2, %8, %9 offset:8\n ds_bpermute_b32 %3, %8, %9 offset:12\n"
                     "ds_bpermute_b32 %4, %8, %9 offset:16\n ds_bpermute_b32 %5, %8, %9 offset:20\n ds_bpermute_b32 %6, %8, %9 offset:24\n ds_bpermute_b32 %7, %8, %9 offset:28\n")
                 "s_waitcnt lgkmcnt(0)\n"
                 : "=&v"(r[0]), "=&v"(r[1]), "=&v"(r[2]), "=&v"(r[3]), "=&v"(r[4]), "=&v"(r[5]), "=&v"(r[6]), "=&v"(r[7])
                 : "v"((int)(threadIdx.x & 63) * 4), "v"(__double2loint(w)));
    v[0] += r[0] + r[7];
  } else if constexpr (OP == BPERM_DEP) {
    int x = __double2loint(v[0]);
    asm volatile(R16("ds_bpermute_b32 %0, %1, %0\n s_waitcnt lgkmcnt(0)\n") : "+v"(x) : "v"((int)(threadIdx.x & 63) * 4));
    v[0] += x;
  } else if constexpr (OP == RCP_IND) {
    asm volatile(R16("v_rcp_f64 %0, %8\n v_rcp_f64 %1, %8\n v_rcp_f64 %2, %8\n v_rcp_f64 %3, %8\n"
                     "v_rcp_f64 %4, %8\n v_rcp_f64 %5, %8\n v_rcp_f64 %6, %8\n v_rcp_f64 %7, %8\n")
                 : "=&v"(v[0]), "=&v"(v[1]), "=&v"(v[2]), "=&v"(v[3]), "=&v"(v[4]), "=&v"(v[5]), "=&v"(v[6]), "=&v"(v[7]) : "v"(w));
  } else if constexpr (OP == RCP_DEP) {
    asm volatile(R16("v_rcp_f64 %0, %0\n") : "+v"(v[0]));
  } else if constexpr (OP == CND_IND) {
    int r[4];
    asm volatile(R16("v_cndmask_b32_e64 %0, 0, %4, vcc\n v_cndmask_b32_e64 %1, 0, %4, vcc\n v_cndmask_b32_e64 %2, 0, %4, vcc\n v_cndmask_b32_e64 %3, 0, %4, vcc\n")
                 : "=&v"(r[0]), "=&v"(r[1]), "=&v"(r[2]), "=&v"(r[3]) : "v"(__double2loint(w)) : "vcc");
    v[0] += r[0] + r[3];
  } else if constexpr (OP == NOP0) {
    asm volatile(R16("s_nop 0\n s_nop 0\n s_nop 0\n s_nop 0\n s_nop 0\n s_nop 0\n s_nop 0\n s_nop 0\n") ::);
  } else if constexpr (OP == MUL_IND) {
    asm volatile(R16("v_mul_f64 %0, %8, %0\n v_mul_f64 %1, %8, %1\n v_mul_f64 %2, %8, %2\n v_mul_f64 %3, %8, %3\n"
                     "v_mul_f64 %4, %8, %4\n v_mul_f64 %5, %8, %5\n v_mul_f64 %6, %8, %6\n v_mul_f64 %7, %8, %7\n")
                 : "+v"(v[0]), "+v"(v[1]), "+v"(v[2]), "+v"(v[3]), "+v"(v[4]), "+v"(v[5]), "+v"(v[6]), "+v"(v[7]) : "v"(w));
  } else if constexpr (OP == FMAC_IND) {
    asm volatile(R16("v_fmac_f64_e32 %0, %8, %8\n v_fmac_f64_e32 %1, %8, %8\n v_fmac_f64_e32 %2, %8, %8\n v_fmac_f64_e32 %3, %8, %8\n"
                     "v_fmac_f64_e32 %4, %8, %8\n v_fmac_f64_e32 %5, %8, %8\n v_fmac_f64_e32 %6, %8, %8\n v_fmac_f64_e32 %7, %8, %8\n")
                 : "+v"(v[0]), "+v"(v[1]), "+v"(v[2]), "+v"(v[3]), "+v"(v[4]), "+v"(v[5]), "+v"(v[6]), "+v"(v[7]) : "v"(w));
  } else if constexpr (OP == MFMA_ASM4 || OP == MFMA_ASM8) {
    // 16 MFMAs round-robin over 4 or 8 accumulators held across calls (no
    // per-call setup); pure issue / pipe throughput
    typedef double v4d __attribute__((ext_vector_type(4)));
    static_assert(sizeof(v4d) == 32, "");
    v4d* acc = reinterpret_cast<v4d*>(v);   // v has room for 8 v4d (see k_pair)
    if constexpr (OP == MFMA_ASM4) {
      asm volatile(R16("v_mfma_f64_16x16x4_f64 %0, %4, %5, %0\n" "v_mfma_f64_16x16x4_f64 %1, %4, %5, %1\n"
                       "v_mfma_f64_16x16x4_f64 %2, %4, %5, %2\n" "v_mfma_f64_16x16x4_f64 %3, %4, %5, %3\n")
                   : "+v"(acc[0]), "+v"(acc[1]), "+v"(acc[2]), "+v"(acc[3]) : "v"(w), "v"(v[32]));
    } else {
      asm volatile(R16("v_mfma_f64_16x16x4_f64 %0, %8, %9, %0\n" "v_mfma_f64_16x16x4_f64 %1, %8, %9, %1\n"
                       "v_mfma_f64_16x16x4_f64 %2, %8, %9, %2\n" "v_mfma_f64_16x16x4_f64 %3, %8, %9, %3\n"
                       "v_mfma_f64_16x16x4_f64 %4, %8, %9, %4\n" "v_mfma_f64_16x16x4_f64 %5, %8, %9, %5\n"
                       "v_mfma_f64_16x16x4_f64 %6, %8, %9, %6\n" "v_mfma_f64_16x16x4_f64 %7, %8, %9, %7\n")
                   : "+v"(acc[0]), "+v"(acc[1]), "+v"(acc[2]), "+v"(acc[3]), "+v"(acc[4]), "+v"(acc[5]), "+v"(acc[6]),
                     "+v"(acc[7]) : "v"(w), "v"(v[32]));
    }
  } else if constexpr (OP == IADD_IND || OP == MOVB32_IND) {
    int r[8];
    for (int j = 0; j < 8; ++j) r[j] = (int)threadIdx.x + j;
    if constexpr (OP == IADD_IND)
      asm volatile(R16("v_add_u32 %0, %0, %8\n v_add_u32 %1, %1, %8\n v_add_u32 %2, %2, %8\n v_add_u32 %3, %3, %8\n"
                       "v_add_u32 %4, %4, %8\n v_add_u32 %5, %5, %8\n v_add_u32 %6, %6, %8\n v_add_u32 %7, %7, %8\n")
                   : "+v"(r[0]), "+v"(r[1]), "+v"(r[2]), "+v"(r[3]), "+v"(r[4]), "+v"(r[5]), "+v"(r[6]), "+v"(r[7])
                   : "v"(__double2loint(w)));
    else
      asm volatile(R16("v_mov_b32 %0, %8\n v_mov_b32 %1, %8\n v_mov_b32 %2, %8\n v_mov_b32 %3, %8\n"
                       "v_mov_b32 %4, %8\n v_mov_b32 %5, %8\n v_mov_b32 %6, %8\n v_mov_b32 %7, %8\n")
                   : "+v"(r[0]), "+v"(r[1]), "+v"(r[2]), "+v"(r[3]), "+v"(r[4]), "+v"(r[5]), "+v"(r[6]), "+v"(r[7])
                   : "v"(__double2loint(w)));
    v[0] += r[0] + r[7];
  } else if constexpr (OP == SALU_IND) {
    int s0 = 1, s1 = 2, s2 = 3, s3 = 4;
    asm volatile(R16("s_add_u32 %0, %0, 3\n s_add_u32 %1, %1, 5\n s_add_u32 %2, %2, 7\n s_add_u32 %3, %3, 9\n"
                     "s_add_u32 %0, %0, 3\n s_add_u32 %1, %1, 5\n s_add_u32 %2, %2, 7\n s_add_u32 %3, %3, 9\n")
                 : "+s"(s0), "+s"(s1), "+s"(s2), "+s"(s3) :: "scc");
    v[0] += s0 + s1 + s2 + s3;
  } else if constexpr (OP == MFMA_PAD || OP == MFMA_PAD_FMA) {
    // 16 MFMAs round-robin over 8 accumulators; after each, either ~60 cycles
    // of s_nop (the wave presents no instruction while the pipe is busy) or
    // 8 independent v_fma_f64 of its own
    typedef double v4d __attribute__((ext_vector_type(4)));
    v4d* acc = reinterpret_cast<v4d*>(v);
    if constexpr (OP == MFMA_PAD) {
      asm volatile(R16("v_mfma_f64_16x16x4_f64 %0, %8, %9, %0\n s_nop 7\n s_nop 6\n"
                       "v_mfma_f64_16x16x4_f64 %1, %8, %9, %1\n s_nop 7\n s_nop 6\n"
                       "v_mfma_f64_16x16x4_f64 %2, %8, %9, %2\n s_nop 7\n s_nop 6\n"
                       "v_mfma_f64_16x16x4_f64 %3, %8, %9, %3\n s_nop 7\n s_nop 6\n"
                       "v_mfma_f64_16x16x4_f64 %4, %8, %9, %4\n s_nop 7\n s_nop 6\n"
                       "v_mfma_f64_16x16x4_f64 %5, %8, %9, %5\n s_nop 7\n s_nop 6\n"
                       "v_mfma_f64_16x16x4_f64 %6, %8, %9, %6\n s_nop 7\n s_nop 6\n"
                       "v_mfma_f64_16x16x4_f64 %7, %8, %9, %7\n s_nop 7\n s_nop 6\n")
                   : "+v"(acc[0]), "+v"(acc[1]), "+v"(acc[2]), "+v"(acc[3]), "+v"(acc[4]), "+v"(acc[5]), "+v"(acc[6]),
                     "+v"(acc[7]) : "v"(w), "v"(v[32]));
    } else {
      double f0 = v[33], f1 = v[34], f2 = v[35], f3 = v[36];
      asm volatile(R16("v_mfma_f64_16x16x4_f64 %[a0], %[w], %[x], %[a0]\n"
                       "v_fma_f64 %[f0], %[w], %[w], %[f0]\n v_fma_f64 %[f1], %[w], %[w], %[f1]\n"
                       "v_fma_f64 %[f2], %[w], %[w], %[f2]\n v_fma_f64 %[f3], %[w], %[w], %[f3]\n"
                       "v_fma_f64 %[f0], %[w], %[w], %[f0]\n v_fma_f64 %[f1], %[w], %[w], %[f1]\n"
                       "v_fma_f64 %[f2], %[w], %[w], %[f2]\n v_fma_f64 %[f3], %[w], %[w], %[f3]\n"
                       "v_mfma_f64_16x16x4_f64 %[a1], %[w], %[x], %[a1]\n"
                       "v_mfma_f64_16x16x4_f64 %[a2], %[w], %[x], %[a2]\n"
                       "v_mfma_f64_16x16x4_f64 %[a3], %[w], %[x], %[a3]\n"
                       "v_mfma_f64_16x16x4_f64 %[a4], %[w], %[x], %[a4]\n"
                       "v_mfma_f64_16x16x4_f64 %[a5], %[w], %[x], %[a5]\n"
                       "v_mfma_f64_16x16x4_f64 %[a6], %[w], %[x], %[a6]\n"
                       "v_mfma_f64_16x16x4_f64 %[a7], %[w], %[x], %[a7]\n")
                   : [a0] "+v"(acc[0]), [a1] "+v"(acc[1]), [a2] "+v"(acc[2]), [a3] "+v"(acc[3]), [a4] "+v"(acc[4]),
                     [a5] "+v"(acc[5]), [a6] "+v"(acc[6]), [a7] "+v"(acc[7]), [f0] "+v"(f0), [f1] "+v"(f1),
                     [f2] "+v"(f2), [f3] "+v"(f3)
                   : [w] "v"(w), [x] "v"(v[32]));
      v[33] = f0 + f1 + f2 + f3;
    }
  } else if constexpr (OP == NOP1) {
    asm volatile(R16("s_nop 1\n s_nop 1\n s_nop 1\n s_nop 1\n s_nop 1\n s_nop 1\n s_nop 1\n s_nop 1\n") ::);
  }
}

// instructions per body() call
constexpr int per_call(int op) {
  return op == MFMA_ASM4 ? 64 : op == MFMA_ASM8 ? 128 : op == MFMA_PAD ? 128 : op == MFMA_PAD_FMA ? 128 : op == MFMA || op == MFMA1 || op == MFMA2 || op == MFMA8 ? 16 : op == FMA_DEP || op == FMACDPP_DEP || op == RCP_DEP || op == BPERM_DEP ? 16
       : op == RLANE_IND || op == CND_IND ? 64 : 128;
}

template <int OA, int OB>
__global__ __launch_bounds__(512) void k_pair(double seed, double* sink, long long* cyc) {
  const int wave = threadIdx.x >> 6;
  double v[40];
  for (int j = 0; j < 40; ++j) v[j] = seed + j * 1e-3 + threadIdx.x * 1e-6;
  const double w = 0.999 + threadIdx.x * 1e-9;
  __syncthreads();
  const long long t0 = (long long)__builtin_amdgcn_s_memtime();
  if (wave < 4) {
    for (int i = 0; i < ITERS; ++i) body<OA>(v, w);
  } else {
    for (int i = 0; i < ITERS; ++i) body<OB>(v, w);
  }
  const long long t1 = (long long)__builtin_amdgcn_s_memtime();
  double s = 0;
  for (int j = 0; j < 40; ++j) s += v[j];
  sink[blockIdx.x * 512 + threadIdx.x] = s;
  if ((threadIdx.x & 63) == 0) cyc[blockIdx.x * 8 + wave] = t1 - t0;
}

static double med(std::vector<long long> v) {
  std::sort(v.begin(), v.end());
  return (double)v[v.size() / 2];
}

template <int OA, int OB>
static void run(double* sink, long long* cyc) {
  auto kern = k_pair<OA, OB>;
  for (int rep = 0; rep < 2; ++rep) {
    hipLaunchKernelGGL(kern, dim3(256), dim3(512), 0, 0, 1.0, sink, cyc);
    (void)hipDeviceSynchronize();
  }
  std::vector<long long> h(256 * 8);
  (void)hipMemcpy(h.data(), cyc, h.size() * sizeof(long long), hipMemcpyDeviceToHost);
  std::vector<long long> a, b;
  for (int i = 0; i < 256; ++i)
    for (int w = 0; w < 8; ++w) (w < 4 ? a : b).push_back(h[i * 8 + w]);
  const double ca = OA == NONE ? 0 : med(a) / (ITERS * (double)per_call(OA));
  const double cb = OB == NONE ? 0 : med(b) / (ITERS * (double)per_call(OB));
  printf("A %-28s %7.2f cyc/instr | B %-28s %7.2f cyc/instr\n", NAMES[OA], ca, NAMES[OB], cb);
}

int main() {
  double* sink;
  long long* cyc;
  (void)hipMalloc(&sink, 256 * 512 * sizeof(double));
  (void)hipMalloc(&cyc, 256 * 8 * sizeof(long long));
  run<MFMA_ASM4, NONE>(sink, cyc);
  run<MFMA_ASM8, NONE>(sink, cyc);
  run<MFMA_ASM4, MFMA_ASM4>(sink, cyc);
  run<MFMA_ASM8, MFMA_ASM8>(sink, cyc);
  run<MFMA_ASM8, FMA_IND>(sink, cyc);
  run<MFMA_ASM8, FMA_DEP>(sink, cyc);
  run<MFMA_ASM8, FMACDPP_IND>(sink, cyc);
  run<MFMA_ASM8, BPERM_DEP>(sink, cyc);
  run<MFMA_ASM8, RCP_DEP>(sink, cyc);
  // round 3: which non-fp64 classes co-issue beside a partner's f64 MFMA stream
  run<NONE, CND_IND>(sink, cyc);
  run<MFMA_ASM8, CND_IND>(sink, cyc);
  run<NONE, RLANE_IND>(sink, cyc);
  run<MFMA_ASM8, RLANE_IND>(sink, cyc);
  run<NONE, IADD_IND>(sink, cyc);
  run<MFMA_ASM8, IADD_IND>(sink, cyc);
  run<NONE, MOVB32_IND>(sink, cyc);
  run<MFMA_ASM8, MOVB32_IND>(sink, cyc);
  run<NONE, SALU_IND>(sink, cyc);
  run<MFMA_ASM8, SALU_IND>(sink, cyc);
  run<NONE, BPERM_IND>(sink, cyc);
  run<MFMA_ASM8, BPERM_IND>(sink, cyc);
  run<MFMA_ASM8, MUL_IND>(sink, cyc);
  run<MFMA_ASM8, RCP_IND>(sink, cyc);
  run<MFMA_ASM8, MOVDPP_IND>(sink, cyc);
  // round 3: an MFMA stream that presents no instruction while the pipe is
  // busy (s_nop padding): does the partner then issue, and does its f64 VALU
  // run beside the matrix core?
  run<MFMA_PAD, NONE>(sink, cyc);
  run<MFMA_PAD, FMA_IND>(sink, cyc);
  run<MFMA_PAD, IADD_IND>(sink, cyc);
  run<MFMA_PAD, CND_IND>(sink, cyc);
  run<MFMA_PAD, RLANE_IND>(sink, cyc);
  run<MFMA_PAD, FMACDPP_IND>(sink, cyc);
  run<MFMA_PAD_FMA, NONE>(sink, cyc);
  run<MFMA1, NONE>(sink, cyc);
  run<MFMA2, NONE>(sink, cyc);
  run<MFMA, NONE>(sink, cyc);
  run<MFMA8, NONE>(sink, cyc);
  run<MFMA1, MFMA1>(sink, cyc);
  run<MFMA, MFMA>(sink, cyc);
  run<MFMA8, MFMA8>(sink, cyc);
  run<MFMA, FMA_IND>(sink, cyc);
  run<MFMA8, FMA_IND>(sink, cyc);
  run<MFMA1, FMA_IND>(sink, cyc);
  run<MFMA, FMA_DEP>(sink, cyc);
  run<MFMA8, FMA_DEP>(sink, cyc);
  run<MFMA8, FMACDPP_IND>(sink, cyc);
  run<MFMA8, RLANE_IND>(sink, cyc);
  run<MFMA8, BPERM_DEP>(sink, cyc);
  run<MFMA8, NOP1>(sink, cyc);
  printf("ISSUE_PROBE_DONE\n");
  return 0;
}
