// chol_wide.hip — the factorisation at any width: bases wider than the
// register kernels take (reduced width > 16 blocks = 255 columns, e.g.
// red_general_freqs / X_<n>_nfreqs models, enterprise_models.py:148-167,
// :436-468), and the partial factorisation of a correlated common process
// wider than chol_mfma_kernel<..., KEEP> takes (> 9 blocks).
//
// One wave per (pulsar, sample), left-looking over block rows (as
// chol_big_kernel), with NB a runtime value: block row i is processed in
// chunks of CW 16x16 blocks held in registers in the MFMA C/D layout; each
// chunk takes the updates A_ij -= U_pi^T U_pj of every finished row p < i
// (four f64 MFMAs per block, U streamed back from a per-workgroup scratch),
// then -- chunk 0 holds the diagonal block -- the two-level LDL^T panel of
// the batched kernels (diag_factor_2l; E = L^-T and the row scales are kept
// in registers for the row's later chunks), V = E^T A and U = D^-1/2 V
// (row_v_2l), and is written back to the scratch.  Per block the same
// operations in the same order as chol_big_kernel / chol_mfma_kernel.
//
// keep > 0: only block rows 0..NB-keep-1 are factored; the trailing keep x
// keep blocks (the common columns + r of a correlated process) take the
// updates of every factored row and are written to keep_out as a dense
// (16 keep)^2 square, pulsar-major -- the layout of chol_mfma_kernel<KEEP>.
#include "ewarp_dev.h"

namespace ewh_dev {
namespace {

constexpr int CW = 8;                // blocks of a block row per register chunk
typedef __attribute__((address_space(1))) v4d gv4d;

__device__ __forceinline__ long long wide_blk(int p, int j, int nb) {   // packed upper block index
  return (long long)p * nb - (long long)p * (p - 1) / 2 + (j - p);
}

// PAIR (round 5): block rows taken two at a time where both are factored --
// each streamed U_pj block is read once for rows i and i + 1 (the U traffic
// of the left-looking update, which bounds this kernel, halves), row i + 1
// takes its p = i update from row i's registers.  Per block the same MFMAs
// on the same operands in the same order as the one-row form (PAIR = false,
// dev mode 34): bit-identical.
template <bool PAIR>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(2, 2)))
void chol_wide_kernel(const CholJob* __restrict__ jobs, int B, long long u0, int b_off,
                      const double* __restrict__ theta, int ldth, double* __restrict__ out_units,
                      double* __restrict__ scratch, long long scr_per_wg, int keep, double* __restrict__ keep_out,
                      int keep_b0, int keep_bs, int rev_arg, double* __restrict__ units_rev) {
  __shared__ double phinv[WIDE_LD_MAX];
  const int lane = threadIdx.x, q = lane >> 4, c = lane & 15;
  // units_rev: the forward and reversed passes of the same units in one grid
  // (first half forward into out_units, second half reversed into units_rev),
  // so a batch of 1024 units fills 2048 SIMD slots instead of 1024
  long long idx = xcd_unit(blockIdx.x, gridDim.x);
  int rev = rev_arg;
  if (units_rev) {
    const long long half = gridDim.x >> 1;
    rev = idx >= half;
    if (rev) {
      idx -= half;
      out_units = units_rev;
    }
  }
  const long long u = u0 + idx;
  const int p = (int)(u / B), b = (int)(u % B);
  const CholJob J = jobs[p];
  const int LD = J.ld, NB = LD >> 4;
  const int nfact = NB - keep;
  // (debug build: the unit's packed U blocks fit its scratch slot, the
  // phi^-1 table its LDS array, the unit lies inside the batch)
  EWH_DCHECK(LD <= WIDE_LD_MAX && LD % 16 == 0 && keep >= 0 && keep < NB, "chol_wide: width within WIDE_LD_MAX");
  EWH_DCHECK([&] { long long sz = 0; for (int pp = 0; pp < nfact; ++pp) sz += NB - pp; return sz * 256; }() <=
                 scr_per_wg, "chol_wide: U blocks fit the scratch slot");
  EWH_DCHECK(b >= b_off && p >= 0, "chol_wide: unit inside the batch");
  // the reversed (verify) pass reads fl(hi + 2 lo) where the input is held
  // to double-double (S_lo / G_lo): the forward pass's input is X - lo, this
  // one's X + lo (to an ulp), so the two straddle the exact input and their
  // difference also shows how much the input's own rounding moves the lnL.
  // Round 5 (r05j): a shared matrix's fl(hi + 2 lo) is formed once
  // (mats_rev): the second load per element had cost the reversed pass 0.49
  // -> 0.80 ms at the system model's 4096 units -- the same value, read once
  const bool rv = rev && J.mats_rev;
  const gdptr A = (gdptr)((rv ? J.mats_rev : J.mats) + (long long)(b - b_off) * J.mstride);
  const gdptr Alo = (rev && !rv && J.mats_lo) ? (gdptr)(J.mats_lo + (long long)(b - b_off) * J.mstride) : nullptr;
  const double* th = theta + (long long)b * ldth;
  __attribute__((address_space(1))) double* scr =
      (__attribute__((address_space(1))) double*)(scratch + (long long)blockIdx.x * scr_per_wg + lane * 4);

  LogAcc lphi;
  for (int a = lane; a < LD; a += 64) {
    double pi = 0.0;
    if (a < J.mreal && J.col_ptr[a] < J.col_ptr[a + 1]) {   // (pads carry no entry)
      double ph = 0.0;
      for (int e = J.col_ptr[a]; e < J.col_ptr[a + 1]; ++e) ph += spec_phi_body(J.spec[e], th);
      pi = 1.0 / ph;
      lphi.add(ph);
    }
    phinv[a] = pi;
  }
  const double lphi_sum = wave_sum(lphi.value());
  __syncthreads();
  // rev (keep == 0 only): the same factorisation in the reversed column order
  // (r stays last) -- pi(a) = LD - 2 - a -- an independent fp64 ordering of
  // the same lnL, which the verify step compares with the forward one
  auto pi = [&](int a) { return (rev && a < LD - 1) ? LD - 2 - a : a; };

  LogAcc ldet;
  bool ok = true;
  double qv = 0.0;
  const int klast = rev ? 16 : __builtin_amdgcn_readfirstlane(J.mreal - 16 * (NB - 1));
  const int KD = 16 * keep;
  double* ko = keep > 0 ? keep_out + ((long long)p * keep_bs + (b - keep_b0)) * ((long long)KD * KD) : nullptr;
  // element (row, col) of block (i, j) held by this lane, register r: A + phi^-1 on the diagonal
  auto load_blk = [&](int i, int j, v4d& R) {
    static_for<0, 4>([&](auto RR) {
      constexpr int r = decltype(RR)::value;
      const long long o = (long long)pi(16 * i + q + 4 * r) * LD + pi(16 * j + c);
      R[r] = Alo ? A[o] + 2.0 * Alo[o] : A[o];
    });
    if (j == i) {
      const double pd = phinv[pi(16 * i + c)];
      static_for<0, 4>([&](auto RR) {
        constexpr int r = decltype(RR)::value;
        R[r] += (q + 4 * r == c) ? pd : 0.0;
      });
    }
  };
#pragma unroll 1
  for (int i = 0; i < NB; ++i) {
    if (PAIR && i + 1 < nfact) {
      // ---- block rows i and i1 = i + 1, both factored (i1 may hold the residual) ----
      const int i1 = i + 1;
      const bool lastr1 = keep == 0 && i1 == NB - 1;
      v4d E0 = {0.0, 0.0, 0.0, 0.0}, E1 = {0.0, 0.0, 0.0, 0.0}, U01 = {0.0, 0.0, 0.0, 0.0};
      double rs0[4] = {1.0, 1.0, 1.0, 1.0}, rs1[4] = {1.0, 1.0, 1.0, 1.0};
#pragma unroll 1
      for (int c0 = i; c0 < NB; c0 += CW) {
        v4d R0[CW], R1[CW];
        static_for<0, CW>([&](auto JJ) {
          constexpr int jj = decltype(JJ)::value;
          const int j = c0 + jj;
          R0[jj] = v4d{0.0, 0.0, 0.0, 0.0};
          R1[jj] = v4d{0.0, 0.0, 0.0, 0.0};
          if (j < NB) load_blk(i, j, R0[jj]);
          if (j >= i1 && j < NB) load_blk(i1, j, R1[jj]);
        });
#pragma unroll 1
        for (int pp = 0; pp < i; ++pp) {
          const v4d Ui = *(const gv4d*)(scr + wide_blk(pp, i, NB) * 256);
          const v4d Ui1 = *(const gv4d*)(scr + wide_blk(pp, i1, NB) * 256);
          static_for<0, CW>([&](auto JJ) {
            constexpr int jj = decltype(JJ)::value;
            const int j = c0 + jj;
            if (j < NB) {
              const v4d Uj = *(const gv4d*)(scr + wide_blk(pp, j, NB) * 256);
              syrk_update(R0[jj], Ui, Uj);
              if (j >= i1) syrk_update(R1[jj], Ui1, Uj);
            }
          });
        }
        // row i: its panel, U (i, j) to the scratch
        if (c0 == i) diag_factor_2l<2, 0, true>(R0[0], E0, rs0, q, c, ldet, ok, 16);
        static_for<0, CW>([&](auto JJ) {
          constexpr int jj = decltype(JJ)::value;
          const int j = c0 + jj;
          if (j > i && j < NB) {
            row_v_2l(E0, R0[jj]);
            static_for<0, 4>([&](auto RR) { R0[jj][decltype(RR)::value] *= rs0[decltype(RR)::value]; });
            *(gv4d*)(scr + wide_blk(i, j, NB) * 256) = R0[jj];
          }
        });
        if (c0 == i) U01 = R0[1];                              // U (i, i1): j = i1 < NB
        // row i1: the update by row i from registers, then its panel
        static_for<0, CW>([&](auto JJ) {
          constexpr int jj = decltype(JJ)::value;
          const int j = c0 + jj;
          if (j >= i1 && j < NB) syrk_update(R1[jj], U01, R0[jj]);
        });
        if (c0 == i) {
          if (lastr1) {
            diag_factor_2l<1, 0, true>(R1[1], E1, rs1, q, c, ldet, ok, klast);
            qv = readlane_d(R1[1][3], 63);
          } else {
            diag_factor_2l<2, 0, true>(R1[1], E1, rs1, q, c, ldet, ok, 16);
          }
        }
        if (!lastr1) {
          static_for<0, CW>([&](auto JJ) {
            constexpr int jj = decltype(JJ)::value;
            const int j = c0 + jj;
            if (j > i1 && j < NB) {
              row_v_2l(E1, R1[jj]);
              static_for<0, 4>([&](auto RR) { R1[jj][decltype(RR)::value] *= rs1[decltype(RR)::value]; });
              *(gv4d*)(scr + wide_blk(i1, j, NB) * 256) = R1[jj];
            }
          });
        }
      }
      ++i;                                                     // (i1 done)
      continue;
    }
    const bool fact = i < nfact;
    const bool lastr = keep == 0 && i == NB - 1;         // the block row holding the residual
    const int pmax = min(i, nfact);
    v4d E = {0.0, 0.0, 0.0, 0.0};
    double rsr[4] = {1.0, 1.0, 1.0, 1.0};
#pragma unroll 1
    for (int c0 = i; c0 < NB; c0 += CW) {
      v4d R[CW];
      static_for<0, CW>([&](auto JJ) {
        constexpr int jj = decltype(JJ)::value;
        const int j = c0 + jj;
        if (j < NB) {
          load_blk(i, j, R[jj]);
        } else {
          R[jj] = v4d{0.0, 0.0, 0.0, 0.0};
        }
      });
#pragma unroll 1
      for (int pp = 0; pp < pmax; ++pp) {
        const v4d Ui = *(const gv4d*)(scr + wide_blk(pp, i, NB) * 256);
        static_for<0, CW>([&](auto JJ) {
          constexpr int jj = decltype(JJ)::value;
          if (c0 + jj < NB) {
            const v4d Uj = *(const gv4d*)(scr + wide_blk(pp, c0 + jj, NB) * 256);
            syrk_update(R[jj], Ui, Uj);
          }
        });
      }
      if (fact) {
        if (c0 == i) {
          // (template arguments pick the panel form: <1, 0, true> is the
          // residual block row, <2, 0, true> an ordinary one)
          if (lastr) {
            diag_factor_2l<1, 0, true>(R[0], E, rsr, q, c, ldet, ok, klast);
            qv = readlane_d(R[0][3], 63);
          } else {
            diag_factor_2l<2, 0, true>(R[0], E, rsr, q, c, ldet, ok, 16);
          }
        }
        static_for<0, CW>([&](auto JJ) {
          constexpr int jj = decltype(JJ)::value;
          const int j = c0 + jj;
          if (j > i && j < NB) {
            row_v_2l(E, R[jj]);
            static_for<0, 4>([&](auto RR) { R[jj][decltype(RR)::value] *= rsr[decltype(RR)::value]; });
            *(gv4d*)(scr + wide_blk(i, j, NB) * 256) = R[jj];
          }
        });
      } else {
        // a kept block row: the updated blocks (i, j >= i) to the dense square
        static_for<0, CW>([&](auto JJ) {
          constexpr int jj = decltype(JJ)::value;
          const int j = c0 + jj;
          if (j < NB) {
            static_for<0, 4>([&](auto RR) {
              constexpr int r = decltype(RR)::value;
              const int row = 16 * (i - nfact) + q + 4 * r, col = 16 * (j - nfact) + c;
              if (i != j || row <= col) {
                ko[(long long)row * KD + col] = R[jj][r];
                ko[(long long)col * KD + row] = R[jj][r];
              }
            });
          }
        });
      }
    }
  }
  const double ldet_v = wave_sum(ldet.value());
  const bool ok_all = __all(ok);
  if (lane == 0) {
    double lnl = J.K[(long long)(b - b_off) * J.kstride] - 0.5 * qv - 0.5 * ldet_v - 0.5 * lphi_sum;
    if (!ok_all || J.fail) lnl = -INFINITY;
    out_units[(long long)p * B + b] = lnl;
  }
}

}  // namespace

long long wide_scratch_per_wg(int nb, int keep) {
  const int nf = nb - keep;
  long long n = 0;
  for (int p = 0; p < nf; ++p) n += nb - p;
  return n * 256;
}

int launch_chol_wide(const CholJob* jobs, int B, long long u0, long long n, int b_off, const double* theta, int ldth,
                     double* units, double* scr, long long scr_per_wg, long long cap, int keep, double* keep_out,
                     int keep_b0, int keep_bs, hipStream_t st, int rev, double* units_rev, bool pair) {
  // one scratch slot per workgroup of a launch; with units_rev two workgroups per unit
  const long long per = units_rev ? std::max<long long>(1, cap / 2) : cap;
  for (long long o = 0; o < n; o += per) {
    const long long m = std::min(per, n - o);
    const dim3 grid((unsigned)(units_rev ? 2 * m : m));
    if (pair)
      hipLaunchKernelGGL(HIP_KERNEL_NAME(chol_wide_kernel<true>), grid, dim3(64), 0, st, jobs, B, u0 + o, b_off, theta,
                         ldth, units, scr, scr_per_wg, keep, keep_out, keep_b0, keep_bs, rev, units_rev);
    else
      hipLaunchKernelGGL(HIP_KERNEL_NAME(chol_wide_kernel<false>), grid, dim3(64), 0, st, jobs, B, u0 + o, b_off, theta,
                         ldth, units, scr, scr_per_wg, keep, keep_out, keep_b0, keep_bs, rev, units_rev);
  }
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? 0 : set_err(EWH_E_HIP, std::string("chol_wide_kernel: ") + hipGetErrorString(e));
}

}  // namespace ewh_dev
