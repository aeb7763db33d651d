// chol_lat.hip — latency form of the fixed-white-noise factorisation for small
// batches (one sampler proposal: PTMCMC / bilby call get_lnlikelihood with a
// single theta, /root/reference/examples/run_example_paramfile.py:27-30,
// /root/reference/enterprise_warp/bilby_warp.py:35).
//
// chol_mfma_kernel gives each (pulsar, sample) unit one wave: at B = 1 the 45
// units of C3 occupy 45 of 1024 SIMDs and each is a ~20 us chain of 472 MFMAs
// and 121 dependent pivots on ONE SIMD.  Here each unit gets a 4-wave
// workgroup (one CU, four SIMDs).  The 16x16 upper blocks (i, j) are dealt to
// the waves by LAT_MAP (below), which keeps the owner of each panel's next
// diagonal block lightly loaded; the owner of a diagonal block factors it (diag_factor_2l, the same
// two-level panel as the batched kernel) and publishes E = L^-T and the row
// scales through LDS; every wave applies them to its blocks of the block row
// (row_v_2l), publishes those U blocks, and takes its trailing updates
// A_ij -= U_bi^T U_bj (syrk_update).  The owner of the next diagonal block
// updates and factors it first (lookahead), so the pivot chain of panel bb+1
// overlaps the other waves' trailing work of panel bb.
//
// Every block sees the same operations in the same order as in
// chol_mfma_kernel (phi^-1 added at load, updates in panel order, the same
// panel code), so the factor, the pivots and q are bit-identical; only the
// log-determinant sum is associated differently (per wave, then across the
// four waves): strict-equal to the batched kernel, not bit-identical.
//
// Sampler I/O is fused in: theta is read straight from the handle's pinned
// (host-mapped) staging and every unit writes its term to pinned host memory
// as well; the host folds the P terms of a sample in pulsar order (the left
// fold of reduce_units_kernel).  One launch per call: no H2D / memset /
// reduction / D2H operations, and no cross-workgroup atomics (a fold by the
// last workgroup cost ~4k cycles of agent-scope fences and atomics).
#include "ewarp_dev.h"

// the diagonal chains' row replication (diag_factor_2l REPL): 2 = by the
// lane swaps of bcast_rows4 (round 6, bit-identical; three interleaved
// rounds, scripts/lat_lib_ab.sh, profiles/r06l/latency_ab.log: B = 1 / 8 /
// 24 30.85 / 37.32 / 79.96 -> 30.35 / 36.89 / 78.40 us per call), 1 = by
// ds_bpermute (until round 5)
#ifndef EWH_LAT_REPL
#define EWH_LAT_REPL 2
#endif

namespace ewh_dev {
namespace {

// Block (i, j) -> wave.  LAT_MAP (the default): per-NB maps annealed by
// scripts/lat_owner_search.py against the panel-time model fitted to the
// round-3 stamps (profiles/r03f/lat_stamps_b1.log): the owner of the next
// diagonal block -- which runs that block's pivot chain (lookahead) before
// its trailing updates -- gets a light share of the trailing blocks, so the
// chain, not that wave's MFMA queue, sets the panel time (model for NB = 8:
// 40.4 k -> 34.2 k cycles over the seven panels).  LAT_VAR_R3 (dev A/B):
// the round-3 map (i + j) mod 4 and prologue.
constexpr unsigned char LAT_MAP[9][8][8] = {{},
  {{0,0,0,0,0,0,0,0}, {0,0,0,0,0,0,0,0}, {0,0,0,0,0,0,0,0}, {0,0,0,0,0,0,0,0}, {0,0,0,0,0,0,0,0}, {0,0,0,0,0,0,0,0}, {0,0,0,0,0,0,0,0}, {0,0,0,0,0,0,0,0}},
  {{0,0,0,0,0,0,0,0}, {0,2,0,0,0,0,0,0}, {0,0,0,0,0,0,0,0}, {0,0,0,0,0,0,0,0}, {0,0,0,0,0,0,0,0}, {0,0,0,0,0,0,0,0}, {0,0,0,0,0,0,0,0}, {0,0,0,0,0,0,0,0}},
  {{2,2,3,0,0,0,0,0}, {0,0,1,0,0,0,0,0}, {0,0,1,0,0,0,0,0}, {0,0,0,0,0,0,0,0}, {0,0,0,0,0,0,0,0}, {0,0,0,0,0,0,0,0}, {0,0,0,0,0,0,0,0}, {0,0,0,0,0,0,0,0}},
  {{0,0,3,1,0,0,0,0}, {0,0,2,3,0,0,0,0}, {0,0,3,2,0,0,0,0}, {0,0,0,1,0,0,0,0}, {0,0,0,0,0,0,0,0}, {0,0,0,0,0,0,0,0}, {0,0,0,0,0,0,0,0}, {0,0,0,0,0,0,0,0}},
  {{1,2,3,0,1,0,0,0}, {0,2,3,1,0,0,0,0}, {0,0,1,0,3,0,0,0}, {0,0,0,3,0,0,0,0}, {0,0,0,0,0,0,0,0}, {0,0,0,0,0,0,0,0}, {0,0,0,0,0,0,0,0}, {0,0,0,0,0,0,0,0}},
  {{0,0,0,1,3,1,0,0}, {0,1,3,2,2,3,0,0}, {0,0,1,2,0,3,0,0}, {0,0,0,0,2,3,0,0}, {0,0,0,0,2,3,0,0}, {0,0,0,0,0,3,0,0}, {0,0,0,0,0,0,0,0}, {0,0,0,0,0,0,0,0}},
  {{1,1,3,1,2,0,3,0}, {0,1,0,2,3,0,2,0}, {0,0,1,3,0,2,0,0}, {0,0,0,1,0,3,2,0}, {0,0,0,0,3,2,0,0}, {0,0,0,0,0,0,2,0}, {0,0,0,0,0,0,2,0}, {0,0,0,0,0,0,0,0}},
  {{2,3,1,1,0,2,0,3}, {0,1,0,2,2,0,3,3}, {0,0,1,2,3,0,0,2}, {0,0,0,1,3,3,0,0}, {0,0,0,0,1,2,0,3}, {0,0,0,0,0,0,3,2}, {0,0,0,0,0,0,3,2}, {0,0,0,0,0,0,0,2}},
};
// Variants: LAT_VAR_FLOW (the default) -- LAT_MAP, theta at kernel entry, the
// panel loop as a dataflow over LDS counters (lat_flow); dev A/B only:
// LAT_VAR_BARRIER -- the same with two block barriers per panel;
// LAT_VAR_R3 -- the round-3 kernel ((i + j) mod 4, theta after the job record).
// LAT_VAR_STALL (dev test only): LAT_VAR_FLOW with every wait running out at
// once, so the stall path (LAT_STALL_BITS -> an error of ewh_lnl_batch) is
// exercised (tests/test_gpu_properties.py).
[[maybe_unused]] constexpr int LAT_VAR_FLOW = 0, LAT_VAR_BARRIER = 1, LAT_VAR_R3 = 2, LAT_VAR_STALL = 3;
constexpr bool lat_pre(int var) { return var != LAT_VAR_R3; }
constexpr bool lat_is_flow(int var) { return var == LAT_VAR_FLOW || var == LAT_VAR_STALL; }
template <int NB, int VAR>
constexpr int lat_owner(int i, int j) { return VAR == LAT_VAR_R3 ? (i + j) & 3 : LAT_MAP[NB][i][j]; }
// wave w owns a block (bb, j > bb) of block row bb
template <int NB, int VAR>
constexpr bool lat_row_owned(int w, int bb) {
  for (int j = bb + 1; j < NB; ++j)
    if (lat_owner<NB, VAR>(bb, j) == w) return true;
  return false;
}
// wave w owns a block (i, j >= i) of row i that panel bb updates after the lookahead block
template <int NB, int VAR>
constexpr bool lat_trail_owned(int w, int bb, int i) {
  for (int j = i; j < NB; ++j)
    if (lat_owner<NB, VAR>(i, j) == w && !(i == bb + 1 && j == bb + 1)) return true;
  return false;
}
template <int NB, int VAR>
constexpr bool lat_any_trail(int w, int bb) {
  for (int i = bb + 1; i < NB; ++i)
    if (lat_trail_owned<NB, VAR>(w, bb, i)) return true;
  return false;
}
// blocks (bb, j > bb) wave w owns
template <int NB, int VAR>
constexpr int lat_row_count(int w, int bb) {
  int n = 0;
  for (int j = bb + 1; j < NB; ++j) n += lat_owner<NB, VAR>(bb, j) == w;
  return n;
}

#ifdef EWH_DEV
// phase stamps (dev mode 22): s_memtime per wave of the first LAT_STAMP_WG
// workgroups -- 0 start, 1 theta staged, 2 phi^-1 ready, 3 + bb after the
// barrier publishing panel bb's E (bb < NB - 1), 10 factorisation done,
// 11 unit term combined
constexpr int LAT_STAMP_WG = 64, LAT_STAMP_N = 16;
__device__ long long g_lat_stamps[LAT_STAMP_WG * 4 * LAT_STAMP_N];
#define LAT_STAMP(I)                                                                        \
  if constexpr (STAMP) {                                                                    \
    if (lane == 0 && blockIdx.x < LAT_STAMP_WG)                                             \
      g_lat_stamps[(blockIdx.x * 4 + (threadIdx.x >> 6)) * LAT_STAMP_N + (I)] =             \
          (long long)__builtin_amdgcn_s_memtime();                                           \
  }
#else
#define LAT_STAMP(I)
#endif

constexpr int LAT_NBUF = 3;
template <int NB>
struct LatLds {
  double phinv[16 * NB];
  double phs[16 * NB];
  double ths[STAGE_THETA_MAX];
  double thr[STAGE_THETA_MAX];   // the whole theta row (prefetched prologue)
  double ldet[4];
  int ok[4];
  double qv;
  // panel k's E = L^-T of the diagonal block, its row scales D^-1/2 and the
  // U blocks (k, j) of the block row, in buffer k % LAT_NBUF (LAT_VAR_FLOW;
  // the barrier form uses buffer 0), and the LDS counters the dataflow
  // waits on instead of block barriers
  double Ef[LAT_NBUF][4][64];
  double Rf[LAT_NBUF][4][64];
  double Uf[LAT_NBUF][NB][4][64];
  int eflag[NB];            // 1: E and scales of panel k published
  int ucount[NB];           // U blocks of block row k published
  int unext[NB];            // 1: U block (k, k + 1) published (the lookahead's operand)
  int done[NB];             // waves through panel k
  int stall;                // a wait ran out (never expected): the unit term becomes LAT_STALL_BITS
};

// LAT_VAR_FLOW synchronisation through LDS counters: a wave publishes with
// one workgroup-scope release add by lane 0 (after the wave's own LDS
// writes), a consumer spins with acquire loads.  Every wait targets data
// produced earlier in some wave's program order (the panel dependency DAG),
// and is bounded: a wait that runs out marks the unit and goes on; the unit's
// term is then the NaN payload LAT_STALL_BITS (ewarp_dev.h), which the host
// turns into an error of ewh_lnl_batch (never a NaN lnL).
constexpr int LAT_SPIN_MAX = 1 << 22;
__device__ __forceinline__ void lat_signal(int* f, int add, int lane) {
  if (lane == 0) __hip_atomic_fetch_add(f, add, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
}
template <bool FORCE = false>
__device__ __forceinline__ void lat_wait(int* f, int target, int* stall) {
  for (int n = 0; __hip_atomic_load(f, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) < target; ++n) {
    if (FORCE || n >= LAT_SPIN_MAX) {
      *stall = 1;
      break;
    }
    // (no s_sleep: a wave spins on its own SIMD; sleeping 64 cycles per poll
    // measured 30.35 vs 30.14 us per B = 1 call, profiles/r03h/lat_ab26.log)
  }
}

__device__ __forceinline__ void lds_put(double (*dst)[64], const v4d& v, int lane) {
  static_for<0, 4>([&](auto R) { dst[decltype(R)::value][lane] = v[decltype(R)::value]; });
}
__device__ __forceinline__ v4d lds_get(const double (*src)[64], int lane) {
  v4d v;
  static_for<0, 4>([&](auto R) { v[decltype(R)::value] = src[decltype(R)::value][lane]; });
  return v;
}

// LAT_VAR_FLOW: the panel loop as a dataflow.  Per panel bb a wave (1) forms
// and publishes its U blocks of block row bb once E_bb is out (the owner of
// (bb, bb) has it in registers), (2) waits for the whole U row, (3) if it
// owns (bb+1, bb+1), updates and factors it and publishes E_{bb+1} at once,
// (4) takes its trailing updates and counts itself through the panel.  No
// block barrier: a wave with little trailing work runs ahead into the next
// panel's row V while others finish theirs.  Buffers rotate over LAT_NBUF
// panels; a writer of buffer k % LAT_NBUF first waits for every wave to be
// through panel k - LAT_NBUF (its last readers).  Same operations per block
// in the same order as the barrier form.
template <int NB, int W, bool STAMP, int VAR>
__device__ __forceinline__ void lat_flow(LatLds<NB>& S, v4d (&C)[NB][NB], v4d& E, double (&rsr)[4], int q, int c,
                                         int lane, LogAcc& ldet, bool& ok, int klast) {
  int* const stall = &S.stall;
  auto factor = [&](auto BBc) {
    constexpr int bb = decltype(BBc)::value;
    diag_factor_2l<NB, bb, true, EWH_LAT_REPL>(C[bb][bb], E, rsr, q, c, ldet, ok, klast);
    if constexpr (bb < NB - 1) {
      if constexpr (bb >= LAT_NBUF) lat_wait<VAR == LAT_VAR_STALL>(&S.done[bb - LAT_NBUF], 4, stall);
      lds_put(S.Ef[bb % LAT_NBUF], E, lane);
      static_for<0, 4>([&](auto R) { S.Rf[bb % LAT_NBUF][decltype(R)::value][lane] = rsr[decltype(R)::value]; });
      lat_signal(&S.eflag[bb], 1, lane);
    } else {
      const double qv = readlane_d(C[bb][bb][3], 63);
      if (lane == 0) S.qv = qv;
    }
  };
  if constexpr (lat_owner<NB, VAR>(0, 0) == W) factor(std::integral_constant<int, 0>{});
  static_for<0, NB - 1>([&](auto BBc) {
    constexpr int bb = decltype(BBc)::value;
    constexpr int buf = bb % LAT_NBUF;
    constexpr int nown = lat_row_count<NB, VAR>(W, bb);
    if constexpr (nown > 0) {
      if constexpr (lat_owner<NB, VAR>(bb, bb) != W) {
        lat_wait<VAR == LAT_VAR_STALL>(&S.eflag[bb], 1, stall);
        E = lds_get(S.Ef[buf], lane);
        static_for<0, 4>([&](auto R) { rsr[decltype(R)::value] = S.Rf[buf][decltype(R)::value][lane]; });
      }
      LAT_STAMP(3 + bb)
      if constexpr (bb >= LAT_NBUF) lat_wait<VAR == LAT_VAR_STALL>(&S.done[bb - LAT_NBUF], 4, stall);
      // block by block, (bb, bb + 1) first: the next diagonal block's owner
      // waits on that one alone
      static_for<bb + 1, NB>([&](auto JJ) {
        constexpr int j = decltype(JJ)::value;
        if constexpr (lat_owner<NB, VAR>(bb, j) == W) {
          row_v_2l(E, C[bb][j]);
          static_for<0, 4>([&](auto R) { C[bb][j][decltype(R)::value] *= rsr[decltype(R)::value]; });
          lds_put(S.Uf[buf][j], C[bb][j], lane);
          if constexpr (j == bb + 1) lat_signal(&S.unext[bb], 1, lane);
        }
      });
      lat_signal(&S.ucount[bb], nown, lane);
    }
    constexpr bool look = lat_owner<NB, VAR>(bb + 1, bb + 1) == W;
    constexpr bool trail = lat_any_trail<NB, VAR>(W, bb);
    constexpr bool own_next = lat_owner<NB, VAR>(bb, bb + 1) == W;
    auto ublk = [&](auto II) -> v4d {
      constexpr int i = decltype(II)::value;
      if constexpr (lat_owner<NB, VAR>(bb, i) == W) return C[bb][i];
      else return lds_get(S.Uf[buf][i], lane);
    };
    if constexpr (look) {
      if constexpr (!own_next) lat_wait<VAR == LAT_VAR_STALL>(&S.unext[bb], 1, stall);
      const v4d u = ublk(std::integral_constant<int, bb + 1>{});
      syrk_update(C[bb + 1][bb + 1], u, u);
      factor(std::integral_constant<int, bb + 1>{});
    }
    if constexpr (trail) lat_wait<VAR == LAT_VAR_STALL>(&S.ucount[bb], NB - 1 - bb, stall);
    static_for<bb + 1, NB>([&](auto II) {
      constexpr int i = decltype(II)::value;
      if constexpr (lat_trail_owned<NB, VAR>(W, bb, i)) {
        const v4d ui = ublk(II);
        static_for<i, NB>([&](auto JJ) {
          constexpr int j = decltype(JJ)::value;
          if constexpr (lat_owner<NB, VAR>(i, j) == W && !(i == bb + 1 && j == bb + 1)) {
            if constexpr (j == i) syrk_update(C[i][j], ui, ui);
            else syrk_update(C[i][j], ui, ublk(JJ));
          }
        });
      }
    });
    lat_signal(&S.done[bb], 1, lane);
  });
}

template <int NB, int W, bool STAMP, int VAR>
__device__ __forceinline__ void lat_wave(LatLds<NB>& S, const CholJob& J, const int* tidx, const double* __restrict__ A,
                                         const double* th, int ldth, const double (&tv)[2], int lane, LogAcc& ldet,
                                         bool& ok) {
  constexpr int LD = 16 * NB;
  const int tid = 64 * W + lane;
  const int q = lane >> 4, c = lane & 15;
  LAT_STAMP(0)
  // ---- prologue: phi^-1 of every column (the arithmetic of chol_mfma_kernel) ----
  // theta -> LDS: the entries the staged records reference (their indices
  // are positions in J.tidx), else the whole row when it fits
  const bool compact = J.urec != nullptr && J.ntidx > 0;
  const bool stage = compact || ldth <= STAGE_THETA_MAX;
  // owned blocks (their latency overlaps the prologue; issuing the theta load
  // ahead of them measured slower: its wait then covered every block load)
  v4d C[NB][NB];
  static_for<0, NB>([&](auto I) {
    constexpr int i = decltype(I)::value;
    static_for<i, NB>([&](auto JJ) {
      constexpr int j = decltype(JJ)::value;
      if constexpr (lat_owner<NB, VAR>(i, j) == W) {
        static_for<0, 4>([&](auto R) {
          constexpr int r = decltype(R)::value;
          C[i][j][r] = A[(long long)(16 * i + q + 4 * r) * LD + 16 * j + c];
        });
      }
    });
  });
  constexpr bool PRE = lat_pre(VAR);
  if constexpr (lat_is_flow(VAR)) {   // (visible to every wave after the prologue's barriers)
    if (tid < NB) {
      S.eflag[tid] = 0;
      S.ucount[tid] = 0;
      S.unext[tid] = 0;
      S.done[tid] = 0;
    }
    if (tid == 0) S.stall = 0;
  }
  static_assert(LD <= 256 && 2 * 256 >= STAGE_THETA_MAX, "one column / record per thread; theta row in two loads");
  if (PRE && J.urec != nullptr && ldth <= STAGE_THETA_MAX) {
    // the theta row arrived in tv (read at kernel entry); this thread's
    // spectrum record, its column's record index and its compact theta index
    // are loaded before the row is waited for, so their latency hides under
    // the PCIe round trip instead of following it
    const bool hasr = tid < J.nu;
    URec R;
    if (hasr) R = J.urec[tid];
    const int ur = tid < J.mreal ? J.urep[tid] : -1;
    const int ti = (compact && tid < J.ntidx) ? tidx[tid] : 0;
    // (S.ths holds what the records index: the compact entries, gathered from
    // the row in S.thr, or the row itself)
    double* row = compact ? S.thr : S.ths;
    if (tid < ldth) row[tid] = tv[0];
    if (tid + 256 < ldth) row[tid + 256] = tv[1];
    __syncthreads();
    if (compact) {
      if (tid < J.ntidx) S.ths[tid] = S.thr[ti];
      __syncthreads();
    }
    LAT_STAMP(1)
    const double* tp = S.ths;
    if (hasr) {
      double ph = 0.0;
      static_for<0, URec::NE>([&](auto E) {   // (constant indices: R stays in registers)
        if (decltype(E)::value < R.ne) ph += spec_phi_body(R.e[decltype(E)::value], tp);
      });
      S.phs[tid] = ph;
    }
    __syncthreads();
    if (tid < LD) {
      double pi = 0.0;
      if (ur >= 0) {
        const double ph = S.phs[ur];
        pi = 1.0 / ph;
        ldet.add(ph);
      }
      S.phinv[tid] = pi;
    }
  } else {
  if (stage) {
    if (compact) {
      if (tid < J.ntidx) S.ths[tid] = th[tidx[tid]];   // (tidx: the job in global memory)
    } else {
      for (int i = tid; i < ldth; i += 256) S.ths[i] = th[i];
    }
    __syncthreads();
  }
  LAT_STAMP(1)
  const double* tp = stage ? S.ths : th;
  if (J.urec != nullptr) {
    for (int u = tid; u < J.nu; u += 256) {
      const URec& R = J.urec[u];
      double ph = 0.0;
      for (int e = 0; e < R.ne; ++e) ph += spec_phi_body(R.e[e], tp);
      S.phs[u] = ph;
    }
    __syncthreads();
    for (int a = tid; a < LD; a += 256) {
      const int ur = a < J.mreal ? J.urep[a] : -1;
      double pi = 0.0;
      if (ur >= 0) {
        const double ph = S.phs[ur];
        pi = 1.0 / ph;
        ldet.add(ph);
      }
      S.phinv[a] = pi;
    }
  } else {
    const bool dedup = J.rep != nullptr;
    if (dedup) {
      for (int i = tid; i < J.nu; i += 256) {
        const int a = J.ulist[i];
        double ph = 0.0;
        for (int e = J.col_ptr[a]; e < J.col_ptr[a + 1]; ++e) ph += spec_phi_body(J.spec[e], tp);
        S.phs[a] = ph;
      }
    }
    __syncthreads();
    for (int a = tid; a < LD; a += 256) {
      double pi = 0.0;
      if (a < J.mreal && J.col_ptr[a] < J.col_ptr[a + 1]) {
        double ph = 0.0;
        if (dedup) {
          ph = S.phs[J.rep[a]];
        } else {
          for (int e = J.col_ptr[a]; e < J.col_ptr[a + 1]; ++e) ph += spec_phi_body(J.spec[e], tp);
        }
        pi = 1.0 / ph;
        ldet.add(ph);
      }
      S.phinv[a] = pi;
    }
  }
  }
  __syncthreads();
  LAT_STAMP(2)
  static_for<0, NB>([&](auto I) {
    constexpr int i = decltype(I)::value;
    if constexpr (lat_owner<NB, VAR>(i, i) == W) {
      const double pd = S.phinv[16 * i + c];
      static_for<0, 4>([&](auto R) {
        constexpr int r = decltype(R)::value;
        C[i][i][r] += (q + 4 * r == c) ? pd : 0.0;
      });
    }
  });
  const int klast = __builtin_amdgcn_readfirstlane(J.mreal - 16 * (NB - 1));
  v4d E;
  double rsr[4];
  // factor diagonal block BB (owner only); publish E and the scales, or q
  auto factor = [&](auto BBc) {
    constexpr int bb = decltype(BBc)::value;
    diag_factor_2l<NB, bb, true, EWH_LAT_REPL>(C[bb][bb], E, rsr, q, c, ldet, ok, klast);
    if constexpr (bb < NB - 1) {
      lds_put(S.Ef[0], E, lane);
      static_for<0, 4>([&](auto R) { S.Rf[0][decltype(R)::value][lane] = rsr[decltype(R)::value]; });
    } else {
      const double qv = readlane_d(C[bb][bb][3], 63);
      if (lane == 0) S.qv = qv;
    }
  };
  if constexpr (lat_is_flow(VAR)) {
    lat_flow<NB, W, STAMP, VAR>(S, C, E, rsr, q, c, lane, ldet, ok, klast);
    return;
  } else {
  if constexpr (lat_owner<NB, VAR>(0, 0) == W) factor(std::integral_constant<int, 0>{});
  static_for<0, NB - 1>([&](auto BBc) {
    constexpr int bb = decltype(BBc)::value;
    __syncthreads();                                       // E, scales of panel bb
    LAT_STAMP(3 + bb)
    constexpr bool row_owned = lat_row_owned<NB, VAR>(W, bb);
    if constexpr (row_owned) {
      if constexpr (lat_owner<NB, VAR>(bb, bb) != W) {
        E = lds_get(S.Ef[0], lane);
        static_for<0, 4>([&](auto R) { rsr[decltype(R)::value] = S.Rf[0][decltype(R)::value][lane]; });
      }
      static_for<bb + 1, NB>([&](auto JJ) {
        constexpr int j = decltype(JJ)::value;
        if constexpr (lat_owner<NB, VAR>(bb, j) == W) row_v_2l(E, C[bb][j]);
      });
      static_for<bb + 1, NB>([&](auto JJ) {
        constexpr int j = decltype(JJ)::value;
        if constexpr (lat_owner<NB, VAR>(bb, j) == W) {
          static_for<0, 4>([&](auto R) { C[bb][j][decltype(R)::value] *= rsr[decltype(R)::value]; });
          lds_put(S.Uf[0][j], C[bb][j], lane);
        }
      });
    }
    __syncthreads();                                       // U blocks of row bb
    auto ublk = [&](auto II) -> v4d {
      constexpr int i = decltype(II)::value;
      if constexpr (lat_owner<NB, VAR>(bb, i) == W) return C[bb][i];
      else return lds_get(S.Uf[0][i], lane);
    };
    // lookahead: the next diagonal block first, then its panel
    if constexpr (lat_owner<NB, VAR>(bb + 1, bb + 1) == W) {
      const v4d u = ublk(std::integral_constant<int, bb + 1>{});
      syrk_update(C[bb + 1][bb + 1], u, u);
      factor(std::integral_constant<int, bb + 1>{});
    }
    static_for<bb + 1, NB>([&](auto II) {
      constexpr int i = decltype(II)::value;
      constexpr bool any = lat_trail_owned<NB, VAR>(W, bb, i);
      if constexpr (any) {
        const v4d ui = ublk(II);
        static_for<i, NB>([&](auto JJ) {
          constexpr int j = decltype(JJ)::value;
          if constexpr (lat_owner<NB, VAR>(i, j) == W && !(i == bb + 1 && j == bb + 1)) {
            if constexpr (j == i) syrk_update(C[i][j], ui, ui);
            else syrk_update(C[i][j], ui, ublk(JJ));
          }
        });
      }
    });
  });
  }
  LAT_STAMP(10)
}

template <int NB, bool STAMP, int VAR>
__global__ __launch_bounds__(256) void chol_lat_kernel(const CholJob* __restrict__ jobs, int B, int P,
                                                       const double* theta, int ldth, double* __restrict__ out_units,
                                                       double* host_units) {
  __shared__ LatLds<NB> S;
  const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
  (void)P;
  const int u = blockIdx.x;
  const int p = u / B, b = u % B;
  // theta first: the whole row when it fits the LDS stage, read from pinned
  // host memory before the job record, so its PCIe round trip overlaps the
  // record and block loads (the round-3 prologue read the compact entries
  // after the record's index list had arrived: two latencies in series)
  double tv[2] = {0.0, 0.0};
  if constexpr (lat_pre(VAR)) {
    const double* t0 = theta + (long long)b * ldth;
    if (ldth <= STAGE_THETA_MAX) {
      if (tid < ldth) tv[0] = t0[tid];
      if (tid + 256 < ldth) tv[1] = t0[tid + 256];
    }
  }
  const CholJob J = jobs[p];
  const double* A = J.mats + (long long)b * J.mstride;
  const double* th = theta + (long long)b * ldth;
  LogAcc ldet;
  bool ok = true;
  switch (w) {
    case 0: lat_wave<NB, 0, STAMP, VAR>(S, J, jobs[p].tidx, A, th, ldth, tv, lane, ldet, ok); break;
    case 1: lat_wave<NB, 1, STAMP, VAR>(S, J, jobs[p].tidx, A, th, ldth, tv, lane, ldet, ok); break;
    case 2: lat_wave<NB, 2, STAMP, VAR>(S, J, jobs[p].tidx, A, th, ldth, tv, lane, ldet, ok); break;
    default: lat_wave<NB, 3, STAMP, VAR>(S, J, jobs[p].tidx, A, th, ldth, tv, lane, ldet, ok); break;
  }
  const double lw = wave_sum(ldet.value());
  const bool okw = __all(ok);
  if (lane == 0) {
    S.ldet[w] = lw;
    S.ok[w] = okw ? 1 : 0;
  }
  __syncthreads();
  LAT_STAMP(11)
  if (tid == 0) {
    double lnl = J.K[(long long)b * J.kstride] - 0.5 * S.qv - 0.5 * (((S.ldet[0] + S.ldet[1]) + S.ldet[2]) + S.ldet[3]);
    if (!(S.ok[0] && S.ok[1] && S.ok[2] && S.ok[3]) || J.fail) lnl = -INFINITY;
    if constexpr (lat_is_flow(VAR)) {
      if (S.stall) lnl = __builtin_bit_cast(double, LAT_STALL_BITS);
    }
    out_units[(long long)p * B + b] = lnl;
    // pinned: the host folds the P terms after the launch.  (A system-scope
    // store, written through at once, measured the same at B = 1 and slower at
    // B = 8: 29.50 / 37.5 vs 29.48 / 35.9 us, round 4.)
    host_units[(long long)p * B + b] = lnl;
  }
  LAT_STAMP(12)
}

template <bool STAMP, int VAR>
int launch_chol_lat_t(int nb, const CholJob* jobs, int B, int P, const double* theta, int ldth, double* units,
                      double* host_units, hipStream_t st) {
  const dim3 grid((unsigned)(P * B)), block(256);
#define EWH_LAT_CASE(N)                                                                                          \
  case N:                                                                                                        \
    hipLaunchKernelGGL(HIP_KERNEL_NAME(chol_lat_kernel<N, STAMP, VAR>), grid, block, 0, st, jobs, B, P, theta,  \
                       ldth, units, host_units);                                                                 \
    break;
  switch (nb) {
    EWH_LAT_CASE(1) EWH_LAT_CASE(2) EWH_LAT_CASE(3) EWH_LAT_CASE(4)
    EWH_LAT_CASE(5) EWH_LAT_CASE(6) EWH_LAT_CASE(7) EWH_LAT_CASE(8)
    default: return 1;
  }
#undef EWH_LAT_CASE
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? 0 : set_err(EWH_E_HIP, std::string("chol_lat_kernel: ") + hipGetErrorString(e));
}

}  // namespace

int launch_chol_lat(int nb, const CholJob* jobs, int B, int P, const double* theta, int ldth, double* units,
                    double* host_units, hipStream_t st, bool stamp, int var) {
#ifdef EWH_DEV
  if (stamp) return launch_chol_lat_t<true, LAT_VAR_FLOW>(nb, jobs, B, P, theta, ldth, units, host_units, st);
  if (var == LAT_VAR_BARRIER)
    return launch_chol_lat_t<false, LAT_VAR_BARRIER>(nb, jobs, B, P, theta, ldth, units, host_units, st);
  if (var == LAT_VAR_R3) return launch_chol_lat_t<false, LAT_VAR_R3>(nb, jobs, B, P, theta, ldth, units, host_units, st);
  if (var == LAT_VAR_STALL)
    return launch_chol_lat_t<false, LAT_VAR_STALL>(nb, jobs, B, P, theta, ldth, units, host_units, st);
#endif
  (void)stamp;
  (void)var;
  return launch_chol_lat_t<false, LAT_VAR_FLOW>(nb, jobs, B, P, theta, ldth, units, host_units, st);
}

#ifdef EWH_DEV
extern "C" int ewh_dev_lat_stamps(long long* out, long long n) {
  if (n > (long long)LAT_STAMP_WG * 4 * LAT_STAMP_N) n = (long long)LAT_STAMP_WG * 4 * LAT_STAMP_N;
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_lat_stamps), (size_t)n * sizeof(long long)) == hipSuccess ? 0 : -1;
}
#endif

}  // namespace ewh_dev
