/*
 * ewarp_hip.h — C ABI of libewarp_hip.so, the MI355X (gfx950) PTA
 * log-likelihood engine behind enterprise_warp_amd.PTA.
 *
 * Drop-in boundary.  In the reference the likelihood is the object built by
 * `signal_base.PTA(models)` at enterprise_warp.py:502 and called as
 * `pta.get_lnlikelihood(params)` at bilby_warp.py:35 (and, through
 * enterprise_extensions' PTSampler, with an ndarray at
 * examples/run_example_paramfile.py:27-30).  The Python class
 * enterprise_warp_amd.pta.PTA keeps that surface and binds these entry
 * points with ctypes.
 *
 *   ewh_create          replaces signal_base.PTA.__init__ + the white-noise
 *                       cache of LogLikelihood (enterprise_warp.py:502-508):
 *                       uploads every pulsar's basis, residuals, TOA errors,
 *                       white-noise tables and spectral table to each listed
 *                       device; when white noise is fixed (Constant
 *                       efac/equad/ecorr set from noise files,
 *                       enterprise_warp.py:504-508) it also computes and
 *                       caches T^T N^-1 T, T^T N^-1 r, r^T N^-1 r, log|N| and
 *                       the timing-model elimination on each device.
 *   ewh_set_fixed_white replaces pta.set_default_params(noisedict)
 *                       (enterprise_warp.py:504-508) for new white-noise
 *                       constants: recomputes the cache in place.
 *   ewh_lnl_batch       replaces B calls of pta.get_lnlikelihood
 *                       (bilby_warp.py:35) — host theta in, host lnL out,
 *                       spread over every device of the handle.
 *   ewh_lnl_units_device  the same on device buffers for a contiguous range
 *                       of (pulsar, sample) units; used for multi-GPU
 *                       sharding (partial sums, then an RCCL all-reduce).
 *   ewh_destroy / ewh_last_error / ewh_version: lifecycle and errors.
 *
 * Conventions
 *  - theta is row-major [B x n_param] float64, column order = the caller's
 *    parameter order (enterprise_warp_amd.PTA.param_names).
 *  - A parameter reference (ewh_pref) is either a column of theta (idx >= 0)
 *    or a constant (idx < 0, value cval).
 *  - Ownership: the caller owns every host buffer for the duration of the
 *    call; the library copies what it needs and keeps no caller pointer.
 *    The library owns every device buffer it allocates (freed in destroy).
 *  - Errors: 0 on success, negative EWH_E* code otherwise; the message is in
 *    the thread-local ewh_last_error().  A failed Cholesky for a sample is
 *    NOT an error: its lnL is -INFINITY (enterprise: LinAlgError -> -np.inf).
 *  - Threads: one handle per host thread (no internal locking).  The HIP
 *    context is touched only inside ewh_create and later calls, never at
 *    library load, so forked sampler workers stay safe.
 */
#ifndef EWARP_HIP_H
#define EWARP_HIP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define EWH_ABI_VERSION 7

enum ewh_status {
  EWH_OK = 0,
  EWH_E_INVALID = -1,   /* bad descriptor / argument */
  EWH_E_HIP = -2,       /* HIP runtime error */
  EWH_E_NOMEM = -3,     /* device allocation failed */
  EWH_E_UNSUPPORTED = -4
};

/* Spectral-entry kinds: phi contribution of one basis column.
 *  POWERLAW  [ent] utils.powerlaw      p0 = log10_A, p1 = gamma           (enterprise_models.py:180)
 *  TURNOVER  powerlaw_bpl              p0 = log10_A, p1 = gamma, p2 = fc  (enterprise_models.py:553-563)
 *  FREESPEC  [ent] free_spectrum       p0 = log10_rho[j]                  (enterprise_models.py:388)
 *  CONST     phi = p0.cval (timing model: 1e40, [ent] utils.tm_prior)
 * Entries of merged columns ([ent] SignalCollection._combine_basis_columns)
 * are summed, as enterprise's KernelMatrix.add does. */
enum ewh_spec_kind {
  EWH_SPEC_POWERLAW = 1,
  EWH_SPEC_TURNOVER = 2,
  EWH_SPEC_FREESPEC = 3,
  EWH_SPEC_CONST = 4
};

typedef struct ewh_pref {
  int32_t idx;   /* >= 0: theta column; < 0: constant */
  int32_t pad_;
  double cval;
} ewh_pref;

typedef struct ewh_spec_entry {
  int32_t kind;  /* ewh_spec_kind */
  int32_t col;   /* basis column 0..n_col-1 */
  ewh_pref p0, p1, p2;
  double f;      /* Fourier frequency (1/s) */
  double df;     /* np.diff(concatenate([0], f[::2])) entry, as [ent] powerlaw */
  double fyr;    /* 1 / Julian year (s^-1), [ent] constants.fyr */
} ewh_spec_entry;

/* One pulsar's data and model tables.  TOAs are sorted; ECORR epochs are
 * contiguous TOA slices ([ent] utils.quant2ind). */
typedef struct ewh_pulsar_desc {
  int32_t n_toa;
  int32_t n_col;          /* basis columns after merging */
  int32_t n_lead_const;   /* leading columns whose phi is constant (timing model) */
  int32_t n_spec;
  const double* basis;    /* n_toa x n_col, row-major */
  const double* resid;    /* n_toa, seconds */
  const double* toaerr;   /* n_toa, seconds */
  /* white noise: N_t = efac^2 sigma_t^2 + 10^(2 log10_tnequad) (+ ECORR blocks) */
  int32_t n_slot;         /* size of the white-noise parameter table */
  const ewh_pref* slots;  /* n_slot */
  const int32_t* efac_slot;   /* n_toa: slot of efac (MeasurementNoise) */
  const int32_t* equad_slot;  /* n_toa: slot of log10_tnequad, -1 = none */
  int32_t n_epoch;
  const int32_t* epoch_start; /* n_epoch, first TOA of the epoch */
  const int32_t* epoch_stop;  /* n_epoch, one past the last TOA */
  const int32_t* epoch_slot;  /* n_epoch: slot of log10_ecorr */
  const ewh_spec_entry* spec; /* n_spec */
  /* theta-dependent basis columns ([ent] BasisGP with basis parameters:
   * chromred 'vary', enterprise_models.py:242-252): column j of group g =
   * col_bgroup[j] >= 0 is used as basis[t][j] * exp(idx_g * ln_chrom[t]),
   * idx_g = bgroup_idx[g], i.e. F * (1400 / nu)^idx.  A pulsar with groups
   * is always evaluated on the varying path (no T^T N^-1 T cache). */
  int32_t n_bgroup;
  const ewh_pref* bgroup_idx;   /* n_bgroup */
  const int32_t* col_bgroup;    /* n_col (-1: fixed column); NULL if n_bgroup == 0 */
  const double* ln_chrom;       /* n_toa: ln(1400 MHz / nu_t); NULL if n_bgroup == 0 */
  /* correlated common process (ewh_pta_desc.common != NULL): the LAST
   * n_common basis columns are the common signal's columns, in the common
   * order g = 0..n_common-1 (after the leading constant-phi columns and the
   * pulsar's other columns).  Their spec entries here are the pulsar's own
   * signals merged onto them (e.g. red noise); the common signal's own phi is
   * in ewh_common_desc. 0 when uncorrelated. */
  int32_t n_common;
} ewh_pulsar_desc;

/* A spatially correlated common process ([ent] FourierBasisCommonGP with an
 * ORF: enterprise_models.py:390-415): Phi couples column g of pulsar a with
 * column g of pulsar b by orf[a][b] * phi_common(g); the pulsars' own
 * signals add to the diagonal.  Requires fixed white noise (this ABI
 * version). */
enum ewh_common_kind {
  EWH_COMMON_CORRELATED = 0,    /* correlated common process in the likelihood */
  EWH_COMMON_OPTSTAT = 1        /* optimal statistic of an uncorrelated (CURN) model, see ewh_optstat */
};

typedef struct ewh_common_desc {
  int32_t n_col;                /* common columns per pulsar (2 x frequencies), <= 31 */
  const double* orf;            /* n_pulsar x n_pulsar, row-major: Gamma_ab (diagonal included) */
  const ewh_spec_entry* spec;   /* CORRELATED: n_col entries, spec[g].col = g: phi_common of column g.
                                 * OPTSTAT: unused (the common signal's entries are part of each
                                 * pulsar's own spec list, as in the CURN likelihood) */
  int32_t kind;                 /* ewh_common_kind */
} ewh_common_desc;

typedef struct ewh_pta_desc {
  int32_t abi_version;    /* EWH_ABI_VERSION */
  int32_t n_pulsar;
  int32_t n_param;        /* theta row length */
  int32_t white_fixed;    /* 1: no white-noise slot references theta -> cache TNT */
  const ewh_pulsar_desc* pulsars;
  const ewh_common_desc* common;   /* NULL: uncorrelated / CURN (per-pulsar Sigma) */
} ewh_pta_desc;

typedef struct ewh_handle ewh_handle;

/* Build the device-resident PTA on the HIP devices device_ids[0..ndev-1]
 * (NULL / 0: device 0).  Each device holds a full replica (bases, tables,
 * fixed-WN cache) and its own stream; a device id may repeat (two contexts
 * on one device: the split is then exercised on a one-GPU host). */
int ewh_create(const ewh_pta_desc* desc, const int32_t* device_ids, int32_t ndev, ewh_handle** out);

/* Number of device contexts of the handle. */
int ewh_num_devices(const ewh_handle* h);

/* New constant white-noise values (the in-place form of the reference's
 * pta.set_default_params(noisedict), enterprise_warp.py:504-508).
 * values: for each pulsar in descriptor order, its n_slot entries in slot
 * order; the value of every constant slot (idx < 0) is replaced, theta-
 * referencing slots ignore theirs.  A fixed-white-noise handle recomputes
 * T^T N^-1 T, d, r^T N^-1 r, log|N| and the timing-model elimination on
 * every device; bases and layout are unchanged. Synchronous. */
int ewh_set_fixed_white(ewh_handle* h, const double* values);

/* lnL for B samples: theta_host [B x n_param], out_host [B]. Synchronous.
 * Several devices: uncorrelated / CURN models split the (pulsar, sample)
 * units into cost-balanced contiguous ranges (one per device); each device
 * receives only the theta entries its range reads and sums its range over
 * its pulsars (pulsar order) into a B-vector, the
 * B-vectors are peer-copied to the first device and added there in device
 * order, and only B doubles return to the host (equal to one device at the
 * strict bound, not bit for bit: the fold is re-associated).  A correlated
 * common process splits the samples.  theta is staged through pinned host
 * memory owned by the handle. */
int ewh_lnl_batch(ewh_handle* h, const double* theta_host, int32_t B, double* out_host);

/* Device variant (the handle's first device) on a contiguous range [unit_begin, unit_end) of units
 * u = pulsar * B + sample.  With a correlated common process the range must
 * be the whole batch [0, n_pulsar * B) (shard samples across devices by
 * passing each one its own theta rows instead).  out_dev[b] = sum of the unit lnL terms of sample
 * b inside the range (0 where the range has none).  Asynchronous on `stream`
 * (a hipStream_t; NULL = the default stream).  theta_dev and out_dev are
 * device pointers. */
int ewh_lnl_units_device(ewh_handle* h, const double* theta_dev, int32_t B,
                         int64_t unit_begin, int64_t unit_end, double* out_dev,
                         void* stream);

/* Measurement entry (bench.py): the white-noise stage of a varying-white-
 * noise batch alone -- per pulsar and sample N^-1, the ECORR terms and the
 * fp64 MFMA contraction G = T^T N^-1 T (with d, r^T N^-1 r) into the
 * handle's scratch, no factorisation -- for B samples on the handle's first
 * device, asynchronous on `stream`.  EWH_E_UNSUPPORTED for fixed white noise
 * or a correlated process. */
int ewh_contract_device(ewh_handle* h, const double* theta_dev, int32_t B, void* stream);

/* Correlated common process, pulsar-partitioned (the exchange step of
 * one proposal spread over several GPUs, one process per
 * GPU).  kd = ewh_keep_dim(h) (0 for other handles): the kept common block
 * of one (pulsar, sample) is kd x kd doubles.
 *   ewh_corr_partial_device: partial factorisations of pulsars
 *     [p_begin, p_end) for samples [0, B): local terms to
 *     local_dev[p * B + b], kept blocks to keep_dev[(p * B + b) * kd * kd]
 *     (pulsar-major: a rank's pulsar range is one contiguous slice of both
 *     arrays; other rows are not written).
 *   -- all-gather keep_dev / local_dev over the ranks (RCCL) --
 *   ewh_corr_finish_device: with every pulsar's rows present, M_g^-1, the
 *     dense Sigma_c and its factorisation; out_dev[b] = lnL.
 * Device pointers on the handle's first device; asynchronous on `stream`.
 * ewh_lnl_batch uses the same split across the handle's devices (peer
 * copies instead of RCCL) when B is smaller than the device count. */
int ewh_keep_dim(const ewh_handle* h);
int ewh_corr_partial_device(ewh_handle* h, const double* theta_dev, int32_t B, int32_t p_begin, int32_t p_end,
                            double* keep_dev, double* local_dev, void* stream);
int ewh_corr_finish_device(ewh_handle* h, const double* theta_dev, int32_t B, const double* keep_dev,
                           const double* local_dev, double* out_dev, void* stream);

/* Optimal statistic (first device of the handle; the reference's results.py:653-795 ->
 * enterprise_extensions OptimalStatistic.compute_os) for B noise-parameter
 * draws, on a handle created with common->kind == EWH_COMMON_OPTSTAT (fixed
 * white noise): per pulsar X = F^T P^-1 r, Z = F^T P^-1 F (F = the common
 * columns, P = N + T phi T^T with the common process included), per pair
 * rho_ab = X_a^T phihat X_b / tr(Z_a phihat Z_b phihat), sig_ab = tr(..)^-1/2,
 * OS = sum rho Gamma / sig^2 / sum Gamma^2 / sig^2, OS_sig = (sum Gamma^2/sig^2)^-1/2.
 * theta_host [B x n_param]; phihat_host [B x n_col] (unit-amplitude spectrum
 * per draw); rho_host / sig_host [B x n_pulsar x n_pulsar] (pairs a < b
 * filled; may be NULL); os_host, os_sig_host [B]. Synchronous. */
int ewh_optstat(ewh_handle* h, const double* theta_host, int32_t B, const double* phihat_host,
                double* rho_host, double* sig_host, double* os_host, double* os_sig_host);

/* Per-pulsar lnL terms of the last call: out_host [n_pulsar x B] (row p =
 * pulsar p).  Units outside the last range read 0. Synchronous. */
int ewh_last_unit_terms(ewh_handle* h, double* out_host, int32_t B);

/* Cost model used for sharding: relative cost of one unit of pulsar p. */
double ewh_unit_cost(const ewh_handle* h, int32_t pulsar);

/* Transfers of the last ewh_lnl_batch: *h2d_bytes = theta bytes copied host
 * -> device over all contexts (each context receives only the theta entries
 * its units read: per column, the sample rows of its unit range); *peer =
 * bit i set when context i > 0 has peer access to the first context's device
 * (enabled in ewh_create where the devices allow it; the partial B-vectors
 * and gathered blocks then move device to device) -- context 0 and contexts
 * on the first device set their bit too.  Either pointer may be NULL.
 * Peer access is process-global: handles hold it by reference count, and
 * ewh_destroy of the last handle holding a direction disables it again (a
 * direction that was on before any handle enabled it is left on). */
int ewh_transfer_stats(const ewh_handle* h, int64_t* h2d_bytes, int64_t* peer);

/* The double-double route since the last query (bases past the register
 * kernels: fixed white noise past 9 blocks, any basis past 16; under kernel
 * mode 29 every fixed-white-noise unit): *checked = units that took it,
 * *refined = units chol_dd_kernel refactored (the verify step flagged them --
 * the forward and reversed fp64 factorisations disagree by more than
 * VERIFY_FRAC = 1/16 of strict, csrc/chol_dd.hip -- or kernel mode 29 sent
 * every unit).  Both are 64-bit counters kept on the device in stream order:
 * replays of a captured ewh_lnl_batch graph count, the capture itself does
 * not.  Synchronises every device of the handle (all streams, so work the
 * caller enqueued with ewh_lnl_units_device on its own stream is counted)
 * and resets both counts.  Either pointer may be NULL.  (Host twin: always
 * 0.)  ABI 7. */
int ewh_refine_stats(ewh_handle* h, int64_t* checked, int64_t* refined);

/* Kernel selection: 0 = auto (register-blocked MFMA factorisation with the
 * two-level LDL^T panel -- the 16x16 diagonal block in 4-row sub-panels by
 * VALU, each closed by one symmetric MFMA rank-4 update, the rest of the
 * block row by MFMA with L^-1 -- when the matrix fits registers; the LDS
 * kernel otherwise; batches of up to ewh_lat_b_max() = 24 samples on one
 * device take the latency kernel, one 4-wave workgroup per (pulsar, sample) with theta read
 * from pinned memory and the unit terms written to pinned memory, folded by
 * the host), 2 = the default without
 * that latency path (batched kernels at every batch size), 1 = force the
 * LDS kernel (unblocked Cholesky; for a
 * correlated common process also the round-1 dense LDS diagonal-block and
 * panel kernels), 27 = every factorisation (full and partial) by the fp64
 * any-width chol_wide_kernel (cross-check of the register, big and
 * double-double kernels), 29 = the double-double factorisation for every unit
 * of a basis past the register kernels (default: only where the forward and
 * reversed fp64 factorisations disagree) and every other uncorrelated unit
 * too -- fixed white noise on the double-double S, varying white noise on an
 * error-free double-double Gram -- the device-side double-double twin of the
 * batch (ABI 7).  In every mode but 1 / 27 an uncorrelated unit whose fp64
 * factorisation returns -inf is refactored in double-double (a -inf result
 * means the double-double factorisation failed too), 7 = default factorisation with the
 * round-1 kernels
 * elsewhere: the contraction (varying white noise: separate epoch-sum
 * kernel, unpipelined tiles) instead of the pipelined one and, for a
 * correlated common process, the right-looking dense update and the LDS
 * Gauss-Jordan M_g inverse.
 * Dev library only (`make dev`: libewarp_hip_dev.so): 15 / 16 = the
 * pipelined contraction with 4 / 8 waves per sample (default: 8 for 144+
 * columns, else 4), 17 = the round-2 one-level panel (NB = 8), 19 = the default with the spectra read through the CSR tables
 * instead of the staged records, 21 = the default with in-kernel phase
 * stamps (NB = 8, ewh_dev_stamps), 22 = the latency kernel with phase
 * stamps (ewh_dev_lat_stamps), 23 = the latency kernel with every wait
 * forced to run out (the stall error path), 24 / 25 = the latency kernel with
 * block barriers instead of the dataflow panel loop / as in round 3, 26 = the
 * C3 kernel at one wave per SIMD with the whole triangle resident, 28 = the
 * C5 row update one 64-row block row per pass with one tile per workgroup
 * (round 3), 30 = the contraction with TwoSum accumulation (up to 10
 * blocks), 31 = the C5 row update one block row per pass with two tiles per
 * workgroup, 32 = the C5 two-row pass with each streamed slab loaded at the
 * top of its step, 33 = the C5 one-proposal (right-looking) schedule with
 * each diagonal block factored in a launch of its own instead of inside the
 * previous trailing update, 34 = the wide / double-double route as in round
 * 5a (separate forward and reversed fp64 launches, 128 MB scratch budgets
 * that cap the launches at 56-624 workgroups), 35 = the varying-white-noise
 * contraction with the blocks' remainder on the first waves (round 4-5a:
 * the waves that also form the ECORR epoch sums), 36 = the contraction
 * without the r-separated Gram (r in the MFMA blocks, as before round 5h),
 * 37 = the wide path's ECORR epoch sums one sample per workgroup (as before
 * round 5h), 38 / 39 = the varying-white-noise contraction up to 10 blocks
 * with blocked instead of TwoSum accumulation, 4 / 8 waves.  Other modes return
 * EWH_E_UNSUPPORTED. */
int ewh_set_kernel_mode(ewh_handle* h, int32_t mode);

/* The largest batch the single-launch latency path serves (LAT_B_MAX; a
 * fixed-white-noise uncorrelated / CURN batch of at most this many samples on
 * one device is one launch of chol_lat_kernel).  0: no latency path (the host
 * twin).  Callers size their persistent small-batch buffers from it. */
int ewh_lat_b_max(void);

void ewh_destroy(ewh_handle* h);
const char* ewh_last_error(void);
int ewh_version(void);

#ifdef __cplusplus
}
#endif

#endif /* EWARP_HIP_H */
