"""Full-size (BASELINE config 3) properties on the GPU: sizes where the oracle
would take minutes, checked through size-independent identities."""
import numpy as np
import pytest

from conftest import check_parity
from enterprise_warp_amd import sharding, synth

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def c3():
    return synth.config_c3()


def test_c3_units_sum_and_sharding(require_gpu, c3):
    """Sum over pulsar terms == lnL; any partition into unit ranges (the
    multi-GPU sharding) sums to the same vector; batch-order independence."""
    import torch
    pta = c3.pta
    B = 512
    X = synth.prior_draws(pta, B, 45)
    full = pta.get_lnlikelihood_batch(X)
    eng = pta.engine()
    terms = eng.unit_terms(B)
    np.testing.assert_allclose(terms.sum(axis=0), full, rtol=1e-12, atol=1e-6)
    th = torch.from_numpy(X).cuda()
    for world in (2, 3, 8):
        acc = torch.zeros(B, dtype=torch.float64, device="cuda")
        for (u0, u1) in sharding.unit_ranges(eng.unit_costs(), B, world):
            part = torch.zeros(B, dtype=torch.float64, device="cuda")
            eng.lnl_units_device(th.data_ptr(), B, u0, u1, part.data_ptr(), torch.cuda.current_stream().cuda_stream)
            torch.cuda.synchronize()
            acc += part
        got = acc.cpu().numpy()
        fin = np.isfinite(full)
        np.testing.assert_allclose(got[fin], full[fin], rtol=1e-12, atol=1e-6)
        assert np.array_equal(~np.isfinite(got), ~fin)
    perm = np.random.default_rng(0).permutation(B)
    np.testing.assert_array_equal(pta.get_lnlikelihood_batch(X[perm]), full[perm])


def test_c3_mfma_vs_lds_full_size(require_gpu, c3):
    pta = c3.pta
    X = synth.near_draws(pta, c3.truth, 64, 3)
    a = pta.get_lnlikelihood_batch(X)
    pta.engine().set_kernel_mode(1)
    b = pta.get_lnlikelihood_batch(X)
    pta.engine().set_kernel_mode(0)
    check_parity(a, b, "C3 mfma vs lds")


def test_c3_pulsar_permutation_invariance(require_gpu, c3):
    """lnL is a sum over pulsars: reversing the pulsar order changes only the
    summation order."""
    from enterprise_warp_amd.pta import PTA
    pta = c3.pta
    X = synth.near_draws(pta, c3.truth, 32, 4)
    a = pta.get_lnlikelihood_batch(X)
    rev = PTA(list(reversed(pta.signal_collections)))
    b = rev.get_lnlikelihood_batch(X)
    check_parity(b, a, "C3 reversed pulsars")


@pytest.mark.parametrize("mode", [0, 1])
def test_c3_chol_vs_oracle(require_gpu, c3, mode):
    """The default register-blocked factorisation (mode 0: two-level blocked
    LDL^T panel) and the LDS Cholesky kernel (mode 1) against the oracle on
    full-size C3 near-truth draws, strict bound."""
    from conftest import oracle_lnl
    pta = c3.pta
    X = synth.near_draws(pta, c3.truth, 16, 7)
    pta.engine().set_kernel_mode(mode)
    try:
        got = pta.get_lnlikelihood_batch(X)
    finally:
        pta.engine().set_kernel_mode(0)
    check_parity(got, oracle_lnl(pta, X), f"C3 mode {mode}")


@pytest.mark.parametrize("name", ["c3_small", "c2_small", "c5_small", "c4_small"])
def test_multi_context_handle(require_gpu, name):
    """ewh_create with a device list: the batch is split over the contexts
    (units by cost for uncorrelated / CURN models, samples for a correlated
    common process).  Per-unit terms equal the single-context ones bit for
    bit; lnL equals it at the strict bound (uncorrelated: each context folds
    its range into a B-vector on its device and the first device adds the
    B-vectors -- a re-associated sum; correlated: bit for bit).  On the
    one-GPU box the lists [0, 0] and [0, 0, 0] exercise the split; a node
    passes [0..7]."""
    from conftest import check_parity, load_golden
    pta, X, _, _ = load_golden(name)
    X = np.vstack([X] * 8)                         # 128 samples: ranges split pulsars mid-row
    one = pta.get_lnlikelihood_batch(X)
    terms1 = pta.engine().unit_terms(len(X))
    for devs in ([0, 0], [0, 0, 0]):
        eng = pta.engine(devices=devs)
        assert eng.num_devices() == len(devs)
        got = pta.get_lnlikelihood_batch(X)
        check_parity(got, one, f"{name} on {devs}")
        if name.startswith("c5"):
            np.testing.assert_array_equal(got, one)
        np.testing.assert_array_equal(eng.unit_terms(len(X)), terms1)
    pta.engine(devices=[0])


def test_multi_context_theta_staging(require_gpu):
    """A handle spanning a node's contexts sends each context only the theta
    entries its units read (ewh_transfer_stats): C3's model on 45 pulsars
    (300-1200 TOAs) over 8 contexts -- the per-pulsar columns once in total,
    the shared CURN columns once per context -- at most 1.2 x B x n_param x 8
    bytes per batch, with the per-pulsar terms bit-identical to one context
    and peer access recorded for every context.  The bound needs P >> 2 ndev:
    each context boundary that splits a pulsar sends that pulsar's columns
    twice, and the 2 CURN columns go to every context (16 pulsars: 1.21 x)."""
    c3s = synth.config_c3(n_psr=45, n_min=300, n_max=1200, epoch_size=8)
    pta = c3s.pta
    B = 256
    X = synth.prior_draws(pta, B, 77)
    one = pta.get_lnlikelihood_batch(X)
    terms1 = pta.engine().unit_terms(B)
    full = B * len(pta.param_names) * 8
    eng = pta.engine(devices=[0] * 8)
    got = pta.get_lnlikelihood_batch(X)
    nbytes, peer = eng.transfer_stats()
    print(f"theta bytes {nbytes} = {nbytes / full:.3f} x full, peer mask {peer:#x}")
    assert nbytes <= 1.2 * full
    assert peer == 0xff
    check_parity(got, one, "C3-45psr on 8 contexts")
    np.testing.assert_array_equal(eng.unit_terms(B), terms1)
    pta.engine(devices=[0])


def test_set_fixed_white_in_place(require_gpu):
    """pta.set_default_params(new white-noise constants) (enterprise_warp.py:
    504-508) updates the cached TNT in place (ewh_set_fixed_white, same
    handle) and equals a PTA built from scratch with those constants."""
    from conftest import check_parity, load_golden, oracle_lnl
    pta, X, lnl, _ = load_golden("c3_small")
    eng = pta.engine()
    before = pta.get_lnlikelihood_batch(X)
    const = pta.constant_values()
    rng = np.random.default_rng(5)
    new = {k: (v * rng.uniform(0.95, 1.05) if k.endswith("_efac") else v + rng.uniform(-0.2, 0.2))
           for k, v in const.items() if k.endswith(("_efac", "_log10_tnequad", "_log10_ecorr"))}
    pta.set_default_params(new)
    assert pta.engine() is eng                      # no rebuild
    got = pta.get_lnlikelihood_batch(X)
    assert not np.array_equal(got, before)
    fresh, _, _, _ = load_golden("c3_small")
    fresh.set_default_params(new)
    np.testing.assert_array_equal(fresh.get_lnlikelihood_batch(X), got)
    check_parity(got[8:], oracle_lnl(pta, X[8:]), "c3_small new white noise")


def test_graph_replay_matches_eager(require_gpu):
    """ewh_lnl_batch captures each single-device batch size above the latency
    path's (B > LAT_B_MAX = 24) into a HIP graph on its first call and
    replays it afterwards; buffer growth (a larger B) invalidates the graphs.
    Every call must equal the first (eager) one; single-theta calls (the
    latency kernel) are deterministic, agree with a 16-sample latency batch
    bit for bit and with the batched value."""
    from conftest import load_golden
    pta, X, _, _ = load_golden("c3_small")
    X32 = np.vstack([X, X])
    big = np.vstack([X] * 32)
    ref = {1: pta.get_lnlikelihood_batch(X[:1]), 16: pta.get_lnlikelihood_batch(X),
           32: pta.get_lnlikelihood_batch(X32)}
    ref[512] = pta.get_lnlikelihood_batch(big)
    for B in (1, 1, 32, 16, 1, 32, 512, 1, 32, 16, 512, 1):
        XX = {1: X[:1], 16: X, 32: X32, 512: big}[B]
        np.testing.assert_array_equal(pta.get_lnlikelihood_batch(XX), ref[B])
    for i in range(16):                                   # single-theta calls (PTMCMC / bilby)
        one = pta.get_lnlikelihood(X[i])                  # (the latency kernel: B = 1 <= LAT_B_MAX)
        assert one == pta.get_lnlikelihood_batch(X[i:i + 1])[0]
        assert one == ref[16][i]                          # (B = 16: the latency kernel too)
        # ... the batched kernels' value up to the re-associated log-determinant sum
        assert abs(one - ref[32][i]) <= 1e-3 * (1e-6 + 1e-10 * abs(ref[32][i]))


def test_correlated_pulsar_partition(require_gpu):
    """Config 5's model, one proposal over several devices (SURVEY.md §8(e)
    exchange step): (1) a handle with 3 contexts and B < 3 splits the pulsars,
    gathers the kept blocks peer-to-peer and finishes on the first context;
    (2) the ABI protocol the torchrun ranks use -- ewh_corr_partial_device on
    pulsar ranges into pulsar-major buffers, then ewh_corr_finish_device.
    Both equal the one-device result bit for bit."""
    import torch
    c5 = synth.config_c5(n_psr=16, n_toa=800, seed=55, epoch_size=8)
    pta = c5.pta
    X = synth.near_draws(pta, c5.truth, 2, 57)
    one = pta.get_lnlikelihood_batch(X)
    pta.engine(devices=[0, 0, 0])
    for B in (1, 2):
        np.testing.assert_array_equal(pta.get_lnlikelihood_batch(X[:B]), one[:B])
    # fewer pulsars than contexts: the first context gets none and still
    # finishes (theta is staged on it regardless)
    c2p = synth.config_c5(n_psr=2, n_toa=300, seed=58, epoch_size=8)
    x2 = synth.near_draws(c2p.pta, c2p.truth, 1, 59)
    ref2 = c2p.pta.get_lnlikelihood_batch(x2)
    c2p.pta.engine(devices=[0, 0, 0])
    np.testing.assert_array_equal(c2p.pta.get_lnlikelihood_batch(x2), ref2)
    eng = pta.engine(devices=[0])
    kd = eng.keep_dim()
    P, B = len(pta.signal_collections), len(X)
    th = torch.from_numpy(X).cuda()
    keep = torch.zeros((P, B, kd, kd), dtype=torch.float64, device="cuda")
    local = torch.zeros((P, B), dtype=torch.float64, device="cuda")
    out = torch.zeros(B, dtype=torch.float64, device="cuda")
    s = torch.cuda.current_stream().cuda_stream
    for p0, p1 in ((0, 5), (5, 11), (11, P)):
        eng.corr_partial_device(th.data_ptr(), B, p0, p1, keep.data_ptr(), local.data_ptr(), s)
    eng.corr_finish_device(th.data_ptr(), B, keep.data_ptr(), local.data_ptr(), out.data_ptr(), s)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(out.cpu().numpy(), one)


@pytest.mark.parametrize("name", ["c3_small", "c3_freesp", "c1_j1832", "c1_system", "full_c3"])
def test_latency_kernel_matches_batched(require_gpu, c3, name):
    """Batches of up to 24 samples (LAT_B_MAX) on one device run
    chol_lat_kernel (one 4-wave workgroup per unit, theta read from pinned
    memory, the pulsar fold and the lnL write fused into the launch).  Its
    factor, pivots and q are the batched kernel's bit for bit; only the
    log-determinant sum is associated differently, so lnL must agree with the
    batched path (kernel mode 2: latency path off) far inside the strict
    bound, with the same -inf pattern, for B = 1 (a sampler's single
    proposal), 5, 8, 12, 16 and 24 (the bound)."""
    from conftest import load_golden
    if name == "full_c3":
        pta = c3.pta
        X = np.vstack([synth.prior_draws(pta, 12, 45), synth.near_draws(pta, c3.truth, 12, 3)])
    else:
        pta, X, _, _ = load_golden(name)
        X = np.vstack([X, X[::-1]])                     # 32 rows (16 golden samples, each twice)
    eng = pta.engine()
    assert eng.lat_b_max() == 24
    worst = 0.0
    for B in (1, 5, 8, 12, 16, 24):
        XX = X[:B]
        eng.set_kernel_mode(2)
        ref = pta.get_lnlikelihood_batch(XX)
        ref_terms = eng.unit_terms(B)
        eng.set_kernel_mode(0)
        got = pta.get_lnlikelihood_batch(XX)
        terms = eng.unit_terms(B)
        assert np.array_equal(np.isfinite(got), np.isfinite(ref)), f"{name} B={B}: -inf pattern differs"
        assert not np.any(np.isnan(got))
        fin = np.isfinite(ref)
        err = np.abs(got[fin] - ref[fin]) / (1e-6 + 1e-10 * np.abs(ref[fin]))
        worst = max(worst, float(err.max()) if err.size else 0.0)
        assert np.all(err <= 1e-3), f"{name} B={B}: latency vs batched {err.max():.3e} of strict"
        tf = np.isfinite(ref_terms)
        assert np.array_equal(tf, np.isfinite(terms))
        np.testing.assert_allclose(terms[tf], ref_terms[tf], rtol=1e-12, atol=1e-9)
        # repeated single-proposal calls are deterministic
        np.testing.assert_array_equal(pta.get_lnlikelihood_batch(XX), got)
    print(f"{name}: latency vs batched max err/strict {worst:.3e}")


def test_correlated_right_looking_small_chunks(require_gpu):
    """Sigma_c of a correlated common process: chunks of up to 12 samples (a
    PTMCMC proposal, a few tempering chains) are factored right-looking (trailing tiles updated in
    parallel after each 64-wide panel), larger chunks left-looking (row
    update, fused with the panel from 64 samples on).  Tile (i, j) takes the
    same K = 64 slabs in the same order either way, so the two give the same
    lnL bit for bit."""
    from conftest import load_golden
    pta, X, _, _ = load_golden("c5_small")
    big = np.vstack([X] * 8)                    # 128 samples: left-looking, fused row update + panel
    left = pta.get_lnlikelihood_batch(big)[:len(X)]
    for B in (1, 3, 4, 12, 13):          # 13: the left-looking small-chunk row update
        got = np.concatenate([pta.get_lnlikelihood_batch(X[i:i + B]) for i in range(0, len(X), B)])
        np.testing.assert_array_equal(got, left)


@pytest.mark.parametrize("n_psr", [16, 20])
def test_correlated_row_pairs_bit_identical(require_gpu, n_psr):
    """Chunks of >= 64 samples update two block rows of Sigma_c per pass
    (dchol_rowpair_kernel: rows k, k + 1 take every p < k together, row
    k + 1 then p = k); chunks of <= 12 factor right-looking.  Per tile the
    same K = 64 slabs in the same order: bit-identical lnL.  16 pulsars: 8
    block rows (the last pair ends the matrix), 20 pulsars: 9 (a single last
    row)."""
    cfg = synth.config_c5(n_psr=n_psr, n_toa=1200, seed=7)
    pta = cfg.pta
    X = synth.prior_draws(pta, 64, 11)
    big = pta.get_lnlikelihood_batch(X)
    small = np.concatenate([pta.get_lnlikelihood_batch(X[i:i + 4]) for i in range(0, 16, 4)])
    assert not np.any(np.isnan(big)) and np.mean(np.isfinite(big)) > 0.5
    np.testing.assert_array_equal(small, big[:16])


@pytest.mark.parametrize("name", ["c4_small", "c3_small", "c2_small", "c5_small", "c5_varwn", "c1_system"])
def test_wide_kernel_matches_register_kernels(require_gpu, name):
    """chol_wide_kernel (fp64, any width: the partial factorisation of a wide
    correlated model, and kernel mode 27's route for every factorisation)
    against the default kernels on the same inputs: chol_big_kernel (c4_small,
    13 blocks: the same operations per block in the same order, unit terms
    equal to ~1 ulp), chol_mfma_kernel (right-looking, one log-determinant
    accumulator) and its KEEP form, at 1e-3 of strict; c1_system (fixed white
    noise, 13 blocks; by default the double-double chol_dd_kernel) on its
    near-truth draws at the strict bound."""
    from conftest import load_golden
    pta, z = load_golden(name, full=True)
    X = z["theta"]
    eng = pta.engine()
    eng.set_kernel_mode(2)                           # (the latency path off: batched kernels only)
    a = pta.get_lnlikelihood_batch(X)
    ta = eng.unit_terms(len(X))
    eng.set_kernel_mode(27)
    try:
        b = pta.get_lnlikelihood_batch(X)
        tb = eng.unit_terms(len(X))
    finally:
        eng.set_kernel_mode(0)
    assert np.array_equal(np.isfinite(a), np.isfinite(b)) and not np.any(np.isnan(b))
    if name == "c1_system":
        check_parity(b[z["near"]], a[z["near"]], "c1_system wide (fp64) vs dd")
        return
    fin = np.isfinite(a)
    err = np.abs(b[fin] - a[fin]) / (1e-6 + 1e-10 * np.abs(a[fin]))
    assert err.max() <= 1e-3, f"{name}: wide vs register {err.max():.3e} of strict"
    if name == "c4_small":
        tf = np.isfinite(ta)
        np.testing.assert_allclose(tb[tf], ta[tf], rtol=1e-14, atol=0)


@pytest.mark.parametrize("name", ["c1_system", "c1_widefix", "c1_wide"])
def test_dd_verify_and_refine(require_gpu, name):
    """Bases past the register kernels (fixed white noise past 9 blocks,
    any basis past 16): by default the forward and the reversed-order fp64
    factorisations (chol_wide_kernel) verify each other and only the units
    on which they disagree by more than a quarter of strict are refactored
    in double-double (chol_dd_kernel); kernel mode 29 takes every unit
    through chol_dd_kernel.  The two agree at the strict bound on every
    golden sample (prior draws included)."""
    from conftest import load_golden
    pta, X, _, _ = load_golden(name)
    eng = pta.engine()
    eng.set_kernel_mode(2)
    a = pta.get_lnlikelihood_batch(X)
    eng.set_kernel_mode(29)
    try:
        b = pta.get_lnlikelihood_batch(X)
    finally:
        eng.set_kernel_mode(0)
    check_parity(a, b, f"{name}: verify-and-refine vs double-double everywhere")


def test_wide_bases_full_size(require_gpu):
    """A basis past every register kernel at a realistic size: one pulsar of
    10k TOAs with red / DM / chromatic noise at 60 frequencies each (X_60_nfreqs,
    enterprise_models.py:148-167; 12 + 360 columns, 24 blocks): white noise
    sampled (contract_wide_kernel + chol_wide_kernel) and fixed (gram_dd +
    schur + chol_wide_kernel), near-truth draws against the oracle, strict."""
    from conftest import oracle_lnl
    psr = synth.make_pulsar("J0000+0060", 10000, seed=60, epoch_size=16)
    terms = {"efac": "by_backend", "equad": "by_backend", "ecorr": "by_backend",
             "spin_noise": "powerlaw_60_nfreqs", "dm_noise": "powerlaw_60_nfreqs", "chromred": "4_60_nfreqs"}
    wn = synth.white_noisedict([psr], 61)
    for fixed in (False, True):
        ns = synth.params_namespace(psr.toas.max() - psr.toas.min(), fixed)
        pta = synth.build_pta([psr], terms, {}, ns, wn if fixed else None)
        truth = synth.truth_values(pta, 62, white=wn)
        synth.simulate_residuals(pta, truth, 63)
        X = synth.near_draws(pta, truth, 6, 64)
        check_parity(pta.get_lnlikelihood_batch(X), oracle_lnl(pta, X), f"wide 372 columns, fixed white {fixed}")
