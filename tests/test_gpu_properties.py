"""Full-size (BASELINE config 3) properties on the GPU: sizes where the oracle
would take minutes, checked through size-independent identities."""
import numpy as np
import pytest

from conftest import lnl_tolerance
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
    assert np.all(np.abs(a - b) <= lnl_tolerance(b))


def test_c3_pulsar_permutation_invariance(require_gpu, c3):
    """lnL is a sum over pulsars: reversing the pulsar order changes only the
    summation order."""
    from enterprise_warp_amd.pta import PTA
    pta = c3.pta
    X = synth.near_draws(pta, c3.truth, 32, 4)
    a = pta.get_lnlikelihood_batch(X)
    rev = PTA(list(reversed(pta.signal_collections)))
    b = rev.get_lnlikelihood_batch(X)
    assert np.all(np.abs(a - b) <= lnl_tolerance(a))


@pytest.mark.parametrize("mode", [0, 2, 3, 4, 5, 6, 8, 9, 10, 11, 12, 13])
def test_c3_chol_variants_vs_oracle(require_gpu, c3, mode):
    """Every register-blocked Cholesky variant (Cholesky / LDL^T panel, looped
    / unrolled, 1-2 waves per SIMD) against the oracle on full-size C3: near-
    truth draws at the strict bound, prior draws (loud red noise, Sigma close
    to singular) at the conditioning-widened bound of conftest.lnl_tolerance."""
    from conftest import oracle_lnl_cond
    pta = c3.pta
    X = np.concatenate([synth.near_draws(pta, c3.truth, 16, 7), synth.prior_draws(pta, 16, 8)])
    pta.engine().set_kernel_mode(mode)
    try:
        got = pta.get_lnlikelihood_batch(X)
    finally:
        pta.engine().set_kernel_mode(0)
    want, cond = oracle_lnl_cond(pta, X)
    fin = np.isfinite(want)
    strict = np.arange(len(X)) < 16
    err = np.abs(got - want)
    assert np.all(err[strict] <= lnl_tolerance(want[strict])), f"mode {mode}: near-truth worst {err[strict].max():.3e}"
    tol = lnl_tolerance(want[fin], cond[fin])
    assert np.all(err[fin] <= tol), f"mode {mode}: worst err/tol {np.max(err[fin] / tol):.3e}"
    assert np.array_equal(np.isfinite(got), fin)
