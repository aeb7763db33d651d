"""Optimal statistic (results.py:653-795 -> enterprise_extensions
OptimalStatistic.compute_os; next-tier row 4 of SURVEY.md §8f).

Parity is unpinned by the reference (enterprise_extensions is absent and the
reference holds no OS fixtures): the oracle's Woodbury restatement is checked
against a dense-covariance computation of X = F^T C^-1 r, Z = F^T C^-1 F, and
the GPU path (ewh_optstat) against the oracle."""
import numpy as np
import pytest

from conftest import load_golden
from oracle import enterprise_ref as ref
from oracle.dense_ref import dense_os_xz

# OS tolerance: rho and sig relative to the largest |rho| / sig of the draw;
# OS and OS_sig relative.  The Schur/Gauss-Jordan route on the device and
# the oracle's cho_solve differ by rounding amplified by cond(Sigma).
OS_RTOL = 1e-7


def _oracle(pta):
    const_ = pta.constant_values()
    o = ref.OraclePTA([c.psr for c in pta.signal_collections], pta.oracle_terms(), fixed_params=const_)
    return o, const_


def _params(pta, const_, x):
    d = dict(const_)
    d.update(pta.map_params(x))
    return d


def test_oracle_os_matches_dense_covariance():
    pta, X, _, _ = load_golden("c3_small")
    o, const_ = _oracle(pta)
    d = _params(pta, const_, X[10])   # near-truth draw (8..15); prior draws 0..7 can be numerically singular
    xi, rho, sig, OS, OS_sig = ref.optimal_statistic(o, d)
    Xs, Zs = zip(*[dense_os_xz(pp, d) for pp in o.pulsars])
    g = next(g for g in o.pulsars[0].gps if g.get("name") == "gw")
    phat = ref.powerlaw(g["f"], 0.0, d["gw_gamma"], 2)
    k = 0
    P = len(Xs)
    for a in range(P):
        for b in range(a + 1, P):
            top = Xs[a] @ (phat * Xs[b])
            bot = np.trace((Zs[a] * phat) @ (Zs[b] * phat))
            assert abs(rho[k] - top / bot) <= 1e-6 * np.max(np.abs(rho))
            assert abs(sig[k] - bot ** -0.5) <= 1e-6 * sig[k]
            k += 1
    assert np.isfinite(OS) and OS_sig > 0
    assert np.all((xi >= 0) & (xi <= np.pi))


def test_os_needs_curn_signal():
    from enterprise_warp_amd.optstat import OptimalStatistic
    pta, _, _, _ = load_golden("c2_small")
    with pytest.raises(ValueError):
        OptimalStatistic(pta, gw_name="gw")


@pytest.mark.gpu
@pytest.mark.parametrize("orf", ["hd", "monopole", "dipole"])
def test_gpu_os_vs_oracle(require_gpu, orf):
    from enterprise_warp_amd.optstat import OptimalStatistic
    pta, X, _, _ = load_golden("c3_small")
    o, const_ = _oracle(pta)
    ost = OptimalStatistic(pta, orf=orf)
    draws = X[[8, 10, 12, 13, 15]]   # near-truth draws
    OS, OS_sig, rho, sig = ost.compute_noise_marginalised_os(draws, want_pairs=True)
    iu = np.triu_indices(len(pta.signal_collections), 1)
    for i, x in enumerate(draws):
        xi, r_w, s_w, os_w, oss_w = ref.optimal_statistic(o, _params(pta, const_, x), orf=orf)
        r_g, s_g = rho[i][iu], sig[i][iu]
        assert np.max(np.abs(r_g - r_w)) <= OS_RTOL * np.max(np.abs(r_w)), (i, r_g, r_w)
        assert np.max(np.abs(s_g - s_w) / s_w) <= OS_RTOL
        assert abs(OS[i] - os_w) <= OS_RTOL * max(abs(os_w), oss_w)
        assert abs(OS_sig[i] - oss_w) <= OS_RTOL * oss_w
    # single-draw surface: enterprise_extensions' (xi, rho, sig, OS, OS_sig)
    xi, r1, s1, os1, oss1 = ost.compute_os(pta.map_params(draws[1]))
    assert os1 == OS[1] and oss1 == OS_sig[1] and len(xi) == len(r1) == len(iu[0])
