"""CPU tests of the PTMCMC surface (enterprise_warp_amd.ptmcmc / model_utils):
PTMCMCSampler's call signature, chain file layout, resume, jump proposals'
proposal ratios, and that the chain samples a known posterior.  The device
likelihood is replaced by an analytic Gaussian here (the GPU test
test_ptmcmc_driver_hypermodel runs the reference's driver flow on device)."""
import inspect

import numpy as np
import pytest

from enterprise_warp_amd import model_utils, parameter
from enterprise_warp_amd.ptmcmc import JumpProposal, PTSampler


class GaussPTA:
    """Stand-in PTA: Uniform(-10, 10) priors, Gaussian likelihood."""

    def __init__(self, mu, sig):
        self.mu, self.sig = np.asarray(mu, float), np.asarray(sig, float)
        self.params = [parameter.Uniform(-10, 10)(f"J0000_red_noise_{n}") for n in ("gamma", "log10_A")] + \
                      [parameter.Uniform(-10, 10)("gw_log10_A")]
        self.param_names = [p.name for p in self.params]
        self.pulsars = ["J0000"]
        self.calls = 0

    def get_lnlikelihood(self, x):
        self.calls += 1
        return float(-0.5 * np.sum(((np.asarray(x) - self.mu) / self.sig) ** 2))

    def get_lnprior(self, x):
        return float(sum(p.get_logpdf(v) for p, v in zip(self.params, x)))


def test_sample_signature_matches_ptmcmcsampler():
    """run_example_paramfile.py:38-43 filters the paramfile's sampler kwargs by
    sample()'s argument names and deletes 'Niter' and 'p0'."""
    args = inspect.getfullargspec(PTSampler.sample).args
    for a in ("p0", "Niter", "SCAMweight", "AMweight", "DEweight", "burn", "thin", "isave", "covUpdate"):
        assert a in args


def test_chain_samples_posterior_and_layout(tmp_path):
    pta = GaussPTA([1.0, -2.0, 0.5], [0.3, 0.5, 0.2])
    s = model_utils.setup_sampler(pta, outdir=str(tmp_path), seed=1)
    x0 = np.hstack([np.atleast_1d(p.sample()) for p in pta.params])
    s.sample(x0, 30000, burn=2000, thin=10, isave=5000, covUpdate=1000)
    ch = np.loadtxt(tmp_path / "chain_1.txt")
    assert ch.shape == (3000, 3 + 4)
    post = ch[1000:]
    np.testing.assert_allclose(post[:, :3].mean(0), pta.mu, atol=0.1)
    np.testing.assert_allclose(post[:, :3].std(0), pta.sig, rtol=0.25)
    # ln posterior = ln likelihood + ln prior; ln likelihood re-evaluates
    lp = np.array([pta.get_lnprior(r[:3]) for r in post[:20]])
    ll = np.array([pta.get_lnlikelihood(r[:3]) for r in post[:20]])
    np.testing.assert_allclose(post[:20, 4], ll, rtol=1e-12)
    np.testing.assert_allclose(post[:20, 3], ll + lp, rtol=1e-12)
    assert 0 < ch[-1, 5] < 1
    assert (tmp_path / "pars.txt").exists() and (tmp_path / "cov.npy").exists()


def test_resume_appends(tmp_path):
    pta = GaussPTA([0, 0, 0], [1, 1, 1])
    s = model_utils.setup_sampler(pta, outdir=str(tmp_path), seed=2)
    s.sample(np.zeros(3), 500, thin=10, isave=100)
    n1 = len(np.loadtxt(tmp_path / "chain_1.txt"))
    s2 = model_utils.setup_sampler(pta, outdir=str(tmp_path), resume=True, seed=3)
    s2.sample(np.zeros(3), 1000, thin=10, isave=100)
    assert n1 == 50 and len(np.loadtxt(tmp_path / "chain_1.txt")) == 100


def test_prior_draw_jump_ratio():
    """lqxy = log p(x_i) - log p(q_i): with a flat prior inside the bounds it
    is 0, and a draw always lands inside the prior."""
    pta = GaussPTA([0, 0, 0], [1, 1, 1])
    jp = JumpProposal(pta, seed=4)
    x = np.array([0.1, 0.2, 0.3])
    for _ in range(50):
        q, lqxy = jp.draw_from_prior(x, 0, 1.0)
        assert np.sum(q != x) <= 1 and lqxy == 0.0 and np.all(np.abs(q) <= 10)
    q, _ = jp.draw_from_gwb_prior(x, 0, 1.0)
    assert np.all(q[:2] == x[:2])


def test_hypermodel_sampler_has_nmodel_jump(tmp_path):
    from enterprise_warp_amd.hypermodel import HyperModel
    hm = HyperModel([GaussPTA([0, 0, 0], [1, 1, 1]), GaussPTA([1, 1, 1], [1, 1, 1])])
    s = hm.setup_sampler(outdir=str(tmp_path), seed=5)
    names = [f.__name__ for f, _ in s._custom]
    assert "draw_from_nmodel_prior" in names
    x = s.sample(hm.initial_sample(rng=0), 300, thin=10, isave=100)
    assert len(x) == len(hm.param_names)


@pytest.mark.parametrize("groups", [None])
def test_parameter_groups(groups):
    pta = GaussPTA([0, 0, 0], [1, 1, 1])
    g = model_utils.get_parameter_groups(pta)
    assert g[0] == [0, 1, 2] and [0, 1] in g and [2] in g
