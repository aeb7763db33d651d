"""Batched Metropolis sampler: the stand-in for the reference's samplers
(PTMCMCSampler via enterprise_extensions `setup_sampler`, bilby's nested
samplers; run_example_paramfile.py:25-57), which are absent from this image.

`BatchedMH` runs B independent random-walk Metropolis chains.  Each iteration
proposes for all chains at once, so the likelihood of the whole batch is ONE
device call (`get_lnlikelihood_batch`) — the batching the GPU path is built
for.  Proposals are Gaussian with the 2.38^2/d-scaled covariance of the
pooled chain history (adapted every `adapt_every` iterations; initially the
prior widths, or `cov` / the paramfile's `mcmc_covm_csv`).  Chains are written
as `chain_1.txt` in the PTMCMCSampler column layout: parameters, ln posterior,
ln likelihood, acceptance rate, 0 (one row per chain per recorded iteration).
"""
import os

import numpy as np


def prior_widths(model):
    w = []
    for p in model.params:
        d = p.prior._defaults
        if "pmin" in d:
            width = (d["pmax"] - d["pmin"]) / np.sqrt(12.0)
        elif "sigma" in d:
            width = d["sigma"]
        else:
            width = 1.0
        w.extend([width] * (p.size or 1))
    return np.array(w)


class BatchedMH:
    def __init__(self, model, nchains=256, outdir=None, seed=0, cov=None, adapt_every=100, scale=None):
        self.model = model
        self.nchains = int(nchains)
        self.outdir = outdir
        self.rng = np.random.default_rng(seed)
        self.ndim = len(model.param_names)
        c = np.diag(prior_widths(model) ** 2) * 0.01 if cov is None else np.asarray(cov, dtype=float)
        self.L = np.linalg.cholesky(c)
        self.scale = (2.38 ** 2 / self.ndim) if scale is None else scale
        self.adapt_every = adapt_every
        self.history = []

    def initial(self):
        X = np.empty((self.nchains, self.ndim))
        for b in range(self.nchains):
            if hasattr(self.model, "initial_sample"):
                X[b] = self.model.initial_sample(self.rng)
            else:
                X[b] = np.hstack([np.atleast_1d(p.sample(self.rng)) for p in self.model.params])
        return X

    def _lnpost(self, X):
        lp = self.model.get_lnprior_batch(X)
        ll = np.full(len(X), -np.inf)
        ok = np.isfinite(lp)
        if ok.any():
            ll[ok] = self.model.get_lnlikelihood_batch(X[ok])
        return lp + ll, ll

    def sample(self, x0=None, niter=1000, thin=10):
        X = self.initial() if x0 is None else np.array(np.broadcast_to(x0, (self.nchains, self.ndim)))
        post, like = self._lnpost(X)
        acc = np.zeros(self.nchains)
        fh = None
        if self.outdir:
            os.makedirs(self.outdir, exist_ok=True)
            fh = open(os.path.join(self.outdir, "chain_1.txt"), "w")
        try:
            for it in range(1, niter + 1):
                Z = self.rng.standard_normal((self.nchains, self.ndim)) @ self.L.T
                P = X + np.sqrt(self.scale) * Z
                pp, pl = self._lnpost(P)
                take = np.log(self.rng.uniform(size=self.nchains)) < (pp - post)
                X[take], post[take], like[take] = P[take], pp[take], pl[take]
                acc += take
                self.history.append(X.copy())
                if self.adapt_every and it % self.adapt_every == 0:
                    H = np.concatenate(self.history[len(self.history) // 2:])
                    c = np.cov(H.T) + 1e-12 * np.eye(self.ndim)
                    try:
                        self.L = np.linalg.cholesky(c)
                    except np.linalg.LinAlgError:
                        pass
                if fh is not None and it % thin == 0:
                    rows = np.column_stack([X, post, like, acc / it, np.zeros(self.nchains)])
                    np.savetxt(fh, rows)
        finally:
            if fh is not None:
                fh.close()
        self.acceptance = acc / max(niter, 1)
        return X, post, like
