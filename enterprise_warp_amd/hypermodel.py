"""`HyperModel`: product-space model selection over several PTAs, the object
the reference's driver builds when a paramfile has more than one `{N}` model
block (examples/run_example_paramfile.py:31-45, enterprise_extensions
`model_utils.HyperModel`, unpinned, absent from this image).

Semantics restated from enterprise_extensions' published HyperModel:
* `param_names`: the union of the models' parameter names in order of first
  appearance, then `nmodel` (Uniform(-0.5, n_models - 0.5));
* `get_lnlikelihood(x)`: nmodel = rint(x[nmodel]); the active model's
  parameters are picked out of x by name and only that model's likelihood is
  evaluated (+ an optional log-weight per model);
* `get_lnprior(x)`: -inf outside the model range, else the sum of every
  model's log-prior over its own parameters.

New here: `get_lnlikelihood_batch(X)` groups a batch of proposals by model and
evaluates each group in one device call of that model's PTA.
"""
import numpy as np

from . import parameter


class HyperModel:
    def __init__(self, models, log_weights=None):
        self.models = dict(models) if isinstance(models, dict) else dict(enumerate(models))
        self.num_models = len(self.models)
        self.log_weights = log_weights
        names, params, seen = [], [], set()
        for m in self.models.values():
            by_name = {}
            for p in m.params:
                if p.size:
                    for i in range(p.size):
                        by_name[f"{p.name}_{i}"] = p
                else:
                    by_name[p.name] = p
            for nm in m.param_names:
                if nm not in seen:
                    seen.add(nm)
                    names.append(nm)
                    if by_name[nm] not in params:
                        params.append(by_name[nm])
        self.nmodel_param = parameter.Uniform(-0.5, self.num_models - 0.5)("nmodel")
        self.param_names = names + ["nmodel"]
        self.params = params + [self.nmodel_param]
        self._idx = {k: np.array([self.param_names.index(n) for n in m.param_names], dtype=int)
                     for k, m in self.models.items()}
        self._inm = len(self.param_names) - 1

    def _model_of(self, x):
        return int(np.rint(x[self._inm]))

    def get_lnlikelihood(self, x):
        x = np.asarray(x, dtype=float)
        k = self._model_of(x)
        lnl = self.models[k].get_lnlikelihood(x[self._idx[k]])
        if self.log_weights is not None:
            lnl += self.log_weights[k]
        return lnl

    def get_lnlikelihood_batch(self, X):
        X = np.atleast_2d(np.asarray(X, dtype=float))
        ks = np.rint(X[:, self._inm]).astype(int)
        out = np.full(len(X), -np.inf)
        for k, m in self.models.items():
            sel = np.flatnonzero(ks == k)
            if len(sel):
                out[sel] = m.get_lnlikelihood_batch(X[np.ix_(sel, self._idx[k])])
                if self.log_weights is not None:
                    out[sel] += self.log_weights[k]
        return out

    def get_lnprior(self, x):
        x = np.asarray(x, dtype=float)
        if self._model_of(x) not in self.models:
            return -np.inf
        return float(sum(m.get_lnprior(x[self._idx[k]]) for k, m in self.models.items()))

    def get_lnprior_batch(self, X):
        X = np.atleast_2d(np.asarray(X, dtype=float))
        ks = np.rint(X[:, self._inm]).astype(int)
        lp = np.zeros(len(X))
        for k, m in self.models.items():
            lp += m.get_lnprior_batch(X[:, self._idx[k]])
        lp[(ks < 0) | (ks >= self.num_models)] = -np.inf
        return lp

    @property
    def pulsars(self):
        out = []
        for m in self.models.values():
            for p in getattr(m, "pulsars", []):
                if p not in out:
                    out.append(p)
        return out

    def setup_sampler(self, outdir="chains", resume=False, sample_nmodel=True, empirical_distr=None, groups=None,
                      human=None, loglkwargs=None, logpkwargs=None, seed=None):
        """enterprise_extensions HyperModel.setup_sampler (run_example_paramfile.py:33):
        the PTMCMC sampler over the union parameters + nmodel, with a prior-draw
        jump on nmodel (enterprise_warp_amd.ptmcmc)."""
        from .ptmcmc import setup_sampler
        return setup_sampler(self, outdir=outdir, resume=resume, empirical_distr=empirical_distr, groups=groups,
                             human=human, loglkwargs=loglkwargs, logpkwargs=logpkwargs, seed=seed)

    def initial_sample(self, rng=None):
        rng = np.random.default_rng(rng)
        x = np.empty(len(self.param_names))
        for k, m in self.models.items():
            for p in m.params:
                v = np.atleast_1d(p.sample(rng))
                for i, val in enumerate(v):
                    nm = f"{p.name}_{i}" if p.size else p.name
                    x[self.param_names.index(nm)] = val
        x[self._inm] = rng.uniform(-0.5, self.num_models - 0.5)
        return x
