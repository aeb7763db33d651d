"""Sampler adapters: `PTABilbyLikelihood`, `get_bilby_prior_dict`.

Same behaviour as enterprise_warp.bilby_warp (bilby_warp.py:3-106):
`log_likelihood()` gathers `timing model_tmparams_*` entries into one vector
parameter and calls `pta.get_lnlikelihood(dict)`; `get_bilby_prior_dict`
translates `pta.params` (uniform / normal / truncatednormal scalars, vector
`jup_orb_elements` and `timing model_tmparams`).  bilby is not installed in
this image; when it is importable the classes subclass / return bilby
objects, otherwise minimal stand-ins with the same attributes are used.

New: `log_likelihood_batch(samples)` evaluates many proposals in one device
call (the hot loop of a batched sampler).
"""
import numpy as np

try:  # pragma: no cover - bilby absent in this image
    import bilby as _bilby
    _Base = _bilby.Likelihood
except Exception:  # noqa: BLE001
    _bilby = None

    class _Base:
        def __init__(self, parameters=None):
            self.parameters = parameters or {}


class PTABilbyLikelihood(_Base):
    def __init__(self, pta, parameters):
        self.pta = pta
        self.parameters = parameters
        self._marginalized_parameters = []

    def _to_dict(self, params):
        tm, tmname, cur = [], None, {}
        for k, v in params.items():
            if "timing model_tmparams" in k:
                tm.append(v)
                if tmname is None:
                    tmname = "_".join(k.split("_")[:-1])
            else:
                cur[k] = v
        if tmname is not None:
            cur[tmname] = tm
        return cur

    def log_likelihood(self):
        return self.pta.get_lnlikelihood(self._to_dict(self.parameters))

    def log_likelihood_batch(self, samples):
        """samples: list of parameter dicts, or an array [B, nparam] in
        pta.param_names order."""
        if isinstance(samples, np.ndarray):
            return self.pta.get_lnlikelihood_batch(samples)
        X = np.vstack([self.pta._theta(self._to_dict(s)) for s in samples])
        return self.pta.get_lnlikelihood_batch(X)

    def get_one_sample(self):
        return {par.name: par.sample() for par in self.pta.params}


class _Prior:
    def __init__(self, kind, name, **kw):
        self.kind, self.name = kind, name
        self.__dict__.update(kw)

    def sample(self, size=None, rng=None):
        rng = rng or np.random.default_rng()
        if self.kind == "Uniform":
            return rng.uniform(self.minimum, self.maximum, size)
        if self.kind == "Normal":
            return rng.normal(self.mu, self.sigma, size)
        import scipy.stats as ss
        a, b = (self.minimum - self.mu) / self.sigma, (self.maximum - self.mu) / self.sigma
        return ss.truncnorm.rvs(a, b, loc=self.mu, scale=self.sigma, size=size, random_state=rng)

    def __repr__(self):
        return f"{self.kind}({self.name})"


def _uniform(lo, hi, name):
    return _bilby.core.prior.Uniform(lo, hi, name) if _bilby else _Prior("Uniform", name, minimum=lo, maximum=hi)


def _normal(mu, sigma, name):
    return _bilby.core.prior.Normal(mu, sigma, name) if _bilby else _Prior("Normal", name, mu=mu, sigma=sigma)


def _truncnorm(mu, sigma, lo, hi, name):
    if _bilby:
        return _bilby.core.prior.TruncatedGaussian(mu, sigma, lo, hi, name)
    return _Prior("TruncatedGaussian", name, mu=mu, sigma=sigma, minimum=lo, maximum=hi)


def get_bilby_prior_dict(pta):
    priors = {}
    for p in pta.params:
        d = p.prior._defaults
        if p.size is None:
            if p.type == "uniform":
                priors[p.name] = _uniform(d["pmin"], d["pmax"], p.name)
            elif p.type == "normal":
                priors[p.name] = _normal(d["mu"], d["sigma"], p.name)
            elif p.type == "truncatednormal":
                priors[p.name] = _truncnorm(d["mu"], d["sigma"], d["minv"], d["maxv"], p.name)
            else:
                raise ValueError(f"{p.name}: scalar prior of type {p.type!r} has no bilby counterpart here "
                                 f"(supported: uniform, normal, truncatednormal)")
        else:
            if p.name == "jup_orb_elements" and p.type == "uniform":
                for i in range(p.size):
                    priors[f"{p.name}_{i}"] = _uniform(-0.05, 0.05, f"{p.name}_{i}")
            elif "timing model_tmparams" in p.name and p.type == "uniform":
                for i in range(p.size):
                    priors[f"{p.name}_{i}"] = _uniform(d["pmin"], d["pmax"], f"{p.name}_{i}")
            else:
                raise ValueError(f"{p.name}: vector prior (size {p.size}, type {p.type!r}) has no bilby "
                                 f"counterpart here (supported: uniform jup_orb_elements / timing-model tmparams)")
    for k in priors:
        if k not in pta.param_names:
            print(f"[!] Warning: Bilby's {k} is not in PTA params")
    return priors
