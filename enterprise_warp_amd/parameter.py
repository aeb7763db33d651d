"""Sampling parameters with enterprise's public surface.

enterprise_warp builds priors with `parameter.Uniform(lo, hi)` (unnamed, the
signal names it `{psr}_{signal}_{key}_{par}`) or `parameter.Uniform(lo,
hi)(name)` (explicitly named, e.g. `gw_log10_A`, enterprise_models.py:366-387),
`parameter.Constant()` for fixed white noise (enterprise_models.py:549) and
`parameter.LinearExp` (:369).  The bilby bridge reads `.name`, `.size`,
`.type` and `.prior._defaults` (bilby_warp.py:51-98); PTMCMC calls
`.sample()` (run_example_paramfile.py:29).  This module provides exactly that
surface; values live on the host, the likelihood engine sees only the flat
theta matrix built from `PTA.param_names`.
"""
import numpy as np

_rng = np.random.default_rng()


class _Prior:
    def __init__(self, **defaults):
        self._defaults = dict(defaults)


class Parameter:
    """A named parameter instance (free or constant)."""

    type = "base"

    def __init__(self, name, size=None, **defaults):
        self.name = name
        self.size = size
        self.prior = _Prior(**defaults)
        self.value = None

    # --- enterprise API ---------------------------------------------------
    def sample(self, rng=None):
        rng = rng or _rng
        shape = () if self.size is None else (self.size,)
        return self._sample(rng, shape)

    def get_logpdf(self, value):
        v = np.asarray(value, dtype=float)
        lp = self._logpdf(v)
        return float(np.sum(lp))

    def get_pdf(self, value):
        return float(np.exp(self.get_logpdf(value)))

    def __repr__(self):
        return f"{self.name}:{type(self).__name__}({self.prior._defaults})"


class UniformParameter(Parameter):
    type = "uniform"

    def _sample(self, rng, shape):
        d = self.prior._defaults
        return rng.uniform(d["pmin"], d["pmax"], size=shape or None)

    def _logpdf(self, v):
        d = self.prior._defaults
        inside = (v >= d["pmin"]) & (v <= d["pmax"])
        with np.errstate(divide="ignore"):
            return np.where(inside, -np.log(d["pmax"] - d["pmin"]), -np.inf)


class NormalParameter(Parameter):
    type = "normal"

    def _sample(self, rng, shape):
        d = self.prior._defaults
        return rng.normal(d["mu"], d["sigma"], size=shape or None)

    def _logpdf(self, v):
        d = self.prior._defaults
        return -0.5 * ((v - d["mu"]) / d["sigma"]) ** 2 - np.log(np.sqrt(2 * np.pi) * d["sigma"])


class TruncNormalParameter(Parameter):
    type = "truncatednormal"

    def _sample(self, rng, shape):
        import scipy.stats as ss
        d = self.prior._defaults
        a, b = (d["minv"] - d["mu"]) / d["sigma"], (d["maxv"] - d["mu"]) / d["sigma"]
        return ss.truncnorm.rvs(a, b, loc=d["mu"], scale=d["sigma"], size=shape or None, random_state=rng)

    def _logpdf(self, v):
        import scipy.stats as ss
        d = self.prior._defaults
        a, b = (d["minv"] - d["mu"]) / d["sigma"], (d["maxv"] - d["mu"]) / d["sigma"]
        return ss.truncnorm.logpdf(v, a, b, loc=d["mu"], scale=d["sigma"])


class LinearExpParameter(Parameter):
    """Uniform in 10**x ([ent] parameter.LinearExp; enterprise_models.py:369)."""

    type = "linearexp"

    def _sample(self, rng, shape):
        d = self.prior._defaults
        return np.log10(rng.uniform(10 ** d["pmin"], 10 ** d["pmax"], size=shape or None))

    def _logpdf(self, v):
        d = self.prior._defaults
        inside = (v >= d["pmin"]) & (v <= d["pmax"])
        with np.errstate(divide="ignore"):
            val = np.log(np.log(10) * 10 ** v / (10 ** d["pmax"] - 10 ** d["pmin"]))
        return np.where(inside, val, -np.inf)


class ConstantParameter(Parameter):
    type = "constant"

    def __init__(self, name, value=None):
        super().__init__(name)
        self.value = value

    def sample(self, rng=None):
        return self.value

    def _logpdf(self, v):
        return np.zeros_like(v)


class ParameterSpec:
    """An unnamed prior, as returned by `Uniform(lo, hi)`.  Calling it with a
    name gives a bound Parameter (enterprise's Parameter-class idiom)."""

    def __init__(self, cls, size=None, **defaults):
        self.cls = cls
        self.size = size
        self.defaults = defaults
        self.name = None

    def __call__(self, name):
        if self.cls is ConstantParameter:
            return ConstantParameter(name, self.defaults.get("value"))
        return self.cls(name, size=self.size, **self.defaults)

    @property
    def is_constant(self):
        return self.cls is ConstantParameter


def Uniform(pmin, pmax, size=None):
    return ParameterSpec(UniformParameter, size=size, pmin=float(pmin), pmax=float(pmax))


def Normal(mu=0.0, sigma=1.0, size=None):
    return ParameterSpec(NormalParameter, size=size, mu=float(mu), sigma=float(sigma))


def TruncNormal(mu=0.0, sigma=1.0, minv=-np.inf, maxv=np.inf, size=None):
    return ParameterSpec(TruncNormalParameter, size=size, mu=float(mu), sigma=float(sigma),
                         minv=float(minv), maxv=float(maxv))


def LinearExp(pmin, pmax, size=None):
    return ParameterSpec(LinearExpParameter, size=size, pmin=float(pmin), pmax=float(pmax))


def Constant(val=None):
    return ParameterSpec(ConstantParameter, value=None if val is None else float(val))


def resolve(spec_or_param, default_name):
    """Turn what a signal factory was given into a bound Parameter.

    * an already-named Parameter (e.g. `Uniform(..)('gw_log10_A')`) keeps its name;
    * a ParameterSpec gets `default_name`;
    * a plain number becomes a Constant with that value."""
    if isinstance(spec_or_param, Parameter):
        return spec_or_param
    if isinstance(spec_or_param, ParameterSpec):
        return spec_or_param(default_name)
    if isinstance(spec_or_param, (int, float, np.floating, np.integer)):
        return ConstantParameter(default_name, float(spec_or_param))
    raise TypeError(f"cannot interpret {spec_or_param!r} as a parameter")
