"""PTMCMC sampler surface: `setup_sampler`, `PTSampler`, `JumpProposal`,
`get_parameter_groups` — the second sampler family of the reference's driver
(examples/run_example_paramfile.py:25-45), which reaches them through
enterprise_extensions `model_utils.setup_sampler` / `HyperModel.setup_sampler`
and PTMCMCSampler's `PTSampler.sample(x0, N, **kwargs)` (both third-party,
unpinned, absent from this image).

Restated from their published behaviour, single temperature (PTMCMCSampler
runs tempering only across MPI ranks):

* the chain advances one proposal at a time; each proposal is drawn from a
  weighted cycle of jumps -- SCAM (one eigen-direction of a parameter group's
  covariance), AM (the whole group, 2.38^2/d-scaled covariance), DE
  (difference of two past states, after `burn` iterations) and any jump added
  with `addProposalToCycle` (prior draws of `JumpProposal`);
* Metropolis-Hastings with the jump's log proposal ratio `lqxy`;
* the group covariances adapt every `covUpdate` iterations from the recent
  chain;
* every `thin`-th state is written to `outDir/chain_1.txt` as
  [parameters, ln posterior, ln likelihood, acceptance rate, PT acceptance]
  (the layout the reference's results.py reads: the last four columns are
  sampler statistics, results.py:431-437, :480), flushed every `isave`
  iterations; `cov.npy` holds the current covariance; `resume=True`
  continues from the last written state.

Every likelihood call is `pta.get_lnlikelihood(x)` on one theta -- the
device call through ewh_lnl_batch with B = 1 (bench.py `sampler_latency`).
"""
import os

import numpy as np


def get_parameter_groups(pta):
    """enterprise_extensions model_utils.get_parameter_groups, restated:
    all parameters, then the parameters of each pulsar, each (log10_A, gamma
    [, fc]) spectral pair, the common-process parameters, and nmodel."""
    names = list(pta.param_names)
    groups = [list(range(len(names)))]

    def add(idx):
        idx = sorted(set(idx))
        if idx and idx not in groups:
            groups.append(idx)

    psrs = getattr(pta, "pulsars", None) or []
    for psr in psrs:
        add([i for i, n in enumerate(names) if n.startswith(psr + "_")])
    prefixes = {}
    for i, n in enumerate(names):
        for tail in ("_log10_A", "_gamma", "_fc"):
            if n.endswith(tail):
                prefixes.setdefault(n[: -len(tail)], []).append(i)
    for idx in prefixes.values():
        if len(idx) > 1:
            add(idx)
    add([i for i, n in enumerate(names) if n.startswith("gw_")])
    if "nmodel" in names:
        add([names.index("nmodel")])
    return groups


class JumpProposal:
    """Prior-draw jumps (enterprise_extensions sampler.JumpProposal): each
    returns (q, lqxy) with lqxy = log p(x_i) - log p(q_i) for the redrawn
    parameter, so the Metropolis-Hastings ratio targets the posterior."""

    def __init__(self, pta, snames=None, empirical_distr=None, seed=None):
        self.pta = pta
        self.rng = np.random.default_rng(seed)
        self.names = list(pta.param_names)
        self.plist = []
        for p in pta.params:
            if p.size:
                self.plist.extend((p, j) for j in range(p.size))
            else:
                self.plist.append((p, None))

    def _draw(self, x, idx):
        q = np.array(x, dtype=float, copy=True)
        if len(idx) == 0:
            return q, 0.0
        i = int(self.rng.choice(idx))
        p, j = self.plist[i]
        v = np.atleast_1d(p.sample(self.rng))
        new = float(v[j] if j is not None else v[0])
        lqxy = self._logpdf(p, x[i]) - self._logpdf(p, new)
        q[i] = new
        return q, float(lqxy)

    @staticmethod
    def _logpdf(p, v):
        return float(np.sum(p._logpdf(np.asarray(v, dtype=float))))

    def _by(self, pred):
        return [i for i, n in enumerate(self.names) if pred(n)]

    def draw_from_prior(self, x, iter, beta):
        return self._draw(x, list(range(len(self.names))))

    def draw_from_red_prior(self, x, iter, beta):
        return self._draw(x, self._by(lambda n: "_red_noise_" in n))

    def draw_from_dm_gp_prior(self, x, iter, beta):
        return self._draw(x, self._by(lambda n: "_dm_gp_" in n))

    def draw_from_gwb_prior(self, x, iter, beta):
        return self._draw(x, self._by(lambda n: n.startswith("gw_")))

    def draw_from_white_prior(self, x, iter, beta):
        return self._draw(x, self._by(lambda n: n.endswith(("_efac", "_log10_tnequad", "_log10_ecorr"))))

    def draw_from_nmodel_prior(self, x, iter, beta):
        return self._draw(x, self._by(lambda n: n == "nmodel"))

    def draw_from_par_prior(self, par_names):
        par_names = [par_names] if isinstance(par_names, str) else list(par_names)
        idx = self._by(lambda n: any(n == pn or n.startswith(pn + "_") for pn in par_names))

        def jump(x, iter, beta):
            return self._draw(x, idx)
        jump.__name__ = "draw_from_" + "_".join(par_names) + "_prior"
        return jump


class PTSampler:
    """PTMCMCSampler-compatible single-temperature sampler (see module doc)."""

    def __init__(self, ndim, logl, logp, cov, groups=None, loglargs=None, loglkwargs=None, logpargs=None,
                 logpkwargs=None, comm=None, outDir="./chains", verbose=True, nowrite=False, resume=False,
                 seed=None):
        self.ndim = int(ndim)
        self.logl, self.logp = logl, logp
        self.loglargs, self.loglkwargs = list(loglargs or []), dict(loglkwargs or {})
        self.logpargs, self.logpkwargs = list(logpargs or []), dict(logpkwargs or {})
        self.cov = np.array(cov, dtype=float)
        self.groups = [list(range(self.ndim))] if groups is None else [list(g) for g in groups]
        self.outDir = outDir
        self.verbose, self.nowrite, self.resume = verbose, nowrite, resume
        self.rng = np.random.default_rng(seed)
        self.propCycle = []
        self._custom = []
        self._set_group_covs()
        if not nowrite:
            os.makedirs(outDir, exist_ok=True)
        self.fname = os.path.join(outDir, "chain_1.txt")

    # ---- proposals --------------------------------------------------------
    def addProposalToCycle(self, func, weight):
        self._custom.append((func, int(weight)))

    def _set_group_covs(self):
        self.U, self.S = [], []
        for g in self.groups:
            c = self.cov[np.ix_(g, g)]
            s, u = np.linalg.eigh(c)
            self.S.append(np.clip(s, 0, None))
            self.U.append(u)

    def covarianceJumpProposalSCAM(self, x, iter, beta):
        q = x.copy()
        k = self.rng.integers(len(self.groups))
        g = self.groups[k]
        j = self.rng.integers(len(g))
        scale = 2.38 if self.rng.uniform() < 0.9 else (0.2 if self.rng.uniform() < 0.5 else 10.0)
        q[g] += scale * np.sqrt(self.S[k][j]) * self.rng.standard_normal() * self.U[k][:, j]
        return q, 0.0

    def covarianceJumpProposalAM(self, x, iter, beta):
        q = x.copy()
        k = self.rng.integers(len(self.groups))
        g = self.groups[k]
        scale = 2.38 / np.sqrt(len(g)) if self.rng.uniform() < 0.9 else (0.2 if self.rng.uniform() < 0.5 else 10.0)
        z = self.rng.standard_normal(len(g)) * np.sqrt(self.S[k])
        q[g] += scale * (self.U[k] @ z)
        return q, 0.0

    def DEJump(self, x, iter, beta):
        q = x.copy()
        if self._nhist < 2:
            return q, 0.0
        a, b = self.rng.choice(self._nhist, 2, replace=False)
        k = self.rng.integers(len(self.groups))
        g = self.groups[k]
        scale = 1.0 if self.rng.uniform() < 0.5 else 2.38 / np.sqrt(2 * len(g))
        q[g] += scale * (self._hist[a, g] - self._hist[b, g])
        return q, 0.0

    def _cycle(self, SCAMweight, AMweight, DEweight, with_de):
        cyc = [self.covarianceJumpProposalSCAM] * int(SCAMweight) + [self.covarianceJumpProposalAM] * int(AMweight)
        if with_de:
            cyc += [self.DEJump] * int(DEweight)
        for f, w in self._custom:
            cyc += [f] * w
        return cyc or [self.covarianceJumpProposalAM]

    # ---- likelihood / prior ----------------------------------------------
    def _lnpost(self, x):
        lp = self.logp(x, *self.logpargs, **self.logpkwargs)
        if not np.isfinite(lp):
            return -np.inf, -np.inf
        ll = self.logl(x, *self.loglargs, **self.loglkwargs)
        return ll + lp, ll

    # ---- driver -----------------------------------------------------------
    def sample(self, p0, Niter, ladder=None, Tmin=1, Tmax=None, Tskip=100, isave=1000, covUpdate=1000,
               SCAMweight=30, AMweight=15, DEweight=50, NUTSweight=0, HMCweight=0, MALAweight=0, burn=10000,
               HMCstepsize=0.1, HMCsteps=300, maxIter=None, thin=10, i0=0, neff=100000, writeHotChains=False,
               hotChain=False):
        """Run the chain from p0 to Niter iterations (PTMCMCSampler.sample's
        signature; the tempering / gradient-based arguments are accepted and
        ignored in a single-temperature run)."""
        x = np.array(p0, dtype=float)
        Niter = int(Niter)
        thin = max(1, int(thin))
        isave = max(thin, int(isave))
        nrec = 0
        mode = "w"
        if self.resume and os.path.exists(self.fname) and os.path.getsize(self.fname) > 0:
            prev = np.atleast_2d(np.loadtxt(self.fname))
            x = prev[-1, : self.ndim].copy()
            nrec = len(prev)
            i0 = nrec * thin
            mode = "a"
            cpath = os.path.join(self.outDir, "cov.npy")
            if os.path.exists(cpath):
                self.cov = np.load(cpath)
                self._set_group_covs()
        nbuf = max(1, min(Niter // thin + 1, 100000))
        self._hist = np.zeros((nbuf, self.ndim))
        self._nhist = 0
        lnprob, lnlike = self._lnpost(x)
        naccept, nprop = 0, 0
        rows = []
        fh = None if self.nowrite else open(self.fname, mode)
        try:
            for it in range(i0, Niter):
                cyc = self._cycle(SCAMweight, AMweight, DEweight, with_de=it >= burn and self._nhist >= 2)
                jump = cyc[self.rng.integers(len(cyc))]
                q, lqxy = jump(x, it, 1.0)
                nprop += 1
                if np.all(np.isfinite(q)):
                    lp_new, ll_new = self._lnpost(q)
                    if np.isfinite(lp_new) and np.log(self.rng.uniform()) < lp_new - lnprob + lqxy:
                        x, lnprob, lnlike = q, lp_new, ll_new
                        naccept += 1
                if (it + 1) % thin == 0:
                    self._hist[self._nhist % nbuf] = x
                    self._nhist = min(self._nhist + 1, nbuf)
                    rows.append(np.concatenate([x, [lnprob, lnlike, naccept / nprop, 0.0]]))
                if covUpdate and (it + 1) % int(covUpdate) == 0 and self._nhist > 2 * self.ndim:
                    H = self._hist[: self._nhist][-min(self._nhist, 1000):]
                    c = np.cov(H.T) + 1e-20 * np.eye(self.ndim)
                    if np.all(np.isfinite(c)):
                        self.cov = c
                        self._set_group_covs()
                if fh is not None and rows and ((it + 1) % isave == 0 or it + 1 == Niter):
                    np.savetxt(fh, np.array(rows))
                    fh.flush()
                    rows = []
                    np.save(os.path.join(self.outDir, "cov.npy"), self.cov)
                if maxIter is not None and it + 1 >= maxIter:
                    break
        finally:
            if fh is not None:
                if rows:
                    np.savetxt(fh, np.array(rows))
                fh.close()
        self.acceptance_rate = naccept / max(nprop, 1)
        if self.verbose:
            print(f"PTSampler: {nprop} proposals, acceptance {self.acceptance_rate:.3f}")
        return x


def setup_sampler(pta, outdir="chains", resume=False, empirical_distr=None, groups=None, human=None,
                  save_ext_dists=False, loglkwargs=None, logpkwargs=None, seed=None):
    """enterprise_extensions model_utils.setup_sampler, restated: parameter
    groups, a diagonal initial covariance (0.1^2; 0.01^2 for nmodel as the
    HyperModel uses), pars.txt / priors.txt in outdir, and the default prior-
    draw jumps (all parameters, red noise, DM, common process)."""
    names = list(pta.param_names)
    ndim = len(names)
    cov = np.diag(np.ones(ndim) * 0.1 ** 2)
    groups = get_parameter_groups(pta) if groups is None else groups
    sampler = PTSampler(ndim, pta.get_lnlikelihood, pta.get_lnprior, cov, groups=groups, outDir=outdir,
                        resume=resume, loglkwargs=loglkwargs, logpkwargs=logpkwargs, seed=seed)
    os.makedirs(outdir, exist_ok=True)
    np.savetxt(os.path.join(outdir, "pars.txt"), names, fmt="%s")
    with open(os.path.join(outdir, "priors.txt"), "w") as fh:
        for p in pta.params:
            fh.write(f"{p!r}\n")
    jp = JumpProposal(pta, empirical_distr=empirical_distr, seed=seed)
    sampler.jp = jp
    sampler.addProposalToCycle(jp.draw_from_prior, 5)
    if any("_red_noise_" in n for n in names):
        sampler.addProposalToCycle(jp.draw_from_red_prior, 10)
    if any("_dm_gp_" in n for n in names):
        sampler.addProposalToCycle(jp.draw_from_dm_gp_prior, 10)
    if any(n.startswith("gw_") for n in names):
        sampler.addProposalToCycle(jp.draw_from_gwb_prior, 10)
    if "nmodel" in names:
        sampler.addProposalToCycle(jp.draw_from_nmodel_prior, 25)
    return sampler
