"""TEST INFRASTRUCTURE ONLY — numpy/scipy restatement of enterprise's PTA lnL.

See oracle/__init__.py for the parity status ("parity unpinned" against
enterprise itself; pinned by known-answer tests and the dense cross-check).

Every function names the enterprise v3.x routine it restates ([ent] = the
third-party `enterprise` package, PyPI `enterprise-pulsar`, unpinned, absent
from /root/reference) and the enterprise_warp call site that reaches it.

Input model: per pulsar, a list of *term specs* (plain dicts, in model order:
timing model first, then common signals, then per-pulsar signals, as
enterprise_warp.init_pta assembles them at enterprise_warp.py:453-500):

  {"kind": "timing_model"}
  {"kind": "efac"|"tnequad"|"ecorr", "selection": "by_backend"|"no_selection"}
  {"kind": "gp", "name": str, "basis": "fourier"|"dm"|"chromatic",
   "nfreqs": int, "Tspan": float, "fref": float, "idx": float,
   "spectrum": "powerlaw"|"turnover"|"free_spectrum", "components": 2,
   "idx_param": name (chromatic basis with a sampled index),
   "pnames": {local: global name} (explicitly named parameters, e.g. gw_*),
   "const": {local: value}, "selection": None | {"flag": f, "value": v}}

Parameter values are looked up by their enterprise names (Appendix A.7 of
SURVEY.md) in a flat dict that also carries the Constant values.
"""
import numpy as np
import scipy.linalg as sl

DAY = 86400.0                      # [ent] constants.day = scipy.constants.day
YR = 365.25 * DAY                  # [ent] constants.yr  = scipy.constants.Julian_year
FYR = 1.0 / YR                     # [ent] constants.fyr


# --------------------------------------------------------------------------
# overlap reduction functions ([ent] utils.hd_orf / monopole_orf / dipole_orf;
# hd_orf_noauto from the reference, enterprise_models.py:565-572)
# --------------------------------------------------------------------------
def orf_value(kind, pos1, pos2):
    same = np.all(pos1 == pos2)
    if kind in ("hd", "hd_noauto"):
        if same:
            return 1.0 if kind == "hd" else 0.0
        omc2 = (1 - np.dot(pos1, pos2)) / 2
        return 1.5 * omc2 * np.log(omc2) - 0.25 * omc2 + 0.5
    if kind == "monopole":
        return 1.0 + 1e-5 if same else 1.0
    if kind == "dipole":
        return 1.0 + 1e-5 if same else float(np.dot(pos1, pos2))
    raise ValueError(kind)


# --------------------------------------------------------------------------
# bases and spectra
# --------------------------------------------------------------------------
def fourier_basis(toas, nmodes, Tspan):
    """[ent] gp_bases.createfourierdesignmatrix_red (no logf / fmin / modes).

    Called through gp_signals.FourierBasisGP from enterprise_models.py:186,
    :279, :325, :418.  Columns 2j = sin, 2j+1 = cos, f_j = j/Tspan."""
    f = 1.0 * np.arange(1, nmodes + 1) / Tspan
    F = np.zeros((len(toas), 2 * nmodes))
    F[:, ::2] = np.sin(2 * np.pi * toas[:, None] * f[None, :])
    F[:, 1::2] = np.cos(2 * np.pi * toas[:, None] * f[None, :])
    return F, np.repeat(f, 2)


def dm_basis(toas, freqs, nmodes, Tspan, fref=1400.0):
    """[ent] gp_bases.createfourierdesignmatrix_dm (enterprise_models.py:206-208)."""
    F, Ff = fourier_basis(toas, nmodes, Tspan)
    return F * ((fref / freqs) ** 2)[:, None], Ff


def chromatic_basis(toas, freqs, nmodes, Tspan, idx=4.0):
    """[ent] gp_bases.createfourierdesignmatrix_chromatic (enterprise_models.py:248-250)."""
    F, Ff = fourier_basis(toas, nmodes, Tspan)
    return F * ((1400.0 / freqs) ** idx)[:, None], Ff


def normed_tm_basis(M):
    """[ent] utils.normed_tm_basis via gp_signals.TimingModel (enterprise_warp.py:453-454)."""
    norm = np.sqrt(np.sum(M ** 2, axis=0))
    with np.errstate(divide="ignore", invalid="ignore"):
        nmat = M / norm
    nmat[:, norm == 0] = 0
    return nmat


def powerlaw(f, log10_A, gamma, components=2):
    """[ent] utils.powerlaw (enterprise_models.py:180, :200, :267, :382)."""
    df = np.diff(np.concatenate((np.array([0]), f[::components])))
    return ((10 ** log10_A) ** 2 / 12.0 / np.pi ** 2 * FYR ** (gamma - 3)
            * f ** (-gamma) * np.repeat(df, components))


def powerlaw_bpl(f, log10_A, gamma, fc, components=2):
    """Restates enterprise_models.py:553-563 (the reference's own turnover law)."""
    df = np.diff(np.concatenate((np.array([0]), f[::components])))
    if fc < 0:
        fc = 10 ** fc
    return ((10 ** log10_A) ** 2 / 12.0 / np.pi ** 2 * FYR ** (-3)
            * ((f + fc) / FYR) ** (-gamma) * np.repeat(df, components))


def free_spectrum(f, log10_rho):
    """[ent] gp_priors.free_spectrum (enterprise_models.py:388)."""
    return np.repeat(10 ** (2 * np.asarray(log10_rho, dtype=float)), 2)


# --------------------------------------------------------------------------
# selections and quantisation
# --------------------------------------------------------------------------
def backend_flags(flags, n):
    """[ent] BasePulsar.backend_flags: first present of group, g, sys, i, f, fe+be."""
    out = np.array(["flag"] * n, dtype=object)
    order = [["group"], ["g"], ["sys"], ["i"], ["f"], ["fe", "be"]]
    for i in range(n):
        for fl in order:
            if all(ff in flags and flags[ff][i] != "" for ff in fl):
                out[i] = "_".join(flags[ff][i] for ff in fl)
                break
    return out.astype(str)


def selection_masks(psr, selection):
    """[ent] selections.by_backend / no_selection (enterprise_models.py:113-116)."""
    n = len(psr.toas)
    if selection == "no_selection":
        return {"": np.ones(n, bool)}
    if selection == "by_backend":
        bf = backend_flags(psr.flags, n)
        return {v: bf == v for v in np.unique(bf)}
    raise ValueError(selection)


def quantization_slices(toas, dt=1.0, nmin=2):
    """[ent] utils.create_quantization_matrix + utils.quant2ind.

    Buckets start at a TOA and take every later TOA within dt seconds of the
    bucket's first TOA; buckets with < nmin TOAs are dropped.  Returns index
    lists into `toas`."""
    isort = np.argsort(toas, kind="mergesort")
    ref = [toas[isort[0]]]
    buckets = [[isort[0]]]
    for i in isort[1:]:
        if toas[i] - ref[-1] < dt:
            buckets[-1].append(i)
        else:
            ref.append(toas[i])
            buckets.append([i])
    return [np.array(b) for b in buckets if len(b) >= nmin]


def pname(psr_name, sig_name, key, par):
    """[ent] gp_signals.BasisGP._do_selection / white_signals naming rule."""
    return "_".join(x for x in [psr_name, sig_name, key, par] if x)


# --------------------------------------------------------------------------
# per-pulsar model
# --------------------------------------------------------------------------
class OraclePulsar:
    """Restates [ent] signal_base.SignalCollection for one pulsar."""

    def __init__(self, psr, terms):
        self.psr = psr
        self.name = psr.name
        self.r = np.asarray(psr.residuals, float)
        self.sigma = np.asarray(psr.toaerrs, float)
        n = len(self.r)
        self.white = []        # (kind, {key: mask}, {key: pname})
        self.gps = []          # dict per GP signal
        self.basis_params = []  # (columns, unscaled F, idx parameter name) of theta-dependent bases
        self.has_tm = False
        cols = []              # unique basis columns (SignalCollection._combine_basis_columns)
        for t in terms:
            k = t["kind"]
            if k == "timing_model":
                self.has_tm = True
                Mn = normed_tm_basis(np.asarray(psr.Mmat, float))
                idx = [self._add_cols(cols, Mn[:, j]) for j in range(Mn.shape[1])]
                self.gps.append({"kind": "tm", "idx": idx})
            elif k in ("efac", "tnequad", "ecorr"):
                masks = selection_masks(psr, t.get("selection", "by_backend"))
                par = {"efac": "efac", "tnequad": "log10_tnequad", "ecorr": "log10_ecorr"}[k]
                names = {key: pname(self.name, "", key, par) for key in masks}
                self.white.append((k, masks, names))
            elif k == "gp":
                self.gps.extend(self._gp(t, cols))
            else:
                raise ValueError(k)
        self.T = np.array(cols).T if cols else np.zeros((n, 0))
        # ECORR epochs (white_signals.EcorrKernelNoise, SM form)
        self.ecorr = []
        for k, masks, names in self.white:
            if k != "ecorr":
                continue
            for key in sorted(masks):
                idx = np.flatnonzero(masks[key])
                for b in quantization_slices(self.psr.toas[idx]):
                    ep = np.sort(idx[b])
                    if ep[-1] - ep[0] + 1 != len(ep):
                        raise ValueError("ERROR: slice does not work")  # [ent] quant2ind
                    self.ecorr.append((slice(ep[0], ep[-1] + 1), names[key]))

    def _add_cols(self, cols, c):
        """First earlier identical column, else append ([ent]
        _combine_basis_columns' linear np.array_equal scan, found by hash)."""
        idx = self.__dict__.setdefault("_colhash", {})
        key = np.ascontiguousarray(c).tobytes()
        for j in idx.get(key, ()):
            if np.array_equal(c, cols[j]):
                return j
        cols.append(c)
        idx.setdefault(key, []).append(len(cols) - 1)
        return len(cols) - 1

    def _gp(self, t, cols):
        psr = self.psr
        toas = np.asarray(psr.toas, float)
        n = len(toas)
        sel = t.get("selection")
        if sel is None:
            masks = {"": np.ones(n, bool)}
        else:
            fl = np.asarray(psr.flags[sel["flag"]])
            masks = {sel["value"]: fl == sel["value"]}
        out = []
        for key in sorted(masks):
            mask = masks[key]
            tt = toas[mask]
            nf, Ts = int(t["nfreqs"]), float(t["Tspan"])
            if t["basis"] == "fourier":
                Fm, Ff = fourier_basis(tt, nf, Ts)
            elif t["basis"] == "dm":
                Fm, Ff = dm_basis(tt, np.asarray(psr.freqs)[mask], nf, Ts, float(t.get("fref", 1400.0)))
            elif t["basis"] == "chromatic" and "idx_param" in t:
                # basis depends on theta ([ent] BasisGP with basis_params):
                # columns are appended unmerged and rebuilt on every call
                Fm, Ff = fourier_basis(tt, nf, Ts)
            elif t["basis"] == "chromatic":
                Fm, Ff = chromatic_basis(tt, np.asarray(psr.freqs)[mask], nf, Ts, float(t.get("idx", 4.0)))
            else:
                raise ValueError(t["basis"])
            F = np.zeros((n, Fm.shape[1]))
            F[mask] = Fm
            if "idx_param" in t:
                idx = list(range(len(cols), len(cols) + F.shape[1]))
                cols.extend(F[:, j] for j in range(F.shape[1]))
                self.basis_params.append((idx, F, t["idx_param"]))
            else:
                idx = [self._add_cols(cols, F[:, j]) for j in range(F.shape[1])]
            names = {}
            for p in {"powerlaw": ["log10_A", "gamma"], "turnover": ["log10_A", "gamma", "fc"],
                      "free_spectrum": ["log10_rho"]}[t["spectrum"]]:
                if p in t.get("const", {}):
                    names[p] = ("const", t["const"][p])
                elif p in t.get("pnames", {}):
                    names[p] = ("name", t["pnames"][p])
                else:
                    names[p] = ("name", pname(self.name, t["name"], key, p))
            out.append({"kind": "gp", "idx": idx, "f": Ff, "spectrum": t["spectrum"],
                        "names": names, "components": int(t.get("components", 2)),
                        "orf": t.get("orf"), "name": t["name"]})
        return out

    # ---- parameters -------------------------------------------------------
    @staticmethod
    def _val(params, ref):
        kind, v = ref
        return v if kind == "const" else params[v]

    def white_ndiag(self, params):
        """[ent] MeasurementNoise + TNEquadNoise get_ndiag (enterprise_models.py:117, :130)."""
        n = len(self.r)
        nd = np.zeros(n)
        have_efac = False
        for k, masks, names in self.white:
            if k == "efac":
                have_efac = True
                for key, m in masks.items():
                    nd[m] += params[names[key]] ** 2 * self.sigma[m] ** 2
            elif k == "tnequad":
                for key, m in masks.items():
                    nd[m] += 10 ** (2 * params[names[key]])
        if not have_efac:
            raise ValueError("model has no MeasurementNoise term")
        return nd

    def gp_values(self, g, params):
        """phi of one GP signal on its own columns (before merging)."""
        nm = g["names"]
        if g["spectrum"] == "powerlaw":
            return powerlaw(g["f"], self._val(params, nm["log10_A"]), self._val(params, nm["gamma"]),
                            g["components"])
        if g["spectrum"] == "turnover":
            return powerlaw_bpl(g["f"], self._val(params, nm["log10_A"]), self._val(params, nm["gamma"]),
                                self._val(params, nm["fc"]), g["components"])
        return free_spectrum(g["f"], self._val(params, nm["log10_rho"]))

    def phi(self, params):
        """[ent] SignalCollection.get_phi: per-column sum over merged signals;
        a common (ORF) signal contributes orf(pos, pos) * phi_gw on its columns
        ([ent] FourierBasisCommonGP.get_phi)."""
        phi = np.zeros(self.T.shape[1])
        for g in self.gps:
            if g["kind"] == "tm":
                phi[g["idx"]] += 1e40                      # [ent] utils.tm_prior
                continue
            if g.get("orf"):
                pos = np.asarray(self.psr.pos, float)
                phi[g["idx"]] += orf_value(g["orf"], pos, pos) * self.gp_values(g, params)
                continue
            nm = g["names"]
            if g["spectrum"] == "powerlaw":
                v = powerlaw(g["f"], self._val(params, nm["log10_A"]), self._val(params, nm["gamma"]),
                             g["components"])
            elif g["spectrum"] == "turnover":
                v = powerlaw_bpl(g["f"], self._val(params, nm["log10_A"]), self._val(params, nm["gamma"]),
                                 self._val(params, nm["fc"]), g["components"])
            else:
                v = free_spectrum(g["f"], self._val(params, nm["log10_rho"]))
            phi[g["idx"]] += v
        return phi

    # ---- N^{-1} products (ShermanMorrison) --------------------------------
    def _sm(self, params):
        D = self.white_ndiag(params)
        ep = [(s, 10 ** (2 * params[nm])) for s, nm in self.ecorr]
        return D, ep

    @staticmethod
    def _solve_2D2(D, ep, X, Z):
        """[ent] ShermanMorrison._solve_2D2: X^T N^{-1} Z."""
        ZNX = np.dot(Z.T / D, X)
        for slc, jv in ep:
            if slc.stop - slc.start > 1:
                ni = 1.0 / D[slc]
                beta = 1.0 / (np.sum(ni) + 1.0 / jv)
                zn = np.dot(ni, Z[slc])
                xn = np.dot(ni, X[slc])
                ZNX -= beta * np.outer(zn.T, xn)
        return ZNX

    @staticmethod
    def _solve_1D1(D, ep, x):
        """[ent] ShermanMorrison._solve_1D1 + _get_logdet: r^T N^{-1} r, log|N|."""
        Nx = x / D
        ld = np.sum(np.log(D))
        for slc, jv in ep:
            if slc.stop - slc.start > 1:
                ni = 1.0 / D[slc]
                beta = 1.0 / (np.sum(ni) + 1.0 / jv)
                Nx[slc] -= beta * np.dot(ni, x[slc]) * ni
                ld += np.log(jv) - np.log(beta)
        return np.dot(x, Nx), ld

    @staticmethod
    def _solve_2D1(D, ep, T, x):
        """[ent] ShermanMorrison._solve_D1 then T^T (.): T^T N^{-1} x."""
        Nx = x / D
        for slc, jv in ep:
            if slc.stop - slc.start > 1:
                ni = 1.0 / D[slc]
                beta = 1.0 / (np.sum(ni) + 1.0 / jv)
                Nx[slc] -= beta * np.dot(ni, x[slc]) * ni
        return np.dot(T.T, Nx)

    def basis(self, params):
        """[ent] SignalCollection.get_basis: theta-dependent chromatic columns
        F * (1400 / nu)^idx rebuilt from the current idx."""
        if not self.basis_params:
            return self.T
        T = self.T.copy()
        nu = np.asarray(self.psr.freqs, float)
        for idx, F, pn in self.basis_params:
            T[:, idx] = F * ((1400.0 / nu) ** params[pn])[:, None]
        return T

    def white_terms(self, params):
        """[ent] get_TNT / get_TNr / get_rNr_logdet."""
        D, ep = self._sm(params)
        T = self.basis(params)
        TNT = self._solve_2D2(D, ep, T, T)
        TNr = self._solve_2D1(D, ep, T, self.r)
        rNr, ldN = self._solve_1D1(D, ep, self.r)
        return TNT, TNr, rNr, ldN


class OraclePTA:
    """Restates [ent] signal_base.PTA + LogLikelihood.__call__, reached at
    bilby_warp.py:35: the per-pulsar path (uncorrelated / CURN,
    `pta._commonsignals` empty) and the correlated one (HD / monopole / dipole
    ORF, FourierBasisCommonGP at enterprise_models.py:390-415).

    `fixed_white=True` mimics enterprise's cache_call: TNT / TNr / rNr /
    log|N| are computed once (white-noise parameters are Constants)."""

    def __init__(self, psrs, terms_per_psr, fixed_params=None):
        self.pulsars = [OraclePulsar(p, t) for p, t in zip(psrs, terms_per_psr)]
        self.fixed = None
        if fixed_params is not None and not any(pp.basis_params for pp in self.pulsars):
            self.fixed = [pp.white_terms(fixed_params) for pp in self.pulsars]

    def correlated(self):
        return any(g.get("orf") for pp in self.pulsars for g in pp.gps)

    def phi_global(self, params):
        """[ent] PTA.get_phi for a correlated common signal: block-diagonal
        per-pulsar phi plus Phi[(a, col_a(j)), (b, col_b(j))] = orf(a, b) *
        phi_common(j) for a != b (get_phicross), as one dense matrix."""
        sizes = [pp.T.shape[1] for pp in self.pulsars]
        off = np.concatenate(([0], np.cumsum(sizes)))
        Phi = np.zeros((off[-1], off[-1]))
        for a, pp in enumerate(self.pulsars):
            Phi[np.arange(off[a], off[a + 1]), np.arange(off[a], off[a + 1])] = pp.phi(params)
        commons = {}
        for a, pp in enumerate(self.pulsars):
            for g in pp.gps:
                if g.get("orf"):
                    commons.setdefault(g["name"], []).append((a, g))
        for name, lst in commons.items():
            for a, ga in lst:
                va = self.pulsars[a].gp_values(ga, params)
                for b, gb in lst:
                    if b == a:
                        continue
                    gam = orf_value(ga["orf"], np.asarray(self.pulsars[a].psr.pos, float),
                                    np.asarray(self.pulsars[b].psr.pos, float))
                    ia = off[a] + np.asarray(ga["idx"])
                    ib = off[b] + np.asarray(gb["idx"])
                    Phi[ia, ib] += gam * va
        return Phi, off

    @staticmethod
    def phiinv_cliques(Phi):
        """[ent] PTA.get_phiinv(method='cliques'): invert each connected
        block (clique) of Phi by cho_factor; log|Phi| from the same factors."""
        from scipy.sparse.csgraph import connected_components
        ncomp, lab = connected_components(Phi != 0, directed=False)
        inv = np.zeros_like(Phi)
        logdet = 0.0
        for c in range(ncomp):
            ix = np.flatnonzero(lab == c)
            sub = Phi[np.ix_(ix, ix)]
            if len(ix) == 1:
                inv[ix[0], ix[0]] = 1.0 / sub[0, 0]
                logdet += np.log(sub[0, 0])
            else:
                cf = sl.cho_factor(sub)
                inv[np.ix_(ix, ix)] = sl.cho_solve(cf, np.eye(len(ix)))
                logdet += 2 * np.sum(np.log(np.diag(cf[0])))
        return inv, logdet

    def lnlikelihood_correlated(self, params):
        """[ent] LogLikelihood.__call__ with pta._commonsignals: Sigma =
        block_diag(TNT_a) + Phi^-1 over all pulsars, one dense Cholesky
        (enterprise: sksparse cholesky, scipy dense fallback)."""
        terms = [self.fixed[i] if self.fixed is not None else pp.white_terms(params)
                 for i, pp in enumerate(self.pulsars)]
        loglike = -0.5 * sum(t[2] + t[3] for t in terms)
        Phi, off = self.phi_global(params)
        try:
            phiinv, logdet_phi = self.phiinv_cliques(Phi)
        except sl.LinAlgError:
            return -np.inf
        Sigma = phiinv
        for a, t in enumerate(terms):
            Sigma[off[a]:off[a + 1], off[a]:off[a + 1]] += t[0]
        TNr = np.concatenate([t[1] for t in terms])
        try:
            cf = sl.cho_factor(Sigma)
            expval = sl.cho_solve(cf, TNr)
        except sl.LinAlgError:
            return -np.inf
        logdet_sigma = 2 * np.sum(np.log(np.diag(cf[0])))
        return loglike + 0.5 * (np.dot(TNr, expval) - logdet_sigma - logdet_phi)

    def lnlikelihood(self, params):
        if self.correlated():
            return self.lnlikelihood_correlated(params)
        loglike = 0.0
        rnr_ld = []
        red = 0.0
        for i, pp in enumerate(self.pulsars):
            if self.fixed is not None:
                TNT, TNr, rNr, ldN = self.fixed[i]
            else:
                TNT, TNr, rNr, ldN = pp.white_terms(params)
            rnr_ld.append((rNr, ldN))
            phi = pp.phi(params)
            phiinv, logdet_phi = 1.0 / phi, np.sum(np.log(phi))
            Sigma = TNT + np.diag(phiinv)
            try:
                cf = sl.cho_factor(Sigma)
                expval = sl.cho_solve(cf, TNr)
            except sl.LinAlgError:
                return -np.inf
            logdet_sigma = np.sum(2 * np.log(np.diag(cf[0])))
            red += 0.5 * (np.dot(TNr, expval) - logdet_sigma - logdet_phi)
        loglike += -0.5 * np.sum([ell for ell in rnr_ld])
        loglike += red
        return loglike



# --------------------------------------------------------------------------
# optimal statistic (results.py:653-795 -> enterprise_extensions
# frequentist.optimal_statistic.OptimalStatistic, unpinned, absent)
# --------------------------------------------------------------------------
def optimal_statistic(opta, params, gw_name="gw", orf="hd", gamma=None):
    """Restates enterprise_extensions OptimalStatistic.get_XZ + compute_os on
    the CURN model: per pulsar, with P = N + T phi T^T (the common process
    included, as the noise-marginalised OS of results.py uses the CURN chain),
      X = F^T P^-1 r,  Z = F^T P^-1 F   (F = the common signal's columns),
    then per pair rho_ab = X_a^T phi^ X_b / tr(Z_a phi^ Z_b phi^),
    sig_ab = tr(...)^-1/2 with phi^ the unit-amplitude power law, and
    OS = sum rho Gamma / sig^2 / sum Gamma^2 / sig^2, OS_sig = (sum Gamma^2 / sig^2)^-1/2.
    gamma: params['gw_gamma'] when None (13/3 if absent).  Returns
    (xi, rho, sig, OS, OS_sig) over pairs a < b in row-major order."""
    if gamma is None:
        gamma = params.get("gw_gamma", 13.0 / 3.0)
    Xs, Zs, pos, freqs = [], [], [], None
    for i, pp in enumerate(opta.pulsars):
        TNT, TNr, _, _ = opta.fixed[i] if opta.fixed is not None else pp.white_terms(params)
        phi = pp.phi(params)
        g = next(g for g in pp.gps if g.get("name") == gw_name)
        idx = np.asarray(g["idx"])
        freqs = g["f"]
        Sigma = TNT + np.diag(1.0 / phi)
        cf = sl.cho_factor(Sigma)
        SigmaTNr = sl.cho_solve(cf, TNr)
        FNT = TNT[idx, :]
        SigmaTNF = sl.cho_solve(cf, FNT.T)
        Xs.append(TNr[idx] - FNT @ SigmaTNr)
        Zs.append(TNT[np.ix_(idx, idx)] - FNT @ SigmaTNF)
        pos.append(np.asarray(pp.psr.pos, float))
    phat = powerlaw(freqs, 0.0, gamma, 2)
    xi, rho, sig, G = [], [], [], []
    P = len(Xs)
    for a in range(P):
        for b in range(a + 1, P):
            top = Xs[a] @ (phat * Xs[b])
            bot = np.trace((Zs[a] * phat[None, :]) @ (Zs[b] * phat[None, :]))
            rho.append(top / bot)
            sig.append(1.0 / np.sqrt(bot))
            G.append(orf_value(orf, pos[a], pos[b]))
            xi.append(np.arccos(np.clip(np.dot(pos[a], pos[b]), -1, 1)))
    rho, sig, G, xi = map(np.array, (rho, sig, G, xi))
    OS = np.sum(rho * G / sig ** 2) / np.sum(G ** 2 / sig ** 2)
    return xi, rho, sig, OS, 1.0 / np.sqrt(np.sum(G ** 2 / sig ** 2))
