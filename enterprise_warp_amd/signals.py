"""Signal (noise / GW term) factories with enterprise's composition idiom.

`StandardModels` (models.py) builds terms exactly where the reference calls
enterprise's factories (enterprise_models.py:116-117, :129-130, :144-145,
:186-187, :206-209, :248-252, :279-284, :325-330, :401-419) and
`init_pta` adds them (`tm + common + per-psr`, enterprise_warp.py:453-500).

An unbound `Signal` is applied to a `Pulsar` to give a bound term; a
`SignalModel` (sum of Signals) applied to a Pulsar gives a
`SignalCollection`, which holds what the likelihood engine needs:

* the basis T (timing model first, then GP bases in model order) with
  identical columns merged and their phi contributions summed, as
  [ent] SignalCollection._combine_basis_columns / get_phi do;
* per column, the list of spectral entries (kind, parameters, f, df);
* the white-noise tables (efac / log10_tnequad per TOA, ECORR epochs).

Parameter naming follows enterprise: `{psr}_{signal}_{selection key}_{par}`
with empty parts dropped; explicitly named parameters keep their name.
"""
import numpy as np

from . import constants as const
from . import parameter as parameter
from .selections import Selection, no_selection


# ----------------------------------------------------------------------------
# spectra
# ----------------------------------------------------------------------------
class Spectrum:
    def __init__(self, kind, params, components=2):
        self.kind = kind
        self.params = params          # local name -> ParameterSpec | Parameter | float
        self.components = int(components)


def powerlaw(log10_A=-16.0, gamma=5.0, components=2):
    """[ent] utils.powerlaw (enterprise_models.py:180, :200, :267, :382)."""
    return Spectrum("powerlaw", {"log10_A": log10_A, "gamma": gamma}, components)


def powerlaw_bpl(log10_A=-16.0, gamma=5.0, fc=-9.0, components=2):
    """The reference's turnover power law (enterprise_models.py:553-563)."""
    return Spectrum("turnover", {"log10_A": log10_A, "gamma": gamma, "fc": fc}, components)


def free_spectrum(log10_rho=None):
    """[ent] gp_priors.free_spectrum (enterprise_models.py:388)."""
    return Spectrum("free_spectrum", {"log10_rho": log10_rho}, 2)


def spectrum_values(kind, f, vals, components=2):
    """Host evaluation of a spectrum (for checks and the bridge; the device
    evaluates the same formulas in spec_phi)."""
    if kind == "powerlaw":
        df = np.diff(np.concatenate((np.array([0]), f[::components])))
        return ((10 ** vals["log10_A"]) ** 2 / 12.0 / np.pi ** 2 * const.fyr ** (vals["gamma"] - 3)
                * f ** (-vals["gamma"]) * np.repeat(df, components))
    if kind == "turnover":
        df = np.diff(np.concatenate((np.array([0]), f[::components])))
        fc = vals["fc"]
        if fc < 0:
            fc = 10 ** fc
        return ((10 ** vals["log10_A"]) ** 2 / 12.0 / np.pi ** 2 * const.fyr ** (-3)
                * ((f + fc) / const.fyr) ** (-vals["gamma"]) * np.repeat(df, components))
    if kind == "free_spectrum":
        return np.repeat(10 ** (2 * np.asarray(vals["log10_rho"], dtype=float)), 2)
    raise ValueError(kind)


# ----------------------------------------------------------------------------
# bases
# ----------------------------------------------------------------------------
class BasisSpec:
    def __init__(self, kind, nmodes, Tspan=None, fref=1400.0, idx=4.0):
        self.kind = kind
        self.nmodes = int(nmodes)
        self.Tspan = Tspan
        self.fref = fref
        self.idx = idx


def createfourierdesignmatrix_red(nmodes=30, Tspan=None):
    return BasisSpec("fourier", nmodes, Tspan)


def createfourierdesignmatrix_dm(nmodes=30, Tspan=None, fref=1400.0):
    """[ent] gp_bases.createfourierdesignmatrix_dm (enterprise_models.py:206-208)."""
    return BasisSpec("dm", nmodes, Tspan, fref=float(fref))


def createfourierdesignmatrix_chromatic(nmodes=30, Tspan=None, idx=4.0):
    """[ent] gp_bases.createfourierdesignmatrix_chromatic (enterprise_models.py:248-250):
    F * (1400 / nu)^idx.  A sampled idx (chromred 'vary') makes the basis
    theta-dependent: its columns are never merged and are rescaled per
    sample on the device (contraction kernels)."""
    if isinstance(idx, (int, float, np.floating, np.integer)):
        idx = float(idx)
    return BasisSpec("chromatic", nmodes, Tspan, idx=idx)


def fourier_matrix(toas, nmodes, Tspan):
    """[ent] gp_bases.createfourierdesignmatrix_red: F[:, 2j] = sin, F[:, 2j+1] = cos."""
    f = 1.0 * np.arange(1, nmodes + 1) / Tspan
    F = np.zeros((len(toas), 2 * nmodes))
    F[:, ::2] = np.sin(2 * np.pi * toas[:, None] * f[None, :])
    F[:, 1::2] = np.cos(2 * np.pi * toas[:, None] * f[None, :])
    return F, np.repeat(f, 2)


def build_basis(spec, toas, freqs):
    """Basis of one GP on the selected TOAs; a sampled chromatic index leaves
    the Fourier columns unscaled (scaled per sample on the device)."""
    Ts = spec.Tspan if spec.Tspan is not None else toas.max() - toas.min()
    F, Ff = fourier_matrix(toas, spec.nmodes, Ts)
    if spec.kind == "dm":
        F = F * ((float(spec.fref) / freqs) ** 2)[:, None]
    elif spec.kind == "chromatic" and isinstance(spec.idx, float):
        F = F * ((1400.0 / freqs) ** spec.idx)[:, None]
    return F, Ff, Ts


def normed_tm_basis(M):
    """[ent] utils.normed_tm_basis (gp_signals.TimingModel, enterprise_warp.py:453-454)."""
    norm = np.sqrt(np.sum(M ** 2, axis=0))
    with np.errstate(divide="ignore", invalid="ignore"):
        nmat = M / norm
    nmat[:, norm == 0] = 0
    return nmat


def _pname(*parts):
    return "_".join(p for p in parts if p)


# ----------------------------------------------------------------------------
# unbound signals and their sums
# ----------------------------------------------------------------------------
class Signal:
    signal_type = "base"

    def __add__(self, other):
        return SignalModel([self]) + other

    def __radd__(self, other):
        return SignalModel([other]) + self

    def __call__(self, psr):
        raise NotImplementedError


class SignalModel:
    def __init__(self, signals):
        self.signals = []
        for s in signals:
            self.signals.extend(s.signals if isinstance(s, SignalModel) else [s])

    def __add__(self, other):
        if other is None:
            return SignalModel(self.signals)
        return SignalModel(self.signals + (other.signals if isinstance(other, SignalModel) else [other]))

    def __call__(self, psr):
        bound = []
        for s in self.signals:
            b = s(psr)
            if b is not None:
                bound.append(b)
        return SignalCollection(psr, bound)


class TimingModel(Signal):
    """[ent] gp_signals.TimingModel(normed=True): basis M/|M|, phi = 1e40."""
    signal_type = "basis"

    def __call__(self, psr):
        return _BoundTM(psr)


class _BoundTM:
    kind = "timing_model"

    def __init__(self, psr):
        self.F = normed_tm_basis(np.asarray(psr.Mmat, dtype=float))
        self.params = []

    def spec(self):
        return {"kind": "timing_model"}


class _White(Signal):
    signal_type = "white noise"

    def __init__(self, kind, prior, selection):
        self.kind, self.prior = kind, prior
        self.selection = selection if selection is not None else Selection(no_selection)

    def __call__(self, psr):
        return _BoundWhite(self, psr)


_WHITE_PAR = {"efac": "efac", "tnequad": "log10_tnequad", "ecorr": "log10_ecorr"}


class _BoundWhite:
    def __init__(self, sig, psr):
        self.kind = sig.kind
        self.selection_name = sig.selection.name
        masks = sig.selection.masks(psr)
        self.masks = {k: masks[k] for k in sorted(masks)}
        par = _WHITE_PAR[sig.kind]
        self.pars = {k: parameter.resolve(sig.prior, _pname(psr.name, k, par)) for k in self.masks}
        self.params = list(self.pars.values())

    def spec(self):
        return {"kind": self.kind, "selection": self.selection_name}


def MeasurementNoise(efac=None, selection=None, name=""):
    """[ent] white_signals.MeasurementNoise: N += efac^2 sigma^2 (enterprise_models.py:117)."""
    return _White("efac", efac if efac is not None else parameter.Uniform(0.5, 1.5), selection)


def TNEquadNoise(log10_tnequad=None, selection=None, name=""):
    """[ent] white_signals.TNEquadNoise: N += 10^(2 q) (enterprise_models.py:130)."""
    return _White("tnequad", log10_tnequad if log10_tnequad is not None else parameter.Uniform(-10, -5), selection)


def EcorrKernelNoise(log10_ecorr=None, selection=None, name=""):
    """[ent] white_signals.EcorrKernelNoise, Sherman-Morrison form (enterprise_models.py:145)."""
    return _White("ecorr", log10_ecorr if log10_ecorr is not None else parameter.Uniform(-10, -5), selection)


class _GP(Signal):
    signal_type = "basis"

    def __init__(self, spectrum, basis, name, selection=None, orf=None):
        self.spectrum, self.basis, self.name = spectrum, basis, name
        self.selection = selection if selection is not None else Selection(no_selection)
        self.orf = orf

    def __call__(self, psr):
        return _BoundGP(self, psr)


class _BoundGP:
    kind = "gp"

    def __init__(self, sig, psr):
        self.name = sig.name
        self.spectrum = sig.spectrum
        self.basis_spec = sig.basis
        self.orf = sig.orf          # None, or the ORF of a correlated common process
        masks = sig.selection.masks(psr)
        self.sel_flag = getattr(sig.selection.func, "flag", None)
        self.sel_value = getattr(sig.selection.func, "value", None)
        toas = np.asarray(psr.toas, float)
        freqs = np.asarray(psr.freqs, float)
        self.parts = []
        self.params = []
        for key in sorted(masks):
            mask = masks[key]
            if not np.any(mask):
                raise ValueError(f"{psr.name}: selection '{key}' of signal {sig.name} selects no TOA")
            Fm, Ff, Ts = build_basis(sig.basis, toas[mask], freqs[mask])
            F = np.zeros((len(toas), Fm.shape[1]))
            F[mask] = Fm
            pars, explicit = {}, {}
            for loc, val in sig.spectrum.params.items():
                explicit[loc] = isinstance(val, parameter.Parameter)
                p = parameter.resolve(val, _pname(psr.name, sig.name, key, loc))
                if sig.spectrum.kind == "free_spectrum" and (p.size or 1) != Fm.shape[1] // 2:
                    raise ValueError(f"{p.name}: size {p.size} != number of frequencies {Fm.shape[1] // 2}")
                pars[loc] = p
            bpar = None
            if sig.basis.kind == "chromatic" and not isinstance(sig.basis.idx, float):
                bpar = parameter.resolve(sig.basis.idx, _pname(psr.name, sig.name, key, "idx"))
                self.params.append(bpar)
            self.parts.append({"key": key, "F": F, "f": Ff, "Tspan": Ts, "pars": pars, "explicit": explicit,
                               "basis_par": bpar})
            self.params.extend(pars.values())

    def spec(self):
        out = []
        b = self.basis_spec
        for part in self.parts:
            d = {"kind": "gp", "name": self.name, "basis": b.kind, "nfreqs": b.nmodes, "Tspan": part["Tspan"],
                 "fref": float(b.fref), "idx": float(b.idx) if part["basis_par"] is None else None, "spectrum": self.spectrum.kind,
                 "components": self.spectrum.components, "pnames": {}, "const": {},
                 "selection": None if self.sel_flag is None else {"flag": self.sel_flag, "value": self.sel_value}}
            for loc, p in part["pars"].items():
                if isinstance(p, parameter.ConstantParameter) and p.value is not None:
                    d["const"][loc] = p.value
                elif part["explicit"][loc]:
                    d["pnames"][loc] = p.name
            if part["basis_par"] is not None:
                d["idx_param"] = part["basis_par"].name
            if self.orf is not None:
                d["orf"] = self.orf
            out.append(d)
        return out


def FourierBasisGP(spectrum, components=20, Tspan=None, name="red_noise", selection=None):
    """[ent] gp_signals.FourierBasisGP (enterprise_models.py:186, :279, :325, :418)."""
    return _GP(spectrum, createfourierdesignmatrix_red(components, Tspan), name, selection)


def BasisGP(spectrum, basis, name="basis_gp", selection=None):
    """[ent] gp_signals.BasisGP (enterprise_models.py:209, :252)."""
    return _GP(spectrum, basis, name, selection)


def FourierBasisCommonGP(spectrum, orf, components=20, Tspan=None, name="common_fourier"):
    """[ent] gp_signals.FourierBasisCommonGP (enterprise_models.py:401-415)."""
    return _GP(spectrum, createfourierdesignmatrix_red(components, Tspan), name, None, orf=orf)


class _Deterministic(Signal):
    def __init__(self, what):
        self.what = what

    def __call__(self, psr):
        raise NotImplementedError(f"{self.what}: deterministic delay signals are out of scope "
                                  "(SURVEY.md §2 row 2: bayes_ephem needs ephemeris data)")


def PhysicalEphemerisSignal(**kw):
    return _Deterministic("PhysicalEphemerisSignal")


# ----------------------------------------------------------------------------
# per-pulsar collection
# ----------------------------------------------------------------------------
class SignalCollection:
    """Bound model of one pulsar ([ent] signal_base.SignalCollection)."""

    def __init__(self, psr, bound):
        self.psr = psr
        self.name = psr.name
        self.bound = bound
        n = len(psr.toas)
        cols = []          # merged basis columns
        entries = []       # per column: list of entry dicts
        by_hash = {}       # column bytes -> candidate indices (same result as a linear np.array_equal scan)
        self.col_bgroup_map = {}   # column -> chromatic-index Parameter (theta-dependent basis)
        self.common = None         # correlated common process: {"name", "orf", "cols", "entries"}
        self.gp_cols = {}          # GP signal name -> its (merged) column indices, in basis order
        self.gp_entries = {}       # GP signal name -> its spectral entries, same order
        self.n_tm = 0
        seen_gp = False

        def add(column, entry):
            key = np.ascontiguousarray(column).tobytes()
            for j in by_hash.get(key, ()):
                if np.array_equal(column, cols[j]):
                    entries[j].append(entry)
                    return j
            cols.append(column)
            entries.append([entry])
            by_hash.setdefault(key, []).append(len(cols) - 1)
            return len(cols) - 1

        for b in bound:
            if isinstance(b, _BoundTM):
                if seen_gp:
                    raise ValueError("the timing model must come first (tm + ..., enterprise_warp.py:466-497)")
                for j in range(b.F.shape[1]):
                    add(b.F[:, j], {"kind": "const", "value": const.TM_PRIOR_VARIANCE})
            elif isinstance(b, _BoundGP):
                seen_gp = True
                comp = b.spectrum.components
                if b.orf is not None:
                    if self.common is not None:
                        raise NotImplementedError(f"{psr.name}: more than one correlated common process")
                    if len(b.parts) != 1 or b.parts[0]["basis_par"] is not None:
                        raise NotImplementedError("a correlated common process must be one unselected Fourier basis")
                    self.common = {"name": b.name, "orf": b.orf, "cols": [], "entries": []}
                for part in b.parts:
                    f = part["f"]
                    df = np.repeat(np.diff(np.concatenate((np.array([0]), f[::comp]))), comp)
                    for j in range(part["F"].shape[1]):
                        e = {"kind": b.spectrum.kind, "pars": part["pars"], "f": f[j], "df": df[j], "mode": j // 2}
                        if b.orf is not None:
                            # [ent] FourierBasisCommonGP: phi(a, a) = orf(a, a) phi_c on the
                            # merged column; cross-pulsar terms in the PTA's common block
                            e["common"] = True
                            self.common["cols"].append(add(part["F"][:, j], e))
                            self.common["entries"].append(e)
                        elif part["basis_par"] is None:
                            col = add(part["F"][:, j], e)
                            self.gp_cols.setdefault(b.name, []).append(col)
                            self.gp_entries.setdefault(b.name, []).append(e)
                        else:   # theta-dependent basis: own column, never merged
                            cols.append(part["F"][:, j])
                            entries.append([e])
                            self.col_bgroup_map[len(cols) - 1] = part["basis_par"]
        self.T = np.array(cols).T if cols else np.zeros((n, 0))
        self.entries = entries
        # theta-dependent basis groups: one per chromatic-index parameter
        self.basis_groups = []
        self.col_bgroup = np.full(len(cols), -1, np.int32)
        for j, p in sorted(self.col_bgroup_map.items()):
            names = [q.name for q in self.basis_groups]
            if p.name not in names:
                self.basis_groups.append(p)
            self.col_bgroup[j] = [q.name for q in self.basis_groups].index(p.name)
        self.ln_chrom = np.log(1400.0 / np.asarray(psr.freqs, float))
        # leading columns whose phi is constant (timing model): eliminated once when white noise is fixed
        nl = 0
        while nl < len(entries) and all(e["kind"] == "const" for e in entries[nl]):
            nl += 1
        self.n_lead_const = nl
        self.white = [b for b in bound if isinstance(b, _BoundWhite)]
        if not any(w.kind == "efac" for w in self.white):
            raise ValueError(f"{psr.name}: model has no MeasurementNoise (efac) term; the white-noise "
                             "covariance would not include the TOA errors")
        for kind in ("efac", "tnequad", "ecorr"):
            if sum(w.kind == kind for w in self.white) > 1:
                raise NotImplementedError(f"{psr.name}: more than one {kind} term")
        # params (free + constant), unique by name, in enterprise's name order
        allp = {}
        for b in bound:
            for p in b.params:
                allp.setdefault(p.name, p)
        self.all_params = [allp[k] for k in sorted(allp)]

    @property
    def params(self):
        return [p for p in self.all_params if not isinstance(p, parameter.ConstantParameter)]

    def oracle_terms(self):
        """Plain-dict term specs for the CPU oracle (tests only)."""
        out = []
        for b in self.bound:
            s = b.spec()
            out.extend(s if isinstance(s, list) else [s])
        return out

    def ecorr_epochs(self):
        """ECORR epochs as (start, stop, Parameter): per selection key (sorted),
        quantise the key's TOAs ([ent] utils.create_quantization_matrix, dt =
        1 s, nmin = 2) and require contiguous TOA slices ([ent] quant2ind)."""
        out = []
        for w in self.white:
            if w.kind != "ecorr":
                continue
            toas = np.asarray(self.psr.toas, float)
            for key, mask in w.masks.items():
                idx = np.flatnonzero(mask)
                if len(idx) == 0:
                    continue
                for bucket in quantize(toas[idx]):
                    ep = np.sort(idx[bucket])
                    if ep[-1] - ep[0] + 1 != len(ep):
                        raise ValueError(f"{self.name}: ECORR epoch is not a contiguous TOA slice "
                                         "(enterprise quant2ind: 'slice does not work')")
                    out.append((int(ep[0]), int(ep[-1]) + 1, w.pars[key]))
        out.sort(key=lambda x: x[0])
        return out


def quantize(toas, dt=1.0, nmin=2):
    """[ent] utils.create_quantization_matrix bucket rule (returns index lists)."""
    isort = np.argsort(toas, kind="mergesort")
    buckets, ref = [[isort[0]]], toas[isort[0]]
    for i in isort[1:]:
        if toas[i] - ref < dt:
            buckets[-1].append(i)
        else:
            ref = toas[i]
            buckets.append([i])
    return [np.array(b) for b in buckets if len(b) >= nmin]
