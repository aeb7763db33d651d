"""Seeded synthetic pulsar timing arrays for the BASELINE.json configurations.

There is no network and no tempo2, so every dataset is synthetic (except
config 1, which reads the TOAs, errors, frequencies and flags of the
reference's example pulsar J1832-0836; a copy of that data file lives in
tests/golden/ref_examples/).  Residuals are drawn from the model itself at a
"truth" parameter point, so likelihood values are realistic.

Configurations:
  C1  J1832-0836 example pulsar, EFAC/EQUAD by backend, red + DM power laws
  C2  1 pulsar x 10,000 TOAs, ECORR, red + DM (30 freqs), varying white noise
  C3  45 pulsars, n = linspace(2000, 20000), ECORR, red + DM (30), CURN gw
      (vary_gamma_14_nfreqs, merged with red noise), FIXED white noise
  C4  30 pulsars, n = linspace(1000, 12000), 6 backends, no ECORR, red + DM +
      one band-noise term (30 each) + CURN 14, varying white noise
"""
from types import SimpleNamespace

import numpy as np

from . import constants as const
from .models import StandardModels
from .pta import PTA
from .pulsar import Pulsar
from .signals import TimingModel

MJD0 = 53000.0


def make_pulsar(name, n_toa, tspan_yr=14.7, seed=0, n_backends=4, epoch_size=16, n_tm=12,
                sigma_range_us=(0.1, 3.0), freq_range=(700.0, 3500.0), pos=None):
    """Synthetic pulsar: epochs of `epoch_size` TOAs (channels) from one
    backend, within 0.15 s of each other (one ECORR epoch each), spread
    uniformly over `tspan_yr` (default 14.7 yr: an integer number of years
    would put Fourier mode Tspan/yr exactly on the yearly astrometric
    timing-model column and make Sigma singular for loud red noise); log-uniform radio frequencies and TOA errors;
    an n_tm-column linear timing model; residuals zero (see simulate)."""
    rng = np.random.default_rng(seed)
    n_ep = max(1, n_toa // epoch_size)
    span = tspan_yr * const.yr
    t_ep = np.sort(rng.uniform(0.0, span, n_ep))
    t_ep[0], t_ep[-1] = 0.0, span                      # every pulsar spans the full baseline
    sizes = np.full(n_ep, min(epoch_size, n_toa))
    sizes[-1] += n_toa - sizes.sum()
    be = rng.integers(0, n_backends, n_ep)
    toas, backend = [], []
    for t, s, b in zip(t_ep, sizes, be):
        toas.append(MJD0 * const.day + t + 0.01 * np.arange(s))
        backend.extend([b] * s)
    toas = np.concatenate(toas)
    backend = np.array(backend)
    n = len(toas)
    freqs = np.exp(rng.uniform(np.log(freq_range[0]), np.log(freq_range[1]), n))
    errs = np.exp(rng.uniform(np.log(sigma_range_us[0]), np.log(sigma_range_us[1]), n)) * 1e-6
    band = np.where(freqs > 2000, "10CM", np.where(freqs > 1000, "20CM", "40CM"))
    group = np.array([f"BE{b}" for b in backend])
    flags = {"group": group, "B": band, "be": group}
    t = (toas - toas.mean()) / (toas.max() - toas.min())
    ph = 2 * np.pi * toas / const.yr
    nu2 = (1400.0 / freqs) ** 2
    cols = [np.ones(n), t, t ** 2, np.sin(ph), np.cos(ph), t * np.sin(ph), t * np.cos(ph), np.cos(2 * ph),
            nu2, nu2 * t, nu2 * t ** 2]
    for b in range(1, n_backends):
        cols.append((backend == b).astype(float))
    while len(cols) < n_tm:
        cols.append(np.sin((len(cols) + 1) * ph / 7.0))
    M = np.array(cols[:n_tm]).T
    if pos is None:
        v = rng.standard_normal(3)
        pos = v / np.linalg.norm(v)
    return Pulsar(name, toas, np.zeros(n), errs, freqs, flags=flags, Mmat=M, pos=pos)


def params_namespace(Tspan, fixed_white, **over):
    """Stand-in for an enterprise_warp Params model block (priors + Tspan)."""
    ns = SimpleNamespace(**StandardModels().priors)
    ns.Tspan = Tspan
    ns.fref = 1400.0
    ns.opts = None
    if fixed_white:
        ns.efac, ns.equad, ns.ecorr = -1.0, -1.0, -1.0
    ns.__dict__.update(over)
    return ns


def build_pta(psrs, per_psr_terms, common_terms, ns, noisedict=None):
    """init_pta's assembly (enterprise_warp.py:453-500) without a paramfile."""
    allm = StandardModels(psr=psrs, params=ns)
    m_all = TimingModel()
    for term, opt in common_terms.items():
        m_all = m_all + getattr(allm, term)(option=opt)
    models = []
    for psr in psrs:
        sm = StandardModels(psr=psr, params=ns)
        m = m_all
        for term, opt in per_psr_terms.items():
            m = m + getattr(sm, term)(option=opt)
        models.append(m(psr))
    pta = PTA(models)
    if noisedict:
        pta.set_default_params(noisedict)
    return pta


def white_noisedict(psrs, seed, ecorr=True, equad=True):
    rng = np.random.default_rng(seed)
    d = {}
    for p in psrs:
        for b in np.unique(p.backend_flags):
            d[f"{p.name}_{b}_efac"] = float(rng.uniform(0.8, 1.3))
            if equad:
                d[f"{p.name}_{b}_log10_tnequad"] = float(rng.uniform(-7.5, -6.5))
            if ecorr:
                d[f"{p.name}_{b}_log10_ecorr"] = float(rng.uniform(-7.2, -6.3))
    return d


def truth_values(pta, seed, white=None):
    """A realistic parameter point: red / DM / band amplitudes 1e-14..1e-13,
    gw 10^-14.3 with gamma 13/3, white noise from `white` or mid-prior."""
    rng = np.random.default_rng(seed)
    v = dict(pta.constant_values())
    if white:
        v.update(white)
    for p in pta.params:
        n = p.name
        if n in v and v[n] is not None:
            continue
        if n.endswith("efac"):
            v[n] = float(rng.uniform(0.9, 1.2))
        elif n.endswith("log10_tnequad"):
            v[n] = float(rng.uniform(-7.5, -6.5))
        elif n.endswith("log10_ecorr"):
            v[n] = float(rng.uniform(-7.2, -6.3))
        elif n == "gw_log10_A":
            v[n] = -14.3
        elif n == "gw_gamma":
            v[n] = 13.0 / 3.0
        elif n.endswith("log10_A"):
            v[n] = float(rng.uniform(-14.5, -13.0))
        elif n.endswith("gamma"):
            v[n] = float(rng.uniform(2.0, 5.0))
        elif n.endswith("fc"):
            v[n] = -8.5
        elif n.endswith("log10_rho"):
            v[n] = np.full(p.size, -7.0)
        else:
            v[n] = float(p.sample(rng))
    return v


def simulate_residuals(pta, values, seed):
    """Draw residuals from the model at `values` (white + ECORR + every GP
    column with phi from its spectra; timing-model columns get no signal)."""
    rng = np.random.default_rng(seed)
    for c in pta.signal_collections:
        psr = c.psr
        n = len(psr.toas)
        D = np.zeros(n)
        for w in c.white:
            for key, m in w.masks.items():
                val = values[w.pars[key].name]
                if w.kind == "efac":
                    D[m] += val ** 2 * psr.toaerrs[m] ** 2
                elif w.kind == "tnequad":
                    D[m] += 10 ** (2 * val)
        r = np.sqrt(D) * rng.standard_normal(n)
        for s0, s1, p in c.ecorr_epochs():
            r[s0:s1] += 10 ** values[p.name] * rng.standard_normal()
        phi = np.zeros(c.T.shape[1])
        for j, ents in enumerate(c.entries):
            for e in ents:
                if e["kind"] == "const" or e.get("common"):
                    continue
                vals = {k: values[p.name] if p.value is None else p.value for k, p in e["pars"].items()}
                if e["kind"] == "free_spectrum":
                    phi[j] += 10 ** (2 * np.atleast_1d(vals["log10_rho"])[e["mode"]])
                else:
                    phi[j] += _spec_single(e["kind"], e["f"], e["df"], vals)
        r += c.T @ (np.sqrt(phi) * rng.standard_normal(len(phi)))
        psr.residuals = r
    if pta.correlated():
        # the common process: per column g, coefficients ~ N(0, Gamma phi_c(g))
        # across pulsars (Gamma from the ORF; a singular Gamma, e.g. HD
        # without auto terms, falls back to its eigen-square-root)
        cl = pta.common_layout()
        w, V = np.linalg.eigh(cl["orf"])
        Lg = V * np.sqrt(np.clip(w, 0, None))[None, :]
        cols = [c.common["cols"] for c in pta.signal_collections]
        for g, e in enumerate(pta.signal_collections[0].common["entries"]):
            vals = {k: values[p.name] if p.value is None else p.value for k, p in e["pars"].items()}
            if e["kind"] == "free_spectrum":
                ph = 10 ** (2 * np.atleast_1d(vals["log10_rho"])[e["mode"]])
            else:
                ph = _spec_single(e["kind"], e["f"], e["df"], vals)
            z = Lg @ rng.standard_normal(len(cols)) * np.sqrt(ph)
            for a, c in enumerate(pta.signal_collections):
                c.psr.residuals = c.psr.residuals + c.T[:, cols[a][g]] * z[a]
    pta._drop_engine()


def _spec_single(kind, f, df, vals):
    if kind == "powerlaw":
        return (10 ** vals["log10_A"]) ** 2 / 12.0 / np.pi ** 2 * const.fyr ** (vals["gamma"] - 3) * f ** (
            -vals["gamma"]) * df
    if kind == "turnover":
        fc = vals["fc"]
        fc = 10 ** fc if fc < 0 else fc
        return (10 ** vals["log10_A"]) ** 2 / 12.0 / np.pi ** 2 * const.fyr ** (-3) * ((f + fc) / const.fyr) ** (
            -vals["gamma"]) * df
    raise ValueError(kind)


def prior_draws(pta, B, seed):
    """B samples from the priors, [B, nparam] in param_names order."""
    rng = np.random.default_rng(seed)
    cols = []
    for p in pta.params:
        d = p.prior._defaults
        size = p.size or 1
        if p.type == "uniform":
            cols.append(rng.uniform(d["pmin"], d["pmax"], (B, size)))
        else:
            cols.append(np.array([np.atleast_1d(p.sample(rng)) for _ in range(B)]))
    return np.hstack(cols)


def near_draws(pta, values, B, seed, scale=0.3):
    """B samples around `values` (Gaussian, clipped to the prior)."""
    rng = np.random.default_rng(seed)
    X = np.empty((B, len(pta.param_names)))
    c = 0
    for p in pta.params:
        size = p.size or 1
        centre = np.atleast_1d(values[p.name])
        d = p.prior._defaults
        x = centre[None, :] + scale * rng.standard_normal((B, size)) * (0.1 if p.name.endswith("efac") else 1.0)
        if p.type == "uniform":
            x = np.clip(x, d["pmin"], d["pmax"])
        X[:, c:c + size] = x
        c += size
    return X


# ----------------------------------------------------------------------------
# configurations
# ----------------------------------------------------------------------------
def config_c2(seed=2, n_toa=10000, fixed_white=False, epoch_size=16):
    psr = make_pulsar("J0000+0002", n_toa, seed=seed, epoch_size=epoch_size)
    ns = params_namespace(psr.toas.max() - psr.toas.min(), fixed_white)
    wn = white_noisedict([psr], seed + 1)
    terms = {"efac": "by_backend", "equad": "by_backend", "ecorr": "by_backend",
             "spin_noise": "powerlaw_30_nfreqs", "dm_noise": "powerlaw_30_nfreqs"}
    pta = build_pta([psr], terms, {}, ns, wn if fixed_white else None)
    truth = truth_values(pta, seed + 2, white=wn)
    simulate_residuals(pta, truth, seed + 3)
    return SimpleNamespace(name="C2", pta=pta, truth=truth, B=4096, theta_seed=4096)


def c3_pulsars(n_psr=45, n_min=2000, n_max=20000, seed=45, epoch_size=16):
    rng = np.random.default_rng(seed)
    ns_ = np.round(np.linspace(n_min, n_max, n_psr)).astype(int)
    out = []
    for i, n in enumerate(ns_):
        v = rng.standard_normal(3)
        out.append(make_pulsar(f"J{i:04d}+{seed:04d}", int(n), seed=seed * 1000 + i, pos=v / np.linalg.norm(v),
                               epoch_size=epoch_size))
    return out


def config_c3(n_psr=45, n_min=2000, n_max=20000, seed=45, epoch_size=16):
    psrs = c3_pulsars(n_psr, n_min, n_max, seed, epoch_size)
    Tspan = max(p.toas.max() for p in psrs) - min(p.toas.min() for p in psrs)
    ns = params_namespace(Tspan, True)
    wn = white_noisedict(psrs, seed + 1)
    terms = {"efac": "by_backend", "equad": "by_backend", "ecorr": "by_backend",
             "spin_noise": "powerlaw_30_nfreqs", "dm_noise": "powerlaw_30_nfreqs"}
    pta = build_pta(psrs, terms, {"gwb": "vary_gamma_14_nfreqs"}, ns, wn)
    truth = truth_values(pta, seed + 2, white=wn)
    simulate_residuals(pta, truth, seed + 3)
    return SimpleNamespace(name="C3", pta=pta, truth=truth, B=4096, theta_seed=seed)


def config_c4(n_psr=30, n_min=1000, n_max=12000, seed=30, epoch_size=16):
    rng = np.random.default_rng(seed)
    psrs = []
    for i, n in enumerate(np.round(np.linspace(n_min, n_max, n_psr)).astype(int)):
        v = rng.standard_normal(3)
        psrs.append(make_pulsar(f"J{i:04d}-{seed:04d}", int(n), seed=seed * 1000 + i, n_backends=6,
                                pos=v / np.linalg.norm(v), epoch_size=epoch_size))
    Tspan = max(p.toas.max() for p in psrs) - min(p.toas.min() for p in psrs)
    ns = params_namespace(Tspan, False)
    terms = {"efac": "by_backend", "equad": "by_backend", "spin_noise": "powerlaw_30_nfreqs",
             "dm_noise": "powerlaw_30_nfreqs", "ppta_band_noise": ["20CM_30_nfreqs"]}
    pta = build_pta(psrs, terms, {"gwb": "vary_gamma_14_nfreqs"}, ns, None)
    wn = white_noisedict(psrs, seed + 1, ecorr=False)
    truth = truth_values(pta, seed + 2, white=wn)
    simulate_residuals(pta, truth, seed + 3)
    return SimpleNamespace(name="C4", pta=pta, truth=truth, B=1024, theta_seed=seed)


def config_c5(n_psr=100, n_toa=20000, seed=100, epoch_size=16, gwb="hd_vary_gamma_14_nfreqs", nfreqs=30,
              fixed_white=True):
    """BASELINE config 5: n_psr x n_toa PTA, fixed white noise + ECORR, red and
    DM noise, and a Hellings-Downs correlated GWB (cross-pulsar Sigma).
    fixed_white=False: efac / equad / ecorr sampled (enterprise_models.py:
    108-146 stacked under the correlated process, :390-403)."""
    rng = np.random.default_rng(seed)
    psrs = []
    for i in range(n_psr):
        v = rng.standard_normal(3)
        psrs.append(make_pulsar(f"J{i:04d}+{seed:04d}", int(n_toa), seed=seed * 1000 + i, pos=v / np.linalg.norm(v),
                                epoch_size=epoch_size))
    Tspan = max(p.toas.max() for p in psrs) - min(p.toas.min() for p in psrs)
    ns = params_namespace(Tspan, fixed_white)
    wn = white_noisedict(psrs, seed + 1)
    terms = {"efac": "by_backend", "equad": "by_backend", "ecorr": "by_backend",
             "spin_noise": f"powerlaw_{nfreqs}_nfreqs", "dm_noise": f"powerlaw_{nfreqs}_nfreqs"}
    pta = build_pta(psrs, terms, {"gwb": gwb}, ns, wn if fixed_white else None)
    truth = truth_values(pta, seed + 2, white=wn)
    simulate_residuals(pta, truth, seed + 3)
    return SimpleNamespace(name="C5", pta=pta, truth=truth, B=512, theta_seed=seed, terms=terms,
                           common={"gwb": gwb})


def config_c1(data_dir, noise_json=None, seed=1832):
    """data_dir: a copy of the reference's examples/ tree (tests/golden/ref_examples)."""
    """The reference's example pulsar (examples/data/J1832-0836.{par,tim},
    examples/example_params/default_model_dynesty.dat +
    default_noise_example_1.json): efac + equad by backend, red + DM power
    laws with the tobs_60days frequency rule; residuals drawn at the
    example noise file's values (examples/example_noisefiles)."""
    import json
    import os
    from .pulsar import pulsar_from_par_tim
    psr = pulsar_from_par_tim(os.path.join(data_dir, "data", "J1832-0836.par"),
                              os.path.join(data_dir, "data", "J1832-0836.tim"))
    ns = params_namespace(psr.toas.max() - psr.toas.min(), False)
    terms = {"efac": "by_backend", "equad": "by_backend", "spin_noise": "powerlaw", "dm_noise": "powerlaw"}
    pta = build_pta([psr], terms, {}, ns, None)
    noise_json = noise_json or os.path.join(data_dir, "example_noisefiles", "J1832-0836_noise.json")
    with open(noise_json) as fh:
        nd = json.load(fh)
    truth = {k.replace("_log10_equad", "_log10_tnequad"): v for k, v in nd.items()}
    simulate_residuals(pta, truth, seed)
    return SimpleNamespace(name="C1", pta=pta, truth=truth, B=64, theta_seed=seed)


def config_wide(fixed_white, n_toa=10000, nfreqs=60, seed=60):
    """A basis past every register kernel at a realistic size: one pulsar of
    10k TOAs with red / DM / chromatic noise at 60 frequencies each
    (X_60_nfreqs, enterprise_models.py:148-167; the reference's own
    determine_nfreqs gives its fake_psr_0 60, :457-462): 12 + 360 columns,
    24 blocks.  White noise fixed (the cached Gram) or sampled."""
    psr = make_pulsar("J0000+0060", n_toa, seed=seed, epoch_size=16)
    terms = {"efac": "by_backend", "equad": "by_backend", "ecorr": "by_backend",
             "spin_noise": f"powerlaw_{nfreqs}_nfreqs", "dm_noise": f"powerlaw_{nfreqs}_nfreqs",
             "chromred": f"4_{nfreqs}_nfreqs"}
    wn = white_noisedict([psr], seed + 1)
    ns = params_namespace(psr.toas.max() - psr.toas.min(), fixed_white)
    pta = build_pta([psr], terms, {}, ns, wn if fixed_white else None)
    truth = truth_values(pta, seed + 2, white=wn)
    simulate_residuals(pta, truth, seed + 3)
    return SimpleNamespace(name="wide", pta=pta, truth=truth, B=1024, theta_seed=seed + 5, terms=terms)


def config_system(data_dir, seed=8):
    """The reference's system_noise_example.dat / system_noise_example.json on
    J1832-0836 (data_dir: a copy of its examples/ tree): efac / equad fixed,
    spin + DM noise, system noise on the PDFB_40CM and CASPSR_40CM groups,
    band noise on 10CM (enterprise_models.py:256-338) -- 13 blocks with fixed
    white noise.  The model of the golden fixture c1_system."""
    c1 = config_c1(data_dir)
    psr = c1.pta.signal_collections[0].psr
    ns = params_namespace(np.ptp(psr.toas), True)
    terms = {"efac": "by_backend", "equad": "by_backend", "spin_noise": "powerlaw", "dm_noise": "powerlaw",
             "system_noise": ["PDFB_40CM", "CASPSR_40CM"], "ppta_band_noise": ["10CM"]}
    wn = {k: v for k, v in c1.truth.items() if k.endswith("_efac") or k.endswith("_log10_tnequad")}
    pta = build_pta([psr], terms, {}, ns, wn)
    truth = truth_values(pta, seed, white=wn)
    simulate_residuals(pta, truth, seed + 1)
    return SimpleNamespace(name="system", pta=pta, truth=truth, B=4096, theta_seed=19, terms=terms)
