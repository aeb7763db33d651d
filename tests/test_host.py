"""CPU tests of the host layer: paramfile semantics, term library, parameter
naming / ordering, basis merging, engine tables, bilby bridge, sharding."""
import os

import numpy as np
import pytest

from conftest import REF_EXAMPLES, load_golden
from enterprise_warp_amd import parameter, sharding, synth, warp
from enterprise_warp_amd.bilby_bridge import get_bilby_prior_dict
from enterprise_warp_amd.selections import backend_flags


@pytest.fixture
def in_examples(monkeypatch):
    monkeypatch.chdir(REF_EXAMPLES)


def test_paramfile_default_model(in_examples):
    """examples/example_params/default_model_dynesty.dat + default_noise_example_1.json."""
    P = warp.Params("example_params/default_model_dynesty.dat", opts=None)
    assert P.sampler == "dynesty" and P.sampler_kwargs == {"dlogz": 0.1, "nlive": 800}
    assert P.array_analysis == "False" and len(P.psrs) == 1 and P.psrs[0].name == "J1832-0836"
    assert P.models[0].model_name == "examp_1"
    pta = warp.init_pta(P)[0]
    bk = ["CASPSR_40CM", "PDFB_10CM", "PDFB_20CM", "PDFB_40CM"]   # -group flags of the .tim
    want = sorted([f"J1832-0836_{b}_efac" for b in bk] + [f"J1832-0836_{b}_log10_tnequad" for b in bk] +
                  ["J1832-0836_red_noise_log10_A", "J1832-0836_red_noise_gamma", "J1832-0836_dm_gp_log10_A",
                   "J1832-0836_dm_gp_gamma"])
    assert pta.param_names == want
    c = pta.signal_collections[0]
    assert c.n_lead_const == 16                  # offset + 10 fitted params + 5 fitted JUMPs
    assert c.T.shape[1] == 16 + 2 * 32 + 2 * 32  # nfreqs 32 from tobs_60days (enterprise_models.py:462)
    pr = {p.name: p.prior._defaults for p in pta.params}
    assert pr["J1832-0836_PDFB_10CM_efac"] == {"pmin": 0.0, "pmax": 10.0}
    assert pr["J1832-0836_red_noise_log10_A"] == {"pmin": -20.0, "pmax": -6.0}


def test_paramfile_fixed_white_noise(in_examples):
    """efac/equad: -1 -> Constants filled from example_noisefiles, including the
    `_log10_equad` -> `_log10_tnequad` alias."""
    P = warp.Params("example_params/fixed_white_noise.dat", opts=None)
    ptas = warp.init_pta(P)
    assert sorted(ptas) == [0, 1]
    p0, p1 = ptas[0], ptas[1]
    assert p0.param_names == ["J1832-0836_dm_gp_gamma", "J1832-0836_dm_gp_log10_A", "J1832-0836_red_noise_gamma",
                              "J1832-0836_red_noise_log10_A"]
    assert "J1832-0836_red_noise_fc" in p1.param_names          # spin_noise: turnover
    assert p0.white_fixed()
    cv = p0.constant_values()
    assert cv["J1832-0836_PDFB_10CM_efac"] == pytest.approx(1.0691290656558021)
    assert cv["J1832-0836_PDFB_10CM_log10_tnequad"] == pytest.approx(-6.2326037554799)
    lay = p0.layout()[0]
    assert all(idx < 0 for idx, _ in lay["slots"])


def test_paramfile_system_noise(in_examples):
    P = warp.Params("example_params/system_noise_example.dat", opts=None)
    pta = warp.init_pta(P)[0]
    names = pta.param_names
    assert "J1832-0836_system_noise_0_PDFB_40CM_log10_A" in names
    assert "J1832-0836_system_noise_1_CASPSR_40CM_gamma" in names
    assert "J1832-0836_band_noise_2_10CM_log10_A" in names
    c = pta.signal_collections[0]
    mask = c.psr.flags["B"] == "10CM"
    # band-noise columns vanish outside the band's TOAs
    band_cols = [j for j, es in enumerate(c.entries) if any("band_noise_2" in e["pars"]["log10_A"].name
                                                             for e in es if e["kind"] == "powerlaw")]
    assert band_cols and np.all(c.T[~mask][:, band_cols] == 0)


def test_universal_white_noise_quirk(in_examples):
    """The examples' `universal: {"white_noise": ...}` names no StandardModels
    method: a pulsar without its own entry fails, as
    in the reference."""
    P = warp.Params("example_params/default_model_dynesty.dat", opts=None)
    P.psrs[0].name = "J0711-0000"
    with pytest.raises(AttributeError):
        warp.init_pta(P)


def test_backend_flag_ranking():
    flags = {"group": np.array(["A", "", ""]), "g": np.array(["x", "y", ""]), "fe": np.array(["", "", "L"]),
             "be": np.array(["", "", "P"])}
    assert list(backend_flags(flags, 3)) == ["A", "y", "L_P"]
    assert list(backend_flags({}, 2)) == ["flag", "flag"]


def test_curn_columns_merge_with_red_noise():
    """CURN (gw, 14 freqs, global Tspan) shares the red-noise Fourier columns:
    m = 12 + 60 + 60 and the 28 shared columns carry two phi entries
    ([ent] SignalCollection._combine_basis_columns)."""
    c = synth.config_c3(n_psr=2, n_min=800, n_max=900).pta.signal_collections[0]
    assert c.T.shape[1] == 132 and c.n_lead_const == 12
    nent = [len(e) for e in c.entries]
    assert sum(1 for k in nent if k == 2) == 28
    gw = [e for es in c.entries for e in es if e["kind"] == "powerlaw" and e["pars"]["log10_A"].name == "gw_log10_A"]
    assert len(gw) == 28


def test_param_order_and_map_params():
    pta, X, _, _ = load_golden("c3_small")
    assert pta.param_names == sorted(pta.param_names)
    d = pta.map_params(X[0])
    assert np.array_equal(pta._theta(d)[0], X[0])
    assert "gw_log10_A" in d and "gw_gamma" in d


def test_lnprior():
    pta, X, _, _ = load_golden("c1_j1832")
    lp = pta.get_lnprior(X[0])
    want = sum(-np.log(p.prior._defaults["pmax"] - p.prior._defaults["pmin"]) for p in pta.params)
    assert lp == pytest.approx(want)
    x = X[0].copy()
    x[0] = 1e9
    assert pta.get_lnprior(x) == -np.inf


def test_constant_without_value_raises():
    c = synth.config_c3(n_psr=2, n_min=600, n_max=700)
    pta = c.pta
    for p in pta._all.values():
        if isinstance(p, parameter.ConstantParameter):
            p.value = None
            break
    with pytest.raises(ValueError, match="has no value"):
        pta.layout()


def test_engine_tables():
    """Engine tables: every TOA has an efac slot, epochs are ordered disjoint
    slices of >= 2 TOAs, every column has a phi entry, timing-model columns
    are CONST 1e40."""
    pta, _, _, _ = load_golden("c2_small")
    L = pta.layout()[0]
    assert np.all(L["efac"] >= 0)
    assert np.all(L["ep_stop"] - L["ep_start"] >= 2)
    assert np.all(L["ep_start"][1:] >= L["ep_stop"][:-1])
    cols = {e[1] for e in L["spec"]}
    assert cols == set(range(L["T"].shape[1]))
    tm = [e for e in L["spec"] if e[1] < L["n_lead"]]
    assert all(e[0] == 4 and e[2] == (-1, 1e40) for e in tm)


def test_bilby_prior_dict():
    pta, _, _, _ = load_golden("c3_small")
    pri = get_bilby_prior_dict(pta)
    assert list(pri) == pta.param_names
    s = pri["gw_gamma"].sample(5)
    assert np.all((s >= 0) & (s <= 10))


@pytest.mark.parametrize("world", [1, 2, 3, 8])
def test_unit_ranges_cover_and_balance(world):
    costs = np.array([1.0, 3.0, 2.0, 5.0, 1.0])
    B = 1000
    r = sharding.unit_ranges(costs, B, world)
    assert r[0][0] == 0 and r[-1][1] == len(costs) * B
    assert all(a[1] == b[0] for a, b in zip(r, r[1:]))
    per = []
    for u0, u1 in r:
        u = np.arange(u0, u1)
        per.append(costs[u // B].sum())
    assert max(per) <= (costs.sum() * B / world) + costs.max() + 1e-9


def test_bundle_roundtrip(tmp_path):
    from enterprise_warp_amd.pulsar import load_bundle, save_bundle
    p = synth.make_pulsar("J1234+5678", 300, seed=3)
    save_bundle(p, tmp_path / "p.npz")
    q = load_bundle(tmp_path / "p.npz")
    assert q.name == p.name and np.array_equal(q.toas, p.toas) and np.array_equal(q.Mmat, p.Mmat)
    assert np.array_equal(q.backend_flags, p.backend_flags)


def test_extra_model_terms_merge():
    d1 = {"J1": {"efac": "by_backend", "system_noise": ["A"]}}
    d2 = {"J1": {"system_noise": ["B"]}, "J2": {"efac": "by_backend"}}
    out = warp.merge_two_noise_model_dicts(d1, d2)
    assert out["J1"]["system_noise"] == ["A", "B"] and out["J2"] == {"efac": "by_backend"}


def test_hd_layout_puts_common_columns_last():
    """Correlated common process: each pulsar's device layout is [timing
    model | own columns | common columns in frequency order]; the common
    signal's phi goes to the PTA-level descriptor with the ORF matrix."""
    from enterprise_warp_amd.models import hd_orf
    c5 = synth.config_c5(n_psr=3, n_toa=300, seed=9, epoch_size=4, gwb="hd_vary_gamma_5_nfreqs", nfreqs=10)
    pta = c5.pta
    assert pta.correlated()
    cl = pta.common_layout()
    assert cl["n_col"] == 10 and cl["kind"] == "hd"
    pos = [c.psr.pos for c in pta.signal_collections]
    assert cl["orf"][0, 0] == 1.0 and np.isclose(cl["orf"][0, 1], hd_orf(pos[0], pos[1]))
    for c, L in zip(pta.signal_collections, pta.layout()):
        m = L["T"].shape[1]
        assert L["n_common"] == 10
        np.testing.assert_array_equal(L["T"][:, m - 10:], c.T[:, c.common["cols"]])
        np.testing.assert_array_equal(L["T"][:, :L["n_lead"]], c.T[:, :L["n_lead"]])
        # red noise merged onto the common columns stays in the pulsar's table
        assert sum(1 for e in L["spec"] if e[1] >= m - 10) == 10


class _MockPTA:
    """Minimal PTA surface (params, param_names, batch lnL / lnprior) with an
    analytic Gaussian likelihood, for the host-side HyperModel / sampler."""

    def __init__(self, names, mu, sig=0.5):
        from enterprise_warp_amd import parameter
        self.params = [parameter.Uniform(-10, 10)(n) for n in names]
        self.param_names = list(names)
        self.mu, self.sig = np.asarray(mu, float), sig

    def get_lnlikelihood_batch(self, X):
        X = np.atleast_2d(X)
        return -0.5 * np.sum((X - self.mu) ** 2, axis=1) / self.sig ** 2

    def get_lnlikelihood(self, x):
        return float(self.get_lnlikelihood_batch(np.asarray(x))[0])

    def get_lnprior_batch(self, X):
        X = np.atleast_2d(X)
        return np.where(np.all(np.abs(X) <= 10, axis=1), -len(self.param_names) * np.log(20.0), -np.inf)

    def get_lnprior(self, x):
        return float(self.get_lnprior_batch(np.asarray(x))[0])


def test_hypermodel_routes_by_nmodel():
    """enterprise_extensions HyperModel semantics (run_example_paramfile.py:31-45):
    union of parameter names in first-appearance order + nmodel; only the
    active model's likelihood; batch == single calls."""
    from enterprise_warp_amd.hypermodel import HyperModel
    a = _MockPTA(["a", "shared"], [1.0, 2.0])
    b = _MockPTA(["shared", "b"], [3.0, -1.0])
    hm = HyperModel([a, b])
    assert hm.param_names == ["a", "shared", "b", "nmodel"]
    X = np.array([[1.0, 2.0, 0.0, 0.2], [0.0, 3.0, -1.0, 0.9], [0.0, 3.0, -1.0, 1.4], [0, 0, 0, 2.0]])
    got = hm.get_lnlikelihood_batch(X)
    assert got[0] == a.get_lnlikelihood([1.0, 2.0]) and got[1] == b.get_lnlikelihood([3.0, -1.0])
    assert got[2] == got[1] and got[3] == -np.inf
    np.testing.assert_array_equal([hm.get_lnlikelihood(x) for x in X[:3]], got[:3])
    lp = hm.get_lnprior_batch(X)
    assert np.isfinite(lp[:3]).all() and lp[3] == -np.inf
    assert lp[0] == hm.get_lnprior(X[0])


def test_batched_sampler_recovers_gaussian(tmp_path):
    from enterprise_warp_amd.sampler import BatchedMH
    m = _MockPTA(["x", "y"], [1.5, -2.0], sig=0.3)
    s = BatchedMH(m, nchains=64, outdir=str(tmp_path), seed=3, adapt_every=50)
    X, post, like = s.sample(niter=400, thin=50)
    H = np.concatenate(s.history[200:])
    np.testing.assert_allclose(H.mean(axis=0), [1.5, -2.0], atol=0.05)
    np.testing.assert_allclose(H.std(axis=0), [0.3, 0.3], rtol=0.15)
    rows = np.loadtxt(tmp_path / "chain_1.txt")
    assert rows.shape == (64 * 8, 2 + 4)
