import json
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(ROOT, "tests", "golden")
REF_EXAMPLES = os.path.join(GOLDEN, "ref_examples")
sys.path.insert(0, ROOT)

# Parity tolerance of the north star (BASELINE.json): 1e-6 absolute / 1e-10
# relative in lnL ("strict").  Near-truth samples (where samplers spend their
# time) and full-size checks are held to strict against the enterprise-order
# oracle.  Prior draws are often so ill-conditioned that the lnL of the fp64
# inputs is not determined to 1e-10 by ANY fp64 ordering (enterprise's own
# LAPACK order misses the exact value by up to 6e5 x strict on
# tests/golden/c2_small); there the GPU is held to ACCURACY: its error
# against a near-exact reference (oracle/ddref.py double-double, or the
# extended-precision, error-free-Gram restatement) must not exceed
# enterprise's own error against it, or strict if that is larger
# (`check_accuracy`).  Independent of the device's own order.
ATOL, RTOL = 1e-6, 1e-10


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device) and libewarp_hip.so")
    config.addinivalue_line("markers", "gpu_ab: kernel A/B variants (dev library libewarp_hip_dev.so, "
                                       "`make -C enterprise_warp_amd/csrc dev`); not part of the driver's -m gpu suite")
    config.addinivalue_line("markers", "gpu_debug: the device-side debug build (build/libewarp_hip_debug.so, "
                                       "`make -C enterprise_warp_amd/csrc debug`); not part of the driver's -m gpu suite")


def pytest_collection_modifyitems(config, items):
    skip = pytest.mark.skip(reason="A/B variant tests need a GPU and the dev library (make dev)")
    for it in items:
        if ("gpu_ab" in it.keywords or "gpu_debug" in it.keywords) and not gpu_available():
            it.add_marker(skip)


def strict_tolerance(ref):
    return ATOL + RTOL * np.abs(np.asarray(ref, dtype=float))


def _finite_pattern(got, want, label):
    got = np.asarray(got, dtype=float)
    want = np.asarray(want, dtype=float)
    assert not np.isnan(got).any(), f"{label}: NaN in GPU lnL at {np.flatnonzero(np.isnan(got))}"
    bad_inf = ~np.isfinite(got) & (got != -np.inf)
    assert not bad_inf.any(), f"{label}: non-finite values other than -inf at {np.flatnonzero(bad_inf)}"
    fin_g, fin_w = np.isfinite(got), np.isfinite(want)
    assert np.array_equal(fin_g, fin_w), \
        f"{label}: -inf pattern differs (gpu -inf at {np.flatnonzero(~fin_g)}, ref -inf at {np.flatnonzero(~fin_w)})"
    return got, want, fin_w


def check_parity(got, want, label):
    """GPU lnL vs a reference at the strict bound: no NaN, every non-finite
    value exactly -inf and exactly where the reference is -inf, finite values
    within 1e-6 + 1e-10 |lnL|.  Prints and returns max err / strict."""
    got, want, fin = _finite_pattern(got, want, label)
    if not fin.any():
        return 0.0
    ratio = np.abs(got[fin] - want[fin]) / strict_tolerance(want[fin])
    print(f"{label}: max err/strict {ratio.max():.3e} over {fin.sum()} samples")
    k = int(np.argmax(ratio))
    assert ratio.max() <= 1.0, f"{label}: {(ratio > 1).sum()} samples outside strict; worst sample " \
                               f"{np.flatnonzero(fin)[k]}: err/strict {ratio[k]:.3e}"
    return float(ratio.max())


def check_accuracy(got, ent, ext, label, near=None, per_sample=False):
    """The parity criterion on prior draws: the GPU is no
    less accurate than enterprise's own fp64 order against the near-exact
    value ext -- max over the samples of |gpu - ext| <= max(max over the
    samples of |ent - ext|, strict) --, per_sample=True: on every sample
    |gpu - ext| <= max(|ent - ext|, strict).  Near-truth samples (near True)
    are held to strict against both references.  The -inf pattern must equal
    the references' exactly; NaN fails.  Prints how many samples the GPU is
    less accurate than enterprise on; returns max |gpu - ext| /
    max(|ent - ext|, strict) over the samples."""
    got, ext, fin = _finite_pattern(got, ext, label + " vs extended")
    ent = np.asarray(ent, dtype=float)
    assert np.array_equal(np.isfinite(ent), fin), f"{label}: the references disagree on -inf"
    if not fin.any():
        return 0.0
    st = strict_tolerance(ext[fin])
    eg = np.abs(got[fin] - ext[fin])
    ee = np.abs(ent[fin] - ext[fin])
    if near is not None:
        nr = np.asarray(near, bool)[fin]
        if nr.any():
            assert np.all(eg[nr] <= st[nr]), f"{label}: near-truth samples outside strict vs the exact value: " \
                                             f"{eg[nr] / st[nr]}"
            en = np.abs(got[fin] - ent[fin])[nr]
            assert np.all(en <= strict_tolerance(ent[fin][nr])), \
                f"{label}: near-truth samples outside strict vs enterprise-order: {en / strict_tolerance(ent[fin][nr])}"
    r = eg / np.maximum(ee, st)
    worse = int(np.sum(r > 1.0))
    print(f"{label}: |gpu-ext|/strict max {np.max(eg / st):.3e}, |ent-ext|/strict max {np.max(ee / st):.3e}; "
          f"samples where the GPU is less accurate than enterprise (beyond strict): {worse} of {fin.sum()} "
          f"(max ratio {r.max():.3f})")
    assert eg.max() <= max(ee.max(), st[int(np.argmax(eg))]), \
        f"{label}: worst GPU error {eg.max():.3e} exceeds enterprise's worst {ee.max():.3e}"
    if per_sample:
        k = int(np.argmax(r))
        assert r.max() <= 1.0, f"{label}: sample {np.flatnonzero(fin)[k]}: GPU error {eg[k]:.3e} exceeds " \
                               f"max(enterprise error {ee[k]:.3e}, strict {st[k]:.3e})"
    return float(r.max())


def oracle_lnl(pta, X):
    """Enterprise-order oracle lnL of every row of X."""
    from oracle.enterprise_ref import OraclePTA
    const = pta.constant_values()
    fixed = const if pta.white_fixed() else None
    o = OraclePTA([c.psr for c in pta.signal_collections], pta.oracle_terms(), fixed_params=fixed)
    out = []
    for x in X:
        d = dict(const)
        d.update(pta.map_params(x))
        out.append(o.lnlikelihood(d))
    return np.array(out)


def reference_lnl(pta, X, exact="auto"):
    """(enterprise-order lnL, near-exact lnL) of every row of X.  exact:
    "dd" -- oracle/ddref.py (double-double, uncorrelated / CURN models),
    "ext" -- the extended-precision restatement with an error-free Gram
    (oracle/device_order_ref.py, np.longdouble), "auto" -- dd when the model
    allows it and the pulsars are few."""
    from oracle.device_order_ref import DeviceOrderPTA
    from oracle.ddref import DDReferencePTA
    from oracle.enterprise_ref import OraclePTA
    const = pta.constant_values()
    fixed = const if pta.white_fixed() else None
    psrs, terms = [c.psr for c in pta.signal_collections], pta.oracle_terms()
    ent = OraclePTA(psrs, terms, fixed_params=fixed)
    if exact == "auto":
        exact = "dd" if not ent.correlated() and len(psrs) <= 4 else "ext"
    ref = DDReferencePTA(psrs, terms) if exact == "dd" else DeviceOrderPTA(psrs, terms, fixed, np.longdouble)
    a, b = [], []
    for x in X:
        d = dict(const)
        d.update(pta.map_params(x))
        a.append(ent.lnlikelihood(d))
        b.append(ref.lnlikelihood(d))
    return np.array(a), np.array(b)


def load_golden(name, full=False):
    """Rebuild (pta, theta, lnl, min_eig) from a committed fixture; full=True
    returns (pta, z) with every stored array (lnl = enterprise order, lnl_dev
    = the device's order in fp64, lnl_exact = near-exact, spread, near)."""
    from enterprise_warp_amd import synth
    from enterprise_warp_amd.pulsar import Pulsar
    z = np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False)
    rec = json.loads(str(z["recipe"]))
    psrs = []
    for i, nm in enumerate(rec["names"]):
        flags = {k: z[f"p{i}_flag_{k}"] for k in rec["flag_names"][i]}
        psrs.append(Pulsar(nm, z[f"p{i}_toas"], z[f"p{i}_residuals"], z[f"p{i}_toaerrs"], z[f"p{i}_freqs"],
                           flags=flags, Mmat=z[f"p{i}_Mmat"], pos=z[f"p{i}_pos"], sort=False))
    ns = synth.params_namespace(rec["Tspan"], rec["fixed_white"])
    pta = synth.build_pta(psrs, rec["per_psr_terms"], rec["common_terms"], ns, rec["noisedict"] or None)
    assert pta.param_names == rec["param_names"]
    if full:
        return pta, {k: z[k] for k in ("theta", "lnl", "lnl_dev", "lnl_exact", "spread", "near", "min_eig")}
    return pta, z["theta"], z["lnl"], z["min_eig"]


GOLDEN_NAMES = ["c1_j1832", "c1_turnover", "c1_system", "c2_small", "c2_chromvary", "c3_small", "c3_freesp",
                "c4_small", "c5_small", "c5_mono", "c5_noauto", "c5_dipo", "c5_varwn", "c1_wide", "c1_widefix"]


def gpu_available():
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:  # noqa: BLE001
        return False


@pytest.fixture(scope="session")
def require_gpu():
    if not gpu_available():
        pytest.fail("this test needs a HIP GPU (run with -m 'not gpu' on CPU-only hosts)")
