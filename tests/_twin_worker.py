"""Subprocess body of tests/test_cpu_twin.py: runs with EWARP_BACKEND=cpu,
so enterprise_warp_amd binds the host twin libewarp_cpu.so (the ctypes
binding is process-global).  Prints one JSON object."""
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, HERE)


def main():
    from conftest import GOLDEN_NAMES, check_accuracy, load_golden
    from enterprise_warp_amd import _lib
    assert _lib.LIB_PATH.endswith("libewarp_cpu.so"), _lib.LIB_PATH
    out = {"lib": os.path.basename(_lib.LIB_PATH), "goldens": {}, "refused": {}}
    for name in GOLDEN_NAMES:
        pta, z = load_golden(name, full=True)
        try:
            got = pta.get_lnlikelihood_batch(z["theta"])
        except _lib.EngineError as e:
            out["refused"][name] = str(e)
            continue
        r = check_accuracy(got, z["lnl"], z["lnl_exact"], name + " (cpu twin)", near=z["near"],
                           per_sample=name == "c2_small")
        out["goldens"][name] = r
    # in-place white noise (ewh_set_fixed_white) == a PTA built with those constants
    pta, X, _, _ = load_golden("c3_small")
    const = pta.constant_values()
    rng = np.random.default_rng(5)
    new = {k: (v * rng.uniform(0.95, 1.05) if k.endswith("_efac") else v + rng.uniform(-0.2, 0.2))
           for k, v in const.items() if k.endswith(("_efac", "_log10_tnequad", "_log10_ecorr"))}
    before = pta.get_lnlikelihood_batch(X)
    pta.set_default_params(new)
    got = pta.get_lnlikelihood_batch(X)
    fresh, _, _, _ = load_golden("c3_small")
    fresh.set_default_params(new)
    out["set_fixed_white_equal"] = bool(np.array_equal(fresh.get_lnlikelihood_batch(X), got))
    out["set_fixed_white_changed"] = bool(not np.array_equal(got, before))
    # unit terms sum to lnL in pulsar order
    terms = pta.engine().unit_terms(len(X))
    out["unit_terms_sum_ok"] = bool(np.allclose(terms.sum(axis=0), got, rtol=1e-13, atol=1e-8))
    # the device entries are refused
    try:
        pta.engine().lnl_units_device(0, len(X), 0, 1, 0, 0)
        out["device_entry_refused"] = False
    except _lib.EngineError:
        out["device_entry_refused"] = True
    print("TWIN_JSON " + json.dumps(out))


if __name__ == "__main__":
    main()
