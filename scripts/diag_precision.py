"""Where does the device's fp64 rounding enter?  (dev library: EWARP_HIP_LIB=
enterprise_warp_amd/libewarp_hip_dev.so).  For golden samples, compares the
device's Gram G = T_aug^T N^-1 T_aug (varying white noise) / cached reduced
matrix S_p (fixed) with numpy's fp64 and extended-precision ones, and
re-evaluates lnL in extended precision from the device's own G / S_p: if
that lands on the device's lnL, the Gram / Schur step carries the error; if
on the exact value, the per-sample factorisation does."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
os.environ.setdefault("EWARP_HIP_LIB", os.path.join(ROOT, "enterprise_warp_amd", "libewarp_hip_dev.so"))

import numpy as np  # noqa: E402

from conftest import load_golden  # noqa: E402
import oracle.device_order_ref as D  # noqa: E402


def lnl_from_G(dop, i, G, p):
    """device-order lnL of pulsar i from a given (m+1)^2 Gram G (in dop's dtype)."""
    dt = dop.dt
    pp = dop.pulsars[i]
    nl = dop.nlead[i]
    m = pp.T.shape[1]
    Sr, logdet, ok = D.lead_schur(G.astype(dt), nl, np.full(nl, D.TM_PHI, dtype=dt))
    return Sr, logdet


def main(names, samples):
    for nm in names:
        pta, z = load_golden(nm, full=True)
        const = pta.constant_values()
        fixed = const if pta.white_fixed() else None
        psrs = [c.psr for c in pta.signal_collections]
        dld = D.DeviceOrderPTA(psrs, pta.oracle_terms(), fixed, np.longdouble)
        eng = pta.engine()
        got = pta.get_lnlikelihood_batch(z["theta"])
        for s in samples:
            x = z["theta"][s]
            d = dict(const)
            d.update(pta.map_params(x))
            pl = D._cast(d, np.longdouble)
            print(f"{nm}[{s}] gpu-exact {got[s] - z['lnl_exact'][s]:+.3e}  ent-exact {z['lnl'][s] - z['lnl_exact'][s]:+.3e}"
                  f"  dev64-exact {z['lnl_dev'][s] - z['lnl_exact'][s]:+.3e}")
            if fixed is None:
                Gg = eng.dev_gram(0, x)[0]
                m = pta.signal_collections[0].T.shape[1]
                ld = Gg.shape[0]
                idx = list(range(m)) + [ld - 1]
                Gg = Gg[np.ix_(idx, idx)]
                Gl, _ = D.gram(dld.pulsars[0], pl, np.longdouble)
                G6, _ = D.gram(dld.pulsars[0], D._cast(d, np.float64), np.float64)
                sc = 1 / np.sqrt(np.abs(np.diag(Gl).astype(float)))
                rel_g = np.max(np.abs((Gg - Gl.astype(float)) * sc[:, None] * sc[None, :]))
                rel_6 = np.max(np.abs((G6 - Gl.astype(float)) * sc[:, None] * sc[None, :]))
                # lnL (extended precision) from the GPU's G
                orig = D.gram
                D.gram = lambda pp, p, dt, G=Gg, ldn=orig(dld.pulsars[0], pl, np.longdouble)[1]: (G.astype(dt), ldn)
                try:
                    lg = D.DeviceOrderPTA(psrs, pta.oracle_terms(), None, np.longdouble).lnlikelihood(d)
                finally:
                    D.gram = orig
                print(f"   G scaled max|gpu-exact| {rel_g:.2e}   numpy fp64 {rel_6:.2e};  "
                      f"lnL(ext, from gpu G) - exact {lg - z['lnl_exact'][s]:+.3e}")
            else:
                for i in range(len(psrs)):
                    S_ld, K_ld, _, own, _, _ = dld.cache[i]
                    n = S_ld.shape[0]
                    Sg, Kg = eng.dev_reduced(i, n)
                    sc = 1 / np.sqrt(np.abs(np.diag(S_ld).astype(float)))
                    rel = np.max(np.abs((Sg - S_ld.astype(float)) * sc[:, None] * sc[None, :]))
                    print(f"   psr {i}: S_p scaled max|gpu-exact| {rel:.2e}, K gpu-exact {Kg - float(K_ld):+.3e}")


if __name__ == "__main__":
    main(sys.argv[1].split(","), [int(v) for v in sys.argv[2].split(",")])
