"""Diagnostic (dev library): gram_dd_units_kernel's G_hi + G_lo of C4 pulsar
p on prior draws, against the host double-double Gram of the same projected
basis (oracle/ddref.dd_gram), and both factored on the host in double-double
(ddref._factor) -- separates the Gram from chol_dd_kernel.  Run with
EWARP_HIP_LIB=enterprise_warp_amd/libewarp_hip_dev.so."""
import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

if __name__ == "__main__":
    from enterprise_warp_amd import _lib, synth
    from oracle import ddref
    from oracle.device_order_ref import project_coef
    from oracle.enterprise_ref import OraclePTA
    cfg = synth.config_c4()
    pta = cfg.pta
    X = synth.prior_draws(pta, cfg.B, cfg.theta_seed)[:64]
    eng = pta.engine()
    lib = _lib.load()
    lib.ewh_dev_gram_dd.argtypes = [C.c_void_p, C.c_int32, C.POINTER(C.c_double), C.c_int32,
                                    C.POINTER(C.c_double), C.POINTER(C.c_double)]
    const = pta.constant_values()
    o = OraclePTA([c.psr for c in pta.signal_collections], pta.oracle_terms(), fixed_params=None)
    r = ddref.DDReferencePTA([c.psr for c in pta.signal_collections], pta.oracle_terms())
    for s, pi in [(0, 0), (5, 0), (38, None), (1, 0)]:
        d = dict(const)
        d.update(pta.map_params(X[s]))
        pis = [pi] if pi is not None else range(len(o.pulsars))
        for p in pis:
            pp = o.pulsars[p]
            T = np.asarray(pp.T, float)
            m = T.shape[1]
            ld = 16 * ((m + 1 + 15) // 16)
            th = np.ascontiguousarray(X[s:s + 1])
            Gh = np.zeros((1, ld, ld))
            Gl = np.zeros((1, ld, ld))
            rc = lib.ewh_dev_gram_dd(eng.h, p, th.ctypes.data_as(C.POINTER(C.c_double)), 1,
                                     Gh.ctypes.data_as(C.POINTER(C.c_double)), Gl.ctypes.data_as(C.POINTER(C.c_double)))
            assert rc == ld, (rc, lib.ewh_last_error())
            idx = list(range(m)) + [ld - 1]
            Gd = (Gh[0][np.ix_(idx, idx)], Gl[0][np.ix_(idx, idx)])
            Xa = np.concatenate([T, np.asarray(pp.r, float)[:, None]], 1)
            nl = 12
            cols = list(range(nl, m + 1))
            Cc = project_coef(Xa, pp.sigma, nl, cols)
            Xp = Xa.copy()
            Xp[:, cols] = Xa[:, cols] - Xa[:, :nl] @ Cc
            # (the original basis too: the reference's own)
            D = pp.white_ndiag(d)
            w = 1.0 / D
            Ghost = ddref.dd_gram(Xp, (w, np.zeros_like(w)))
            rel = np.abs((Gd[0] - Ghost[0]) + (Gd[1] - Ghost[1])) / np.sqrt(np.outer(np.diag(Ghost[0]), np.diag(Ghost[0])))
            ldn = np.sum(np.log(D))
            vd = r._factor(r.pulsars[p], d, Gd, ldn)
            vh = r._factor(r.pulsars[p], d, Ghost, ldn)
            vo = r._factor(r.pulsars[p], d, ddref.dd_gram(Xa, (w, np.zeros_like(w))), ldn)
            if pi is not None or not np.isclose(vd, vh, rtol=0, atol=1e-6 + 1e-10 * abs(vh)):
                print(f"draw {s} psr {p}: max scaled |G_dev - G_host| {rel.max():.3e} at "
                      f"{np.unravel_index(np.argmax(rel), rel.shape)}; host dd factor of device G {vd!r}, "
                      f"of host G {vh!r}, of the original basis {vo!r}", flush=True)
