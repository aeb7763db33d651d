"""TEST INFRASTRUCTURE ONLY: host-oracle evaluations of a full-size synthetic
configuration spread over the job's usable cores.

The at-scale parity tests (tests/test_gpu_parity.py) compare whole bench
batches -- 4096 C3 prior draws, 1024 C4 prior draws -- with the oracle.  One
core evaluates the enterprise-order oracle at ~75-230 C3 draws/s, so the
draws go to spawned single-threaded workers.  A worker rebuilds the seeded
model itself (the same host, the same seeds: the arrays the device saw) and
keeps it for the next task, so a pytest session pays the build once per
worker.  Workers never touch a GPU (they import numpy / scipy / the oracle
and the model builder only; torch is not initialised there).

Kinds of value per draw:
  "ent"  -- oracle/enterprise_ref.py, enterprise's own fp64 order
            (cho_factor; -inf on LinAlgError), the reference's call
            pta.get_lnlikelihood (/root/reference/enterprise_warp/bilby_warp.py:35);
  "dd"   -- oracle/ddref.py, double-double (uncorrelated / CURN models);
  "ext"  -- oracle/device_order_ref.py in np.longdouble with the error-free
            Gram (the near-exact value for varying white noise);
  "lmin" -- per draw, min over pulsars of lambda_min(H_p) - delta_p, where H_p
            is enterprise's Sigma_p = T^T N^-1 T + diag(1/phi) (timing model
            in, phi_tm = 1e40) scaled to unit diagonal from the error-free
            Gram, and delta_p = m_p (n_p + m_p) u the fp64 backward-error bound
            of forming and factoring it (u = 2^-53): a draw with a negative
            value is ambiguous in finiteness (tests/test_gpu_parity.py::
            test_c4_bench_inf_sets_at_scale), returned with the argmin pulsar;
  "ent_psr" -- per pulsar, 1 where enterprise's cho_factor of Sigma_p
            succeeds, 0 where it raises (the pulsar that makes the draw -inf);
  "entv_psr" -- the same for two further legitimate fp64 orders of
            enterprise's own algorithm: column block 0 = TNT with the TOAs
            summed in reverse order and the lower Cholesky factor, block 1 =
            the original TNT with the lower factor.
"""
import math
import os

import numpy as np

_CACHE = {}
U64 = 2.0 ** -53


def usable_cpus():
    """min(affinity, cgroup quota) -- bench.host_cpu_info's rule -- capped at
    16 (the GPU box gives one GPU's job 16 cores)."""
    aff = len(os.sched_getaffinity(0))
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as fh:
            q, per = fh.read().split()[:2]
            if q != "max":
                quota = float(q) / float(per)
    except OSError:
        pass
    n = aff if quota is None else max(1, min(aff, int(math.floor(quota + 1e-9))))
    return max(1, min(16, n))


def _model(cfg_name):
    if cfg_name not in _CACHE:
        from enterprise_warp_amd import synth
        cfg = {"c3": synth.config_c3, "c4": synth.config_c4, "c2": synth.config_c2}[cfg_name]()
        _CACHE.clear()                     # one model per worker at a time (memory)
        _CACHE[cfg_name] = {"cfg": cfg, "X": {}}
    return _CACHE[cfg_name]


def _draws(ent, seed, B):
    if (seed, B) not in ent["X"]:
        from enterprise_warp_amd import synth
        ent["X"][(seed, B)] = synth.prior_draws(ent["cfg"].pta, B, seed)
    return ent["X"][(seed, B)]


def _oracle(ent, kind):
    key = "o_" + kind
    if key not in ent:
        pta = ent["cfg"].pta
        psrs, terms = [c.psr for c in pta.signal_collections], pta.oracle_terms()
        const = pta.constant_values()
        fixed = const if pta.white_fixed() else None
        if kind in ("ent", "ent_psr", "entv_psr"):
            from oracle.enterprise_ref import OraclePTA
            ent[key] = OraclePTA(psrs, terms, fixed_params=fixed)
        elif kind == "dd":
            from oracle.ddref import DDReferencePTA
            ent[key] = DDReferencePTA(psrs, terms)
        else:
            from oracle.enterprise_ref import OraclePTA
            from oracle.device_order_ref import DeviceOrderPTA
            ent[key] = (DeviceOrderPTA(psrs, terms, fixed, np.longdouble) if kind == "ext"
                        else OraclePTA(psrs, terms, fixed_params=None))
    return ent[key]


def sigma_lambda_min(opta, params):
    """(min_p lambda_min(H_p) - delta_p, argmin p) for enterprise's Sigma_p
    (see the module docstring), from the error-free Gram in extended precision."""
    from oracle.device_order_ref import gram
    best, arg = np.inf, -1
    for i, pp in enumerate(opta.pulsars):
        G, _ = gram(pp, {k: np.longdouble(v) if np.ndim(v) == 0 else v for k, v in params.items()},
                    np.longdouble, "blas")
        m = pp.T.shape[1]
        S = np.array(G[:m, :m], dtype=np.longdouble)
        S[np.arange(m), np.arange(m)] += 1 / np.asarray(pp.phi(params), dtype=np.longdouble)
        sc = 1 / np.sqrt(np.diag(S))
        H = np.asarray(S * sc[:, None] * sc[None, :], dtype=np.float64)
        lam = float(np.linalg.eigvalsh(H)[0])
        delta = m * (len(pp.r) + m) * U64
        if lam - delta < best:
            best, arg = lam - delta, i
    return best, arg


def _psr_ok(opta, i, params):
    import scipy.linalg as sl
    pp = opta.pulsars[i]
    TNT = opta.fixed[i][0] if opta.fixed is not None else pp.white_terms(params)[0]
    try:
        sl.cho_factor(TNT + np.diag(1.0 / pp.phi(params)))
        return 1.0
    except sl.LinAlgError:
        return 0.0


def _psr_ok_variants(opta, i, params):
    """(reversed-TOA TNT + lower factor, original TNT + lower factor) finiteness."""
    import scipy.linalg as sl
    pp = opta.pulsars[i]
    if opta.fixed is not None:
        TNT = opta.fixed[i][0]
        D, ep = pp._sm(params)
    else:
        TNT = pp.white_terms(params)[0]
        D, ep = pp._sm(params)
    n = len(D)
    T = pp.basis(params)[::-1]
    ep_r = [(slice(n - sl_.stop, n - sl_.start), j) for sl_, j in ep]
    TNT_r = pp._solve_2D2(D[::-1].copy(), ep_r, T, T)
    pinv = np.diag(1.0 / pp.phi(params))
    out = []
    for A in (TNT_r + pinv, TNT + pinv):
        try:
            sl.cho_factor(A, lower=True)
            out.append(1.0)
        except sl.LinAlgError:
            out.append(0.0)
    return out


def _task(args):
    cfg_name, seed, B, idx, kind = args
    from threadpoolctl import threadpool_limits
    with threadpool_limits(limits=1):
        ent = _model(cfg_name)
        pta = ent["cfg"].pta
        X = _draws(ent, seed, B)
        o = _oracle(ent, kind)
        const = pta.constant_values()
        out = []
        for i in idx:
            d = dict(const)
            d.update(pta.map_params(X[i]))
            if kind == "lmin":
                out.append(sigma_lambda_min(o, d))
            elif kind == "ent_psr":
                out.append(tuple(_psr_ok(o, p, d) for p in range(len(o.pulsars))))
            elif kind == "entv_psr":
                v = [_psr_ok_variants(o, p, d) for p in range(len(o.pulsars))]
                out.append(tuple(a for a, _ in v) + tuple(b for _, b in v))
            else:
                out.append((o.lnlikelihood(d),))
        return out


def map_reference(cfg_name, seed, B, idx, kind, procs=None):
    """Oracle values (kind, module docstring) of draws idx of
    synth.prior_draws(config, B, seed), in idx order, over `procs` spawned
    workers (default: usable_cpus()).  Returns an array: one column for lnL
    kinds, two (value, pulsar) for "lmin"."""
    import multiprocessing as mp
    idx = [int(i) for i in idx]
    if not idx:
        return np.zeros((0, 2 if kind == "lmin" else 1))
    n = min(procs or usable_cpus(), len(idx))
    chunks = [idx[k::n] for k in range(n)]
    ctx = mp.get_context("spawn")
    with ctx.Pool(n) as pool:
        res = pool.map(_task, [(cfg_name, seed, B, c, kind) for c in chunks])
    out = np.zeros((len(idx), len(res[0][0])))
    for k, r in enumerate(res):
        out[k::n] = np.array(r, dtype=float)
    return out
