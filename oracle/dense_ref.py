"""TEST INFRASTRUCTURE ONLY — brute-force dense Gaussian lnL.

Independent of the Woodbury / Sherman-Morrison route in enterprise_ref: builds
the full n x n covariance C = N + U J U^T + T phi T^T explicitly and evaluates
-1/2 r^T C^{-1} r - 1/2 log|C| with a dense Cholesky.  The timing-model prior
must be finite here (phi_tm = tm_var, e.g. 1e-12 s^2), because phi_tm = 1e40
cannot be represented densely.

Relation to enterprise's convention: enterprise omits
-1/2 n log 2pi, so `dense_lnl` omits it too; the Woodbury form equals
-1/2 r^T C^-1 r - 1/2 log|C| exactly, so for the same finite phi_tm the two
agree to rounding.
"""
import numpy as np
import scipy.linalg as sl


def dense_lnl(oracle_pulsar, params, tm_var=None):
    """lnL of one pulsar from the dense covariance.

    oracle_pulsar: enterprise_ref.OraclePulsar; tm_var overrides phi of the
    timing-model columns (required when the model has a timing model)."""
    pp = oracle_pulsar
    D, ep = pp._sm(params)
    n = len(D)
    C = np.diag(D)
    for slc, jv in ep:
        C[slc, slc] += jv
    phi = pp.phi(params)
    if tm_var is not None:
        for g in pp.gps:
            if g["kind"] == "tm":
                phi[g["idx"]] = tm_var
    T = pp.basis(params)
    C += (T * phi[None, :]) @ T.T
    cf = sl.cho_factor(C, lower=True)
    x = sl.cho_solve(cf, pp.r)
    return -0.5 * np.dot(pp.r, x) - np.sum(np.log(np.diag(cf[0])))


def woodbury_lnl(oracle_pulsar, params, tm_var=None):
    """The same pulsar through the enterprise route, with phi_tm = tm_var."""
    pp = oracle_pulsar
    TNT, TNr, rNr, ldN = pp.white_terms(params)
    phi = pp.phi(params)
    if tm_var is not None:
        for g in pp.gps:
            if g["kind"] == "tm":
                phi[g["idx"]] = tm_var
    Sigma = TNT + np.diag(1.0 / phi)
    cf = sl.cho_factor(Sigma)
    expval = sl.cho_solve(cf, TNr)
    return (-0.5 * (rNr + ldN)
            + 0.5 * (TNr @ expval - 2 * np.sum(np.log(np.diag(cf[0]))) - np.sum(np.log(phi))))


def dense_lnl_pta(oracle_pta, params, tm_var):
    """lnL of a whole (possibly correlated) PTA from the dense covariance
    C = blockdiag_a(N_a) + T Phi T^T over all TOAs, with Phi the global prior
    (cross-pulsar ORF terms included) and a finite timing-model variance."""
    o = oracle_pta
    Phi, off = o.phi_global(params)
    for a, pp in enumerate(o.pulsars):
        for g in pp.gps:
            if g["kind"] == "tm":
                ix = off[a] + np.asarray(g["idx"])
                Phi[ix, ix] = tm_var
    ns = [len(pp.r) for pp in o.pulsars]
    toff = np.concatenate(([0], np.cumsum(ns)))
    n = toff[-1]
    C = np.zeros((n, n))
    T = np.zeros((n, off[-1]))
    r = np.concatenate([pp.r for pp in o.pulsars])
    for a, pp in enumerate(o.pulsars):
        D, ep = pp._sm(params)
        sl_ = slice(toff[a], toff[a + 1])
        C[sl_, sl_] = np.diag(D)
        for slc, jv in ep:
            s0, s1 = toff[a] + slc.start, toff[a] + slc.stop
            C[s0:s1, s0:s1] += jv
        T[sl_, off[a]:off[a + 1]] = pp.basis(params)
    C += T @ Phi @ T.T
    cf = sl.cho_factor(C, lower=True)
    x = sl.cho_solve(cf, r)
    return -0.5 * np.dot(r, x) - np.sum(np.log(np.diag(cf[0])))


def woodbury_lnl_pta(oracle_pta, params, tm_var):
    """The enterprise route (Sigma = blockdiag(TNT) + Phi^-1) with the same
    finite timing-model variance, for comparison with dense_lnl_pta."""
    o = oracle_pta
    Phi, off = o.phi_global(params)
    for a, pp in enumerate(o.pulsars):
        for g in pp.gps:
            if g["kind"] == "tm":
                ix = off[a] + np.asarray(g["idx"])
                Phi[ix, ix] = tm_var
    Phiinv = np.linalg.inv(Phi)
    _, logdet_phi = np.linalg.slogdet(Phi)
    terms = [pp.white_terms(params) for pp in o.pulsars]
    S = Phiinv.copy()
    for a, t in enumerate(terms):
        S[off[a]:off[a + 1], off[a]:off[a + 1]] += t[0]
    d = np.concatenate([t[1] for t in terms])
    cf = sl.cho_factor(S)
    x = sl.cho_solve(cf, d)
    return (-0.5 * sum(t[2] + t[3] for t in terms)
            + 0.5 * (d @ x - 2 * np.sum(np.log(np.diag(cf[0]))) - logdet_phi))


def dense_os_xz(oracle_pulsar, params, gw_name="gw"):
    """X = F^T C^-1 r and Z = F^T C^-1 F of the optimal statistic from the
    dense covariance (enterprise_extensions OptimalStatistic.get_XZ computes
    the same through Woodbury).  C = N + T_gp phi T_gp^T + M phi_tm M^T is
    taken in the limit phi_tm -> inf (the 1e40 of [ent] utils.tm_prior):
    C^-1 = A - A M (M^T A M)^-1 M^T A with A = (N + T_gp phi T_gp^T)^-1."""
    pp = oracle_pulsar
    D, ep = pp._sm(params)
    C = np.diag(D)
    for slc, jv in ep:
        C[slc, slc] += jv
    phi = pp.phi(params)
    T = pp.basis(params)
    tm = np.zeros(T.shape[1], bool)
    for g in pp.gps:
        if g["kind"] == "tm":
            tm[g["idx"]] = True
    C += (T[:, ~tm] * phi[None, ~tm]) @ T[:, ~tm].T
    A = sl.cho_solve(sl.cho_factor(C), np.eye(len(D)))
    M = T[:, tm]
    AM = A @ M
    Cinv = A - AM @ np.linalg.solve(M.T @ AM, AM.T)
    g = next(g for g in pp.gps if g.get("name") == gw_name)
    F = T[:, np.asarray(g["idx"])]
    return F.T @ Cinv @ pp.r, F.T @ Cinv @ F
