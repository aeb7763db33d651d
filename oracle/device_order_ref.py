"""TEST INFRASTRUCTURE ONLY — the likelihood in the DEVICE's order of operations.

`enterprise_ref` restates enterprise's own order (the full Sigma = TNT +
diag(1/phi) factored by LAPACK `cho_factor`, timing-model columns included).
libewarp_hip.so computes the same quantity in another order
(enterprise_warp_amd/csrc/ewarp_hip.hip):

* the residual is the LAST column of the basis, so one Gram matrix
  G = [T r]^T N^-1 [T r] carries TNT, d = TNr and rNr, and the last pivot of
  the factorisation of G + diag(1/phi, 0) is q = rNr - d^T Sigma^-1 d;
* at create, every theta-independent basis column and r lose their
  least-squares component along the timing-model columns M (weights
  1/sigma^2): X' = X - M C.  With phi_M = 1e40 this is an exact
  reparametrisation of the same likelihood (`project_coef`);
* varying white noise: G (fp64 contraction) + diag(1/phi) -- timing model
  included -- is factored in one go;
* fixed white noise: G is summed in double-double and the constant-phi
  (timing-model) leading block is eliminated ONCE in double-double
  (`schur_kernel`), leaving the reduced matrix S (rounded to fp64) with the
  residual last; per sample only S + diag(1/phi_own, 0) is factored;
* the factorisation is an LDL^T in 16-wide block rows with a two-level panel
  (`ldl_two_level`: the diagonal block in 4-row sub-panels, each closed by a
  symmetric rank-4 update of the rows below; the rest of the block row by
  L^-1 = E^T; trailing update A -= U^T U with U = D^-1/2 L^-1 A);
* a correlated common process (HD / monopole / dipole ORF) keeps each
  pulsar's common block after eliminating its own columns, inverts
  M_g = Gamma phi_c(g) + diag(phi_own(., g)) per common column by
  Gauss-Jordan, and factors the dense Sigma_c = blockdiag(S^G_a) + [M_g^-1]
  (DESIGN.md §4b);
* lnL_p = K - q/2 - 1/2 sum log d_k - 1/2 sum log phi.

Every function takes a numpy dtype.  With `np.float64` this is the device's
ordering in fp64.  With `np.longdouble` (x86 80-bit extended, eps 1.1e-19)
it is a near-exact value of the same likelihood for the same fp64 inputs --
no projection (the reference value is the ORIGINAL basis's), the Gram error
free (`exact_gram`: an Ozaki split into 18-bit slices whose products and
sums are exact in fp64 BLAS, summed in extended precision), the timing-model
elimination and the factorisation in extended precision -- against which
every ordering's error is measured (tests/conftest.py `check_accuracy`).

Model tables (bases, selections, epochs, spectra, parameter names) come from
`enterprise_ref.OraclePulsar`; only the arithmetic order differs.
"""
import numpy as np

from .enterprise_ref import FYR, OraclePTA, orf_value

TM_PHI = 1e40        # [ent] utils.tm_prior


def _cast(params, dt):
    out = {}
    for k, v in params.items():
        if v is None:
            continue
        a = np.asarray(v)
        out[k] = a.astype(dt) if a.ndim else dt(a)
    return out


def _spectrum(g, p, dt):
    """phi of one GP signal on its own columns, in dtype dt (the formulas of
    enterprise_ref.powerlaw / powerlaw_bpl / free_spectrum)."""
    f = np.asarray(g["f"], dtype=dt)
    val = lambda ref: dt(ref[1]) if ref[0] == "const" else p[ref[1]]  # noqa: E731
    nm = g["names"]
    comp = g["components"]
    df = np.diff(np.concatenate((np.zeros(1, dt), f[::comp])))
    df = np.repeat(df, comp)
    pi2 = dt(np.pi) ** 2 if dt is np.float64 else np.arccos(dt(-1)) ** 2
    fyr = dt(FYR)
    if g["spectrum"] == "powerlaw":
        A, gam = val(nm["log10_A"]), val(nm["gamma"])
        return dt(10) ** (2 * A) / 12 / pi2 * fyr ** (gam - 3) * f ** (-gam) * df
    if g["spectrum"] == "turnover":
        A, gam, fc = val(nm["log10_A"]), val(nm["gamma"]), val(nm["fc"])
        if fc < 0:
            fc = dt(10) ** fc
        return dt(10) ** (2 * A) / 12 / pi2 * fyr ** (-3) * ((f + fc) / fyr) ** (-gam) * df
    rho = val(nm["log10_rho"])
    return np.repeat(dt(10) ** (2 * np.asarray(rho, dtype=dt)), 2)


def phi_columns(pp, p, dt, with_common=True):
    """Per-column phi of one pulsar ([ent] SignalCollection.get_phi), in dt.
    with_common=False leaves out a correlated common signal (it lives in the
    cross-pulsar M_g blocks of the device)."""
    phi = np.zeros(pp.T.shape[1], dtype=dt)
    for g in pp.gps:
        if g["kind"] == "tm":
            phi[g["idx"]] += dt(TM_PHI)
            continue
        if g.get("orf"):
            if with_common:
                pos = np.asarray(pp.psr.pos, float)
                phi[g["idx"]] += dt(orf_value(g["orf"], pos, pos)) * _spectrum(g, p, dt)
            continue
        phi[g["idx"]] += _spectrum(g, p, dt)
    return phi


def _fma(a, b, c):
    """fp64 fused multiply-add, emulated through the x87 extended product
    (double rounding differs from a true FMA on ~1 in 2^11 operations)."""
    return (np.asarray(a, dtype=np.longdouble) * b + c).astype(np.float64)


def gram_device_fma(pp, p, nl=0):
    """fp64 Gram in the contraction kernels' accumulation order
    (contract2_kernel) on the projected basis: per entry one accumulator, TOA
    rows (padded to whole 32-row tiles) taken 4 at a time as sequential FMAs
    of (w_t T_ti) T_tj; ECORR epoch sums s_e as an FMA chain over the epoch's
    TOAs, then the epoch rows with weights -beta_e through the same
    accumulator."""
    n = len(pp.r)
    Dd = np.zeros(n)
    sig2 = np.asarray(pp.sigma, float) ** 2
    for k, masks, names in pp.white:
        for key, m in masks.items():
            if k == "efac":
                ef = float(p[names[key]])
                Dd[m] += (ef * ef) * sig2[m]
            elif k == "tnequad":
                Dd[m] += 10.0 ** (2.0 * float(p[names[key]]))
    w = 1.0 / Dd
    T = np.asarray(pp.basis({k: float(v) for k, v in p.items() if np.ndim(v) == 0}), dtype=float)
    X = np.concatenate([T, np.asarray(pp.r, float)[:, None]], axis=1)
    if nl:
        X = projected(pp, X, nl)
    m1 = X.shape[1]
    acc = np.zeros((m1, m1))

    def rows(acc, R, wr):
        npad = (len(R) + 31) // 32 * 32
        Rp = np.zeros((npad, m1))
        Rp[:len(R)] = R
        wp = np.zeros(npad)
        wp[:len(R)] = wr
        A = Rp * wp[:, None]
        for t in range(npad):
            acc = _fma(A[t][:, None], Rp[t][None, :], acc)
        return acc

    acc = rows(acc, X, w)
    ldn = np.sum(np.log(Dd))
    if pp.ecorr:
        S, nb = [], []
        for slc, nm in pp.ecorr:
            J = 10.0 ** (2.0 * float(p[nm]))
            sw = 0.0
            e = np.zeros(m1)
            for t in range(slc.start, slc.stop):
                sw = sw + w[t]
                e = _fma(np.full(m1, w[t]), X[t], e)
            beta = 1.0 / (sw + 1.0 / J)
            S.append(e)
            nb.append(-beta)
            ldn += np.log(J) - np.log(beta)
        acc = rows(acc, np.array(S), np.array(nb))
    return acc, ldn


_SPLIT = 134217729.0     # 2^27 + 1 (Veltkamp)


def two_prod(a, b):
    """a * b = p + e exactly (Dekker's TwoProduct by Veltkamp splitting; fp64)."""
    a = np.asarray(a, float)
    b = np.asarray(b, float)
    p = a * b
    ca, cb = _SPLIT * a, _SPLIT * b
    ah = ca - (ca - a)
    bh = cb - (cb - b)
    al, bl = a - ah, b - bh
    e = ((ah * bh - p) + ah * bl + al * bh) + al * bl
    return p, e


def _slices(A, k=4, beta=18):
    """A (n x m, fp64) = sum of k column-aligned slices (+ a remainder below
    2^(e_j - k beta) that is dropped): slice s of column j is a multiple of
    2^(e_j - beta (s + 1)) with |slice| < 2^(e_j - beta s), max |A_:j| < 2^e_j.
    A product of two slices is an integer of <= 2 beta bits times a power of
    two common to the whole dot product, so a sum of n <= 2^17 of them is exact
    in fp64 whatever order BLAS adds them in (Ozaki et al. 2012)."""
    A = np.asarray(A, float)
    mx = np.max(np.abs(A), axis=0) if A.shape[0] else np.zeros(A.shape[1])
    e = np.where(mx > 0, np.floor(np.log2(np.where(mx > 0, mx, 1.0))) + 1, 0.0)
    out, R = [], A.copy()
    for s in range(k):
        sigma = 1.5 * np.exp2(e - beta * (s + 1) + 52)
        S = (R + sigma) - sigma
        out.append(S)
        R = R - S
    return out


def exact_product(A, B, k=4):
    """A^T B to ~2^-72 of max|A_:i| max|B_:j| per term, exact sums (longdouble)."""
    if A.shape[0] > 1 << 17:
        raise ValueError("exact_product: at most 2^17 rows")
    SA, SB = _slices(A, k), _slices(B, k)
    out = np.zeros((A.shape[1], B.shape[1]), dtype=np.longdouble)
    for s in range(k):
        for t in range(k - s):
            out += (SA[s].T @ SB[t]).astype(np.longdouble)
    return out


def exact_gram(X, D):
    """G = X^T diag(1/D) X for fp64 X and extended-precision D, error free up
    to ~2^-64 relative per term: w = 1/D as w_hi + w_lo, X w_hi = A_hi + A_lo
    exactly (TwoProduct), A_hi^T X by `exact_product`, the small remainder
    (A_lo + X w_lo)^T X by one fp64 product."""
    X = np.asarray(X, float)
    w = 1 / np.asarray(D, dtype=np.longdouble)
    w_hi = w.astype(np.float64)
    w_lo = (w - w_hi).astype(np.float64)
    A_hi, A_lo = two_prod(X, w_hi[:, None])
    A_lo = A_lo + X * w_lo[:, None]
    return exact_product(A_hi, X) + (A_lo.T @ X).astype(np.longdouble)


def project_coef(X, sigma, nl, cols):
    """C of the create-time timing-model projection (ewarp_hip.hip
    projection_coef): (M^T W0 M)^-1 M^T W0 X[:, cols], W0 = 1/sigma^2, M = the
    first nl columns; columns of M without weight are left out."""
    M = X[:, :nl]
    w0 = 1.0 / np.asarray(sigma, float) ** 2
    G0 = (M * w0[:, None]).T @ M
    B = (M * w0[:, None]).T @ X[:, cols]
    dmax = np.max(np.diag(G0)) if nl else 0.0
    use = np.zeros(nl, bool)
    L = np.zeros((nl, nl))
    for kk in range(nl):
        v = G0[kk, kk] - L[kk, :kk] @ L[kk, :kk]
        if not v > 1e-12 * dmax:
            continue
        use[kk] = True
        L[kk, kk] = np.sqrt(v)
        for i in range(kk + 1, nl):
            L[i, kk] = (G0[i, kk] - L[i, :kk] @ L[kk, :kk]) / L[kk, kk]
    C = np.zeros((nl, len(cols)))
    u = np.flatnonzero(use)
    if len(u):
        Lu = L[np.ix_(u, u)]
        y = np.linalg.solve(Lu, B[u])
        C[u] = np.linalg.solve(Lu.T, y)
    return C


def projected(pp, X, nl):
    """X' = X - M C on the theta-independent columns and r (last column of X)."""
    cache = pp.__dict__.setdefault("_proj_cache", {})
    if nl not in cache:
        chrom = set()
        for idx, _, _ in pp.basis_params:
            chrom.update(np.atleast_1d(idx).tolist())
        cols = [j for j in range(nl, X.shape[1] - 1) if j not in chrom] + [X.shape[1] - 1]
        cache[nl] = (cols, project_coef(X, pp.sigma, nl, cols))
    cols, C = cache[nl]
    X = X.copy()
    X[:, cols] = X[:, cols] - X[:, :nl] @ C
    return X


def gram(pp, p, dt, mode="blas", nl=0):
    """G = [T r]^T N^-1 [T r] (ShermanMorrison form of EcorrKernelNoise) and
    log|N|, in dt.  mode "blas": one matrix product (error free for
    dt = longdouble: `exact_gram`); "reverse": the TOAs summed in reverse
    order; "device": gram_device_fma (fp64 only).  nl > 0: on the basis
    projected off its first nl (timing-model) columns (the device's basis)."""
    if mode == "device":
        return gram_device_fma(pp, p, nl)
    n = len(pp.r)
    D = np.zeros(n, dtype=dt)
    sig2 = np.asarray(pp.sigma, dtype=dt) ** 2
    for k, masks, names in pp.white:
        for key, m in masks.items():
            if k == "efac":
                D[m] += p[names[key]] ** 2 * sig2[m]
            elif k == "tnequad":
                D[m] += dt(10) ** (2 * p[names[key]])
    T = np.asarray(pp.basis({k: float(v) for k, v in p.items() if np.ndim(v) == 0}), dtype=float)
    X = np.concatenate([T, np.asarray(pp.r, float)[:, None]], axis=1)
    if nl:
        X = projected(pp, X, nl)
    if dt is np.longdouble and mode == "blas":
        G = exact_gram(X, D)
        Xd = X.astype(dt)
    else:
        Xd = X.astype(dt)
        if mode == "reverse":
            Xd, D = Xd[::-1], D[::-1]
        G = Xd.T @ (Xd / D[:, None])
        if mode == "reverse":
            Xd, D = Xd[::-1], D[::-1]
    ldn = np.sum(np.log(D))
    for slc, nm in pp.ecorr:
        J = dt(10) ** (2 * p[nm])
        ni = 1 / D[slc]
        beta = 1 / (np.sum(ni) + 1 / J)
        sv = ni @ Xd[slc]
        G -= beta * np.outer(sv, sv)
        ldn += np.log(J) - np.log(beta)
    return G, ldn


def lead_schur(G, nlead, phi_lead, device=False):
    """`schur_kernel`: add 1/phi to the leading block's diagonal, eliminate it
    by a sequential Cholesky; returns (reduced G, sum log L_kk, ok).
    device=True (fp64): the kernel's arithmetic -- row k scaled by 1/sqrt(pivot),
    updates as fused multiply-adds."""
    G = G.copy()
    idx = np.arange(nlead)
    G[idx, idx] += 1 / phi_lead
    logdet = G.dtype.type(0)
    ok = True
    for k in range(nlead):
        piv = G[k, k]
        ok &= bool(piv > 0)
        d = np.sqrt(piv)
        logdet += np.log(d)
        if device:
            row = G[k, k + 1:] * (1.0 / d)
            G[k + 1:, k + 1:] = _fma(-row[:, None], row[None, :], G[k + 1:, k + 1:])
        else:
            row = G[k, k + 1:] / d
            G[k + 1:, k + 1:] -= np.outer(row, row)
    return G[nlead:, nlead:], logdet, ok


def ldl_blocked(A, npiv, bs=16):
    """LDL^T in bs-wide block rows (the register kernels' blocked panel):
    within a block row the pivots are eliminated one at a time across the
    whole row (= L^-1 applied to the off-diagonal blocks), the row is scaled
    to U = D^-1/2 V and the trailing matrix takes A -= U^T U.  Pivots are
    0..npiv-1; the rest of the matrix (the residual corner / a kept block) is
    returned updated.  Returns (pivots d, updated A)."""
    A = A.copy()
    n = A.shape[0]
    d = []
    for k0 in range(0, npiv, bs):
        k1 = min(k0 + bs, n)
        kend = min(k1, npiv)
        for k in range(k0, kend):
            dk = A[k, k]
            d.append(dk)
            w = A[k, k + 1:] / dk
            # rows k+1..k1-1 of this block row take row k (columns > k)
            A[k + 1:k1, k + 1:] -= np.outer(A[k + 1:k1, k], w)
        if k1 < n:
            dv = np.array(d[k0:kend], dtype=A.dtype)
            U = A[k0:kend, k1:] / np.sqrt(dv)[:, None]
            A[k1:, k1:] -= U.T @ U
    return np.array(d, dtype=A.dtype), A


def chol_unblocked(A, npiv):
    """Sequential right-looking Cholesky (scipy cho_factor's pivot order, no
    blocking): pivots d_k = L_kk^2 and the updated trailing corner."""
    A = A.copy()
    d = []
    for k in range(npiv):
        dk = A[k, k]
        d.append(dk)
        row = A[k, k + 1:] / np.sqrt(dk)
        A[k + 1:, k + 1:] -= np.outer(row, row)
    return np.array(d, dtype=A.dtype), A


def ldl_two_level(A, npiv, bs=16, sub=4):
    """The register kernels' LDL^T (ewarp_dev.h panel_ldl_row, PANEL_2L) in
    bs-wide block rows: the diagonal block (held in full) is eliminated in
    sub-row sub-panels -- within one, each pivot updates the sub-panel's rows
    below it (multipliers from the lower triangle) and E = L^-T takes the
    column operation; a closed sub-panel is scaled to U_s = D_s^-1/2 V_s and
    the rest of the block takes D -= U_s^T U_s --, the rest of the block row
    becomes U = D^-1/2 E^T A and the trailing matrix takes A -= U^T U.
    Pivots 0..npiv-1; the rest (the residual corner / a kept block) is
    returned updated.  Returns (pivots d, updated A)."""
    A = A.copy()
    n = A.shape[0]
    d = []
    for k0 in range(0, npiv, bs):
        k1 = min(k0 + bs, n)
        kend = min(k1, npiv)
        m = k1 - k0
        D = A[k0:k1, k0:k1].copy()
        E = np.eye(m, dtype=A.dtype)
        rs = np.ones(m, dtype=A.dtype)
        ar = np.arange(m)
        for s0 in range(0, kend - k0, sub):
            s1 = min(s0 + sub, m)
            pe = min(s1, kend - k0)
            for kk in range(s0, pe):
                dk = D[kk, kk]
                d.append(dk)
                nw = -D[kk, :] / dk
                E += np.outer(E[:, kk], np.where(ar > kk, nw, 0))
                rows = np.arange(kk + 1, s1)
                D[rows, :] += np.outer(D[rows, kk], nw)
            rs[s0:pe] = 1 / np.sqrt(np.diag(D)[s0:pe])
            if s1 < m and pe == s1:
                U = D[s0:s1, :] * rs[s0:s1, None]
                D[s1:, :] -= (U.T @ U)[s1:, :]
        nr = kend - k0
        A[k0:k1, k0:k1] = D
        if k1 < n:
            U = (E.T @ A[k0:k1, k1:])[:nr] * rs[:nr, None]
            A[k1:, k1:] -= U.T @ U
    return np.array(d, dtype=A.dtype), A


def _block_layout(nown, ncom):
    """Reduced layout of the device (ewarp_hip.hip ewh_create):
    [own | pad | r] or, with a common block, [own | pad to 16 | common | pad | r].
    Returns (size, gstart)."""
    if ncom:
        gstart = 16 * ((nown + 15) // 16)
        return 16 * ((gstart + ncom + 1 + 15) // 16), gstart
    return 16 * ((nown + 1 + 15) // 16), nown


class DeviceOrderPTA:
    """The device's ordering of the same likelihood (fixed or varying white
    noise, uncorrelated / CURN or correlated common process), or -- with
    other arguments -- further correct orderings of it."""

    def __init__(self, psrs, terms_per_psr, fixed_params=None, dtype=np.float64, gram_mode="blas",
                 factor="ldl2"):
        """dtype float64 with factor "ldl2" (default) is the device's order:
        projected basis, two-level blocked LDL^T, varying white noise factored
        with the timing model in, fixed white noise through a double-double
        (here: extended-precision, error-free) Gram and timing-model
        elimination; gram_mode "device" restates the contraction kernels' FMA
        accumulation order, "blas" uses one matrix product.  factor "ldl16"
        (the round-2 one-level panel) or "chol" (unblocked Cholesky), or
        gram_mode "reverse": another correct fp64 ordering (original basis,
        timing model eliminated first).  dtype longdouble: the near-exact
        reference (original basis, error-free Gram, extended precision)."""
        self.o = OraclePTA(psrs, terms_per_psr, fixed_params=None)
        self.dt = dtype
        self.gram_mode = gram_mode
        self.factor = {"ldl2": ldl_two_level, "ldl16": ldl_blocked,
                       "chol": lambda A, npiv, bs=16: chol_unblocked(A, npiv)}[factor]
        self.device = dtype is np.float64 and factor == "ldl2" and gram_mode in ("blas", "device")
        self.pulsars = self.o.pulsars
        self.nlead = []
        for pp in self.pulsars:
            tm = [g for g in pp.gps if g["kind"] == "tm"]
            nl = len(set(tm[0]["idx"])) if tm else 0
            if tm and sorted(set(tm[0]["idx"])) != list(range(nl)):
                raise ValueError("timing-model columns must lead the basis")
            self.nlead.append(nl)
        self.white_fixed = fixed_params is not None and not any(pp.basis_params for pp in self.pulsars)
        self.cache = None
        if self.white_fixed:
            p = _cast(fixed_params, dtype)
            self.cache = [self._reduce(i, p) for i in range(len(self.pulsars))]

    def correlated(self):
        return self.o.correlated()

    # ---- per pulsar: G, lead elimination, reduced layout -----------------
    def _common_cols(self, pp):
        for g in pp.gps:
            if g.get("orf"):
                return list(g["idx"])
        return []

    def _reduce(self, i, p):
        """Gram + timing-model elimination of pulsar i: (S in the device's
        reduced layout, K, ok, own column ids, common column ids)."""
        pp = self.pulsars[i]
        dt = self.dt
        m = pp.T.shape[1]
        nl = self.nlead[i]
        com = self._common_cols(pp) if self.correlated() else []
        own = [j for j in range(nl, m) if j not in set(com)]
        if self.device:
            # gram_dd_kernel + schur_kernel: double-double Gram of the projected
            # basis and elimination (restated error free / in extended precision)
            pl = _cast(p, np.longdouble)
            G, ldn = gram(pp, pl, np.longdouble, "blas", nl=nl)
            phi_lead = np.full(nl, TM_PHI, dtype=np.longdouble)
            Sr, logdet, ok = lead_schur(G, nl, phi_lead)
            K = -ldn / 2 - logdet - np.sum(np.log(phi_lead)) / 2
            Sr, K = Sr.astype(np.float64), np.float64(K)
        else:
            G, ldn = gram(pp, p, dt, self.gram_mode)
            phi_lead = np.full(nl, TM_PHI, dtype=dt)           # constant-phi leading block
            Sr, logdet, ok = lead_schur(G, nl, phi_lead)
            K = -ldn / 2 - logdet - np.sum(np.log(phi_lead)) / 2
        # Sr indexes columns nl..m (r last); lay it out as the device does
        size, gstart = _block_layout(len(own), len(com))
        pos = np.full(size, -1)
        pos[:len(own)] = [j - nl for j in own]
        pos[gstart:gstart + len(com)] = [j - nl for j in com]
        pos[size - 1] = m - nl
        S = np.zeros((size, size), dtype=dt)
        S[np.arange(size), np.arange(size)] = 1
        live = pos >= 0
        S[np.ix_(live, live)] = Sr[np.ix_(pos[live], pos[live])]
        return S, K, ok, own, com, gstart

    # ---- lnL ------------------------------------------------------------
    def _full(self, i, p):
        """Varying white noise on the device: G of the projected basis +
        diag(1/phi) factored with the timing model in, layout [T | pad | r]."""
        pp = self.pulsars[i]
        G, ldn = gram(pp, p, np.float64, self.gram_mode, nl=self.nlead[i])
        m = pp.T.shape[1]
        size = 16 * ((m + 1 + 15) // 16)
        S = np.eye(size)
        S[:m, :m] = G[:m, :m]
        S[:m, -1] = G[:m, m]
        S[-1, :m] = G[m, :m]
        S[-1, -1] = G[m, m]
        return S, np.float64(-ldn / 2), True, list(range(m)), [], m

    def lnlikelihood(self, params):
        p = _cast(params, self.dt)
        if self.correlated():
            return float(self._lnl_correlated(p))
        tot = self.dt(0)
        for i, pp in enumerate(self.pulsars):
            if self.white_fixed:
                S, K, ok, own, _, _ = self.cache[i]
            elif self.device:
                S, K, ok, own, _, _ = self._full(i, p)
            else:
                S, K, ok, own, _, _ = self._reduce(i, p)
            phi = phi_columns(pp, p, self.dt)[own]
            A = S.copy()
            idx = np.arange(len(own))
            A[idx, idx] += 1 / phi
            d, A = self.factor(A, A.shape[0] - 1)
            if not ok or not np.all(d > 0):
                return -np.inf
            q = A[-1, -1]
            tot += K - q / 2 - np.sum(np.log(d)) / 2 - np.sum(np.log(phi)) / 2
        return float(tot)

    def min_eig(self, params):
        """Conditioning of what the device factors for this sample: min over
        pulsars of lambda_min of the unit-diagonal-scaled S + diag(1/phi_own)
        (own columns, timing model eliminated), fp64.  Informational: near 0
        means two correct fp64 orderings may differ widely (the `spread`)."""
        if self.correlated():
            return float("nan")
        p = _cast(params, np.float64)
        mins = []
        for i, pp in enumerate(self.pulsars):
            S, K, ok, own, _, _ = self.cache[i] if self.white_fixed else self._reduce(i, p)
            S = np.array(S[:len(own), :len(own)], dtype=np.float64)
            S[np.arange(len(own)), np.arange(len(own))] += 1 / np.asarray(phi_columns(pp, p, np.float64)[own])
            sc = 1 / np.sqrt(np.abs(np.diag(S)))
            mins.append(np.linalg.eigvalsh(S * sc[:, None] * sc[None, :])[0])
        return float(min(mins))

    def partial(self, i, params):
        """Step 1 of the correlated likelihood for pulsar i (what
        ewh_corr_partial_device computes): its local term K_i - 1/2 log|Sigma_LL|
        - 1/2 log|phi_L| (-inf when the own block is not positive definite) and
        its kept block, as one (nc + 1)^2 array [[S^G, d'], [d'^T, rho]]."""
        dt = self.dt
        p = params if all(isinstance(v, (np.ndarray, dt)) for v in params.values()) else _cast(params, dt)
        pp = self.pulsars[i]
        S, K, ok, own, com, gstart = self.cache[i] if self.white_fixed else self._reduce(i, p)
        nc = len(com)
        phi = phi_columns(pp, p, dt, with_common=False)[own]
        A = S.copy()
        idx = np.arange(len(own))
        A[idx, idx] += 1 / phi
        d, A = self.factor(A, gstart)
        local = K - np.sum(np.log(d)) / 2 - np.sum(np.log(phi)) / 2 if ok and np.all(d > 0) else dt(-np.inf)
        kb = A[gstart:, gstart:]
        keep = np.zeros((nc + 1, nc + 1), dtype=dt)
        keep[:nc, :nc] = kb[:nc, :nc]
        keep[:nc, nc] = kb[:nc, -1]
        keep[nc, :nc] = kb[-1, :nc]
        keep[nc, nc] = kb[-1, -1]
        return local, keep

    def finish(self, params, locals_, keeps):
        """Step 2 (ewh_corr_finish_device): from every pulsar's local term and
        kept block, M_g^-1, the dense Sigma_c, its factorisation, lnL."""
        dt = self.dt
        p = _cast(params, dt)
        P = len(self.pulsars)
        if not np.all(np.isfinite(np.asarray(locals_, dtype=float))):
            return dt(-np.inf)
        nc = keeps[0].shape[0] - 1
        own_phi_common = [phi_columns(pp, p, dt, with_common=False)[self._common_cols(pp)] for pp in self.pulsars]
        pp0 = self.pulsars[0]
        gc = next(g for g in pp0.gps if g.get("orf"))
        phic = _spectrum(gc, p, dt)
        pos = [np.asarray(pp.psr.pos, float) for pp in self.pulsars]
        Gam = np.array([[orf_value(gc["orf"], pos[a], pos[b]) for b in range(P)] for a in range(P)], dtype=dt)
        N = P * nc
        Sc = np.zeros((N + 1, N + 1), dtype=dt)
        mlog = dt(0)
        for g in range(nc):
            M = Gam * phic[g] + np.diag(np.array([own_phi_common[a][g] for a in range(P)], dtype=dt))
            Minv, ld, ok = _gauss_jordan(M)
            if not ok:
                return dt(-np.inf)
            mlog += ld
            ix = np.arange(P) * nc + g
            Sc[np.ix_(ix, ix)] += Minv
        for a, kp in enumerate(keeps):
            s = slice(a * nc, (a + 1) * nc)
            Sc[s, s] += kp[:nc, :nc]
            Sc[s, N] = kp[:nc, nc]
            Sc[N, s] = kp[nc, :nc]
            Sc[N, N] += kp[nc, nc]
        d, A = self.factor(Sc, N)
        if not np.all(d > 0):
            return dt(-np.inf)
        return sum(locals_) - (np.sum(np.log(d)) + A[N, N] + mlog) / 2

    def _lnl_correlated(self, p):
        parts = [self.partial(i, p) for i in range(len(self.pulsars))]
        return self.finish(p, [q[0] for q in parts], [q[1] for q in parts])


def _gauss_jordan(M):
    """M^-1 and log|M| by in-place Gauss-Jordan without pivoting
    (`common_minv_reg_kernel`)."""
    M = M.copy()
    n = M.shape[0]
    ld = M.dtype.type(0)
    ok = True
    for k in range(n):
        piv = M[k, k]
        ok &= bool(piv > 0)
        ld += np.log(piv) if piv > 0 else 0
        pinv = 1 / piv
        colk = M[:, k].copy()
        rowk = M[k, :] * pinv
        M -= np.outer(colk, rowk)
        M[k, :] = rowk
        M[:, k] = -colk * pinv
        M[k, k] = pinv
    return M, ld, ok
