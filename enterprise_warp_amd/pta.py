"""`PTA`: the drop-in for enterprise's `signal_base.PTA` on the likelihood path.

Reference boundary: `pta = signal_base.PTA(models)` (enterprise_warp.py:502),
`pta.set_default_params(noisedict)` (:508), `pta.param_names` (:511, :515),
`pta.params` (bilby_warp.py:51; run_example_paramfile.py:29) and
`pta.get_lnlikelihood(params)` with a dict (bilby_warp.py:35) or an ndarray in
`param_names` order (PTSampler via run_example_paramfile.py:27-30).

Every likelihood call goes to libewarp_hip.so (hand-written gfx950 kernels)
through the C ABI in include/ewarp_hip.h; there is no CPU path.  New in this
framework: `get_lnlikelihood_batch(X[B, nparam])` evaluates a batch of sampler
proposals in one device call, and `engine()` exposes the device-pointer entry
used for multi-GPU sharding (bench.py, enterprise_warp_amd/sharding.py).
"""
import ctypes as C

import numpy as np

from . import _lib
from . import constants as const
from . import parameter as parameter
from .signals import SignalCollection


class PTA:
    def __init__(self, init, lnlikelihood=None):
        if isinstance(init, SignalCollection):
            init = [init]
        self._collections = list(init)
        names = [c.name for c in self._collections]
        if len(set(names)) != len(names):
            raise ValueError("duplicate pulsar names in PTA")
        self._engine = None
        self._engine_devices = None
        self._rebuild_params()

    # ------------------------------------------------------------------ params
    def _rebuild_params(self):
        allp = {}
        for c in self._collections:
            for p in c.all_params:
                q = allp.setdefault(p.name, p)
                if q is not p and type(q) is not type(p):
                    raise ValueError(f"parameter {p.name} defined with two different priors")
        self._all = allp
        self._params = [allp[k] for k in sorted(allp) if not isinstance(allp[k], parameter.ConstantParameter)]
        self._index = {}
        ct = 0
        for p in self._params:
            n = p.size if p.size else 1
            self._index[p.name] = ct
            ct += n
        self._nparam = ct

    @property
    def params(self):
        return list(self._params)

    @property
    def param_names(self):
        out = []
        for p in self._params:
            if p.size:
                out.extend(f"{p.name}_{i}" for i in range(p.size))
            else:
                out.append(p.name)
        return out

    @property
    def pulsars(self):
        return [c.name for c in self._collections]

    @property
    def signal_collections(self):
        return list(self._collections)

    def map_params(self, xs):
        """ndarray in param_names order -> {name: value} ([ent] PTA.map_params)."""
        xs = np.asarray(xs, dtype=float)
        ret, ct = {}, 0
        for p in self._params:
            n = p.size if p.size else 1
            ret[p.name] = xs[ct:ct + n] if n > 1 else float(xs[ct])
            ct += n
        return ret

    def set_default_params(self, params):
        """Set Constant values from a noise dictionary (enterprise_warp.py:504-508).

        Compatibility alias: the reference's example
        noise files name EQUAD `{psr}_{backend}_log10_equad` while
        TNEquadNoise's parameter is `..._log10_tnequad`; a `_log10_equad` key
        fills the matching `_log10_tnequad` Constant when that key is absent."""
        keyed = dict(params)
        for k, v in params.items():
            if k.endswith("_log10_equad"):
                keyed.setdefault(k[: -len("_log10_equad")] + "_log10_tnequad", v)
        changed = set()
        for p in self._all.values():
            if isinstance(p, parameter.ConstantParameter) and p.name in keyed:
                val = float(keyed[p.name])
                if p.value != val:
                    was_set = p.value is not None
                    p.value = val
                    changed.add(p.name if was_set else None)
        if not changed:
            return
        white = {p.name for c in self._collections for w in c.white for p in w.params}
        if self._engine is not None and None not in changed and changed <= white:
            # new white-noise constants only: recompute the cached TNT etc. in
            # place (ewh_set_fixed_white) instead of rebuilding the engine
            self._engine.set_fixed_white(self)
        else:
            self._drop_engine()

    def get_lnprior(self, params):
        d = params if isinstance(params, dict) else self.map_params(params)
        return float(sum(p.get_logpdf(d[p.name]) for p in self._params))

    def get_lnprior_batch(self, X):
        """log-prior of every row of X [B, nparam] (param_names order)."""
        X = np.atleast_2d(np.asarray(X, dtype=float))
        lp = np.zeros(len(X))
        for p in self._params:
            i = self._index[p.name]
            v = X[:, i:i + p.size] if p.size else X[:, i]
            q = np.asarray(p._logpdf(v), dtype=float)
            lp += q.sum(axis=1) if q.ndim == 2 else q
        return lp

    def _theta(self, X):
        """dict / ndarray / batch -> theta matrix [B, nparam] (param_names order)."""
        if isinstance(X, dict):
            row = np.empty(self._nparam)
            for p in self._params:
                i = self._index[p.name]
                if p.name in X:
                    v = np.atleast_1d(np.asarray(X[p.name], dtype=float))
                elif p.size and all(f"{p.name}_{j}" in X for j in range(p.size)):
                    v = np.array([X[f"{p.name}_{j}"] for j in range(p.size)], dtype=float)
                else:
                    raise KeyError(f"missing value for parameter {p.name}")
                row[i:i + (p.size or 1)] = v
            return row[None, :]
        X = np.asarray(X, dtype=float)
        if X.ndim == 1:
            X = X[None, :]
        if X.shape[1] != self._nparam:
            raise ValueError(f"expected {self._nparam} parameters per sample, got {X.shape[1]}")
        return np.ascontiguousarray(X)

    # -------------------------------------------------------------- likelihood
    def get_lnlikelihood(self, params, **kwargs):
        return float(self.get_lnlikelihood_batch(self._theta(params))[0])

    def get_lnlikelihood_batch(self, X):
        th = self._theta(X)
        return self.engine().lnl_batch(th)

    def engine(self, device=None, devices=None):
        """The device-resident likelihood (created on first use, after
        set_default_params; re-created when the device list or non-white
        constants change).  devices: HIP device ids the handle spreads every
        batch over (get_lnlikelihood_batch then uses the whole node);
        device: shorthand for [device].  Default: the current list, else [0]."""
        if devices is None and device is not None:
            devices = [device]
        if devices is None:
            devices = self._engine_devices if self._engine_devices is not None else [0]
        devices = [int(d) for d in devices]
        if self._engine is None or self._engine_devices != devices:
            self._drop_engine()
            self._engine = Engine(self, devices)
            self._engine_devices = devices
        return self._engine

    def _drop_engine(self):
        if self._engine is not None:
            self._engine.close()
        self._engine = None

    # ----------------------------------------------------------------- layout
    def _pref(self, p, elem=None):
        if isinstance(p, parameter.ConstantParameter):
            if p.value is None:
                raise ValueError(f"Constant parameter {p.name} has no value: call set_default_params "
                                 "(noise files) first")
            return (-1, float(p.value))
        return (self._index[p.name] + (elem or 0), 0.0)

    def white_fixed(self):
        return all(isinstance(p, parameter.ConstantParameter)
                   for c in self._collections for w in c.white for p in w.params)

    def correlated(self):
        """True if the model has a spatially correlated common process
        (FourierBasisCommonGP with an ORF, enterprise_models.py:390-415)."""
        return any(c.common is not None for c in self._collections)

    def common_layout(self):
        """ORF matrix and spectral entries of the correlated common process;
        checks that every pulsar carries it with the same frequencies."""
        from .models import orf_matrix
        cs = [c.common for c in self._collections]
        if any(c is None for c in cs):
            raise ValueError("a correlated common process must be present in every pulsar")
        ref = cs[0]
        for c in cs[1:]:
            if c["orf"] != ref["orf"] or len(c["cols"]) != len(ref["cols"]) or \
                    not np.allclose([e["f"] for e in c["entries"]], [e["f"] for e in ref["entries"]], rtol=0, atol=0):
                raise ValueError("the correlated common process differs between pulsars (ORF, Tspan or nfreqs)")
        spec = []
        for g, e in enumerate(ref["entries"]):
            spec.append(self._spec_tuple(e, g))
        G = orf_matrix(ref["orf"], [c.psr.pos for c in self._collections])
        return {"orf": np.ascontiguousarray(G), "spec": spec, "n_col": len(ref["cols"]), "kind": ref["orf"]}

    def _spec_tuple(self, e, j):
        if e["kind"] == "const":
            return (_lib.SPEC_CONST, j, (-1, e["value"]), (-1, 0.0), (-1, 0.0), 0.0, 0.0)
        if e["kind"] == "powerlaw":
            pa = e["pars"]
            return (_lib.SPEC_POWERLAW, j, self._pref(pa["log10_A"]), self._pref(pa["gamma"]), (-1, 0.0),
                    e["f"], e["df"])
        if e["kind"] == "turnover":
            pa = e["pars"]
            return (_lib.SPEC_TURNOVER, j, self._pref(pa["log10_A"]), self._pref(pa["gamma"]),
                    self._pref(pa["fc"]), e["f"], e["df"])
        if e["kind"] == "free_spectrum":
            p = e["pars"]["log10_rho"]
            if isinstance(p, parameter.ConstantParameter):
                vals = np.atleast_1d(p.value)
                ref = (-1, float(vals[e["mode"]] if len(vals) > 1 else vals[0]))
            else:
                ref = self._pref(p, e["mode"])
            return (_lib.SPEC_FREESPEC, j, ref, (-1, 0.0), (-1, 0.0), e["f"], 0.0)
        raise ValueError(e["kind"])

    def basis_varies(self):
        """True if some basis depends on theta (chromred 'vary'): no TNT cache."""
        return any(c.basis_groups for c in self._collections)

    def layout(self, common_last=None):
        """Host-side per-pulsar tables for the engine (plain numpy).
        common_last: name of an uncorrelated GP signal whose columns go last
        (the optimal-statistic layout, enterprise_warp_amd.optstat)."""
        out = []
        corr = self.correlated()
        for c in self._collections:
            psr = c.psr
            slots, efac, equad, ep_start, ep_stop, ep_slot = self._white_tables(c)
            # column order: [leading constant-phi | own | common (g order)] when the
            # PTA has a correlated common process (the device keeps the common
            # block for the cross-pulsar factorisation, include/ewarp_hip.h)
            m = c.T.shape[1]
            ncom = 0
            order = np.arange(m)
            if corr or common_last:
                com = list(c.common["cols"]) if corr else list(c.gp_cols[common_last])
                if any(j < c.n_lead_const for j in com) or len(set(com)) != len(com):
                    raise ValueError(f"{c.name}: common columns overlap the timing model or each other")
                own = [j for j in range(m) if j not in set(com)]
                order = np.array(own + com)
                ncom = len(com)
            pos = np.empty(m, int)
            pos[order] = np.arange(m)
            spec = []
            for j, ents in enumerate(c.entries):
                for e in ents:
                    if e.get("common"):
                        continue                      # in the PTA's common descriptor (correlated)
                    spec.append(self._spec_tuple(e, int(pos[j])))
            bgroups = [self._pref(p) for p in c.basis_groups]
            out.append(dict(name=c.name, T=np.ascontiguousarray(c.T[:, order], dtype=float), n_common=ncom,
                            bgroups=bgroups, col_bgroup=np.ascontiguousarray(c.col_bgroup[order], np.int32),
                            ln_chrom=np.ascontiguousarray(c.ln_chrom, dtype=float),
                            resid=np.ascontiguousarray(psr.residuals, dtype=float),
                            toaerr=np.ascontiguousarray(psr.toaerrs, dtype=float),
                            n_lead=c.n_lead_const, slots=slots, efac=efac, equad=equad,
                            ep_start=ep_start, ep_stop=ep_stop, ep_slot=ep_slot, spec=spec))
        return out

    def _white_tables(self, c):
        """White-noise slot table of one pulsar (theta column or constant per
        distinct efac / equad / ecorr parameter) and the per-TOA / per-epoch
        slot indices (include/ewarp_hip.h ewh_pulsar_desc)."""
        n = len(c.psr.toas)
        slots, slot_of = [], {}

        def slot(p):
            if p.name not in slot_of:
                slot_of[p.name] = len(slots)
                slots.append(self._pref(p))
            return slot_of[p.name]

        efac = np.full(n, -1, np.int32)
        equad = np.full(n, -1, np.int32)
        for w in c.white:
            if w.kind == "ecorr":
                continue
            tgt = efac if w.kind == "efac" else equad
            for key, mask in w.masks.items():
                tgt[mask] = slot(w.pars[key])
        if np.any(efac < 0):
            raise ValueError(f"{c.name}: some TOAs are not covered by the efac selection")
        eps = c.ecorr_epochs()
        ep_start = np.array([e[0] for e in eps], np.int32)
        ep_stop = np.array([e[1] for e in eps], np.int32)
        ep_slot = np.array([slot(e[2]) for e in eps], np.int32)
        return slots, efac, equad, ep_start, ep_stop, ep_slot

    # ---------------------------------------------------------------- helpers
    def constant_values(self):
        return {p.name: p.value for p in self._all.values() if isinstance(p, parameter.ConstantParameter)}

    def oracle_terms(self):
        return [c.oracle_terms() for c in self._collections]

    def summary(self):
        lines = [f"PTA with {len(self._collections)} pulsars, {self._nparam} free parameters"]
        for c in self._collections:
            lines.append(f"  {c.name}: n_toa={len(c.psr.toas)} basis={c.T.shape[1]} (tm {c.n_lead_const}) "
                         f"white={[w.kind for w in c.white]}")
        return "\n".join(lines)

    def __repr__(self):
        return self.summary()


def _as_ptr(a, ctype):
    return a.ctypes.data_as(C.POINTER(ctype))


class Engine:
    """Owner of one libewarp_hip handle (one or several devices)."""

    def __init__(self, pta, devices=0, optstat=None):
        """devices: a HIP device id or a list of them (one replica per entry;
        a repeated id gives two contexts on one device).  optstat: None, or
        {"signal": name, "orf": P x P matrix} for an optimal-statistic handle
        (ewh_optstat; see enterprise_warp_amd.optstat)."""
        self.lib = _lib.load()
        self.pta = pta
        self.devices = [int(devices)] if np.isscalar(devices) else [int(d) for d in devices]
        self.device = self.devices[0]
        lay = pta.layout(common_last=optstat["signal"] if optstat else None)
        self.n_pulsar = len(lay)
        self.n_param = pta._nparam
        keep = []
        descs = (_lib.PulsarDesc * len(lay))()
        for i, L in enumerate(lay):
            n, m = L["T"].shape
            slots = (_lib.Pref * max(1, len(L["slots"])))()
            for k, (idx, cv) in enumerate(L["slots"]):
                slots[k] = _lib.Pref(idx, 0, cv)
            spec = (_lib.SpecEntry * max(1, len(L["spec"])))()
            for k, (kind, col, p0, p1, p2, f, df) in enumerate(L["spec"]):
                spec[k] = _lib.SpecEntry(kind, col, _lib.Pref(p0[0], 0, p0[1]), _lib.Pref(p1[0], 0, p1[1]),
                                         _lib.Pref(p2[0], 0, p2[1]), f, df, const.fyr)
            bg = (_lib.Pref * max(1, len(L["bgroups"])))()
            for k, (idx, cv) in enumerate(L["bgroups"]):
                bg[k] = _lib.Pref(idx, 0, cv)
            arrs = [L["T"], L["resid"], L["toaerr"], L["efac"], L["equad"], L["ep_start"], L["ep_stop"],
                    L["ep_slot"], L["col_bgroup"], L["ln_chrom"]]
            keep.extend(arrs + [slots, spec, bg])
            descs[i] = _lib.PulsarDesc(
                n, m, L["n_lead"], len(L["spec"]),
                _as_ptr(L["T"], C.c_double), _as_ptr(L["resid"], C.c_double), _as_ptr(L["toaerr"], C.c_double),
                len(L["slots"]), slots, _as_ptr(L["efac"], C.c_int32), _as_ptr(L["equad"], C.c_int32),
                len(L["ep_start"]), _as_ptr(L["ep_start"], C.c_int32), _as_ptr(L["ep_stop"], C.c_int32),
                _as_ptr(L["ep_slot"], C.c_int32), spec,
                len(L["bgroups"]), bg, _as_ptr(L["col_bgroup"], C.c_int32), _as_ptr(L["ln_chrom"], C.c_double),
                L["n_common"])
        self.white_fixed = pta.white_fixed() and not pta.basis_varies()
        common = None
        self.correlated = pta.correlated()
        if optstat:
            orf = np.ascontiguousarray(optstat["orf"], dtype=float)
            keep.append(orf)
            common = _lib.CommonDesc(L["n_common"], _as_ptr(orf, C.c_double), None, _lib.COMMON_OPTSTAT)
            keep.append(common)
        elif self.correlated:
            cl = pta.common_layout()
            cspec = (_lib.SpecEntry * cl["n_col"])()
            for k, (kind, col, p0, p1, p2, f, df) in enumerate(cl["spec"]):
                cspec[k] = _lib.SpecEntry(kind, col, _lib.Pref(p0[0], 0, p0[1]), _lib.Pref(p1[0], 0, p1[1]),
                                          _lib.Pref(p2[0], 0, p2[1]), f, df, const.fyr)
            keep.extend([cl["orf"], cspec])
            common = _lib.CommonDesc(cl["n_col"], _as_ptr(cl["orf"], C.c_double), cspec, _lib.COMMON_CORRELATED)
            keep.append(common)
        d = _lib.PtaDesc(_lib.EWH_ABI_VERSION, len(lay), self.n_param, int(self.white_fixed), descs,
                         C.pointer(common) if common is not None else None)
        h = C.c_void_p()
        ids = (C.c_int32 * len(self.devices))(*self.devices)
        _lib.check(self.lib.ewh_create(C.byref(d), ids, len(self.devices), C.byref(h)))
        self.h = h
        self.n_slots = [len(L["slots"]) for L in lay]
        del keep
        # sampler-sized calls (one theta per call: PTMCMC / bilby) go through
        # persistent buffers whose addresses are bound once -- building two
        # ctypes pointers per call costs ~5 us, a tenth of the call
        # the latency kernel's batch bound, from the library (LAT_B_MAX)
        self.SMALL_B = max(1, int(self.lib.ewh_lat_b_max()))
        self._small = np.empty((self.SMALL_B, max(1, self.n_param)))
        self._small_out = np.empty(self.SMALL_B)
        self._small_fn = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_void_p, C.c_int32, C.c_void_p)(
            ("ewh_lnl_batch", self.lib))
        self._small_args = (self.h, self._small.ctypes.data, self._small_out.ctypes.data)

    def lat_b_max(self):
        """The latency path's batch bound (ewh_lat_b_max; 0: none)."""
        return int(self.lib.ewh_lat_b_max())

    def lnl_batch(self, theta):
        theta = np.ascontiguousarray(theta, dtype=float)
        B = theta.shape[0]
        if not self.h:
            raise _lib.EngineError("engine is closed")
        if B <= self.SMALL_B and self.n_param > 0:
            self._small[:B] = theta
            h, tp, op = self._small_args
            rc = self._small_fn(h, tp, B, op)
            if rc:
                _lib.check(rc)
            return self._small_out[:B].copy()
        out = np.empty(B)
        _lib.check(self.lib.ewh_lnl_batch(self.h, _as_ptr(theta, C.c_double), B, _as_ptr(out, C.c_double)))
        return out

    def set_fixed_white(self, pta):
        """Push the PTA's current white-noise constants (ewh_set_fixed_white)."""
        vals = []
        for c in pta.signal_collections:
            vals.extend(cv for _, cv in pta._white_tables(c)[0])
        arr = np.ascontiguousarray(vals if vals else [0.0], dtype=float)
        _lib.check(self.lib.ewh_set_fixed_white(self.h, _as_ptr(arr, C.c_double)))

    def num_devices(self):
        return int(self.lib.ewh_num_devices(self.h))

    def dev_gram(self, p, theta):
        """Dev library only: G = T_aug^T N^-1 T_aug of pulsar p per sample."""
        theta = np.ascontiguousarray(np.atleast_2d(theta), dtype=float)
        B = theta.shape[0]
        ld = 16 * ((self.pta.signal_collections[p].T.shape[1] + 1 + 15) // 16)
        G = np.empty((B, ld, ld))
        rc = self.lib.ewh_dev_gram(self.h, int(p), _as_ptr(theta, C.c_double), B, _as_ptr(G, C.c_double))
        if rc < 0:
            _lib.check(rc)
        return G

    def dev_reduced(self, p, n):
        """Dev library only: the cached reduced matrix S_p (n x n) and K_p."""
        S = np.empty((n, n))
        K = np.empty(1)
        rc = self.lib.ewh_dev_reduced(self.h, int(p), _as_ptr(S, C.c_double), _as_ptr(K, C.c_double))
        if rc < 0:
            _lib.check(rc)
        return S, float(K[0])

    def lnl_units_device(self, theta_ptr, B, u0, u1, out_ptr, stream=None):
        _lib.check(self.lib.ewh_lnl_units_device(self.h, C.c_void_p(theta_ptr), int(B), int(u0), int(u1),
                                                 C.c_void_p(out_ptr), C.c_void_p(stream or 0)))

    def contract_device(self, theta_ptr, B, stream=None):
        """Measurement entry (ewh_contract_device): the white-noise stage of a
        varying-white-noise batch alone (N^-1, ECORR, the fp64 MFMA
        contraction), no factorisation."""
        _lib.check(self.lib.ewh_contract_device(self.h, C.c_void_p(theta_ptr), int(B), C.c_void_p(stream or 0)))

    def keep_dim(self):
        """Side of the kept common block of one (pulsar, sample) (0 when the
        model has no correlated common process)."""
        return int(self.lib.ewh_keep_dim(self.h))

    def corr_partial_device(self, theta_ptr, B, p0, p1, keep_ptr, local_ptr, stream=None):
        """Pulsar-partitioned step 1 (ewh_corr_partial_device): pulsars
        [p0, p1) into the pulsar-major keep [P, B, kd, kd] / local [P, B]."""
        _lib.check(self.lib.ewh_corr_partial_device(self.h, C.c_void_p(theta_ptr), int(B), int(p0), int(p1),
                                                    C.c_void_p(keep_ptr), C.c_void_p(local_ptr),
                                                    C.c_void_p(stream or 0)))

    def corr_finish_device(self, theta_ptr, B, keep_ptr, local_ptr, out_ptr, stream=None):
        """Pulsar-partitioned step 2 (ewh_corr_finish_device) on the gathered arrays."""
        _lib.check(self.lib.ewh_corr_finish_device(self.h, C.c_void_p(theta_ptr), int(B), C.c_void_p(keep_ptr),
                                                   C.c_void_p(local_ptr), C.c_void_p(out_ptr),
                                                   C.c_void_p(stream or 0)))

    def optstat(self, theta, phihat, want_pairs=True):
        """ewh_optstat: (rho [B, P, P], sig [B, P, P], OS [B], OS_sig [B])."""
        theta = np.ascontiguousarray(theta, dtype=float)
        phihat = np.ascontiguousarray(phihat, dtype=float)
        B = theta.shape[0]
        P = self.n_pulsar
        rho = np.zeros((B, P, P)) if want_pairs else None
        sig = np.zeros((B, P, P)) if want_pairs else None
        os_, os_sig = np.empty(B), np.empty(B)
        _lib.check(self.lib.ewh_optstat(self.h, _as_ptr(theta, C.c_double), B, _as_ptr(phihat, C.c_double),
                                        _as_ptr(rho, C.c_double) if want_pairs else None,
                                        _as_ptr(sig, C.c_double) if want_pairs else None,
                                        _as_ptr(os_, C.c_double), _as_ptr(os_sig, C.c_double)))
        return rho, sig, os_, os_sig

    def unit_terms(self, B):
        out = np.empty((self.n_pulsar, B))
        _lib.check(self.lib.ewh_last_unit_terms(self.h, _as_ptr(out, C.c_double), int(B)))
        return out

    def transfer_stats(self):
        """(theta bytes host -> device of the last batch, peer-access mask of
        the contexts) -- ewh_transfer_stats."""
        b, m = C.c_int64(), C.c_int64()
        _lib.check(self.lib.ewh_transfer_stats(self.h, C.byref(b), C.byref(m)))
        return int(b.value), int(m.value)

    def refine_stats(self):
        """(units on the double-double route, units chol_dd_kernel refactored)
        since the last query -- ewh_refine_stats (synchronises, resets)."""
        c, r = C.c_int64(), C.c_int64()
        _lib.check(self.lib.ewh_refine_stats(self.h, C.byref(c), C.byref(r)))
        return int(c.value), int(r.value)

    def unit_costs(self):
        return np.array([self.lib.ewh_unit_cost(self.h, p) for p in range(self.n_pulsar)])

    def set_kernel_mode(self, mode):
        _lib.check(self.lib.ewh_set_kernel_mode(self.h, int(mode)))

    def close(self):
        # (the small-batch path's bound arguments hold the raw handle: drop
        # them with it, so a closed engine raises instead of passing a freed
        # handle to ewh_lnl_batch)
        self._small_args = None
        if getattr(self, "h", None):
            self.lib.ewh_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
