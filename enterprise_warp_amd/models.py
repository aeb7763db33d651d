"""Noise / GW term library with the reference's names, options and priors.

Mirrors `enterprise_warp.enterprise_models.StandardModels`
(enterprise_models.py:19-536): the noise-model JSON names a method, its value
is the method's `option`, and the method returns a Signal built with the
factories in signals.py.  Prior bounds come from `params` (paramfile labels,
defaults in `StandardModels.priors`, enterprise_models.py:65-84).

Deliberate differences:
* system_noise / ppta_band_noise build their flag selections directly; the
  reference's `selection_factory` code-object trick fails on Python >= 3.10
  (SURVEY.md Appendix B.4).
* a numeric chromred option without `_nfreqs` is converted to float (the
  reference passes the string through).
* `gwb` keeps the reference's behaviour for '+'-joined options (only the last
  sub-signal survives, Appendix B.3) unless `combine_plus_terms=True`.
"""
import os

import numpy as np

from . import constants as const
from . import parameter
from . import selections
from . import signals


class StandardModels:
    """Standard single-pulsar and common terms (enterprise_models.py:19)."""

    combine_plus_terms = False

    def __init__(self, psr=None, params=None):
        self.psr = psr
        self.params = params
        self.sys_noise_count = 0
        self.priors = {
            "efac": [0., 10.],
            "equad": [-10., -5.],
            "ecorr": [-10., -5.],
            "sn_lgA": [-20., -6.],
            "sn_gamma": [0., 10.],
            "sn_fc": [-10., -6.],
            "dmn_lgA": [-20., -6.],
            "dmn_gamma": [0., 10.],
            "chrom_idx": [0., 6.],
            "syn_lgA": [-20., -6.],
            "syn_gamma": [0., 10.],
            "gwb_lgA": [-20., -6.],
            "gwb_lgA_prior": "uniform",
            "gwb_lgrho": [-10., -4.],
            "gwb_gamma": [0., 10.],
            "gwb_gamma_prior": "uniform",
            "red_general_freqs": "tobs_60days",
            "red_general_nfouriercomp": 2,
        }
        if psr is not None and not isinstance(psr, list) and not hasattr(psr, "sys_flags"):
            psr.sys_flags, psr.sys_flagvals = [], []

    # ---- paramfile plumbing (enterprise_models.py:90-104) -----------------
    def get_label_attr_map(self):
        out = {}
        for key, val in self.priors.items():
            if isinstance(val, (list, tuple)):
                out[key + ":"] = [key] + [type(val[0])] * len(val)
            else:
                out[key + ":"] = [key, type(val)]
        return out

    def get_default_prior(self, key):
        return self.priors[key]

    # ---- white noise (enterprise_models.py:108-146) ------------------------
    def _selection(self, option, what):
        if option not in selections.REGISTRY:
            raise ValueError(f"{what} option must be an enterprise selection function name, got {option!r}")
        return selections.Selection(selections.REGISTRY[option])

    def efac(self, option="by_backend"):
        se = self._selection(option, "EFAC")
        return signals.MeasurementNoise(efac=interpret_white_noise_prior(self.params.efac), selection=se)

    def equad(self, option="by_backend"):
        se = self._selection(option, "EQUAD")
        return signals.TNEquadNoise(log10_tnequad=interpret_white_noise_prior(self.params.equad), selection=se)

    def ecorr(self, option="by_backend"):
        se = self._selection(option, "ECORR")
        return signals.EcorrKernelNoise(log10_ecorr=interpret_white_noise_prior(self.params.ecorr), selection=se)

    # ---- red / DM / chromatic (enterprise_models.py:148-254) --------------
    def option_nfreqs(self, option, sel_func_name=None, selection_flag=None, selection=None):
        """Strip an `<n>_nfreqs` suffix from `option` (enterprise_models.py:148-167)."""
        has = isinstance(option, str) and "_nfreqs" in option
        if has:
            parts = option.split("_")
            i = parts.index("nfreqs") - 1
            nfreqs = int(parts[i])
            del parts[i]
            del parts[parts.index("nfreqs")]
            option = "_".join(parts)
            if option.replace(".", "", 1).isdigit():
                option = float(option)
        if selection_flag is not None:
            self.psr.sys_flags.append(selection_flag)
            self.psr.sys_flagvals.append(option)
        if not has:
            nfreqs = self.determine_nfreqs(sel_func_name=sel_func_name, selection=selection)
        return option, nfreqs

    def _pl(self, lgA, gamma, turnover=False):
        lA = parameter.Uniform(lgA[0], lgA[1])
        gm = parameter.Uniform(gamma[0], gamma[1])
        comp = self.params.red_general_nfouriercomp
        if turnover:
            fc = parameter.Uniform(self.params.sn_fc[0], self.params.sn_fc[1])
            return signals.powerlaw_bpl(log10_A=lA, gamma=gm, fc=fc, components=comp)
        return signals.powerlaw(log10_A=lA, gamma=gm, components=comp)

    def spin_noise(self, option="powerlaw"):
        option, nfreqs = self.option_nfreqs(option)
        if option not in ("powerlaw", "turnover"):
            raise ValueError(f"spin_noise option {option!r}")
        pl = self._pl(self.params.sn_lgA, self.params.sn_gamma, turnover=option == "turnover")
        return signals.FourierBasisGP(spectrum=pl, Tspan=self.params.Tspan, name="red_noise", components=nfreqs)

    def dm_noise(self, option="powerlaw"):
        option, nfreqs = self.option_nfreqs(option)
        if option not in ("powerlaw", "turnover"):
            raise ValueError(f"dm_noise option {option!r}")
        pl = self._pl(self.params.dmn_lgA, self.params.dmn_gamma, turnover=option == "turnover")
        basis = signals.createfourierdesignmatrix_dm(nmodes=nfreqs, Tspan=self.params.Tspan,
                                                     fref=float(self.params.fref))
        return signals.BasisGP(pl, basis, name="dm_gp")

    def chromred(self, option="vary"):
        option, nfreqs = self.option_nfreqs(option)
        turnover = isinstance(option, str) and "turnover" in option
        if turnover:
            parts = option.split("_")
            del parts[parts.index("turnover")]
            option = "_".join(parts)
        pl = self._pl(self.params.dmn_lgA, self.params.dmn_gamma, turnover=turnover)
        if option == "vary":
            idx = parameter.Uniform(self.params.chrom_idx[0], self.params.chrom_idx[1])
        else:
            idx = float(option)
        basis = signals.createfourierdesignmatrix_chromatic(nmodes=nfreqs, Tspan=self.params.Tspan, idx=idx)
        return signals.BasisGP(pl, basis, name="chromatic_gp")

    # ---- system / band noise (enterprise_models.py:256-338) ----------------
    def _flag_terms(self, option, flag, prefix):
        """One FourierBasisGP per flag value, on that value's TOAs with their own
        span (enterprise_models.py:263-290 / :301-336)."""
        total = None
        for term in option:
            value, nfreqs = term, None
            if isinstance(term, str) and "_nfreqs" in term:
                parts = term.split("_")
                i = parts.index("nfreqs") - 1
                nfreqs = int(parts[i])
                del parts[i]
                del parts[parts.index("nfreqs")]
                value = "_".join(parts)
            turnover = isinstance(value, str) and "turnover" in value
            if turnover:
                parts = value.split("_")
                del parts[parts.index("turnover")]
                value = "_".join(parts)
            sel = selections.flag_value_selection(flag, value)
            self.psr.sys_flags.append(flag)
            self.psr.sys_flagvals.append(value)
            if nfreqs is None:
                nfreqs = self.determine_nfreqs(sel_func_name=f"{prefix}_selection_{self.sys_noise_count}",
                                               selection=sel)
            tspan = self.determine_tspan(selection=sel)
            pl = self._pl(self.params.syn_lgA, self.params.syn_gamma, turnover=turnover)
            t = signals.FourierBasisGP(spectrum=pl, Tspan=tspan, name=f"{prefix}_{self.sys_noise_count}",
                                       selection=selections.Selection(sel), components=nfreqs)
            total = t if total is None else total + t
            self.sys_noise_count += 1
        return total

    def system_noise(self, option=()):
        return self._flag_terms(list(option), "group", "system_noise")

    def ppta_band_noise(self, option=()):
        return self._flag_terms(list(option), "B", "band_noise")

    # ---- common signals (enterprise_models.py:342-432) --------------------
    def gwb(self, option="hd_vary_gamma"):
        name = "gw"
        optsp = option.split("+")
        total = None
        for opt in optsp:
            if "_nfreqs" in opt:
                nfreqs = int(opt.split("_")[opt.split("_").index("nfreqs") - 1])
            else:
                nfreqs = self.determine_nfreqs(common_signal=True)
            if "_gamma" in opt:
                amp_name = f"{name}_log10_A"
                if (len(optsp) > 1 and "hd" in opt) or "namehd" in opt:
                    amp_name += "_hd"
                elif (len(optsp) > 1 and ("varorf" in opt or "interporf" in opt)) or "nameorf" in opt:
                    amp_name += "_orf"
                if self.params.gwb_lgA_prior == "uniform":
                    lgA = parameter.Uniform(self.params.gwb_lgA[0], self.params.gwb_lgA[1])(amp_name)
                elif self.params.gwb_lgA_prior == "linexp":
                    lgA = parameter.LinearExp(self.params.gwb_lgA[0], self.params.gwb_lgA[1])(amp_name)
                else:
                    raise ValueError(f"gwb_lgA_prior {self.params.gwb_lgA_prior!r}")
                gam_name = f"{name}_gamma"
                if "vary_gamma" in opt:
                    gamma = parameter.Uniform(self.params.gwb_gamma[0], self.params.gwb_gamma[1])(gam_name)
                elif "fixed_gamma" in opt:
                    gamma = parameter.Constant(4.33)(gam_name)
                else:
                    sp = opt.split("_")
                    gamma = parameter.Constant(float(sp[sp.index("gamma") - 1]))(gam_name)
                spec = signals.powerlaw(log10_A=lgA, gamma=gamma)
            elif "freesp" in opt:
                rho = parameter.Uniform(self.params.gwb_lgrho[0], self.params.gwb_lgrho[1],
                                        size=nfreqs)(f"{name}_log10_rho")
                spec = signals.free_spectrum(log10_rho=rho)
            else:
                raise ValueError(f"gwb option {opt!r} names no spectrum (_gamma or freesp)")
            if "hd" in opt:
                orf = "hd_noauto" if "noauto" in opt else "hd"
                gwname = "gw_hd" if (len(optsp) > 1 or "namehd" in opt) else "gw"
                gwb = signals.FourierBasisCommonGP(spec, orf, components=nfreqs, name=gwname, Tspan=self.params.Tspan)
            elif "mono" in opt:
                gwb = signals.FourierBasisCommonGP(spec, "monopole", components=nfreqs, name="gw",
                                                   Tspan=self.params.Tspan)
            elif "dipo" in opt:
                gwb = signals.FourierBasisCommonGP(spec, "dipole", components=nfreqs, name="gw",
                                                   Tspan=self.params.Tspan)
            else:
                gwb = signals.FourierBasisGP(spec, components=nfreqs, name="gw", Tspan=self.params.Tspan)
            if self.combine_plus_terms and total is not None:
                total = total + gwb
            else:
                total = gwb            # reference behaviour: last term wins (Appendix B.3)
        return total

    def bayes_ephem(self, option="default"):
        return signals.PhysicalEphemerisSignal(use_epoch_toas=True)

    # ---- frequency / span rules (enterprise_models.py:436-536) ------------
    def determine_nfreqs(self, sel_func_name=None, cadence=60, common_signal=False, selection=None):
        rgf = str(self.params.red_general_freqs)
        if rgf.isdigit():
            n = int(rgf)
        elif rgf == "tobs_60days":
            tobs = self.determine_tspan(common_signal=common_signal, selection=selection)
            n = int(np.round((1. / cadence / const.day - 1 / tobs) / (1 / tobs)))
        else:
            raise ValueError(f"red_general_freqs {rgf!r}")
        opts = getattr(self.params, "opts", None)
        if opts is not None and getattr(opts, "mpi_regime", 0) != 2:
            self.save_nfreqs_information(sel_func_name, n)
        return n

    def determine_tspan(self, sel_func_name=None, common_signal=False, selection=None):
        if common_signal:
            if not isinstance(self.psr, list):
                raise ValueError("Expecting a list of pulsars in self.psr for a common signal")
            return np.max([np.max(p.toas) for p in self.psr]) - np.min([np.min(p.toas) for p in self.psr])
        if selection is None or getattr(selection, "value", None) is None:
            toas = self.psr.toas
        else:
            masks = selection(self.psr)
            if len(masks) != 1:
                raise NotImplementedError
            toas = self.psr.toas[list(masks.values())[0]]
        if len(toas) == 0:
            raise ValueError(f"{self.psr.name}: selection {getattr(selection, '__name__', '')} selects no TOA")
        return np.max(toas) - np.min(toas)

    def save_nfreqs_information(self, sel_func_name, n_freqs):
        out = getattr(self.params, "output_dir", None)
        if not out or not os.path.isdir(out):
            return
        fname = "no_selection" if sel_func_name is None else sel_func_name
        with open(os.path.join(out, fname + "_nfreqs.txt"), "w") as fh:
            fh.write(f"no selection;-;{n_freqs}\n")


def interpret_white_noise_prior(prior):
    """Two numbers -> Uniform(lo, hi); one number -> Constant (value from the
    noise files), enterprise_models.py:540-549."""
    if not np.isscalar(prior):
        return parameter.Uniform(prior[0], prior[1])
    return parameter.Constant()


def hd_orf(pos1, pos2):
    """[ent] utils.hd_orf (enterprise_models.py:397)."""
    if np.all(pos1 == pos2):
        return 1.0
    omc2 = (1 - np.dot(pos1, pos2)) / 2
    return 1.5 * omc2 * np.log(omc2) - 0.25 * omc2 + 0.5


def hd_orf_noauto(pos1, pos2):
    """enterprise_models.py:565-572: HD with zero auto-correlation."""
    if np.all(pos1 == pos2):
        return 0.0
    omc2 = (1 - np.dot(pos1, pos2)) / 2
    return 1.5 * omc2 * np.log(omc2) - 0.25 * omc2 + 0.5


def monopole_orf(pos1, pos2):
    """[ent] utils.monopole_orf (enterprise_models.py:405); the 1e-5 on the
    auto term keeps Gamma invertible (enterprise's regularisation)."""
    return 1.0 + 1e-5 if np.all(pos1 == pos2) else 1.0


def dipole_orf(pos1, pos2):
    """[ent] utils.dipole_orf (enterprise_models.py:411)."""
    return 1.0 + 1e-5 if np.all(pos1 == pos2) else float(np.dot(pos1, pos2))


ORFS = {"hd": hd_orf, "hd_noauto": hd_orf_noauto, "monopole": monopole_orf, "dipole": dipole_orf}


def orf_matrix(kind, positions):
    """Gamma_ab = orf(pos_a, pos_b) over the PTA's pulsars (diagonal included)."""
    f = ORFS[kind]
    P = len(positions)
    G = np.empty((P, P))
    for a in range(P):
        for b in range(P):
            G[a, b] = f(np.asarray(positions[a], float), np.asarray(positions[b], float))
    return G
