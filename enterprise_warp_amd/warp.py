"""Paramfile + noise-model assembly: `Params`, `init_pta` and helpers.

Same file formats and semantics as enterprise_warp.enterprise_warp:
* `parse_commandline` — the same optparse flags (enterprise_warp.py:24-71);
* `Params(prfile, opts, custom_models_obj, init_pulsars)` — `label: values`
  lines typed by a label map extended with the term library's prior keys,
  `{N}` model blocks, defaults, noise-model JSON (`model_name`, `universal`,
  `common_signals`, per-pulsar dicts) (enterprise_warp.py:90-435);
* `init_pta(params)` -> {model_id: PTA}: timing model + common signals +
  per-pulsar terms, constants fixed from noise files (enterprise_warp.py:437-519).

Pulsar loading does not use tempo2 (out of scope): `datadir` may hold `.npz`
pulsar bundles (pulsar.save_bundle) or `.par`/`.tim` pairs, read by
pulsar.pulsar_from_par_tim (synthetic design matrix; residuals drawn from the
white noise with a seed derived from the pulsar name — DESIGN.md §Data).
"""
import ast
import glob
import json
import optparse
import os
import zlib

import numpy as np

from . import pulsar as pulsar_io
from .models import StandardModels
from .pta import PTA
from .signals import TimingModel


def parse_commandline(argv=None):
    p = optparse.OptionParser()
    p.add_option("-n", "--num", help="Pulsar number", default=0, type=int)
    p.add_option("-p", "--prfile", help="Parameter file", type=str)
    p.add_option("-d", "--drop", help="Drop pulsar --num in a full-PTA run (0/1)", default=0, type=int)
    p.add_option("-c", "--clearcache", help="Clear pulsar cache (0/1)", default=0, type=int)
    p.add_option("-m", "--mpi_regime", help="0: no MPI, 1: MPI preparation, 2: MPI run", default=0, type=int)
    p.add_option("-w", "--wipe_old_output", help="Wipe the output directory (0/1)", default=0, type=int)
    p.add_option("-x", "--extra_model_terms", help="Extra noise terms (dict literal)", default=None, type=str)
    opts, _ = p.parse_args(argv)
    return opts


class ModelParams:
    """Per-model parameter holder ({N} blocks, enterprise_warp.py:73-88)."""

    def __init__(self, model_id):
        self.model_id = model_id


def _to_bool(s):
    if isinstance(s, bool):
        return s
    return str(s).strip().lower() in ("1", "true", "yes", "y")


def _auto(s):
    for cast in (int, float):
        try:
            return cast(s)
        except ValueError:
            pass
    if s in ("True", "False"):
        return s == "True"
    return s


class Params:
    BASE_LABELS = {
        "paramfile_label:": ["paramfile_label", str], "datadir:": ["datadir", str], "out:": ["out", str],
        "overwrite:": ["overwrite", str], "array_analysis:": ["array_analysis", str],
        "noisefiles:": ["noisefiles", str], "noise_model_file:": ["noise_model_file", str],
        "sampler:": ["sampler", str], "nsamp:": ["nsamp", int], "setupsamp:": ["setupsamp", _to_bool],
        "mcmc_covm_csv:": ["mcmc_covm_csv", str], "psrlist:": ["psrlist", str], "ssephem:": ["ssephem", str],
        "clock:": ["clock", str], "AMweight:": ["AMweight", int], "DMweight:": ["DMweight", int],
        "SCAMweight:": ["SCAMweight", int], "tm:": ["tm", str], "fref:": ["fref", str],
    }

    def __init__(self, input_file_name, opts=None, custom_models_obj=None, init_pulsars=True, pulsars=None):
        self.input_file_name = input_file_name
        self.base_dir = os.path.dirname(os.path.abspath(input_file_name))
        self.opts = opts
        self.psrs = []
        self.Tspan = None
        self.custom_models_obj = custom_models_obj
        self.noise_model_obj = custom_models_obj if custom_models_obj is not None else StandardModels
        self.sampler_kwargs = {}
        self.label_attr_map = dict(self.BASE_LABELS)
        self.label_attr_map.update(self.noise_model_obj().get_label_attr_map())
        self.model_ids = []
        self.models = {}
        model_id = None
        with open(input_file_name) as fh:
            for line in fh:
                inner = line[line.find("{") + 1:line.find("}")]
                if "{" in line and inner.isdigit():
                    model_id = int(inner)
                    self.create_model(model_id)
                    continue
                if not line.strip() or line[0] == "#":
                    continue
                row = line.split()
                label, data = row[0], row[1:]
                if label in self.label_attr_map:
                    attr, types = self.label_attr_map[label][0], self.label_attr_map[label][1:]
                    if len(types) == 1 and len(data) > 1:
                        types = types * len(data)
                    values = [int(d) if t is type(None) else t(d) for t, d in zip(types, data)]
                elif "sampler" in self.__dict__ and label.endswith(":"):
                    # sampler keyword (the reference types these from bilby's
                    # IMPLEMENTED_SAMPLERS defaults, enterprise_warp.py:156-167)
                    attr = label[:-1]
                    values = [_auto(d) for d in data]
                    self.sampler_kwargs[attr] = values if len(values) > 1 else values[0]
                else:
                    raise KeyError(f"{input_file_name}: unknown paramfile label {label!r}")
                target = self.__dict__ if model_id is None else self.models[model_id].__dict__
                target[attr] = values if len(values) > 1 else values[0]
        if not self.models:
            self.create_model(0)
        self.label = os.path.basename(os.path.normpath(getattr(self, "out", "out")))
        self.override_params_using_opts()
        self.set_default_params()
        self.read_modeldicts()
        self.update_sampler_kwargs()
        if pulsars is not None:
            self.psrs = list(pulsars)
            self._finish_pulsars()
            self.clone_all_params_to_models()
        elif init_pulsars:
            self.init_pulsars()
            self.clone_all_params_to_models()

    def _path(self, p):
        return p if os.path.isabs(p) or os.path.exists(p) else os.path.join(self.base_dir, p)

    def override_params_using_opts(self):
        if self.opts is None:
            return
        for key in self.models:
            for opt, val in vars(self.opts).items():
                if opt in self.models[key].__dict__ and val is not None:
                    self.models[key].__dict__[opt] = val
                    self.label += f"_{opt}_{val}"

    def clone_all_params_to_models(self):
        """Give every model the global attributes it does not set itself
        (enterprise_warp.py:203-206 copies them all; model blocks in the
        reference's examples only set noise_model_file, so the two agree)."""
        for key, val in list(self.__dict__.items()):
            if key == "models":
                continue
            for m in self.models.values():
                if key not in m.__dict__ or key in ("psrs", "Tspan", "output_dir", "opts"):
                    m.__dict__[key] = val
        for m in self.models.values():
            m.__dict__.setdefault("model_name", "Untitled")

    def create_model(self, model_id):
        self.model_ids.append(model_id)
        self.models[model_id] = ModelParams(model_id)

    def update_sampler_kwargs(self):
        for k in list(self.sampler_kwargs):
            if k in self.__dict__:
                self.sampler_kwargs[k] = self.__dict__[k]

    def set_default_params(self):
        d = self.__dict__
        d.setdefault("ssephem", "DE436")
        d.setdefault("clock", None)
        d.setdefault("setupsamp", False)
        if "psrlist" in d and isinstance(d["psrlist"], str):
            self.psrlist = [str(x) for x in np.atleast_1d(np.loadtxt(self._path(d["psrlist"]), dtype=str))]
        else:
            d.setdefault("psrlist", [])
        d.setdefault("psrcachefile", None)
        d.setdefault("tm", "default")
        d.setdefault("inc_events", True)
        d.setdefault("fref", 1400)
        d["mcmc_covm"] = None
        if "mcmc_covm_csv" in d and os.path.isfile(self._path(d["mcmc_covm_csv"])):
            import pandas as pd
            d["mcmc_covm"] = pd.read_csv(self._path(d["mcmc_covm_csv"]), index_col=0)
        for key, val in self.noise_model_obj().priors.items():
            d.setdefault(key, val)
        for m in self.models.values():
            m.modeldict = {}

    def read_modeldicts(self):
        extra = None
        if self.opts is not None and getattr(self.opts, "extra_model_terms", None):
            extra = ast.literal_eval(self.opts.extra_model_terms)

        def load(holder, mkey=None):
            nm = read_json_dict(self._path(holder.noise_model_file))
            holder.common_signals = nm.pop("common_signals")
            holder.model_name = nm.pop("model_name")
            holder.universal = nm.pop("universal")
            if extra is not None and (mkey is None or len(self.models) == 1 or (len(self.models) == 2 and mkey == 1)):
                nm = merge_two_noise_model_dicts(nm, extra)
            holder.noisemodel = nm

        if "noise_model_file" in self.__dict__:
            load(self)
        for mkey, m in self.models.items():
            if "noise_model_file" in m.__dict__:
                load(m, mkey)
        self.label_models = "_".join(getattr(m, "model_name", getattr(self, "model_name", "Untitled"))
                                     for m in self.models.values())

    def _load_all_pulsars(self):
        datadir = self._path(self.datadir)
        bundles = sorted(glob.glob(os.path.join(datadir, "*.npz")))
        if bundles:
            return [pulsar_io.load_bundle(b) for b in bundles]
        parfiles = sorted(glob.glob(os.path.join(datadir, "*.par")))
        timfiles = sorted(glob.glob(os.path.join(datadir, "*.tim")))
        if len(parfiles) != len(timfiles):
            raise ValueError("there should be the same number of .par and .tim files")
        out = []
        for p, t in zip(parfiles, timfiles):
            psr = pulsar_io.pulsar_from_par_tim(p, t)
            rng = np.random.default_rng(zlib.crc32(psr.name.encode()))
            psr.residuals = rng.standard_normal(len(psr.toas)) * psr.toaerrs
            psr.parfile_name, psr.timfile_name = p, t
            out.append(psr)
        return out

    def init_pulsars(self):
        allp = self._load_all_pulsars()
        if str(getattr(self, "array_analysis", "False")) == "True":
            sel = []
            for num, psr in enumerate(allp):
                if self.psrlist and psr.name not in self.psrlist:
                    continue
                if self.opts is not None and self.opts.drop and self.opts.num == num:
                    continue
                sel.append(psr)
            self.psrs = sel
        else:
            num = self.opts.num if self.opts is not None else 0
            self.psrs = [allp[num]]
        self._finish_pulsars()

    def _finish_pulsars(self):
        tmin = min(p.toas.min() for p in self.psrs)
        tmax = max(p.toas.max() for p in self.psrs)
        self.Tspan = tmax - tmin
        out = getattr(self, "out", "out/")
        lab = f"{self.label_models}_{getattr(self, 'paramfile_label', 'v1')}/"
        if str(getattr(self, "array_analysis", "False")) == "True":
            self.output_dir = os.path.join(out, lab)
        else:
            num = self.opts.num if self.opts is not None else 0
            self.output_dir = os.path.join(out, lab, f"{num}_{self.psrs[0].name}/")
        if self.opts is not None and self.opts.mpi_regime != 2:
            if os.path.exists(self.output_dir) and self.opts.wipe_old_output:
                import shutil
                shutil.rmtree(self.output_dir)
            os.makedirs(self.output_dir, exist_ok=True)


def init_pta(params_all):
    """{model_id: PTA} (enterprise_warp.py:437-519)."""
    ptas = {}
    for ii, params in params_all.models.items():
        allpsr_model = params_all.noise_model_obj(psr=params_all.psrs, params=params)
        if params.tm == "default":
            tm = TimingModel()
        else:
            raise NotImplementedError(f"tm: {params.tm} (the reference's ridge_regression branch references "
                                      "undefined functions, SURVEY.md Appendix B.5)")
        m_all = tm
        for term, option in params.common_signals.items():
            m_all = m_all + getattr(allpsr_model, term)(option=option)
        models = []
        for psr in params_all.psrs:
            single = params_all.noise_model_obj(psr=psr, params=params)
            terms = params.noisemodel[psr.name] if psr.name in params.noisemodel else params.universal
            m_sep = m_all
            for term, option in terms.items():
                if not hasattr(single, term):
                    raise AttributeError(f"{type(single).__name__} has no noise term {term!r} "
                                         f"(requested for {psr.name})")
                m_sep = m_sep + getattr(single, term)(option=option)
            models.append(m_sep(psr))
        pta = PTA(models)
        if "noisefiles" in params.__dict__:
            pta.set_default_params(get_noise_dict([p.name for p in params_all.psrs],
                                                  params_all._path(params.noisefiles)))
        if params.opts is not None and params.opts.mpi_regime != 2 and getattr(params, "output_dir", None):
            np.savetxt(os.path.join(params.output_dir, "pars.txt"), pta.param_names, fmt="%s")
        ptas[ii] = pta
    return ptas


def get_noise_dict(psrlist, noisefiles):
    """{param: value} from every `*.json` in `noisefiles` whose path names a
    pulsar of `psrlist` (enterprise_warp.py:543-557)."""
    out = {}
    for ff in sorted(glob.glob(os.path.join(noisefiles, "*.json"))):
        if any(p in ff for p in psrlist):
            with open(ff) as fh:
                out.update(json.load(fh))
    return out


def get_noise_dict_psr(psrname, noisefiles):
    with open(os.path.join(noisefiles, psrname + "_noise.json")) as fh:
        return json.load(fh)


def read_json_dict(json_file):
    with open(json_file) as fh:
        return dict(json.load(fh))


def merge_two_noise_model_dicts(dict1, dict2):
    """Merge {psr: {term: option}} dicts; list options are unioned
    (enterprise_warp.py:591-606)."""
    for psr, terms in dict2.items():
        if psr not in dict1:
            dict1[psr] = terms
            continue
        for term, val in terms.items():
            if term in dict1[psr] and isinstance(dict1[psr][term], list):
                dict1[psr][term] = sorted(set(dict1[psr][term] + list(val)))
            else:
                dict1[psr][term] = val
    return dict1
