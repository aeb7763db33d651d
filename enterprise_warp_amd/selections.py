"""TOA selections, as enterprise_warp uses them.

`StandardModels.efac/equad/ecorr(option)` accept the name of an
[ent] enterprise.signals.selections function (enterprise_models.py:113-115,
:125-128, :140-143); system / band noise build per-flag selections with
`selection_factory` (enterprise_models.py:576-642).  A selection maps a pulsar
to {key: boolean TOA mask}; keys become part of parameter names.
"""
import numpy as np


def backend_flags(flags, n):
    """[ent] Pulsar.backend_flags: per TOA, the first present flag of
    `group`, `g`, `sys`, `i`, `f`, `fe`+`be` (joined by '_'), else 'flag'."""
    out = ["flag"] * n
    order = (("group",), ("g",), ("sys",), ("i",), ("f",), ("fe", "be"))
    for i in range(n):
        for names in order:
            if all(nm in flags and flags[nm][i] != "" for nm in names):
                out[i] = "_".join(flags[nm][i] for nm in names)
                break
    return np.array(out, dtype=str)


def no_selection(psr):
    return {"": np.ones(len(psr.toas), dtype=bool)}


def by_backend(psr):
    bf = psr.backend_flags
    return {v: bf == v for v in np.unique(bf)}


def _by_flag(flag):
    def sel(psr):
        vals = np.asarray(psr.flags.get(flag, np.array([""] * len(psr.toas))), dtype=str)
        return {v: vals == v for v in np.unique(vals)}
    sel.__name__ = "by_" + flag
    return sel


by_band = _by_flag("B")
by_frontend = _by_flag("fe")


def by_telescope(psr):
    tel = np.asarray(getattr(psr, "telescope", np.array(["unknown"] * len(psr.toas))), dtype=str)
    return {v: tel == v for v in np.unique(tel)}


def flag_value_selection(flag, value):
    """The selection `selection_factory` builds for one system/band-noise term:
    {value: flags[flag] == value} (enterprise_models.py:596-610)."""
    def sel(psr):
        vals = np.asarray(psr.flags.get(flag, np.array([""] * len(psr.toas))), dtype=str)
        return {str(value): vals == str(value)}
    sel.__name__ = f"flag_{flag}_{value}"
    sel.flag, sel.value = flag, str(value)
    return sel


# names accepted as an efac/equad/ecorr option (enterprise selection functions)
REGISTRY = {
    "no_selection": no_selection,
    "by_backend": by_backend,
    "by_band": by_band,
    "by_frontend": by_frontend,
    "by_telescope": by_telescope,
}


class Selection:
    """Wrapper matching enterprise's `selections.Selection(func)`."""

    def __init__(self, func):
        self.func = func
        self.name = getattr(func, "__name__", "selection")

    def masks(self, psr):
        return self.func(psr)
