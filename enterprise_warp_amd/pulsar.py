"""Pulsar data objects (the input side of the likelihood).

In the reference, pulsars come from `enterprise.pulsar.Pulsar(par, tim,
ephem, clk)` through libstempo/tempo2 (enterprise_warp.py:382-383,
:409-411) or from a pickled list of them (`.pkl` datadir, :350-355).  tempo2
is out of scope, so this module provides:

* `Pulsar` — the attributes the likelihood reads from an enterprise Pulsar:
  name, toas [s], residuals [s], toaerrs [s], freqs [MHz], flags, Mmat
  (design matrix), pos (unit vector), backend_flags.  TOAs are sorted on
  construction, as enterprise sorts them (its `_isort`).
* a `.npz` "pulsar bundle" format (`save_bundle` / `load_bundle`): the
  tempo2-free replacement of the `.pkl` datadir.
* `.tim` / `.par` readers.  Without tempo2 there are no post-fit residuals
  and no design matrix: `pulsar_from_par_tim` builds a synthetic linear
  timing model with one column per fitted `.par` parameter (offset, spin,
  astrometry, DM, JUMPs) and leaves the residuals to the caller (the
  synthetic generator draws them from the noise model).
"""
import numpy as np

from . import constants as const
from .selections import backend_flags as _backend_flags


class Pulsar:
    def __init__(self, name, toas, residuals, toaerrs, freqs, flags=None, Mmat=None, pos=None,
                 fitpars=None, telescope=None, sort=True):
        toas = np.asarray(toas, dtype=float)
        n = len(toas)
        isort = np.argsort(toas, kind="mergesort") if sort else np.arange(n)
        self.name = str(name)
        self.toas = toas[isort]
        self.residuals = np.asarray(residuals, dtype=float)[isort]
        self.toaerrs = np.asarray(toaerrs, dtype=float)[isort]
        self.freqs = np.asarray(freqs, dtype=float)[isort]
        self.flags = {k: np.asarray(v, dtype=str)[isort] for k, v in (flags or {}).items()}
        M = np.ones((n, 1)) if Mmat is None else np.asarray(Mmat, dtype=float)
        self.Mmat = M[isort]
        self.pos = np.asarray(pos if pos is not None else [1.0, 0.0, 0.0], dtype=float)
        self.fitpars = list(fitpars) if fitpars is not None else ["Offset"] + [f"p{i}" for i in range(1, M.shape[1])]
        if telescope is not None:
            self.telescope = np.asarray(telescope, dtype=str)[isort]
        self._bf = None

    @property
    def backend_flags(self):
        if self._bf is None:
            self._bf = _backend_flags(self.flags, len(self.toas))
        return self._bf

    def __repr__(self):
        return f"Pulsar({self.name}, n_toa={len(self.toas)}, n_tm={self.Mmat.shape[1]})"


# ----------------------------------------------------------------------------
# bundle format
# ----------------------------------------------------------------------------
def save_bundle(psr, path):
    flag_names = sorted(psr.flags)
    np.savez(path, name=np.array(psr.name), toas=psr.toas, residuals=psr.residuals, toaerrs=psr.toaerrs,
             freqs=psr.freqs, Mmat=psr.Mmat, pos=psr.pos, fitpars=np.array(psr.fitpars, dtype=str),
             flag_names=np.array(flag_names, dtype=str),
             **{"flag__" + k: psr.flags[k] for k in flag_names})


def load_bundle(path):
    with np.load(path, allow_pickle=False) as z:
        flags = {str(k): z["flag__" + str(k)] for k in z["flag_names"]}
        return Pulsar(str(z["name"]), z["toas"], z["residuals"], z["toaerrs"], z["freqs"], flags=flags,
                      Mmat=z["Mmat"], pos=z["pos"], fitpars=[str(x) for x in z["fitpars"]], sort=False)


# ----------------------------------------------------------------------------
# .tim / .par readers (tempo2 FORMAT 1)
# ----------------------------------------------------------------------------
_TIM_SKIP = {"FORMAT", "MODE", "C", "#", "JUMP", "TIME", "EFAC", "EQUAD", "INCLUDE", "SKIP", "NOSKIP", "END"}


def read_tim(path):
    """Parse a tempo2 FORMAT-1 .tim file.

    Returns dict(names, freqs [MHz], mjd [days, float64], errs [us], sites,
    flags {name: array of str}).  Flags missing on a TOA read ''."""
    rows = []
    with open(path) as fh:
        for line in fh:
            s = line.strip()
            if not s or s.split()[0] in _TIM_SKIP or s.startswith("#") or s.startswith("C "):
                continue
            tok = s.split()
            if len(tok) < 5:
                continue
            fl = {}
            rest = tok[5:]
            i = 0
            while i < len(rest):
                if rest[i].startswith("-") and not _isnum(rest[i]):
                    key = rest[i][1:]
                    val = rest[i + 1] if i + 1 < len(rest) else ""
                    fl[key] = val
                    i += 2
                else:
                    i += 1
            rows.append((tok[0], float(tok[1]), float(tok[2]), float(tok[3]), tok[4], fl))
    keys = sorted({k for r in rows for k in r[5]})
    return {
        "names": np.array([r[0] for r in rows]),
        "freqs": np.array([r[1] for r in rows]),
        "mjd": np.array([r[2] for r in rows]),
        "errs": np.array([r[3] for r in rows]),
        "sites": np.array([r[4] for r in rows]),
        "flags": {k: np.array([r[5].get(k, "") for r in rows], dtype=str) for k in keys},
    }


def _isnum(s):
    try:
        float(s)
        return True
    except ValueError:
        return False


def read_par(path):
    """Parse a tempo2 .par file: {'name', 'values': {key: str}, 'fit': [keys
    with fit flag 1], 'jumps': [(flag, value) of fitted JUMPs], 'ra', 'dec'}."""
    vals, fit, jumps = {}, [], []
    with open(path) as fh:
        for line in fh:
            s = line.strip()
            if not s or s.startswith("#") or s.startswith("C "):
                continue
            tok = s.split()
            key = tok[0]
            if key == "JUMP":
                # JUMP -flag value offset fitflag
                if len(tok) >= 5 and tok[1].startswith("-") and tok[-1] == "1":
                    jumps.append((tok[1][1:], tok[2]))
                continue
            vals[key] = tok[1] if len(tok) > 1 else ""
            if len(tok) >= 3 and tok[2] == "1" and key not in ("START", "FINISH"):
                fit.append(key)
    name = vals.get("PSRJ", vals.get("PSR", "unknown"))
    return {"name": name, "values": vals, "fit": fit, "jumps": jumps}


def _radec_to_pos(ra, dec):
    def sexa(x, hours):
        sign = -1.0 if x.strip().startswith("-") else 1.0
        parts = [abs(float(p)) for p in x.replace("-", "").split(":")]
        while len(parts) < 3:
            parts.append(0.0)
        v = parts[0] + parts[1] / 60 + parts[2] / 3600
        return sign * v * (15.0 if hours else 1.0)
    try:
        a = np.deg2rad(sexa(ra, True))
        d = np.deg2rad(sexa(dec, False))
    except Exception:
        return np.array([1.0, 0.0, 0.0])
    return np.array([np.cos(d) * np.cos(a), np.cos(d) * np.sin(a), np.sin(d)])


def synthetic_design_matrix(toas, freqs, flags, par):
    """A linear timing model with the column count tempo2 would produce:
    offset + one column per fitted .par parameter + one per fitted JUMP.
    Column shapes are physically motivated stand-ins (NOT tempo2 derivatives):
    spin F0/F1/F2: t, t^2, t^3; RAJ/DECJ/PMRA/PMDEC/PX: annual / semi-annual
    harmonics (times t for proper motion); DM, DM1, DM2: nu^-2 * t^k;
    JUMP: indicator of the flag value."""
    t = (toas - toas.mean()) / (toas.max() - toas.min() + 1.0)
    ph = 2 * np.pi * toas / const.yr
    nu2 = (1400.0 / freqs) ** 2
    cols = [np.ones_like(t)]
    names = ["Offset"]
    for key in par["fit"]:
        if key == "F0":
            c = t
        elif key == "F1":
            c = t ** 2
        elif key == "F2":
            c = t ** 3
        elif key in ("RAJ", "ELONG", "RA"):
            c = np.sin(ph)
        elif key in ("DECJ", "ELAT", "DEC"):
            c = np.cos(ph)
        elif key in ("PMRA", "PMELONG"):
            c = t * np.sin(ph)
        elif key in ("PMDEC", "PMELAT"):
            c = t * np.cos(ph)
        elif key == "PX":
            c = np.cos(2 * ph)
        elif key == "DM":
            c = nu2
        elif key.startswith("DM") and key[2:].isdigit():
            c = nu2 * t ** int(key[2:])
        else:
            c = np.sin((len(cols) + 1) * ph / 3.0)
        cols.append(c)
        names.append(key)
    for flag, val in par["jumps"]:
        fv = flags.get(flag, np.array([""] * len(toas)))
        cols.append((fv == val).astype(float))
        names.append(f"JUMP_{flag}_{val}")
    return np.array(cols).T, names


def pulsar_from_par_tim(parfile, timfile, residuals=None):
    """Pulsar from tempo2 files without tempo2: TOAs, errors, frequencies and
    flags from the .tim; name, sky position and the fitted-parameter list
    from the .par; synthetic design matrix; residuals zero unless given."""
    tim = read_tim(timfile)
    par = read_par(parfile)
    toas = tim["mjd"] * const.day
    M, names = synthetic_design_matrix(toas, tim["freqs"], tim["flags"], par)
    pos = _radec_to_pos(par["values"].get("RAJ", "0:0:0"), par["values"].get("DECJ", "0:0:0"))
    res = np.zeros_like(toas) if residuals is None else residuals
    return Pulsar(par["name"], toas, res, tim["errs"] * 1e-6, tim["freqs"], flags=tim["flags"], Mmat=M,
                  pos=pos, fitpars=names, telescope=tim["sites"])
