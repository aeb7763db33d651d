"""Optimal statistic on the GPU: the reference's noise-marginalised OS
(results.py:653-795: `OptimalStatisticWarp` calling enterprise_extensions
`OptimalStatistic(psrs, pta=pta, orf=orf).compute_os(params)` once per chain
draw) as one batched device call over all draws.

    os = OptimalStatistic(pta, orf="hd")                 # pta: the CURN model ('gw' signal)
    xi, rho, sig, OS, OS_sig = os.compute_os(params)     # enterprise_extensions' return tuple
    OS, OS_sig = os.compute_noise_marginalised_os(X)     # X [N, nparam] chain draws

Per pulsar the handle factors Sigma = TNT + phi^-1 (the CURN prior, common
process included, exactly the likelihood's Sigma) with the common columns
last, and reads X = F^T P^-1 r and Z = F^T P^-1 F off the kept block
(include/ewarp_hip.h: ewh_optstat); the pair sums and the ORF-weighted
combination run on the device too.
"""
import numpy as np

from .models import orf_matrix
from .pta import Engine

FYR = 1.0 / (365.25 * 86400.0)


def unit_powerlaw(f, df, gamma):
    """[ent] utils.powerlaw with log10_A = 0 (enterprise_extensions' phiIJ)."""
    return 1.0 / (12.0 * np.pi ** 2) * FYR ** (gamma - 3.0) * f ** (-gamma) * df


class OptimalStatistic:
    def __init__(self, pta, orf="hd", gw_name="gw", gamma_common=None, device=0):
        self.pta = pta
        self.gw_name = gw_name
        cols = [c.gp_cols.get(gw_name) for c in pta.signal_collections]
        if any(c is None for c in cols) or len({len(c) for c in cols}) != 1:
            raise ValueError(f"every pulsar needs the uncorrelated common signal {gw_name!r} (a CURN model)")
        ents = pta.signal_collections[0].gp_entries[gw_name]
        self.freqs = np.array([e["f"] for e in ents])
        self.df = np.array([e["df"] for e in ents])
        self.psrlocs = np.array([c.psr.pos for c in pta.signal_collections], dtype=float)
        self.orf_name = orf
        self.orf = orf_matrix(orf, self.psrlocs)
        self.gamma_common = gamma_common
        self.engine = Engine(pta, device, optstat={"signal": gw_name, "orf": self.orf})
        self._igam = pta.param_names.index(f"{gw_name}_gamma") if f"{gw_name}_gamma" in pta.param_names else None

    def _phihat(self, X):
        if self.gamma_common is not None:
            g = np.full(len(X), float(self.gamma_common))
        elif self._igam is not None:
            g = X[:, self._igam]
        else:
            const = self.pta.constant_values().get(f"{self.gw_name}_gamma")
            g = np.full(len(X), 13.0 / 3.0 if const is None else const)
        return unit_powerlaw(self.freqs[None, :], self.df[None, :], g[:, None])

    def compute_noise_marginalised_os(self, X, want_pairs=False):
        X = np.atleast_2d(np.asarray(X, dtype=float))
        rho, sig, os_, os_sig = self.engine.optstat(X, self._phihat(X), want_pairs=want_pairs)
        return (os_, os_sig, rho, sig) if want_pairs else (os_, os_sig)

    def compute_os(self, params=None):
        """(xi, rho, sig, OS, OS_sig) over pairs a < b, as enterprise_extensions."""
        x = self.pta._theta(params)
        os_, os_sig, rho, sig = self.compute_noise_marginalised_os(x, want_pairs=True)
        P = len(self.psrlocs)
        iu = np.triu_indices(P, 1)
        xi = np.arccos(np.clip(np.einsum("ij,ij->i", self.psrlocs[iu[0]], self.psrlocs[iu[1]]), -1, 1))
        return xi, rho[0][iu], sig[0][iu], float(os_[0]), float(os_sig[0])
