"""Work partitioning over GPUs (one process per GPU).

The likelihood of a batch is a sum over units u = pulsar * B + sample, each
one (pulsar, sample) factorisation; units are independent (uncorrelated and
CURN models share theta, not matrices — SURVEY.md §8(e)).  Each rank takes a
contiguous range of units with equal total cost, evaluates its partial lnL
vector for all B samples, and one RCCL all-reduce (sum) of the B-vector
completes the batch.
"""
import numpy as np


def unit_ranges(unit_costs, B, world):
    """Split units [0, P*B) into `world` contiguous ranges of ~equal cost.

    unit_costs: cost of one unit of each pulsar (length P).  Returns a list of
    (begin, end) pairs covering every unit exactly once."""
    c = np.asarray(unit_costs, dtype=float)
    P = len(c)
    if world <= 1:
        return [(0, P * B)]
    cum_psr = np.concatenate([[0.0], np.cumsum(c * B)])   # cost before pulsar p
    total = cum_psr[-1]
    bounds = [0]
    for r in range(1, world):
        target = total * r / world
        p = int(np.searchsorted(cum_psr, target, side="right") - 1)
        p = min(max(p, 0), P - 1)
        within = (target - cum_psr[p]) / c[p] if c[p] > 0 else 0.0
        u = p * B + int(round(within))
        bounds.append(min(max(u, bounds[-1]), P * B))
    bounds.append(P * B)
    return [(bounds[i], bounds[i + 1]) for i in range(world)]
