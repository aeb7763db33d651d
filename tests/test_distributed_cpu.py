"""The N>1 path on CPU: world_size-2 gloo processes split the (pulsar, sample)
units with sharding.unit_ranges, each sums its partial lnL vector (unit
terms from the CPU oracle here — the device call needs a GPU) and one
all-reduce(sum) must reproduce the full likelihood vector (the same
protocol bench.py runs over RCCL)."""
import os
import socket

import numpy as np
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _unit_terms():
    from conftest import load_golden
    from oracle.enterprise_ref import OraclePTA
    pta, X, lnl, _ = load_golden("c3_small")
    const = pta.constant_values()
    o = OraclePTA([c.psr for c in pta.signal_collections], pta.oracle_terms(), fixed_params=const)
    B = len(X)
    terms = np.zeros((len(o.pulsars), B))
    for b, x in enumerate(X):
        d = dict(const)
        d.update(pta.map_params(x))
        for p in range(len(o.pulsars)):
            sub = OraclePTA.__new__(OraclePTA)
            sub.pulsars, sub.fixed = [o.pulsars[p]], [o.fixed[p]]
            terms[p, b] = sub.lnlikelihood(d)
    return terms, lnl


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import sys
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from enterprise_warp_amd import sharding
    terms, lnl = _unit_terms()
    P, B = terms.shape
    u0, u1 = sharding.unit_ranges(np.ones(P), B, world)[rank]
    part = np.zeros(B)
    for u in range(u0, u1):
        part[u % B] += terms[u // B, u % B]
    t = torch.from_numpy(part)
    dist.all_reduce(t)
    if rank == 0:
        q.put((t.numpy().copy(), lnl))
    dist.barrier()
    dist.destroy_process_group()


def test_gloo_world2_sharded_sum_equals_full():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    got, want = q.get(timeout=300)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    np.testing.assert_allclose(got, want, rtol=1e-11, atol=1e-6)
