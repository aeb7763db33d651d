"""The pulsar-partitioned exchange of a correlated common process (SURVEY.md
§8(e), config 5) on CPU: world_size-2 gloo processes each run step 1 (the
partial factorisations of their pulsars: local terms + kept common blocks, in
the pulsar-major layout of ewh_corr_partial_device), one all-gather moves the
slices, and step 2 (M_g^-1, dense Sigma_c, factorisation) on the gathered
arrays must reproduce the one-process likelihood.  The arithmetic is the
device-order restatement (oracle/device_order_ref.py); on the GPU the same
protocol runs through ewh_corr_partial_device / ewh_corr_finish_device over
RCCL (bench.py --config c5 --partition pulsars) and between the contexts of
one handle (ewh_lnl_batch, tests/test_gpu_properties.py)."""
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


def _setup():
    import sys
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from conftest import load_golden
    from oracle.device_order_ref import DeviceOrderPTA
    pta, z = load_golden("c5_small", full=True)
    const = pta.constant_values()
    dop = DeviceOrderPTA([c.psr for c in pta.signal_collections], pta.oracle_terms(), const, np.float64)
    X = z["theta"][8:12]
    return pta, dop, const, X, z


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    pta, dop, const, X, z = _setup()
    P, B = len(dop.pulsars), len(X)
    p0, p1 = P * rank // world, P * (rank + 1) // world
    kd = None
    local = np.zeros((P, B))
    keep = None
    for b, x in enumerate(X):
        d = dict(const)
        d.update(pta.map_params(x))
        for p in range(p0, p1):
            lv, kb = dop.partial(p, d)
            if keep is None:
                kd = kb.shape[0]
                keep = np.zeros((P, B, kd, kd))
            local[p, b] = lv
            keep[p, b] = kb
    # all-gather of the pulsar slices (equal-size chunks: pad to ceil(P / world))
    per = -(-P // world)
    send_k = torch.zeros((per, B, kd, kd), dtype=torch.float64)
    send_l = torch.zeros((per, B), dtype=torch.float64)
    send_k[: p1 - p0] = torch.from_numpy(keep[p0:p1])
    send_l[: p1 - p0] = torch.from_numpy(local[p0:p1])
    got_k = [torch.zeros_like(send_k) for _ in range(world)]
    got_l = [torch.zeros_like(send_l) for _ in range(world)]
    dist.all_gather(got_k, send_k)
    dist.all_gather(got_l, send_l)
    for r in range(world):
        a0, a1 = P * r // world, P * (r + 1) // world
        keep[a0:a1] = got_k[r][: a1 - a0].numpy()
        local[a0:a1] = got_l[r][: a1 - a0].numpy()
    out = []
    for b, x in enumerate(X):
        d = dict(const)
        d.update(pta.map_params(x))
        out.append(dop.finish(d, list(local[:, b]), [keep[p, b] for p in range(P)]))
    if rank == 0:
        q.put(np.array(out, dtype=float))
    dist.barrier()
    dist.destroy_process_group()


def test_gloo_world2_pulsar_partition_equals_full():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = q.get(timeout=300)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    pta, dop, const, X, z = _setup()
    full = []
    for x in X:
        d = dict(const)
        d.update(pta.map_params(x))
        full.append(dop.lnlikelihood(d))
    np.testing.assert_array_equal(got, np.array(full))
    np.testing.assert_allclose(got, z["lnl"][8:12], rtol=1e-10, atol=1e-6)
