"""Benchmark: lnL evaluations / s on BASELINE config 3 (45-pulsar CURN PTA,
fixed white noise, 4096 sampler proposals per GPU per step).

    python bench.py [--gpus N] [--steps K] [--warmup W]
    torchrun --nproc-per-node N bench.py --gpus N ...      (one process per GPU)

A step = one batched likelihood evaluation of B = 4096 * N proposals over all
45 pulsars: the (pulsar, proposal) units are split into N contiguous ranges of
equal cost (enterprise_warp_amd.sharding), each rank runs its range on its
GPU (ewh_lnl_units_device, inputs resident in HBM), and one RCCL all-reduce of
the B-vector of partial lnL completes the batch.  Per-GPU work is fixed as N
grows (weak scaling).  Rank 0 prints ONE JSON line.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "lnL evals/sec (whole node), 45-psr CURN batched; % fp64 MFMA peak"
FP64_MFMA_PEAK_TFLOPS = 78.6   # MI355X dense fp64 matrix (datasheet)
HBM_PEAK_GBS = 8000.0


def algorithmic_flops_per_unit(m):
    """F_chol = m^3/3 and F_solve = 2 m^2 per (pulsar, sample)
    with m = the pulsar's basis columns (timing model included, as enterprise
    factors Sigma); the fixed-WN contraction is cached and not counted."""
    m = np.asarray(m, dtype=float)
    return m ** 3 / 3.0 + 2.0 * m ** 2


def _cpu_worker(args):
    """One single-threaded process timing the oracle on C3 (spawned before
    the parent touches the GPU)."""
    seconds, seed = args
    import os as _os
    _os.environ["OMP_NUM_THREADS"] = "1"
    from threadpoolctl import threadpool_limits
    from enterprise_warp_amd import synth
    from oracle.enterprise_ref import OraclePTA
    with threadpool_limits(limits=1):
        cfg = synth.config_c3()
        pta = cfg.pta
        const = pta.constant_values()
        o = OraclePTA([c.psr for c in pta.signal_collections], pta.oracle_terms(), fixed_params=const)
        X = synth.prior_draws(pta, 512, seed)
        n, t0 = 0, time.perf_counter()
        while time.perf_counter() - t0 < seconds:
            d = dict(const)
            d.update(pta.map_params(X[n % len(X)]))
            o.lnlikelihood(d)
            n += 1
        return n, time.perf_counter() - t0


def cpu_baseline(seconds, procs):
    """The oracle (numpy/scipy restatement of enterprise's likelihood, TNT
    cached as enterprise caches it for fixed white noise), `procs` single-
    threaded processes evaluating independent proposals (SURVEY.md §8(d) mode
    (ii)); aggregate evals/s."""
    import multiprocessing as mp
    ctx = mp.get_context("spawn")
    with ctx.Pool(procs) as pool:
        res = pool.map(_cpu_worker, [(seconds, 100 + i) for i in range(procs)])
    total = sum(n / dt for n, dt in res)
    per = [n / dt for n, dt in res]
    return {"value": total, "unit": "lnL evals/s", "cores": procs, "kind": "port",
            "sample": f"{procs} single-threaded processes x {seconds:.0f} s of full 45-pulsar C3 evaluations "
                      f"(oracle/enterprise_ref.py, cached TNT); {sum(n for n, _ in res)} evaluations, "
                      f"per-process {np.mean(per):.1f} evals/s"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch-per-gpu", type=int, default=4096)
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--cpu-procs", type=int, default=min(16, len(os.sched_getaffinity(0))))
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--kernel-mode", type=int, default=0, help="0 auto (MFMA), 1 LDS fallback")
    ap.add_argument("--config", default="c3", choices=["c3", "c5"],
                    help="c3: the headline 45-pulsar CURN batch (default); c5: 100-pulsar HD-correlated PTA")
    args = ap.parse_args()
    if args.config == "c5":
        return main_c5(args)

    import torch
    import torch.distributed as dist
    from enterprise_warp_amd import sharding, synth

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # CPU baseline first: worker processes are spawned before this process
    # initialises the GPU (no forked child ever carries a HIP context)
    cpu = None
    if world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(args.cpu_seconds, args.cpu_procs)
    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    else:
        torch.cuda.set_device(0)
    dev = torch.device("cuda", local if world > 1 else 0)

    cfg = synth.config_c3()
    pta = cfg.pta
    B = args.batch_per_gpu * world
    X = synth.prior_draws(pta, B, cfg.theta_seed)      # same seed on every rank
    theta = torch.from_numpy(X).to(dev)
    eng = pta.engine(device=dev.index)
    eng.set_kernel_mode(args.kernel_mode)
    costs = eng.unit_costs()
    u0, u1 = sharding.unit_ranges(costs, B, world)[rank]
    out = torch.zeros(B, dtype=torch.float64, device=dev)
    stream = torch.cuda.current_stream(dev)

    def step():
        eng.lnl_units_device(theta.data_ptr(), B, u0, u1, out.data_ptr(), stream.cuda_stream)
        if world > 1:
            dist.all_reduce(out)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]
    t0 = time.perf_counter()
    for i in range(args.steps):
        ev[i][0].record(stream)
        eng.lnl_units_device(theta.data_ptr(), B, u0, u1, out.data_ptr(), stream.cuda_stream)
        ev[i][1].record(stream)
        if world > 1:
            dist.all_reduce(out)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    elapsed = time.perf_counter() - t0
    launch_ms = float(np.mean([a.elapsed_time(b) for a, b in ev]))
    t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed = float(t.item())
    lnl = out.cpu().numpy()

    # roofline of the dominant kernel (chol_mfma): algorithmic flops of this
    # rank's units / average duration of its likelihood launch
    m_psr = np.array([c.T.shape[1] for c in pta.signal_collections])
    f_unit = algorithmic_flops_per_unit(m_psr)
    flops = 0.0
    for p in range(len(m_psr)):
        lo, hi = max(u0, p * B), min(u1, (p + 1) * B)
        flops += max(0, hi - lo) * f_unit[p]
    achieved = flops / (launch_ms * 1e-3) / 1e12
    traffic = None
    pmc = os.path.join(ROOT, "profiles", "pmc_chol.json")
    if os.path.exists(pmc):
        with open(pmc) as fh:
            traffic = json.load(fh).get("hbm_bytes_per_launch")

    if rank == 0:
        value = B * args.steps / elapsed
        rec = {
            "metric": METRIC, "value": value, "unit": "lnL evals/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": 1e3 * elapsed / args.steps, "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "f64",
            "data": "synthetic: seeded 45-pulsar CURN PTA (SURVEY.md §8(d) C3), theta from the priors",
            "config": {"workload": "C3: 45 psr, n=2000..20000 TOAs (495k), ECORR, RN+DM 30 freqs, CURN 14 freqs "
                                   "merged, fixed white noise (TNT cached), basis m=132",
                       "global_batch": B, "batch_per_gpu": args.batch_per_gpu, "n_pulsars": len(m_psr),
                       "parallelism": f"units{world}", "finite_fraction": float(np.mean(np.isfinite(lnl)))},
            "roofline": {"bound": "mfma", "achieved": achieved, "peak": FP64_MFMA_PEAK_TFLOPS, "unit": "TFLOP/s",
                         "frac": achieved / FP64_MFMA_PEAK_TFLOPS, "traffic": traffic,
                         "kernel": "chol_mfma_kernel<8,1,2,8> (blocked LDL^T panel: diagonal block by VALU + DPP, row by MFMA with L^-1)", "launch_ms": launch_ms,
                         "flops_per_launch": flops},
        }
        if cpu is not None:
            rec["cpu_baseline"] = cpu
        print(json.dumps(rec), flush=True)
    if world > 1:
        dist.destroy_process_group()


def main_c5(args):
    """BASELINE config 5 (100 pulsars x 20k TOAs, Hellings-Downs GWB, fixed
    white noise).  Samples are sharded over ranks (each rank evaluates its own
    proposals over all pulsars: the cross-pulsar factorisation needs every
    pulsar of a sample, and sample sharding has no data-path exchange), so
    per-GPU work is fixed as N grows (weak scaling)."""
    import torch
    import torch.distributed as dist
    from enterprise_warp_amd import synth
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    else:
        torch.cuda.set_device(0)
    dev = torch.device("cuda", local if world > 1 else 0)
    cfg = synth.config_c5()
    pta = cfg.pta
    Bg = cfg.B
    X = synth.prior_draws(pta, Bg * world, cfg.theta_seed)[rank * Bg:(rank + 1) * Bg]
    theta = torch.from_numpy(np.ascontiguousarray(X)).to(dev)
    eng = pta.engine(device=dev.index)
    out = torch.zeros(Bg, dtype=torch.float64, device=dev)
    stream = torch.cuda.current_stream(dev)
    U = len(pta.signal_collections) * Bg
    for _ in range(args.warmup):
        eng.lnl_units_device(theta.data_ptr(), Bg, 0, U, out.data_ptr(), stream.cuda_stream)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        eng.lnl_units_device(theta.data_ptr(), Bg, 0, U, out.data_ptr(), stream.cuda_stream)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    elapsed = time.perf_counter() - t0
    t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed = float(t.item())
    lnl = out.cpu().numpy()
    P = len(pta.signal_collections)
    nc = pta.common_layout()["n_col"]
    m = np.array([c.T.shape[1] for c in pta.signal_collections])
    # algorithmic work per sample: enterprise's sparse factorisation of the
    # global Sigma = local eliminations (m_a^3/3 each) + the dense common
    # block ((P n_c + 1)^3 / 3)
    flops = Bg * (float(np.sum(m ** 3 / 3.0)) + (P * nc + 1) ** 3 / 3.0)
    achieved = flops * args.steps / elapsed / 1e12
    if rank == 0:
        rec = {"metric": "lnL evals/sec (whole node), 100-psr HD-correlated PTA (BASELINE config 5)",
               "value": Bg * world * args.steps / elapsed, "unit": "lnL evals/s", "n_gpus": world,
               "steps": args.steps, "warmup": args.warmup, "ms_per_step": 1e3 * elapsed / args.steps,
               "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f64",
               "data": "synthetic: seeded 100-pulsar x 20k-TOA PTA, HD GWB 14 freqs (SURVEY.md §8(d) C5)",
               "config": {"workload": "C5: 100 psr x 20k TOAs, ECORR, RN+DM 30 freqs, HD GWB 14 freqs, fixed WN; "
                                      "dense common block 2801^2 per sample",
                          "global_batch": Bg * world, "batch_per_gpu": Bg, "n_pulsars": P,
                          "parallelism": f"samples{world}", "finite_fraction": float(np.mean(np.isfinite(lnl)))},
               "roofline": {"bound": "mfma", "achieved": achieved, "peak": FP64_MFMA_PEAK_TFLOPS, "unit": "TFLOP/s",
                            "frac": achieved / FP64_MFMA_PEAK_TFLOPS, "traffic": None,
                            "kernel": "whole step (partial chol + M_g^-1 + dense factorisation)"}}
        print(json.dumps(rec), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
