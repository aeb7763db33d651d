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


def host_cpu_info():
    """Cores this process may use and what they are: sched_getaffinity, the
    cgroup CPU quota (cgroup v2 cpu.max / v1 cfs quota), lscpu model /
    sockets / cores per socket.  usable = min(affinity, quota)."""
    import math
    import subprocess
    aff = len(os.sched_getaffinity(0))
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as fh:
            q, per = fh.read().split()[:2]
            if q != "max":
                quota = float(q) / float(per)
    except OSError:
        try:
            with open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us") as fh:
                q = float(fh.read())
            with open("/sys/fs/cgroup/cpu/cpu.cfs_period_us") as fh:
                per = float(fh.read())
            if q > 0:
                quota = q / per
        except OSError:
            pass
    usable = aff if quota is None else max(1, min(aff, int(math.floor(quota + 1e-9))))
    info = {"affinity_cpus": aff, "cgroup_quota_cpus": quota, "usable_cpus": usable}
    try:
        out = subprocess.run(["lscpu"], capture_output=True, text=True, timeout=20).stdout
        kv = dict(line.split(":", 1) for line in out.splitlines() if ":" in line)
        info.update({"model": kv.get("Model name", "").strip(), "sockets": kv.get("Socket(s)", "").strip(),
                     "cores_per_socket": kv.get("Core(s) per socket", "").strip(),
                     "threads_per_core": kv.get("Thread(s) per core", "").strip(),
                     "online_cpus": kv.get("CPU(s)", "").strip()})
    except Exception:  # noqa: BLE001
        pass
    return info


def _cpu_worker(args):
    """Time the oracle on C3 for `seconds` with `threads` BLAS threads
    (spawned before the parent touches the GPU)."""
    seconds, seed, threads = args
    import os as _os
    _os.environ["OMP_NUM_THREADS"] = str(threads)
    from threadpoolctl import threadpool_limits
    from enterprise_warp_amd import synth
    from oracle.enterprise_ref import OraclePTA
    with threadpool_limits(limits=threads):
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


def cpu_baseline(seconds, procs=None):
    """The CPU likelihood on the same host, SURVEY.md §8(d): the oracle
    (numpy/scipy restatement of enterprise's lnL, TNT cached as enterprise
    caches it for fixed white noise) timed in two modes over the host's
    usable cores -- (i) one process, BLAS threads = usable cores;
    (ii) one single-threaded process per usable core, independent
    proposals -- and the better aggregate reported."""
    import multiprocessing as mp
    info = host_cpu_info()
    n = procs or info["usable_cpus"]
    ctx = mp.get_context("spawn")
    with ctx.Pool(1) as pool:
        n1, dt1 = pool.map(_cpu_worker, [(seconds, 100, n)])[0]
    mode1 = n1 / dt1
    with ctx.Pool(n) as pool:
        res = pool.map(_cpu_worker, [(seconds, 100 + i, 1) for i in range(n)])
    mode2 = sum(k / dt for k, dt in res)
    best = max(mode1, mode2)
    return {"value": best, "unit": "lnL evals/s", "cores": n, "kind": "port",
            "mode_i_one_process_blas_threads": mode1, "mode_ii_single_thread_processes": mode2,
            "best_mode": "i" if mode1 >= mode2 else "ii", "host": info,
            "sample": f"full 45-pulsar C3 evaluations of oracle/enterprise_ref.py (cached TNT, scipy cho_factor) "
                      f"on {n} usable cores ({info.get('model', '?')}): mode (i) 1 process x {n} BLAS threads x "
                      f"{seconds:.0f} s = {n1} evaluations; mode (ii) {n} single-threaded processes x {seconds:.0f} s "
                      f"= {sum(k for k, _ in res)} evaluations; value = the better mode"}


def contraction_work(pta):
    """SURVEY.md §8(d) per (pulsar, sample), varying white noise: algorithmic
    flops of T^T N^-1 T, T^T N^-1 r, r^T N^-1 r, log|N| (+ ECORR terms) --
    F = n m (m + 1) + 2 n m + 3 n + 2 n (m + 1) + E (m + 1)^2 -- and the bytes
    the N-weighted basis read streams: B_bytes = 8 n m + 20 n (T, r, sigma,
    backend and epoch indices once per sample; B_tile = 1).  Summed over
    pulsars."""
    flops = bytes_ = 0.0
    for c in pta.signal_collections:
        n, m = c.T.shape
        E = len(c.ecorr_epochs())
        flops += n * m * (m + 1) + 2 * n * m + 3 * n + (2 * n * (m + 1) + E * (m + 1) ** 2 if E else 0)
        bytes_ += 8 * n * m + 20 * n
    return flops, bytes_


def secondary_configs(dev, steps=5):
    """BASELINE configs 2 and 4 (white noise varying every call), measured in
    this run on this GPU: lnL evals/s of the full batch (ewh_lnl_units_device,
    HIP events around `steps` launches) and, for the contraction stage alone
    (ewh_contract_device: N^-1, ECORR, the fp64 MFMA T^T N^-1 T), its
    algorithmic fp64 rate against the MFMA peak and the N-weighted basis
    stream in GB/s against HBM peak."""
    import torch
    from enterprise_warp_amd import synth
    out = {}
    for name, make in (("c2", synth.config_c2), ("c4", synth.config_c4)):
        cfg = make()
        pta, B = cfg.pta, cfg.B
        X = synth.prior_draws(pta, B, cfg.theta_seed)
        th = torch.from_numpy(X).to(dev)
        eng = pta.engine(device=dev.index)
        U = len(pta.signal_collections) * B
        res = torch.zeros(B, dtype=torch.float64, device=dev)
        st = torch.cuda.current_stream(dev)

        def timed(fn):
            fn()
            torch.cuda.synchronize(dev)
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(st)
            for _ in range(steps):
                fn()
            b.record(st)
            torch.cuda.synchronize(dev)
            return a.elapsed_time(b) / steps

        ms = timed(lambda: eng.lnl_units_device(th.data_ptr(), B, 0, U, res.data_ptr(), st.cuda_stream))
        cms = timed(lambda: eng.contract_device(th.data_ptr(), B, st.cuda_stream))
        f, by = contraction_work(pta)
        tf = f * B / (cms * 1e-3) / 1e12
        gbs = by * B / (cms * 1e-3) / 1e9
        out[name] = {"evals_per_s": B / (ms * 1e-3), "ms_per_batch": ms, "batch": B,
                     "finite_fraction": float(np.mean(np.isfinite(res.cpu().numpy()))),
                     "contraction": {"ms": cms, "share_of_batch": cms / ms,
                                     "algorithmic_tflops": tf, "fp64_mfma_frac": tf / FP64_MFMA_PEAK_TFLOPS,
                                     "basis_stream_GBs": gbs, "hbm_frac": gbs / HBM_PEAK_GBS,
                                     "flops_per_sample": f, "bytes_per_sample": by}}
        pta._drop_engine()
        del th, res
    out["note"] = ("configs 2 and 4 at their stated sizes, prior draws, white noise varying every call; "
                   "contraction = ewh_contract_device alone (wn_weights + contract2_kernel); the basis stream "
                   "is the algorithmic bytes each sample's workgroup reads (T is L2/MALL resident across samples)")
    return out


def secondary_c5(dev, steps=3, steps_one=20):
    """BASELINE config 5 (100 psr x 20k TOAs, Hellings-Downs GWB, fixed white
    noise) on this GPU: evals/s of 512-proposal batches, and the latency of
    one proposal (the right-looking dense factorisation), HIP events around
    ewh_lnl_units_device.  Algorithmic work as main_c5."""
    import torch
    from enterprise_warp_amd import synth
    cfg = synth.config_c5()
    pta = cfg.pta
    eng = pta.engine(device=dev.index)
    P = len(pta.signal_collections)
    st = torch.cuda.current_stream(dev)
    res = {}
    for B, n in ((cfg.B, steps), (1, steps_one)):
        X = synth.prior_draws(pta, B, cfg.theta_seed)
        th = torch.from_numpy(X).to(dev)
        out = torch.zeros(B, dtype=torch.float64, device=dev)
        eng.lnl_units_device(th.data_ptr(), B, 0, P * B, out.data_ptr(), st.cuda_stream)
        torch.cuda.synchronize(dev)
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(st)
        for _ in range(n):
            eng.lnl_units_device(th.data_ptr(), B, 0, P * B, out.data_ptr(), st.cuda_stream)
        b.record(st)
        torch.cuda.synchronize(dev)
        ms = a.elapsed_time(b) / n
        res[f"B{B}"] = {"ms_per_batch": ms, "evals_per_s": B / (ms * 1e-3),
                        "finite_fraction": float(np.mean(np.isfinite(out.cpu().numpy())))}
    nc = pta.common_layout()["n_col"]
    m = np.array([c.T.shape[1] for c in pta.signal_collections])
    f = float(np.sum(m ** 3 / 3.0)) + (P * nc + 1) ** 3 / 3.0
    res[f"B{cfg.B}"]["fp64_mfma_frac"] = f * cfg.B / (res[f"B{cfg.B}"]["ms_per_batch"] * 1e-3) / 1e12 / \
        FP64_MFMA_PEAK_TFLOPS
    res["note"] = ("config 5 at its stated size, prior draws; B1 = one PTMCMC proposal (right-looking dense "
                   "Sigma_c); algorithmic work per sample sum_a m_a^3/3 + (P n_gw + 1)^3 / 3")
    pta._drop_engine()
    return res


def kernel_sources_sha():
    """sha256 of the sources of the factorisation kernel (ewarp_dev.h and its
    instantiating translation unit): ties a committed PMC profile to this tree."""
    import hashlib
    hsh = hashlib.sha256()
    for f in ("ewarp_dev.h", "chol_small.hip"):
        with open(os.path.join(ROOT, "enterprise_warp_amd", "csrc", f), "rb") as fh:
            hsh.update(fh.read())
    return hsh.hexdigest()[:16]


def sampler_latency(pta, cfg, batches=(1, 16, 256, 4096), reps=50):
    """The drop-in as samplers call it: host theta in, host lnL out through
    ewh_lnl_batch (pinned staging, H2D, launches, D2H, stream sync), one
    process, C3.  PTMCMC / bilby call one theta at a time
    (run_example_paramfile.py:27-30, bilby_warp.py:35).  B4096 is the
    headline batch with its host transfers included (the headline `value`
    keeps theta and lnL resident in HBM)."""
    from enterprise_warp_amd import synth
    out = {}
    for B in batches:
        X = synth.prior_draws(pta, B, 7 + B)
        pta.get_lnlikelihood_batch(X)
        ts = []
        for _ in range(reps if B < 4096 else 10):
            t0 = time.perf_counter()
            pta.get_lnlikelihood_batch(X)
            ts.append(time.perf_counter() - t0)
        med = float(np.median(ts))
        out[f"B{B}"] = {"ms_median": 1e3 * med, "ms_p90": 1e3 * float(np.percentile(ts, 90)),
                        "evals_per_s": B / med}
    x = synth.prior_draws(pta, 1, 3)[0]
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        pta.get_lnlikelihood(x)
        ts.append(time.perf_counter() - t0)
    out["get_lnlikelihood_single_ms_median"] = 1e3 * float(np.median(ts))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch-per-gpu", type=int, default=4096)
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--cpu-procs", type=int, default=None, help="default: every usable core (affinity / cgroup quota)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-latency", action="store_true")
    ap.add_argument("--no-secondary", action="store_true", help="skip the C2 / C4 / C5 secondary measurements")
    ap.add_argument("--no-c5", action="store_true", help="skip the C5 secondary measurement (~40 s of model build)")
    ap.add_argument("--kernel-mode", type=int, default=0, help="0 auto (MFMA), 1 LDS fallback")
    ap.add_argument("--config", default="c3", choices=["c3", "c5"],
                    help="c3: the headline 45-pulsar CURN batch (default); c5: 100-pulsar HD-correlated PTA")
    ap.add_argument("--partition", default="samples", choices=["samples", "pulsars"],
                    help="c5 only: shard samples (no exchange) or pulsars (all-gather of the kept common blocks, "
                         "then the dense factorisation on every rank: one proposal over N GPUs)")
    ap.add_argument("--c5-batch", type=int, default=None, help="c5 proposals per step (default 512 / 1 for pulsars)")
    ap.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                    help="nccl (= RCCL, the default); gloo only to rehearse the multi-rank path")
    ap.add_argument("--same-device", action="store_true",
                    help="every rank on cuda:0 (rehearsal on a one-GPU box; needs --dist-backend gloo)")
    ap.add_argument("--verify", action="store_true",
                    help="rank 0 checks the reduced lnL of the first samples against the single-device entry")
    args = ap.parse_args()
    if args.same_device and args.dist_backend != "gloo":
        ap.error("--same-device needs --dist-backend gloo (RCCL takes one rank per GPU)")
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
    # --same-device (rehearsal of the multi-rank path on a one-GPU box, with
    # --dist-backend gloo): every rank on cuda:0
    gpu = 0 if (world == 1 or args.same_device) else local
    if world > 1:
        torch.cuda.set_device(gpu)
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", gpu))
        else:
            dist.init_process_group(args.dist_backend)
    else:
        torch.cuda.set_device(0)
    dev = torch.device("cuda", gpu)

    cfg = synth.config_c3()
    pta = cfg.pta
    B = args.batch_per_gpu * world
    X = synth.prior_draws(pta, B, cfg.theta_seed)      # same seed on every rank
    theta = torch.from_numpy(X).to(dev)
    eng = pta.engine(device=dev.index)
    eng.set_kernel_mode(args.kernel_mode)
    costs = eng.unit_costs()
    u0, u1 = sharding.unit_ranges(costs, B, world)[rank]
    stream = torch.cuda.current_stream(dev)
    # two output buffers: the all-reduce of step i (RCCL's stream) overlaps
    # the likelihood launch of step i+1 (this stream); step i+2 reuses the
    # buffer only after that all-reduce (work.wait(): a stream dependency for
    # RCCL, not a host wait)
    outs = [torch.zeros(B, dtype=torch.float64, device=dev) for _ in range(2)]
    works = [None, None]

    def step(i, ev=None):
        k = i & 1
        if works[k] is not None:
            works[k].wait()
            works[k] = None
        if ev is not None:
            ev[0].record(stream)
        eng.lnl_units_device(theta.data_ptr(), B, u0, u1, outs[k].data_ptr(), stream.cuda_stream)
        if ev is not None:
            ev[1].record(stream)
        if world > 1:
            works[k] = dist.all_reduce(outs[k], async_op=True)

    def drain():
        for k in range(2):
            if works[k] is not None:
                works[k].wait()
                works[k] = None

    for i in range(args.warmup):
        step(i)
    drain()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]
    t0 = time.perf_counter()
    for i in range(args.steps):
        step(i, ev[i])
    drain()
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
    lnl = outs[(args.steps - 1) & 1].cpu().numpy()
    verify = None
    if args.verify and rank == 0:
        # the reduced batch against the single-device entry (ewh_lnl_batch,
        # pulsar-order device fold) on its first samples: strict bound
        nv = min(B, 256)
        ref = pta.get_lnlikelihood_batch(X[:nv])
        fin = np.isfinite(ref)
        same_inf = bool(np.array_equal(fin, np.isfinite(lnl[:nv])))
        err = np.abs(lnl[:nv][fin] - ref[fin]) / (1e-6 + 1e-10 * np.abs(ref[fin]))
        verify = {"samples": nv, "max_err_over_strict": float(err.max()) if err.size else 0.0,
                  "inf_pattern_equal": same_inf}

    # roofline of the dominant kernel (chol_mfma): algorithmic flops of this
    # rank's units / average duration of its likelihood launch
    m_psr = np.array([c.T.shape[1] for c in pta.signal_collections])
    f_unit = algorithmic_flops_per_unit(m_psr)
    flops = 0.0
    for p in range(len(m_psr)):
        lo, hi = max(u0, p * B), min(u1, (p + 1) * B)
        flops += max(0, hi - lo) * f_unit[p]
    achieved = flops / (launch_ms * 1e-3) / 1e12
    # HBM bytes per launch of this kernel from the committed PMC pass, used
    # only when that pass profiled these very kernel sources (sha match)
    traffic, traffic_src = None, None
    pmc = os.path.join(ROOT, "profiles", "pmc_chol.json")
    if os.path.exists(pmc):
        with open(pmc) as fh:
            rec_pmc = json.load(fh)
        if rec_pmc.get("kernel_sources_sha") == kernel_sources_sha():
            traffic = rec_pmc.get("hbm_bytes_per_launch")
            traffic_src = f"profiles/{rec_pmc.get('tag')}/pmc_summary.json (kernel sources sha " \
                          f"{rec_pmc['kernel_sources_sha']})"

    latency = None
    if rank == 0 and not args.no_latency:
        latency = sampler_latency(pta, cfg)
    secondary = None
    if rank == 0 and world == 1 and not args.no_secondary:
        pta._drop_engine()
        secondary = secondary_configs(dev)
        if not args.no_c5:
            secondary["c5"] = secondary_c5(dev)
    if rank == 0:
        value = B * args.steps / elapsed
        rec = {
            "metric": METRIC, "value": value, "unit": "lnL evals/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": 1e3 * elapsed / args.steps, "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "f64",
            "data": "synthetic: seeded 45-pulsar CURN PTA (SURVEY.md §8(d) C3), theta from the priors",
            "config": {"workload": "C3: 45 psr, n=2000..20000 TOAs (495k) over 14.7 yr, ECORR, RN+DM 30 freqs, "
                                   "CURN 14 freqs merged, fixed white noise (TNT cached), basis m=132",
                       "global_batch": B, "batch_per_gpu": args.batch_per_gpu, "n_pulsars": len(m_psr),
                       "parallelism": f"units{world}", "finite_fraction": float(np.mean(np.isfinite(lnl)))},
            "roofline": {"bound": "mfma", "achieved": achieved, "peak": FP64_MFMA_PEAK_TFLOPS, "unit": "TFLOP/s",
                         "frac": achieved / FP64_MFMA_PEAK_TFLOPS, "traffic": traffic, "traffic_source": traffic_src,
                         "kernel": "chol_mfma_kernel<8,2,25> (two-level blocked LDL^T panel: 4-row sub-panels by "
                                   "fused DPP multiply-adds, each closed by one MFMA rank-4 update; rest of the "
                                   "block row by MFMA with L^-1)",
                         "kernel_sources_sha": kernel_sources_sha(), "launch_ms": launch_ms,
                         "flops_per_launch": flops},
        }
        if secondary is not None:
            rec["secondary"] = secondary
        if cpu is not None:
            rec["cpu_baseline"] = cpu
            rec["gpu_over_cpu"] = {"per_gpu": value / world / cpu["value"],
                                   "note": "one GPU against the CPU cores this job is given (its node share); "
                                           "a whole node is 8 such shares, so the node-level ratio at perfect "
                                           "scaling is the same figure (SCALE_rNN measures the real curve)"}
        if latency is not None:
            rec["sampler_latency"] = latency
        if verify is not None:
            rec["verify"] = verify
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
    if args.partition == "pulsars":
        return c5_pulsar_partition(args, cfg, world, rank, dev)
    Bg = args.c5_batch or cfg.B
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


def c5_pulsar_partition(args, cfg, world, rank, dev):
    """Config 5, the exchange step of SURVEY.md §8(e): rank r runs the partial
    factorisations of pulsars [r per, (r+1) per) (ewh_corr_partial_device,
    pulsar-major buffers), one RCCL all-gather moves the kept common blocks
    and local terms, every rank assembles and factors Sigma_c
    (ewh_corr_finish_device).  B proposals per step (default 1: a PTMCMC
    proposal spread over the node)."""
    import torch
    import torch.distributed as dist
    from enterprise_warp_amd import synth
    pta = cfg.pta
    B = args.c5_batch or 1
    X = synth.prior_draws(pta, B, cfg.theta_seed)
    theta = torch.from_numpy(X).to(dev)
    eng = pta.engine(device=dev.index)
    kd = eng.keep_dim()
    P = len(pta.signal_collections)
    per = -(-P // world)
    p0, p1 = min(P, rank * per), min(P, (rank + 1) * per)
    keep = torch.zeros((world * per, B, kd, kd), dtype=torch.float64, device=dev)
    local = torch.zeros((world * per, B), dtype=torch.float64, device=dev)
    out = torch.zeros(B, dtype=torch.float64, device=dev)
    stream = torch.cuda.current_stream(dev)

    def step():
        eng.corr_partial_device(theta.data_ptr(), B, p0, p1, keep.data_ptr(), local.data_ptr(), stream.cuda_stream)
        if world > 1:
            dist.all_gather_into_tensor(keep, keep[rank * per:(rank + 1) * per].clone())
            dist.all_gather_into_tensor(local, local[rank * per:(rank + 1) * per].clone())
        eng.corr_finish_device(theta.data_ptr(), B, keep.data_ptr(), local.data_ptr(), out.data_ptr(),
                               stream.cuda_stream)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed = float(t.item())
    lnl = out.cpu().numpy()
    if rank == 0:
        rec = {"metric": "lnL evals/sec, 100-psr HD-correlated PTA, pulsar-partitioned (BASELINE config 5)",
               "value": B * args.steps / elapsed, "unit": "lnL evals/s", "n_gpus": world, "steps": args.steps,
               "warmup": args.warmup, "ms_per_step": 1e3 * elapsed / args.steps, "higher_is_better": True,
               "scaling": "strong", "vs_baseline": None, "dtype": "f64",
               "data": "synthetic: seeded 100-pulsar x 20k-TOA PTA, HD GWB 14 freqs (SURVEY.md §8(d) C5)",
               "config": {"workload": "C5, pulsars sharded, kept blocks all-gathered over RCCL",
                          "global_batch": B, "n_pulsars": P, "parallelism": f"pulsars{world}",
                          "gather_bytes_per_step": int(world * per * B * (kd * kd + 1) * 8),
                          "finite_fraction": float(np.mean(np.isfinite(lnl)))}}
        print(json.dumps(rec), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
