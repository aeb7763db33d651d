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

Launch contract: `--gpus N` is authoritative.  Started from
plain `python` with N > 1 and no WORLD_SIZE in the environment, this process
is a launcher: it runs the CPU baseline (before anything touches a GPU), then
starts N rank processes of this script (RANK = LOCAL_RANK = r, WORLD_SIZE = N,
MASTER_ADDR = 127.0.0.1, a free MASTER_PORT) and exits with the first non-zero
rank status (the other ranks are then terminated).  Started by torchrun
(WORLD_SIZE set), `--gpus` must equal WORLD_SIZE or the run exits non-zero.
"""
import argparse
import json
import os
import socket
import subprocess
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


def secondary_wide(dev, steps=3):
    """Bases past the register kernels, where the reference's own rules lead
    (X_<n>_nfreqs, enterprise_models.py:148-167; determine_nfreqs gives its
    fake_psr_0 60 frequencies, :457-462; its system_noise_example, :256-338):
    the 372-column 10k-TOA pulsar with white noise fixed and sampled (B =
    1024) and the system-noise J1832 model (13 blocks, fixed white noise, B =
    4096).  Per case, on prior and near-truth draws: ms per batch, evals/s and
    the share of units the verify step sends to chol_dd_kernel
    (ewh_refine_stats); the fp64 chol_wide factorisation alone (kernel mode
    27) against the fp64 MFMA peak (algorithmic m^3/3 + 2 m^2 per unit, m
    the basis width); every unit in double-double (mode 29); for sampled
    white noise the contraction (ewh_contract_device) against §8(d)'s
    contraction flops."""
    import torch
    from enterprise_warp_amd import synth
    ref_examples = os.path.join(ROOT, "tests", "golden", "ref_examples")
    st = torch.cuda.current_stream(dev)
    out = {}
    for name, make in (("w372_fixed", lambda: synth.config_wide(True)),
                       ("w372_varwn", lambda: synth.config_wide(False)),
                       ("system", lambda: synth.config_system(ref_examples))):
        cfg = make()
        pta, B = cfg.pta, cfg.B
        eng = pta.engine(device=dev.index)
        P = len(pta.signal_collections)
        U = P * B
        m = np.array([c.T.shape[1] for c in pta.signal_collections])
        f_chol = float(np.sum(algorithmic_flops_per_unit(m))) * B
        res = torch.zeros(B, dtype=torch.float64, device=dev)

        def timed(fn, n=steps):
            fn()
            torch.cuda.synchronize(dev)
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(st)
            for _ in range(n):
                fn()
            b.record(st)
            torch.cuda.synchronize(dev)
            return a.elapsed_time(b) / n

        rec = {"batch": B, "columns": int(m.max()), "white_fixed": bool(pta.white_fixed())}
        draws = (("prior", synth.prior_draws(pta, B, cfg.theta_seed)),
                 ("near", synth.near_draws(pta, cfg.truth, B, cfg.theta_seed + 1)))
        for kind, X in draws:
            th = torch.from_numpy(X).to(dev)
            run = lambda: eng.lnl_units_device(th.data_ptr(), B, 0, U, res.data_ptr(), st.cuda_stream)  # noqa: E731
            eng.refine_stats()
            ms = timed(run)
            checked, refined = eng.refine_stats()
            rec[kind] = {"ms_per_batch": ms, "evals_per_s": B / (ms * 1e-3),
                         "refined_share": refined / checked if checked else None,
                         "finite_fraction": float(np.mean(np.isfinite(res.cpu().numpy())))}
            if kind == "prior":
                eng.set_kernel_mode(27)
                try:
                    ms27 = timed(run)
                finally:
                    eng.set_kernel_mode(29)
                try:
                    ms29 = timed(run, 1)
                finally:
                    eng.set_kernel_mode(0)
                rec["all_fp64_chol_wide"] = {"ms_per_batch": ms27}
                rec["all_double_double"] = {"ms_per_batch": ms29, "us_per_unit": 1e3 * ms29 / U}
                if not pta.white_fixed():
                    cms = timed(lambda: eng.contract_device(th.data_ptr(), B, st.cuda_stream))
                    fc, by = contraction_work(pta)
                    rec["contraction"] = {"ms": cms, "fp64_mfma_frac": fc * B / (cms * 1e-3) / 1e12 /
                                          FP64_MFMA_PEAK_TFLOPS, "flops_per_sample": fc}
                    ms27 -= cms
                rec["all_fp64_chol_wide"].update(
                    factorisation_ms=ms27, fp64_mfma_frac=f_chol / (ms27 * 1e-3) / 1e12 / FP64_MFMA_PEAK_TFLOPS)
            del th
        out[name] = rec
        pta._drop_engine()
        del res
    out["note"] = ("prior / near: the default route (verify-and-refine: forward + reversed fp64 chol_wide, "
                   "chol_dd_kernel on the units whose two orders disagree); refined_share = units refactored "
                   "in double-double / units on the route; all_fp64_chol_wide = kernel mode 27 (one fp64 "
                   "factorisation per unit, the contraction subtracted for sampled white noise), fp64_mfma_frac "
                   "on m^3/3 + 2 m^2 per unit; all_double_double = kernel mode 29")
    return out


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


CPU_JSON_ENV = "EWARP_BENCH_CPU_JSON"   # launcher -> rank 0: the CPU baseline it measured
LAUNCHER_ENV = "EWARP_BENCH_LAUNCHER"   # set in the ranks bench.py itself starts


def verify_default(flag, world):
    """--verify / --no-verify as given; by default on exactly when the run has
    more than one rank (the driver runs plain `bench.py --gpus N`: a
    multi-rank line must carry its own correctness evidence)."""
    return (world > 1) if flag is None else bool(flag)


def device_identity(index):
    """PCI bus id and UUID of device `index` of this process (hipDeviceGetPCIBusId
    through the HIP runtime torch loaded; torch's device properties)."""
    import ctypes
    import torch
    ident = {"index": int(index), "pci_bus_id": None, "uuid": None}
    try:
        ident["uuid"] = str(torch.cuda.get_device_properties(index).uuid)
    except Exception:  # noqa: BLE001
        pass
    hip = None
    try:   # the runtime already mapped into this process (never a second copy)
        with open("/proc/self/maps") as fh:
            paths = sorted({ln.split()[-1] for ln in fh if "libamdhip64.so" in ln})
        if paths:
            hip = ctypes.CDLL(paths[0], mode=os.RTLD_NOLOAD | ctypes.RTLD_GLOBAL)
    except OSError:
        hip = None
    if hip is not None:
        buf = ctypes.create_string_buffer(64)
        if hip.hipDeviceGetPCIBusId(buf, 64, int(index)) == 0:
            ident["pci_bus_id"] = buf.value.decode()
    return ident


def run_problems(devices, same_device, verify, verify_on):
    """What makes a bench line invalid (rank 0 exits non-zero on any): two
    ranks on one device without --same-device, a missing or failed verify
    block where it was asked for (the reduced lnL against the single-device
    entry: max error > strict, or a different -inf pattern)."""
    out = []
    keys = [d.get("pci_bus_id") or d.get("uuid") or f"index{d.get('index')}" for d in devices]
    if len(devices) > 1 and not same_device and len(set(keys)) < len(keys):
        out.append(f"ranks share a device without --same-device: {keys}")
    if verify_on:
        if verify is None:
            out.append("verify requested but not run")
        else:
            if not verify["max_err_over_strict"] <= 1.0:
                out.append(f"verify: max error {verify['max_err_over_strict']:.3e} x strict")
            if not verify["inf_pattern_equal"]:
                out.append("verify: -inf pattern differs from the single-device entry")
    return out


def free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def rank_environments(n, port, base=None):
    """Environment of each of the n rank processes the launcher starts: the
    env:// rendezvous torch.distributed reads (what torchrun would set for one
    node), one rank per GPU, LOCAL_RANK = RANK."""
    base = dict(os.environ if base is None else base)
    envs = []
    for r in range(n):
        e = dict(base)
        e.update(RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n), GROUP_RANK="0",
                 MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        e[LAUNCHER_ENV] = "1"
        e.pop(CPU_JSON_ENV, None)
        envs.append(e)
    return envs


def resolve_world(gpus, environ):
    """(world, launch): the world size of this run and whether this process
    must start the rank processes itself.  WORLD_SIZE set (torchrun, or our
    own launcher) wins, but must equal --gpus when that is given; without it,
    --gpus N > 1 makes this process the launcher."""
    ws = environ.get("WORLD_SIZE")
    if ws is not None:
        ws = int(ws)
        if gpus is not None and gpus != ws:
            raise SystemExit(f"bench.py: --gpus {gpus} but WORLD_SIZE={ws}: the launcher and the flag disagree")
        return ws, False
    n = 1 if gpus is None else int(gpus)
    if n < 1:
        raise SystemExit(f"bench.py: --gpus {n} < 1")
    return n, n > 1


def launch(n, argv, cpu=None, script=None):
    """Start n rank processes of this script (nothing in this process has
    touched a GPU), wait for all of them; on the first non-zero exit terminate
    the others and return that status.  Rank 0 prints the JSON line; the CPU
    baseline measured here reaches it through a temporary file."""
    import tempfile
    envs = rank_environments(n, free_port())
    tmp = None
    if cpu is not None:
        fd, tmp = tempfile.mkstemp(prefix="ewarp_cpu_", suffix=".json")
        with os.fdopen(fd, "w") as fh:
            json.dump(cpu, fh)
        envs[0][CPU_JSON_ENV] = tmp
    script = os.path.abspath(script or __file__)
    procs = [subprocess.Popen([sys.executable, script] + list(argv), env=e) for e in envs]
    rc = 0
    try:
        while True:
            states = [p.poll() for p in procs]
            bad = [s for s in states if s not in (None, 0)]
            if bad:
                rc = bad[0] if bad[0] > 0 else 128 - bad[0]
                print(f"bench.py launcher: a rank exited with status {bad[0]}; stopping the others",
                      file=sys.stderr, flush=True)
                break
            if all(s == 0 for s in states):
                break
            time.sleep(0.1)
    finally:
        for p in procs:
            if p.poll() is None:
                p.terminate()
        for p in procs:
            try:
                p.wait(timeout=30)
            except subprocess.TimeoutExpired:
                p.kill()
                p.wait()
        if tmp is not None:
            os.unlink(tmp)
    return rc


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None,
                    help="GPUs (= rank processes) of this run; default WORLD_SIZE, else 1 (see the launch contract)")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch-per-gpu", type=int, default=4096)
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--cpu-procs", type=int, default=None, help="default: every usable core (affinity / cgroup quota)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-latency", action="store_true")
    ap.add_argument("--no-secondary", action="store_true", help="skip the C2 / C4 / C5 secondary measurements")
    ap.add_argument("--no-c5", action="store_true", help="skip the C5 secondary measurement (~40 s of model build)")
    ap.add_argument("--no-wide", action="store_true", help="skip the wide-basis secondary measurement")
    ap.add_argument("--only-wide", action="store_true",
                    help="measure only the wide-basis secondary block (prints it as one JSON line) and exit")
    ap.add_argument("--kernel-mode", type=int, default=0, help="0 auto (MFMA), 1 LDS fallback")
    ap.add_argument("--config", default="c3", choices=["c3", "c5"],
                    help="c3: the headline 45-pulsar CURN batch (default); c5: 100-pulsar HD-correlated PTA")
    ap.add_argument("--partition", default="samples", choices=["samples", "pulsars"],
                    help="c5 only: shard samples (no exchange) or pulsars (all-gather of the kept common blocks, "
                         "then the dense factorisation on every rank: one proposal over N GPUs)")
    ap.add_argument("--c5-batch", type=int, default=None, help="c5 proposals per step (default 512 / 1 for pulsars)")
    ap.add_argument("--c3-partition", default="units", choices=["units", "samples"],
                    help="c3: units = contiguous (pulsar-major) unit ranges of equal cost per rank + one RCCL "
                         "all-reduce of the B-vector per step (default); samples = every rank evaluates all "
                         "pulsars for its own batch_per_gpu proposals, no collective (SURVEY.md 8(e): report both)")
    ap.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                    help="nccl (= RCCL, the default); gloo only to rehearse the multi-rank path")
    ap.add_argument("--same-device", action="store_true",
                    help="every rank on cuda:0 (rehearsal on a one-GPU box; needs --dist-backend gloo)")
    ap.add_argument("--verify", dest="verify", action="store_true", default=None,
                    help="rank 0 checks the reduced lnL of the first samples against the single-device entry "
                         "(default with more than one rank; DESIGN.md §5)")
    ap.add_argument("--no-verify", dest="verify", action="store_false",
                    help="skip that check (a multi-rank line then carries no correctness evidence)")
    args = ap.parse_args()
    if args.same_device and args.dist_backend != "gloo":
        ap.error("--same-device needs --dist-backend gloo (RCCL takes one rank per GPU)")
    world, spawn = resolve_world(args.gpus, os.environ)
    args.verify = verify_default(args.verify, world)
    if spawn:
        # launcher: the CPU baseline on this job's cores first, then the ranks
        cpu = None
        if args.config == "c3" and not args.no_cpu_baseline:
            cpu = cpu_baseline(args.cpu_seconds, args.cpu_procs)
        sys.exit(launch(world, sys.argv[1:], cpu))
    if args.config == "c5":
        return main_c5(args)
    if args.only_wide:
        import torch
        torch.cuda.set_device(0)
        print(json.dumps({"secondary": {"wide": secondary_wide(torch.device("cuda", 0))}}), flush=True)
        return

    import torch
    import torch.distributed as dist
    from enterprise_warp_amd import sharding, synth

    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # CPU baseline first: worker processes are spawned before this process
    # initialises the GPU (no forked child ever carries a HIP context).  With
    # N ranks from our launcher it was measured there, on the job's cores
    cpu = None
    if world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(args.cpu_seconds, args.cpu_procs)
    elif rank == 0 and os.environ.get(CPU_JSON_ENV):
        with open(os.environ[CPU_JSON_ENV]) as fh:
            cpu = json.load(fh)
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
    rccl_world = dist.get_world_size() if world > 1 else 1
    if rccl_world != world:
        raise SystemExit(f"bench.py: the process group has {rccl_world} ranks, --gpus / WORLD_SIZE say {world}")
    # every rank's device identity (PCI bus id / UUID), gathered to all
    devices = [device_identity(gpu)]
    if world > 1:
        devices = [None] * world
        dist.all_gather_object(devices, device_identity(gpu))

    cfg = synth.config_c3()
    pta = cfg.pta
    B = args.batch_per_gpu * world
    X = synth.prior_draws(pta, B, cfg.theta_seed)      # same seed on every rank
    theta = torch.from_numpy(X).to(dev)
    eng = pta.engine(device=dev.index)
    eng.set_kernel_mode(args.kernel_mode)
    P = len(pta.signal_collections)
    samples = args.c3_partition == "samples"
    if samples:
        # replicas: rank r takes proposals [r bpg, (r + 1) bpg) of the global
        # batch, all pulsars, and needs no exchange (its lnL are complete)
        bl = args.batch_per_gpu
        theta = theta[rank * bl:(rank + 1) * bl].contiguous()
        ranges = [(r * bl, (r + 1) * bl) for r in range(world)]     # (sample ranges)
        B_run, u0, u1 = bl, 0, P * bl
    else:
        costs = eng.unit_costs()
        ranges = sharding.unit_ranges(costs, B, world)
        B_run = B
        u0, u1 = ranges[rank]
    stream = torch.cuda.current_stream(dev)
    # two output buffers: the all-reduce of step i (RCCL's stream) overlaps
    # the likelihood launch of step i+1 (this stream); step i+2 reuses the
    # buffer only after that all-reduce (work.wait(): a stream dependency for
    # RCCL, not a host wait)
    outs = [torch.zeros(B_run, dtype=torch.float64, device=dev) for _ in range(2)]
    works = [None, None]

    def step(i, ev=None):
        k = i & 1
        if works[k] is not None:
            works[k].wait()
            works[k] = None
        if ev is not None:
            ev[0].record(stream)
        eng.lnl_units_device(theta.data_ptr(), B_run, u0, u1, outs[k].data_ptr(), stream.cuda_stream)
        if ev is not None:
            ev[1].record(stream)
        if world > 1 and not samples:
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
    # every rank's wall time and launch time (the max over ranks is `value`'s clock)
    t = torch.zeros(2 * world, dtype=torch.float64, device=dev)
    t[2 * rank], t[2 * rank + 1] = elapsed, launch_ms
    if world > 1:
        dist.all_reduce(t)
    per_rank = t.cpu().numpy().reshape(world, 2)
    elapsed = float(per_rank[:, 0].max())
    lnl = outs[(args.steps - 1) & 1].cpu().numpy()
    verify, problems = None, []
    if args.verify and rank == 0:
        # the reduced batch against the single-device entry (ewh_lnl_batch,
        # pulsar-order device fold) on its first samples: strict bound
        nv = min(B_run, 256)
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
        lo, hi = max(u0, p * B_run), min(u1, (p + 1) * B_run)
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
        if not args.no_wide:
            secondary["wide"] = secondary_wide(dev)
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
                       "parallelism": f"{'samples' if samples else 'units'}{world}",
                       "finite_fraction": float(np.mean(np.isfinite(lnl)))},
            "rccl_world": rccl_world,
            "dist": {"backend": args.dist_backend if world > 1 else None, "same_device": bool(args.same_device),
                     "devices": devices,
                     "launcher": "bench.py" if os.environ.get(LAUNCHER_ENV) else
                     ("torchrun" if os.environ.get("TORCHELASTIC_RUN_ID") else None),
                     "partition": args.c3_partition,
                     ("sample_ranges" if samples else "unit_ranges"): [list(r) for r in ranges],
                     "rank_elapsed_s": per_rank[:, 0].tolist(), "rank_launch_ms": per_rank[:, 1].tolist()},
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
            rec["gpu_over_cpu"] = {"per_gpu": value / world / cpu["value"], "job": value / cpu["value"],
                                   "note": f"job = this run's {world} GPU(s) against the {cpu['cores']} CPU cores "
                                           f"the same job is given (measured in this run); per_gpu = job / {world}"}
        if latency is not None:
            rec["sampler_latency"] = latency
        if verify is not None:
            rec["verify"] = verify
        problems = run_problems(devices, args.same_device, verify, args.verify)
        if problems:
            rec["problems"] = problems
        print(json.dumps(rec), flush=True)
        if problems:
            print("bench.py: " + "; ".join(problems), file=sys.stderr, flush=True)
    if world > 1:
        dist.destroy_process_group()
    if rank == 0 and problems:
        sys.exit(3)


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
    gpu = 0 if (world == 1 or args.same_device) else local
    torch.cuda.set_device(gpu)
    if world > 1:
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", gpu))
        else:
            dist.init_process_group(args.dist_backend)
        if dist.get_world_size() != world:
            raise SystemExit(f"bench.py: the process group has {dist.get_world_size()} ranks, WORLD_SIZE {world}")
    dev = torch.device("cuda", gpu)
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
               "value": Bg * world * args.steps / elapsed, "unit": "lnL evals/s", "n_gpus": world, "rccl_world": world,
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
               "value": B * args.steps / elapsed, "unit": "lnL evals/s", "n_gpus": world, "rccl_world": world,
               "steps": args.steps,
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
