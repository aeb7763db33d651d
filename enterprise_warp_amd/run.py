"""Paramfile driver: the reference's examples/run_example_paramfile.py flow on
the MI355X likelihood.

    python -m enterprise_warp_amd.run --prfile params.dat [--num N] [--niter K] [--nchains B]

Params -> init_pta (one PTA per `{N}` model block) -> for `sampler:
ptmcmcsampler` the reference's PTMCMC branch (run_example_paramfile.py:25-45:
model_utils.setup_sampler / HyperModel.setup_sampler, x0 from the priors,
sampler.sample(x0, nsamp, **sampler kwargs that sample() takes), one theta
per device call); otherwise, or with --batched, the batched Metropolis
sampler (B chains per device call; bilby is not installed).  Chains go to the
paramfile's output directory as chain_1.txt with pars.txt beside it.
"""
import inspect
import optparse
import os
import sys

import numpy as np

from . import warp
from .hypermodel import HyperModel
from .sampler import BatchedMH


def parse_commandline(argv=None):
    """warp.parse_commandline's options (the reference's, enterprise_warp.py:24-69)
    plus the sampler's own: --niter, --nchains, --seed."""
    p = optparse.OptionParser()
    p.add_option("-n", "--num", default=0, type=int)
    p.add_option("-p", "--prfile", type=str)
    p.add_option("-d", "--drop", default=0, type=int)
    p.add_option("-c", "--clearcache", default=0, type=int)
    p.add_option("-m", "--mpi_regime", default=0, type=int)
    p.add_option("-w", "--wipe_old_output", default=0, type=int)
    p.add_option("-x", "--extra_model_terms", default=None, type=str)
    p.add_option("--niter", type=int, default=None, help="iterations (default: the paramfile's nsamp)")
    p.add_option("--nchains", type=int, default=256, help="chains evaluated per device call")
    p.add_option("--seed", type=int, default=0)
    p.add_option("--batched", action="store_true", help="batched Metropolis even for sampler: ptmcmcsampler")
    opts, _ = p.parse_args(argv)
    return opts


def main(argv=None):
    opts = parse_commandline(argv)
    eo = opts
    params = warp.Params(opts.prfile, opts=opts)
    ptas = warp.init_pta(params)
    model = ptas[0] if len(ptas) == 1 else HyperModel(ptas)
    if len(ptas) > 1:
        print("Super model parameters:", model.param_names)
    outdir = getattr(params, "output_dir", None)
    if outdir:
        os.makedirs(outdir, exist_ok=True)
        np.savetxt(os.path.join(outdir, "pars.txt"), model.param_names, fmt="%s")
    cov = None
    covm = getattr(params, "mcmc_covm_csv", None)
    if covm and os.path.exists(params._path(covm)):
        import pandas as pd
        df = pd.read_csv(params._path(covm), index_col=0)
        names = list(model.param_names)
        if all(n in df.index for n in names):
            cov = df.loc[names, names].to_numpy()
    niter = eo.niter if eo.niter is not None else int(getattr(params, "nsamp", 1000))
    if getattr(params, "sampler", "") == "ptmcmcsampler" and not eo.batched:
        # the reference's PTMCMC branch, call for call
        from . import model_utils
        if len(ptas) == 1:
            sampler = model_utils.setup_sampler(ptas[0], resume=False, outdir=outdir or "chains", seed=eo.seed)
            x0 = np.hstack([np.atleast_1d(p.sample()) for p in ptas[0].params])
        else:
            sampler = model.setup_sampler(resume=False, outdir=outdir or "chains", seed=eo.seed)
            x0 = model.initial_sample()
        accepted = inspect.getfullargspec(sampler.sample).args
        kw = {k: v for k, v in params.sampler_kwargs.items() if k in accepted and k not in ("Niter", "p0")}
        x = sampler.sample(x0, niter, **kw)
        like = model.get_lnlikelihood(x)
        post = like + model.get_lnprior(x)
        print(f"{niter} PTMCMC iterations; acceptance {sampler.acceptance_rate:.3f}; final ln posterior {post:.6f}")
        return x[None, :], np.array([post]), np.array([like])
    sampler = BatchedMH(model, nchains=eo.nchains, outdir=outdir, seed=eo.seed, cov=cov)
    X, post, like = sampler.sample(niter=niter)
    best = int(np.argmax(post))
    print(f"{niter} iterations x {eo.nchains} chains; mean acceptance {sampler.acceptance.mean():.3f}; "
          f"max ln posterior {post[best]:.6f}")
    return X, post, like


if __name__ == "__main__":
    main()
