"""Diagnostic (round 6): which stage sets the varying-white-noise route's
error on C2 prior draws -- the device-order fp64 restatement
(oracle/device_order_ref.py: the contraction kernels' FMA order, projected
basis, two-level LDL^T) against the same fp64 Gram factored in double-double
(oracle/ddref._factor), both against the CPU double-double value and beside
enterprise's order, in units of strict.  CPU only.

    python scripts/diag_varying_error.py [sample ...]
"""
import sys, numpy as np
sys.path.insert(0,'/root/repo'); sys.path.insert(0,'/root/repo/tests')
from enterprise_warp_amd import synth
from oracle import ddref
from oracle.device_order_ref import gram, DeviceOrderPTA
from oracle.enterprise_ref import OraclePTA
cfg=synth.config_c2(); pta=cfg.pta
X=synth.prior_draws(pta,cfg.B,cfg.theta_seed)
const=pta.constant_values()
psrs=[c.psr for c in pta.signal_collections]; terms=pta.oracle_terms()
r=ddref.DDReferencePTA(psrs,terms); o=OraclePTA(psrs,terms,None)
dev=DeviceOrderPTA(psrs,terms,None,np.float64,gram_mode="device")
for s in ([int(a) for a in sys.argv[1:]] or [42, 47, 142, 207, 346]):
    d=dict(const); d.update(pta.map_params(X[s]))
    ex=r.lnlikelihood(d); en=o.lnlikelihood(d); dv=dev.lnlikelihood(d)
    pp=dev.pulsars[0]
    G,ldn=gram(pp,{k:np.float64(v) for k,v in d.items()},np.float64,"device",nl=dev.nlead[0])
    hyb=r._factor(r.pulsars[0],d,(np.asarray(G,float),np.zeros_like(G)),ldn)
    st=1e-6+1e-10*abs(ex)
    print(s,"ent %.2f dev-order %.2f devG+ddfactor %.2f (x strict from exact)"%(abs(en-ex)/st,abs(dv-ex)/st,abs(hyb-ex)/st))
