"""TEST INFRASTRUCTURE ONLY — CPU oracle for the enterprise PTA log-likelihood.

Nothing in the product package (`enterprise_warp_amd`) imports this package.
Only `tests/`, `__graft_entry__.smoke()` and the `cpu_baseline` leg of
`bench.py` may use it, and only as the checker / CPU baseline, never as the
thing measured or shipped.

Parity status
-------------
The arithmetic of the reference path lives in the third-party package
`enterprise` (PyPI `enterprise-pulsar`, version unpinned by the reference's
setup.py:8-21), reached from the reference at enterprise_warp.py:502 and
bilby_warp.py:35.  It is not vendored under /root/reference and is not
installed in this image, so no enterprise-produced lnL value exists anywhere.

* `enterprise_ref` restates enterprise v3.x's published algorithm
  (signal_base.LogLikelihood, white_signals.*, gp_signals.*, gp_bases.*,
  utils.powerlaw / create_quantization_matrix, ShermanMorrison) with numpy /
  scipy, following the reference's call sites in enterprise_models.py.
* `dense_ref` is an independent brute-force check of the same mathematics
  (dense C = N + U J U^T + T phi T^T, finite timing-model prior).
* Pinned only by: known-answer tests (closed-form white-noise lnL, powerlaw
  values, the reference's own `determine_nfreqs` rule on its example data:
  J1832-0836 -> 32, fake_psr_0 -> 60), the reference's example noise file and
  noise models, and the dense cross-check.  Against enterprise itself the
  oracle is **parity unpinned** (see DESIGN.md §Oracle).
"""
