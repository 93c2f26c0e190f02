"""ORACLE — test infrastructure only.

This package is a CPU (torch fp64) restatement of the reference's Discrete-KG
hot path and of the external posterior semantics it calls into.  It exists to
CHECK the MI355X product in ``decoupled-kg_amd/`` and to provide the CPU
baseline leg of ``bench.py``.

Rules (see DESIGN.md "Oracle"):
  * Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s
    ``cpu_baseline`` leg may import anything from here, and only as the
    checker / the timed CPU baseline.  The product (``dkg_amd``) never imports
    it and has no CPU fallback.
  * Every function cites the reference file:line it restates.  The reference
    is pure Python (torch 2.1 CPU + BoTorch@c14808f + GPyTorch 1.11 +
    linear_operator 0.5.1, ``requirements.txt:14-17``,
    ``requirements-full.txt:27``).  BoTorch / GPyTorch / linear_operator are
    not installable here (no network), so their semantics at the reference's
    call sites are restated in ``oracle/gp.py`` and ``oracle/fit.py``.

Pinning: ``tests/test_oracle_kats.py`` checks this restatement against every
known-answer test of ``tests/modules/acquisition/test_discretekg.py`` in the
reference (epigraph and expectation KATs exactly; end-to-end KG KATs via the
``oracle/fit.py`` restatement of ``fit_gpytorch_mll``).
"""
