"""TEST INFRASTRUCTURE ONLY -- the CPU oracle for the pruning likelihood path.

Nothing under ``oracle/`` is part of the product.  Only ``tests/``,
``__graft_entry__.smoke()`` and the ``cpu_baseline`` leg of ``bench.py`` may
import, call, link or execute it, and only as the checker / reported CPU
baseline -- never as the thing measured or shipped.  The product path
(``phylostan_amd``) never imports this package and fails loudly when its HIP
library is missing.

Contents
--------
``stan_restatement``  literal site -> node -> category loops restating the Stan
                      code that ``phylostan/generate_script.py`` emits
                      (likelihood ``:961-1055``, P-matrices ``:755-892``,
                      Weibull rates ``:249-282``).  Pure Python loops: small
                      cases only.
``numpy_pruner``      vectorised (over patterns) twin of the same likelihood
                      plus the analytic reverse (pre-order) pass that produces
                      dlogL/dP, the branch-length gradient and the rate /
                      mixture / root-frequency gradients.  Restates the
                      pre-order algorithm of ``pruner/tree.cpp:228-242`` and
                      ``eigen/eigen.j2:143-167`` (with the ``times[i]`` factor
                      of ``eigen.j2:165`` removed -- see SURVEY.md 8a).
``cpu_pruner.c``      the same algorithm in plain C (fp64, optional OpenMP
                      over patterns), built into ``oracle/liboracle_cpu.so``
                      by ``oracle/Makefile``; used for larger parity cases and
                      as the timed ``cpu_baseline`` (kind "port").

Pinning (see DESIGN.md "Oracle")
--------------------------------
* JC69 likelihood + gradient: pinned to the reference's only known-answer
  test, the closed-form 3-taxon log-likelihood of ``eigen/test_ll_3tax.py``
  (fixture ``tests/golden/kat_3tax.json``, generated from the reference's own
  formula by ``tests/golden/make_golden.py``).
* Input layout (pattern compression, tip encoding, node numbering, peel/map
  order): pinned to fixtures produced by the reference's own
  ``phylostan/utils.py`` functions run in this container.
* HKY/GTR eigen path: the reference delegates to Stan Math
  (``eigenvalues_sym``/``eigenvectors_sym``) which is absent here; P-matrices
  are pinned against ``scipy.linalg.expm(Q t)`` and gradients against central
  finite differences -- "parity unpinned" by the reference for these two.
"""
