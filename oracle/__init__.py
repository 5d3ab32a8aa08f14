"""TEST INFRASTRUCTURE ONLY — the CPU oracle for the divrec hot path.

This package restates, in numpy / plain Python, the reference algorithms of
amtsyplov/diversity-recommendations that the HIP path replaces (each function
cites the reference file:line it follows). It is the checker, never the thing
measured or shipped: only ``tests/``, ``__graft_entry__.smoke()`` and the
``cpu_baseline`` leg of ``bench.py`` may import it. The product path
(``divrec`` under ``diversity-recommendations_amd/``) never imports it and
fails loudly when the HIP library is unavailable.

Pinning: ``tests/golden/*.npz`` were produced by importing the reference
itself (``tests/golden/make_golden.py``, run with PYTHONPATH=/root/reference in
the build container); ``tests/test_oracle_golden.py`` checks every function
here against those vectors, bit-exactly where the reference is deterministic.
"""
from .divrec_oracle import *  # noqa: F401,F403
