"""divrec — MI355X-native hot path of amtsyplov/diversity-recommendations.

Drop-in for the reference's ``divrec.models`` / ``divrec.losses`` /
``divrec.metrics`` / ``divrec.datasets`` / ``divrec.train`` API. Compute runs
in hand-written HIP kernels for gfx950 (``divrec._lib/libdivrec_hip.so``,
C ABI in ``include/divrec_hip.h``); there is no CPU fallback.
"""
__version__ = "0.1.0"
