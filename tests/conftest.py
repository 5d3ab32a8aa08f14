"""pytest configuration: `gpu` marker and import paths.

The product package lives in ``diversity-recommendations_amd/divrec`` (the
directory name is not importable, so its parent is put on sys.path); the CPU
oracle (test infrastructure) is the top-level ``oracle`` package.
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG_PARENT = os.path.join(ROOT, "diversity-recommendations_amd")
for p in (ROOT, PKG_PARENT):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a ROCm GPU (MI355X) and the HIP library")
