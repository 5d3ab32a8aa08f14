"""The C-ABI library builds, loads on a CPU-only host and exports every symbol
that include/divrec_hip.h declares; argument checks run before any HIP call,
so their error codes and messages are testable here. No compute calls."""
import ctypes
import os
import re

import pytest
import torch

from divrec import _backend, ops

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "divrec_hip.h")


def declared_functions():
    text = open(HEADER).read()
    return sorted(set(re.findall(r"^\s*(?:int|size_t|const char\*)\s+(dr_\w+)\(", text, re.M)))


def test_header_declares_all_bound_symbols():
    assert set(declared_functions()) == set(_backend.SIGNATURES)


def test_library_exports_every_declared_symbol():
    lib = _backend.load_library()
    for name in declared_functions():
        assert hasattr(lib, name), name
    # and exports them with C linkage (no mangling)
    raw = ctypes.CDLL(str(_backend.lib_path()))
    for name in declared_functions():
        assert getattr(raw, name) is not None


def test_version_and_error_string():
    lib = _backend.load_library()
    assert lib.dr_version() >= 100
    assert isinstance(lib.dr_last_error(), bytes)


def test_argument_errors_without_gpu():
    lib = _backend.load_library()
    # k out of range -> DR_EINVAL with a message; nothing touches the device
    rc = lib.dr_score_topk(None, None, 10, None, 10, 0, 64, 0, None, None, None, None, None, 0, None)
    assert rc == -1 and b"k must be" in lib.dr_last_error()
    rc = lib.dr_score_topk(None, None, 10, None, 10, 0, 48, 10, None, None, None, None, None, 0, None)
    assert rc == -1 and b"d must be" in lib.dr_last_error()
    rc = lib.dr_ild_embedding(None, 3, 5, 500, None, 10, 128, 0, None, None)
    assert rc == -1
    rc = lib.dr_topk_merge(None, None, 3, 10, 1000, 10, None, None, None)
    assert rc == -1
    rc = lib.dr_mmr_rerank(None, None, 4, 2000, None, 10, 128, 10, 0.5, None, None)
    assert rc == -1 and b"C must be" in lib.dr_last_error()
    # empty inputs are a no-op success
    assert lib.dr_gather_dot(None, None, 0, 64, None, None, 0, None, None) == 0


def test_workspace_query_is_host_only():
    lib = _backend.load_library()
    ws = lib.dr_score_topk_workspace(1_000_000, 10_000_000, 128, 100)
    # candidate buffers: n_users_pad * CAP(512) * 8 B for the single chunk, + counts
    assert ws >= 1_000_000 * 512 * 8
    assert lib.dr_score_topk_workspace(10, 10, 48, 10) == 0  # unsupported d


@pytest.mark.skipif(torch.cuda.is_available(), reason="checks the no-GPU behaviour")
def test_ops_fail_loudly_without_gpu():
    t = torch.zeros(4, 64)
    with pytest.raises(RuntimeError, match="no CPU fallback"):
        ops.gather_dot(t, t, torch.zeros(2, dtype=torch.int64), torch.zeros(2, dtype=torch.int64))
