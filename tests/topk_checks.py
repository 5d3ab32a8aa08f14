"""Shared checks for top-K lists on float tables (test helpers, CPU only).

A float score depends on the summation order, so two correct implementations
(the reference's torch.sum, numpy's pairwise sum, the fp32 MFMA fmaf chain,
the bf16 MFMA) may order near-ties differently. The bar: a
list must equal the reference's wherever the reference's neighbouring exact
scores are separated by more than the score tolerance, and where it differs
it must still be a valid top-k of the exact scores within that tolerance.
"""
import numpy as np

# fp32 dot product of width d: |computed - exact| <= c * eps32 * sum_j |u_j i_j|
# with c ~ d in the worst case; measured fmaf chains stay below ~1.5e-7 *
# sum|u_j i_j| (cdna_hip_programming.md, FP32-input MFMA) and torch's / numpy's
# blocked sums below that. 4e-7 covers both sides of a comparison.
FP32_REL = 4e-7


def fp32_row_tol(U, I, rel=FP32_REL):
    """Per-user score tolerance: rel * max_i sum_j |U[u,j] I[i,j]|."""
    A = np.abs(U.astype(np.float64)) @ np.abs(I.astype(np.float64)).T
    return rel * A.max(axis=1)


def gap_check(got, ref, U, I, frozen_csr, tol):
    """Number of users whose list differs from ``ref``; asserts each such list
    is a valid top-k of the exact (float64) scores within ``tol`` (a scalar or
    one value per user)."""
    S = U.astype(np.float64) @ I.astype(np.float64).T
    tol = np.broadcast_to(np.asarray(tol, dtype=np.float64), (ref.shape[0],))
    bad = 0
    for u in range(ref.shape[0]):
        if np.array_equal(got[u], ref[u]):
            continue
        s = S[u].copy()
        if frozen_csr is not None:
            rowptr, cols = frozen_csr
            s[cols[rowptr[u]:rowptr[u + 1]]] = -np.inf
        t = tol[u]
        gs = s[got[u]]
        assert len(set(got[u].tolist())) == len(got[u]), u  # no duplicates
        assert np.all(np.isfinite(gs)), u                    # no excluded item
        assert np.all(np.diff(gs) <= 2 * t), u               # sorted within tol
        kth = np.sort(s)[::-1][len(ref[u]) - 1]
        assert np.all(gs >= kth - 2 * t), u
        must = np.nonzero(s > kth + 2 * t)[0]
        assert set(must.tolist()) <= set(got[u].tolist()), u
        bad += 1
    return bad
