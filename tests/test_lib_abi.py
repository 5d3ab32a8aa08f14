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
    return sorted(set(re.findall(r"^\s*(?:int|size_t|double|const char\*)\s+(dr_\w+)\(", text, re.M)))


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


def test_build_id_is_the_source_hash():
    """The loaded library carries the hash of the sources it was compiled from
    (dr_build_id), equal to the in-tree sources' hash: the GPU records
    (tests, smoke, bench lines) name exactly which kernels ran."""
    from divrec import _buildid

    bid = _backend.build_id()
    assert re.fullmatch(r"[0-9a-f]{16}", bid)
    assert bid == _buildid.source_hash()


def test_stale_library_is_refused(tmp_path, monkeypatch):
    """A library built from other sources than the tree's is refused at load."""
    import shutil

    stale = tmp_path / "libdivrec_hip.so"
    shutil.copy(_backend.lib_path(), stale)
    monkeypatch.setattr(_backend, "_LIB", None)
    monkeypatch.setenv("DIVREC_HIP_LIB", str(stale))
    monkeypatch.setattr(_backend, "source_hash", lambda: "0" * 16)
    with pytest.raises(RuntimeError, match="stale"):
        _backend.load_library()


def test_argument_errors_without_gpu():
    lib = _backend.load_library()
    # k out of range -> DR_EINVAL with a message; nothing touches the device
    bf16, f32 = _backend.DR_BF16, _backend.DR_F32
    rc = lib.dr_score_topk(None, None, 10, None, 10, 0, bf16, 64, 0, None, None, None, None, None,
                           0, None)
    assert rc == -1 and b"k must be" in lib.dr_last_error()
    rc = lib.dr_score_topk(None, None, 10, None, 10, 0, bf16, 48, 10, None, None, None, None, None,
                           0, None)
    assert rc == -1 and b"d must be" in lib.dr_last_error()
    rc = lib.dr_score_topk(None, None, 10, None, 10, 0, f32, 512, 10, None, None, None, None, None,
                           0, None)
    assert rc == -1 and b"fp32 d must be" in lib.dr_last_error()
    rc = lib.dr_score_topk(None, None, 10, None, 10, 0, _backend.DR_I32, 64, 10, None, None, None,
                           None, None, 0, None)
    assert rc == -1 and b"DR_BF16 or DR_F32" in lib.dr_last_error()
    rc = lib.dr_ild_embedding(None, 3, 5, 500, None, 10, 128, 0, None, None, None)
    assert rc == -1
    rc = lib.dr_topk_merge(None, None, 3, 10, 1000, 2000, None, None, None)
    assert rc == -1 and b"k_out must be <= 1024" in lib.dr_last_error()
    rc = lib.dr_topk_merge(None, None, 3, 10, 1000, 10, None, None, None)
    assert rc == -1 and b"null pointer" in lib.dr_last_error()  # 3 x 1000 > 2048 is accepted
    rc = lib.dr_mmr_rerank(None, None, 4, 2000, None, 10, 128, 10, 0.5, None, None, None)
    assert rc == -1 and b"C must be" in lib.dr_last_error()
    rc = lib.dr_mmr_rerank(None, None, 4, 100, None, 0, 128, 10, 0.5, None, None, None)
    assert rc == -1 and b"empty item table" in lib.dr_last_error()
    # empty inputs are a no-op success
    assert lib.dr_gather_dot(None, 0, None, 0, 0, 64, None, None, 0, None, None, None) == 0
    rc = lib.dr_gather_dot(None, -1, None, 0, 0, 64, None, None, 3, None, None, None)
    assert rc == -1 and b"sizes" in lib.dr_last_error()


def test_workspace_query_is_host_only():
    lib = _backend.load_library()
    bf16, f32 = _backend.DR_BF16, _backend.DR_F32
    ws = lib.dr_score_topk_workspace(1_000_000, 10_000_000, bf16, 128, 100)
    # candidate buffers: n_users_pad * CAP(512) * 8 B for the single chunk, + counts
    assert ws >= 1_000_000 * 512 * 8
    assert lib.dr_score_topk_workspace(10, 10, bf16, 48, 10) == 0  # unsupported d
    assert lib.dr_score_topk_workspace(10, 10, f32, 512, 10) == 0  # no fp32 instance at 512
    # fp32 rows are twice as wide: same geometry as bf16 at 2d (k=1000 needs CAP 2048)
    assert lib.dr_score_topk_workspace(4096, 2000, f32, 64, 1000) == \
        lib.dr_score_topk_workspace(4096, 2000, bf16, 128, 1000)
    assert lib.dr_score_topk_workspace(4096, 2000, bf16, 128, 1000) >= 4096 * 2048 * 8


def test_score_widths_and_padding_host_logic():
    assert ops.score_width(torch.float32, 100) == 128
    assert ops.score_width(torch.bfloat16, 100) == 128
    assert ops.score_width(torch.bfloat16, 300) == 512
    assert ops.score_width(torch.float32, 16) == 32
    with pytest.raises(ValueError):
        ops.score_width(torch.float32, 300)
    t = torch.arange(6, dtype=torch.float32).reshape(2, 3)
    p = ops.pad_columns(t, 8)
    assert p.shape == (2, 8) and torch.equal(p[:, :3], t) and not p[:, 3:].any()
    assert ops.pad_columns(t, 3) is t


@pytest.mark.skipif(torch.cuda.is_available(), reason="checks the no-GPU behaviour")
def test_ops_fail_loudly_without_gpu():
    t = torch.zeros(4, 64)
    with pytest.raises(RuntimeError, match="no CPU fallback"):
        ops.gather_dot(t, t, torch.zeros(2, dtype=torch.int64), torch.zeros(2, dtype=torch.int64))


def test_workspace_reflects_split_tail_plan():
    """The planner (host only) splits the grid tail: 1M users at d=128 are 977
    user blocks for 256 workgroup slots, so 768 blocks scan the 10M catalog
    whole and each of the 209 tail blocks is split into 6 chunks, whose extra
    candidate buffers (5 x 209 x 1024 rows of CAP 512 keys) the workspace
    holds; with the split off (scan_split = 1) only one buffer per user
    remains (DESIGN.md §3.1 grid tail). The seeded plan's sample scan keeps
    dense tile maxima in the same region: 2441 tiles of the 78K-row sample x
    the padded users x 4 B, larger than the buffers here (sample_dense = 0:
    the compaction path, buffers only)."""
    lib = _backend.load_library()
    bf16 = _backend.DR_BF16
    one = (1_000_000 + 448) * 512 * 8  # padded users x CAP x 8 B
    extra = 5 * 209 * 1024 * 512 * 8
    dense = (1_000_000 + 448) * (10_000_000 // 128 // 32) * 4
    with _backend.plan_knobs(scan_slots=256):
        assert dense <= lib.dr_score_topk_workspace(1_000_000, 10_000_000, bf16, 128, 100) < dense + 200_000_000
    # a budget below the matrix (2 GiB) falls back to the compaction path's buffers
    with _backend.plan_knobs(scan_slots=256, sample_dense=2):
        assert lib.dr_score_topk_workspace(1_000_000, 10_000_000, bf16, 128, 100) < dense
    with _backend.plan_knobs(scan_slots=256, sample_dense=0):
        split = lib.dr_score_topk_workspace(1_000_000, 10_000_000, bf16, 128, 100)
        assert one + extra <= split < one + extra + 200_000_000
        with _backend.plan_knobs(scan_split=1):
            whole = lib.dr_score_topk_workspace(1_000_000, 10_000_000, bf16, 128, 100)
        assert one <= whole < one + 100_000_000
        # a grid of exactly one full round has no tail to split
        full = lib.dr_score_topk_workspace(256 * 1024, 10_000_000, bf16, 128, 100)
        assert full < 256 * 1024 * 512 * 8 + 100_000_000


def test_plan_knobs_set_restore_and_no_environment(monkeypatch):
    """The planner knobs live in the library (dr_set_plan_knob), NaN = default;
    plan_knobs restores the previous values; environment variables of the
    round-4 knob names change nothing (the product reads no environment)."""
    import math
    lib = _backend.load_library()
    bf16 = _backend.DR_BF16
    assert all(math.isnan(lib.dr_get_plan_knob(i)) for i in range(11))
    assert lib.dr_set_plan_knob(11, 1.0) == -1  # DR_EINVAL: unknown knob
    out = (ctypes.c_int64 * 13)()
    assert lib.dr_score_topk_plan(1_000_000, 10_000_000, bf16, 128, 100, out, 13) == 0
    base = list(out)
    monkeypatch.setenv("DIVREC_GUESS_STRIDE", "64")
    monkeypatch.setenv("DIVREC_SCAN_SPLIT", "1")
    assert lib.dr_score_topk_plan(1_000_000, 10_000_000, bf16, 128, 100, out, 13) == 0
    assert list(out) == base
    with _backend.plan_knobs(scan_split=1):  # no split: the 10M catalog is then not seeded
        assert lib.dr_score_topk_plan(1_000_000, 10_000_000, bf16, 128, 100, out, 13) == 0
        assert out[3] == 1 and out[7] == 0 and base[3] > 1 and base[7] == 128
    with _backend.plan_knobs(guess_stride=64):
        assert lib.dr_get_plan_knob(4) == 64.0
        assert lib.dr_score_topk_plan(1_000_000, 10_000_000, bf16, 128, 100, out, 13) == 0
        assert out[7] == 64
    assert math.isnan(lib.dr_get_plan_knob(4)) and math.isnan(lib.dr_get_plan_knob(1))
    with pytest.raises(ValueError):
        with _backend.plan_knobs(no_such_knob=1):
            pass


def test_seeded_topk_argument_errors_and_workspace():
    """dr_score_topk_seeded (caller thresholds) checks its arguments before any
    HIP call, and its workspace holds one seeded plan (no sample regions)."""
    lib = _backend.load_library()
    bf16 = _backend.DR_BF16
    rc = lib.dr_score_topk_seeded(None, None, 10, None, 10, 0, bf16, 64, 0, None, None, None,
                                  None, None, None, 0, None)
    assert rc == -1 and b"k must be" in lib.dr_last_error()
    rc = lib.dr_score_topk_seeded(None, None, 10, None, 10, 0, bf16, 64, 5, None, None, None,
                                  None, None, None, 0, None)
    assert rc == -1 and b"null pointer" in lib.dr_last_error()
    assert lib.dr_score_topk_seeded(None, None, 0, None, 10, 0, bf16, 64, 5, None, None, None,
                                    None, None, None, 0, None) == 0  # no users: no-op
    ws = lib.dr_score_topk_seeded_workspace(1_000_000, 1_250_000, bf16, 128, 100)
    assert ws >= (1_000_000 + 448) * 512 * 8
    assert lib.dr_score_topk_seeded_workspace(10, 10, bf16, 48, 10) == 0


def test_headline_plans_on_a_256_cu_device():
    """The plans of the benchmark shapes on 256 CUs (MI355X; this CPU host
    reports no device, and the planner then assumes 256): the headline's
    stride-128 guess with a 6-way split tail over the 4th round's 209 blocks,
    config 2's two unsplit rounds at stride 32, the 8-way shard's stride 32,
    and k = 1000's stride 128 (tests/test_real_plans.py runs them on the GPU)."""
    if torch.cuda.is_available():
        pytest.skip("plans depend on the device's CU count")
    bf = torch.bfloat16
    p = ops.score_topk_plan(1_000_000, 10_000_000, bf, 128, 100)
    assert (p["users_per_wg"], p["user_blocks"], p["head_blocks"], p["tail_chunks"],
            p["sample_stride"], p["sample_rank"]) == (1024, 977, 768, 6, 128, 10)
    p = ops.score_topk_plan(1_000_000, 1_000_000, bf, 64, 100)
    assert (p["users_per_wg"], p["user_blocks"], p["tail_chunks"], p["sample_stride"],
            p["sample_rank"]) == (2048, 489, 1, 32, 17)
    assert ops.score_topk_plan(1_000_000, 1_250_000, bf, 128, 100)["sample_stride"] == 32
    assert ops.score_topk_plan(1_000_000, 5_000_000, bf, 128, 100)["sample_stride"] == 64
    p = ops.score_topk_plan(1_000_000, 10_000_000, bf, 128, 1000)
    assert (p["sample_stride"], p["cap"]) == (128, 2048)
    # long lists: whole-catalog units end compacted to 1024 keys (a 1024-key
    # finalize instead of 2048); 977 blocks on 256 CUs: no split pays here
    assert (p["tail_chunks"], p["head_keys"], p["tail_keys"]) == (1, 1024, 1024)
    assert ops.score_topk_plan(1_000_000, 10_000_000, bf, 128, 100)["head_keys"] == 256
    assert ops.score_topk_plan(1000, 100_000, bf, 128, 100)["sample_stride"] == 0  # plain scan


def test_distributed_stride_mirrors_the_planner():
    """divrec.distributed.sample_stride (the global-threshold sample of the
    item-sharded multi-GPU path) must pick the single-GPU guess's stride for
    the whole catalog: compared with dr_score_topk_plan over catalog lengths
    around every switch point and k below / above the long-list bound."""
    from divrec.distributed import sample_stride

    for n in (1 << 18, 1 << 20, 4_194_303, 4_194_304, 5_000_000, 8_388_607, 8_388_608,
              10_000_000, 2 ** 23 + 1):
        for k in (10, 100, 255, 256, 1000):
            p = ops.score_topk_plan(4096, n, torch.bfloat16, 128, k)
            if p["sample_stride"]:
                assert sample_stride(n, k) == p["sample_stride"], (n, k)


def test_distributed_guess_ranks_mirror_the_planner():
    """divrec.distributed.guess_ranks (the global two-tier thresholds) must give
    the single-GPU guess's first-tier and safe ranks (dr_score_topk_plan's
    first_tier_rank and sample_rank) for the same sample fraction."""
    from divrec.distributed import guess_ranks

    for n in (1 << 18, 1_000_000, 1_250_000, 5_000_000, 10_000_000):
        for k in (10, 50, 100, 1000):
            p = ops.score_topk_plan(4096, n, torch.bfloat16, 128, k)
            if p["sample_stride"]:
                assert guess_ranks(k, p["sample_rows"] / n) == (p["first_tier_rank"],
                                                                p["sample_rank"]), (n, k)


def test_staged_scans_take_catalogs_above_2_28_rows():
    """the staged (d <= 64 bf16, d = 32 fp32) scans used to refuse
    catalog slices above 2^28 rows (a staged block named its tile in 23 bits).
    The tile is now named relative to its stage, so the call gets past the
    argument checks at 2^28 + 32 rows and its workspace and plan exist; the
    scan itself is exact there (tests/test_real_plans.py)."""
    lib = _backend.load_library()
    n = (1 << 28) + 32
    for dtype, d in ((_backend.DR_BF16, 32), (_backend.DR_BF16, 64), (_backend.DR_F32, 32)):
        assert lib.dr_score_topk_workspace(64, n, dtype, d, 10) > 0
        out = (ctypes.c_int64 * 13)()
        assert lib.dr_score_topk_plan(64, n, dtype, d, 10, out, 13) == 0
        rc = lib.dr_score_topk(None, None, 64, None, n, 0, dtype, d, 10, None, None, None, None,
                               None, 0, None)
        assert rc == -1 and b"null pointer" in lib.dr_last_error()


def test_small_catalogs_keep_every_key():
    """Small catalogs (<= 2048 rows) of calls with at most 16384 users plan a
    candidate buffer that holds every row (CAP >= n_items), so the scan never
    compacts and the finalize sorts all keys (round 6; config 1's 943 x 1682
    shape), and split the catalog into stage-long chunks over more CUs.
    Larger calls keep the compacting plan."""
    f32, bf = torch.float32, torch.bfloat16
    p = ops.score_topk_plan(943, 1682, f32, 32, 10)
    assert (p["cap"], p["head_keys"], p["tail_keys"], p["sample_stride"]) == (2048, 1682, 1682, 0)
    # the one user block's catalog split into stage-long chunks (no chunk compacts)
    assert (p["head_blocks"], p["tail_chunks"], p["chunk_items"]) == (0, 3, 896)
    p = ops.score_topk_plan(16384, 500, bf, 128, 100)
    assert (p["cap"], p["head_keys"]) == (512, 500)
    assert ops.score_topk_plan(16385, 500, bf, 128, 100)["head_keys"] != 500  # too many users
    assert ops.score_topk_plan(943, 2049, bf, 64, 10)["cap"] == 1024  # too many rows
    p = ops.score_topk_plan(100, 300, bf, 64, 600)  # k above the catalog: rank k still reached
    assert p["head_keys"] >= 600 and p["tail_keys"] >= 600
    p = ops.score_topk_plan(300, 2000, bf, 128, 1000)  # long lists: split chunks gather every key
    assert p["tail_chunks"] > 1 and p["tail_keys"] == 2000
    # bf16 d = 512 has no CAP-2048 instance: compacting plan
    assert ops.score_topk_plan(943, 1682, bf, 512, 10)["cap"] < 2048
