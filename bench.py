"""Headline benchmark: scored pairs/s + ILD-eval users/s, 1M users x 10M items,
d=128, top-100 (BASELINE.json metric; configs[3], the 10M-item catalog).

    python bench.py [--gpus N] [--steps K] [--warmup W]
    torchrun --nproc-per-node N --master-addr 127.0.0.1 ... bench.py --gpus N

One step = one pass of the hot path over the whole synthetic workload:
  score_topk (bf16 MFMA scores of every user of this rank's user slice x every
  item of its item shard, fused top-k) -> [item shards > 1: all_to_all of the
  partial top-k lists inside the rank's grid row over RCCL + merge] -> cosine
  ILD of the final top-k lists of this rank's users.
Ranks form a (N/S) x S grid (divrec.distributed.grid_layout): the S ranks of
a row row-shard the item table contiguously and share one user slice. S =
--item-shards (default N: pure 8-way item row-sharding at N=8, the north-star
layout). At N >= 4 the (N/2) x 2 grid is timed too and reported beside the
line as `grid_alt` (fewer, longer item shards: less survivor work per rank).
Inputs are resident in HBM before timing (the item table is also replicated
for the ILD gathers); the total work is fixed, so scaling is "strong".
value = U*I / step time (max over ranks).

Rank 0 prints ONE JSON line. The `roofline` object is for the dominant kernel
(score_topk: bound = MFMA, achieved = 2*U*I_shard*d flop / average HIP-event
time of the call on its stream); `traffic` comes from a committed rocprofv3 PMC
summary (profiles/pmc_traffic.json) when one exists for this exact config.
`cpu_baseline` (N=1 only) times the reference's per-user loop restated in
torch (oracle.reference_loop_topk: set difference, torch.full, embedding
gather + sum(u*i), argsort, slice) on all of this host's CPU share, on a
bounded user sample, with the vectorised torch GEMM + topk beside it.

Secondary workloads (single GPU, one JSON line each, same schema; the driver
runs the default only): ``--workload score1m`` (BASELINE configs[1]: 1M x 1M,
d=64, top-100), ``gather`` (the MatrixFactorization.forward row gather on
1M x 1M fp32 tables, HBM roofline), ``bpr`` (configs[2]: one BPR training step
= fused gather + loss + gradient scatter + dense Adam over both tables) and
``mmr`` (configs[4]: the top-1000 scan of the 10M-item catalog, MMR re-rank
of those 1000 candidates to 100 per user, and the ILD of the re-ranked lists;
users sharded over the ranks under torchrun, one all_reduce for the mean ILD).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "diversity-recommendations_amd"))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from divrec import ops  # noqa: E402
from divrec.distributed import (exchange_partials, global_mean, global_thresholds,  # noqa: E402
                               grid_layout, shard_range, thresholded_exchange)

MFMA_BF16_PEAK_TFLOPS = 2500.0  # MI355X dense bf16 (MI355X_MICROARCH.md)
MFMA_F32_PEAK_TFLOPS = 157.3  # v_mfma_f32_32x32x2_f32 (= the fp32 vector rate, MI355X_MICROARCH.md)
HBM_PEAK_GBS = 8000.0
ATOMIC_F32_GBS = 1300.0  # chip-wide global_atomic_add_f32 rate (MI355X_MICROARCH.md)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--users", type=int, default=1_000_000)
    ap.add_argument("--items", type=int, default=10_000_000)
    ap.add_argument("--dim", type=int, default=128)
    ap.add_argument("--k", type=int, default=100)
    ap.add_argument("--ild-kind", default="cosine")
    ap.add_argument("--cpu-budget-s", type=float, default=15.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--item-shards", type=int, default=0,
                    help="ranks that row-shard the item table per user slice (0 = the world "
                         "size: pure item sharding)")
    ap.add_argument("--local-thresholds", action="store_true",
                    help="item shards keep their local top-k (no global sample thresholds)")
    ap.add_argument("--no-alt-grid", action="store_true",
                    help="skip timing the (N/2) x 2 grid beside the main layout (N >= 4)")
    ap.add_argument("--backend", default="nccl", choices=["nccl", "gloo"],
                    help="process-group backend (gloo: multi-rank rehearsal on one GPU)")
    ap.add_argument("--same-device", action="store_true",
                    help="every rank on cuda:0 (rehearsing N ranks on a one-GPU box)")
    ap.add_argument("--check-users", type=int, default=0,
                    help="after timing, recompute this many of each rank's final users "
                         "over the whole catalog on one device and require identical lists")
    ap.add_argument("--fp64-check-users", type=int, default=1024,
                    help="world size 1: check this many of the timed call's lists (head, "
                         "split-tail and last user blocks) against float64 scores of the "
                         "same tables (gap-aware rule; 0 = off)")
    ap.add_argument("--workload", default="catalog",
                    choices=["catalog", "score1m", "gather", "bpr", "mmr", "fp32", "ml100k",
                             "excl"])
    ap.add_argument("--candidates", type=int, default=1000, help="mmr: top-C candidates per user")
    ap.add_argument("--mmr-k", type=int, default=100, help="mmr: re-ranked list length")
    ap.add_argument("--mmr-lambda", type=float, default=0.5)
    return ap.parse_args()


def gen_table(rows: int, d: int, seed: int, device, block: int = 1 << 20) -> torch.Tensor:
    """N(0, 1/sqrt(d)) rows in bf16, generated per 1M-row block with its own
    seed so any contiguous shard is identical whatever the world size."""
    out = torch.empty((rows, d), dtype=torch.bfloat16, device=device)
    scale = 1.0 / d ** 0.5
    for b0 in range(0, rows, block):
        g = torch.Generator(device=device).manual_seed(seed * 100_003 + b0 // block)
        n = min(block, rows - b0)
        out[b0 : b0 + n] = (torch.randn((n, d), generator=g, device=device) * scale).to(torch.bfloat16)
    return out


def host_cpu():
    """(threads used, visible logical CPUs, CPU model) of this host. The
    threads are this process's CPU share (OMP_NUM_THREADS, 16 on the GPU box,
    whose os.cpu_count() shows the whole machine), at most os.cpu_count()."""
    visible = os.cpu_count() or 1
    share = int(os.environ.get("OMP_NUM_THREADS", visible) or visible)
    model = "unknown"
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    return max(1, min(share, visible)), visible, model


def cpu_baseline(U: torch.Tensor, I: torch.Tensor, recs: torch.Tensor, k: int, budget_s: float):
    """The reference's per-user scoring loop, restated in torch with the same
    ops (oracle.reference_loop_topk), timed on this host's CPU share over a
    bounded user sample; the vectorised CPU form and the ILD loop beside it."""
    sys.path.insert(0, ROOT)
    import oracle

    threads, visible, model = host_cpu()
    torch.set_num_threads(threads)
    Uh = U[:64].float().cpu()
    Ih = I.float().cpu()
    n_items = Ih.shape[0]
    t0 = time.perf_counter()
    oracle.reference_loop_topk(Uh, Ih, k, users=[0])
    per_user = time.perf_counter() - t0
    n_users = int(max(1, min(16, budget_s * 0.8 // max(per_user, 1e-3))))
    t0 = time.perf_counter()
    oracle.reference_loop_topk(Uh, Ih, k, users=list(range(1, 1 + n_users)))
    dt = time.perf_counter() - t0
    pairs_per_s = n_users * n_items / dt
    # vectorised CPU: torch fp32 block GEMM + topk, all threads
    n_vec = 64
    t0 = time.perf_counter()
    torch.topk(Uh[:n_vec] @ Ih.T, k, dim=1)
    vec_dt = time.perf_counter() - t0
    # ILD (cosine, from embeddings): per-user pairwise sum of the reference formula
    rh = recs[:2000].long().cpu().numpy()
    Ihn = Ih.numpy()
    t0 = time.perf_counter()
    oracle.ild_embedding_f64(rh, Ihn, "cosine")
    ild_dt = time.perf_counter() - t0
    return {
        "value": pairs_per_s,
        "unit": "scored pairs/s",
        "cores": threads,
        "kind": "port",
        "cpu_model": model,
        "cpus_visible": visible,
        "sample": f"oracle.reference_loop_topk (the reference get_model_recommendations loop "
                  f"restated in torch: frozenset difference, LongTensor, torch.full, embedding "
                  f"gather + sum(u*i), argsort, slice, tolist) for {n_users} users x {n_items} "
                  f"items in {dt:.1f}s on {threads} threads; ILD: oracle.ild_embedding_f64, the "
                  f"VECTORISED float64 form (one Gram matrix per list), not the reference's "
                  f"itertools.combinations loop (~43 users/s at k = 100), on "
                  f"{len(rh)} users -> {len(rh) / ild_dt:.0f} users/s",
        "ild_users_per_s": len(rh) / ild_dt,
        "ild_kind": "vectorised float64 (oracle.ild_embedding_f64), not the reference's pair loop",
        "vectorized": {"value": n_vec * n_items / vec_dt, "unit": "scored pairs/s",
                       "cores": torch.get_num_threads(),
                       "sample": f"torch fp32 ({n_vec} x {Ih.shape[1]}) @ ({Ih.shape[1]} x {n_items}) "
                                 f"+ topk({k}), {vec_dt:.2f}s (a stronger CPU baseline than the "
                                 f"reference's per-user loop)"},
    }


_PEAKS = None
_PEAK_COLD = None  # the MFMA probe run before any timed work (a cold chip)


def _probe_lib():
    import ctypes

    path = os.path.join(ROOT, "tools", "_peaks", "libdivrec_peaks.so")
    if not os.path.exists(path):
        return None
    lib = ctypes.CDLL(path)
    lib.dr_peak_mfma.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_void_p,
                                 ctypes.c_void_p]
    lib.dr_peak_copy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int,
                                 ctypes.c_void_p]
    return lib


def _probe_timed(fn, reps=3):
    fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / 1e3 / reps


def _mfma_probe_tflops(lib, dev):
    """tools/peaks.hip: back-to-back v_mfma_f32_32x32x16_bf16 on random bf16
    operands at the scan's occupancy (8 waves/CU, 4 accumulators/wave),
    ~5-ms launches."""
    stream = torch.cuda.current_stream(dev).cuda_stream
    cus = torch.cuda.get_device_properties(dev).multi_processor_count
    g = torch.Generator(device=dev).manual_seed(99)
    src = torch.randn(8 << 20, generator=g, device=dev).to(torch.bfloat16)  # 16 MiB
    out = torch.empty(cus * 512, device=dev)
    iters = 40000
    t = _probe_timed(lambda: lib.dr_peak_mfma(src.data_ptr(), cus, iters, out.data_ptr(), stream))
    return cus * 8 * 4 * iters * 2.0 * 32 * 32 * 16 / t / 1e12


def cold_mfma_probe(dev):
    """Run the MFMA probe once BEFORE the timed region, on a chip that has not
    yet run the sustained scan (the probe after the timed
    scan runs on a hot, clocked-down chip and flatters the fraction)."""
    global _PEAK_COLD
    lib = _probe_lib()
    if lib is not None and _PEAK_COLD is None:
        _PEAK_COLD = _mfma_probe_tflops(lib, dev)
    return _PEAK_COLD


def achievable_peaks(dev):
    """The box's own peaks (tools/peaks.hip): back-to-back bf16 MFMA on random
    operands at the scan's occupancy, and a float4 HBM copy. Measured once per
    process after the timed region (the "hot" MFMA figure; the "cold" one is
    cold_mfma_probe's, before it); None if the probe library is not built."""
    global _PEAKS
    if _PEAKS is not None:
        return _PEAKS
    lib = _probe_lib()
    if lib is None:
        return None
    stream = torch.cuda.current_stream(dev).cuda_stream
    cus = torch.cuda.get_device_properties(dev).multi_processor_count
    hot = _mfma_probe_tflops(lib, dev)
    nbytes = 2 << 30
    a = torch.empty(nbytes, dtype=torch.uint8, device=dev)
    b = torch.empty_like(a)
    t_copy = min(_probe_timed(lambda: lib.dr_peak_copy(a.data_ptr(), b.data_ptr(), nbytes, cus * wg, stream))
                 for wg in (8, 32))  # best of two grid sizes
    del a, b
    _PEAKS = {"mfma_bf16_tflops": hot, "mfma_bf16_tflops_cold": _PEAK_COLD,
              "hbm_copy_gbs": 2 * nbytes / t_copy / 1e9,
              "probe": "tools/peaks.hip: v_mfma_f32_32x32x16_bf16 back-to-back on random operands, "
                       "8 waves/CU, 4 accumulators/wave, ~5-ms launches; float4 copy of 2 GiB"}
    return _PEAKS


HBM_ACHIEVABLE_GBS = 6290.0  # MI355X_MICROARCH.md: float4 copy, measured (79 % of 8 TB/s)


def with_measured(roof: dict, dev, key: str) -> dict:
    """Add an achievable peak and the fraction of it to a roofline object.
    MFMA: the box's own back-to-back bf16 MFMA loop on random operands (the
    clock it holds under that load is below the one the 2.5 PF spec assumes).
    HBM: the guide's measured 6.29 TB/s copy rate (this repo's probe copy,
    reported beside it, reaches less: a lower bound, not the ceiling)."""
    pk = achievable_peaks(dev)
    if key == "hbm_copy_gbs":
        roof["peak_achievable"] = HBM_ACHIEVABLE_GBS
        roof["frac_of_achievable"] = roof["achieved"] / HBM_ACHIEVABLE_GBS
        roof["achievable_source"] = "MI355X_MICROARCH.md (float4 copy, 6.29 TB/s)"
        if pk:
            roof["probe_copy_gbs"] = pk["hbm_copy_gbs"]
    elif pk:
        hot, cold = pk[key], pk.get(key + "_cold")
        # the larger of the two probe figures (usually the cold chip's): the
        # conservative fraction; both are reported
        best = max(hot, cold) if cold else hot
        roof["peak_achievable"] = best
        roof["frac_of_achievable"] = roof["achieved"] / best
        roof["peak_achievable_hot"] = hot
        roof["frac_of_achievable_hot"] = roof["achieved"] / hot
        if cold:
            roof["peak_achievable_cold"] = cold
            roof["frac_of_achievable_cold"] = roof["achieved"] / cold
        roof["achievable_source"] = pk["probe"] + ("; hot = after the timed region, cold = before "
                                                   "any timed work, peak_achievable = the larger")
    return roof


def same_build(rec: dict) -> bool:
    """A committed profile record describes the binary this process runs only
    if it carries the loaded library's build id (the source hash, stamped by
    tools/pmc_kernels.py / tools/pmc_mfma.py from the profiled run's own bench
    line); records of other builds, or without an id, are not used."""
    from divrec import _backend

    return bool(rec.get("build_id")) and rec.get("build_id") == _backend.build_id()


def load_traffic(cfg_key: str):
    """HBM bytes per dr_score_topk call from a committed PMC summary
    (tools/gpu_pmc.sh + tools/pmc_traffic.py) for exactly this config and build."""
    for name in ("pmc_traffic.json", f"pmc_traffic_{cfg_key}.json"):
        path = os.path.join(ROOT, "profiles", name)
        if not os.path.exists(path):
            continue
        try:
            with open(path) as f:
                rec = json.load(f)
            if rec.get("config") == cfg_key and same_build(rec):
                return rec.get("hbm_bytes_per_launch")
        except (OSError, ValueError):
            pass
    return None


def pmc_traffic(workload: str, config: str, kernel: str, group: int = 0, per_step: int = 1):
    """HBM bytes per step of one kernel from a committed per-dispatch PMC
    summary (tools/gpu_pmc_kernels.sh -> tools/pmc_kernels.py ->
    profiles/pmc_<workload>.json), read only when its config matches. The
    kernel's dispatches come in groups of `reps` calls (one group per phase
    of the workload, in launch order); `per_step` = dispatches per call, or 0:
    every dispatch of the pass belongs to the workload's `reps` calls (a call
    whose dispatch count varies, e.g. dr_score_topk's guess tiers)."""
    path = os.path.join(ROOT, "profiles", f"pmc_{workload}.json")
    try:
        with open(path) as f:
            rec = json.load(f)
    except (OSError, ValueError):
        return None
    if rec.get("config") != config or not same_build(rec):
        return None
    reps, total, found = int(rec["reps"]), 0.0, False
    for prefix in kernel.split("|"):  # every instantiation of every named kernel
        for name, k in rec["kernels"].items():
            if not name.startswith(prefix):
                continue
            if per_step == 0:
                part = k["hbm_bytes"]
            else:
                part = k["hbm_bytes"][group * reps * per_step:(group + 1) * reps * per_step]
                if len(part) != reps * per_step:
                    return None
            total, found = total + sum(part) / reps, True
    return total if found else None


SCAN_KERNELS = ("score_scan_kernel|sample_rows_kernel|topk_threshold_kernel|topk_finalize_kernel"
                "|topk_finalize_stream_kernel")
N_SIMDS = 256 * 4  # MI355X: 256 CUs x 4 SIMDs


def pmc_mfma(workload: str, config: str, kernel: str = "score_scan_kernel"):
    """MFMA utilisation of the scan from a committed rocprofv3 counter pass
    (tools/gpu_pmc_mfma.sh -> tools/pmc_mfma.py -> profiles/pmc_mfma_<workload>.json):
    SQ_VALU_MFMA_BUSY_CYCLES (cycles, = 32 per v_mfma_f32_32x32x16_bf16 on its
    SIMD; MI355X_MICROARCH.md, per-instruction constants) over the SIMD-cycles
    of the dispatches, GRBM_GUI_ACTIVE / 8 x 1024 SIMDs (GRBM sums the 8 XCDs).
    Read only when the config matches; None otherwise."""
    path = os.path.join(ROOT, "profiles", f"pmc_mfma_{workload}.json")
    try:
        with open(path) as f:
            rec = json.load(f)
    except (OSError, ValueError):
        return None
    if rec.get("config") != config or not same_build(rec):
        return None
    ks = rec.get("kernels", {})
    k = ks.get(kernel)
    if not k:
        return None
    # the instantiation with the most MFMA work (the seeded main scan)
    inst = max((n for n in ks if n.startswith(kernel + "<")),
               key=lambda n: ks[n]["mfma_busy_cycles"], default=None)
    out = {"mfma_busy_frac": k["mfma_busy_frac"], "effective_clock_ghz": k.get("clock_ghz"),
           "mfma_busy_cycles": k["mfma_busy_cycles"], "simd_cycles": k["simd_cycles"],
           "busy_over_flops": k.get("busy_over_expected"),
           "scope": f"every {kernel} dispatch of one call (sample scan, seeded scan, rescan)",
           "source": f"profiles/pmc_mfma_{workload}.json ({k.get('counters')})",
           "build_id": rec["build_id"]}
    if inst:
        out["main_scan"] = {"kernel": inst, "mfma_busy_frac": ks[inst]["mfma_busy_frac"]}
    return out


def provenance() -> dict:
    """The build id (source hash) of the loaded libdivrec_hip.so; divrec._backend
    has already refused a library built from other sources than the tree's."""
    from divrec import _backend

    return {"build_id": _backend.build_id()}


# --------------------------------------------------------------------------- rank launcher
def rank_envs(n: int, port: int, base=None) -> list:
    """The environment of each of n ranks on this node, as torchrun sets it
    (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_*; rendezvous on 127.0.0.1).
    Pure host logic: no device is touched."""
    base = dict(os.environ if base is None else base)
    envs = []
    for r in range(n):
        e = dict(base)
        e.update(RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                 GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        e.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")  # dmabuf IPC (RCCL between processes)
        envs.append(e)
    return envs


def free_port() -> int:
    import socket

    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        return sk.getsockname()[1]


def launch_ranks(n: int, cmd: list, envs: list, poll_s: float = 0.5) -> int:
    """Run `cmd` once per rank as child processes (one per GPU), from a parent
    that has made no GPU call (it only waits). Rank 0's stdout is this
    process's stdout (the one JSON line); the other ranks' stdout goes to
    stderr. The first rank to fail ends the job: the others are terminated
    (exact PIDs) and its exit code is returned; 0 when every rank succeeded."""
    import subprocess

    if torch.cuda.is_initialized():
        raise RuntimeError("launch_ranks: the parent must not initialise the GPU")
    procs = [subprocess.Popen(cmd, env=envs[r], stdout=None if r == 0 else sys.stderr)
             for r in range(n)]
    rc = 0
    try:
        while True:
            codes = [p.poll() for p in procs]
            failed = [c for c in codes if c not in (None, 0)]
            if failed:
                rc = failed[0]
                break
            if all(c == 0 for c in codes):
                break
            time.sleep(poll_s)
    finally:
        live = [p for p in procs if p.poll() is None]
        for p in live:
            p.terminate()
        for p in live:
            try:
                p.wait(timeout=20)
            except subprocess.TimeoutExpired:
                p.kill()
                p.wait()
    return rc


def maybe_launch(args) -> int | None:
    """`--gpus N > 1` outside torchrun (no WORLD_SIZE): start N ranks of this
    same command, one process per GPU, and return the job's exit code. Under
    torchrun (WORLD_SIZE set), or at N = 1, None: run in this process."""
    if args.gpus <= 1 or "WORLD_SIZE" in os.environ:
        return None
    cmd = [sys.executable, "-u", os.path.abspath(__file__)] + sys.argv[1:]
    return launch_ranks(args.gpus, cmd, rank_envs(args.gpus, free_port()))


def time_layout(args, world: int, dev, S: int, record_recs: bool = True):
    """Time the catalog step on a (world/S) x S grid of ranks: warmup, barrier,
    exactly args.steps timed steps, barrier; max over ranks. Returns a dict
    with the step time, per-kernel HIP-event times and this rank's data."""
    lay = grid_layout(S) if world > 1 else None
    U_n, I_n, d, k = args.users, args.items, args.dim, args.k
    # (user slice) x (item shard) of this rank in the grid; the item table is
    # also replicated in full for the ILD gathers
    u_lo, u_hi = lay.user_range(U_n) if lay else (0, U_n)
    lo, hi = lay.item_range(I_n) if lay else (0, I_n)
    users = gen_table(U_n, d, 1, dev)[u_lo:u_hi].contiguous()
    items = gen_table(I_n, d, 2, dev)
    shard = items[lo:hi]
    torch.cuda.synchronize()
    ev = {n: [] for n in ("topk0", "topk1", "ild0", "ild1")}

    def step(record: bool):
        e = [torch.cuda.Event(enable_timing=True) for _ in range(4)] if record else None
        if e:
            e[0].record()
        if S > 1 and not args.local_thresholds:
            # shards keep only items above per-user thresholds guessed from a
            # sample of the whole catalog (divrec.distributed.global_thresholds)
            thr = global_thresholds(users, shard, lo, hi, I_n, k, lay.group)  # [2, n]: tiers
            s, i = ops.score_topk(users, shard, k, item_base=lo, init_thr=thr[0])
        else:
            s, i = ops.score_topk(users, shard, k, item_base=lo)
        if e:
            e[1].record()
        if S > 1:  # partial lists of this rank's sub-slice from its row, merged
            if args.local_thresholds:
                ps, pi = exchange_partials(s, i, lay.group)
                s, i = ops.topk_merge(ps, pi, k)
            else:  # exchange + merge + verification (exact fallback if a guess failed)
                s, i = thresholded_exchange(users, shard, lo, hi, I_n, k, lay.group,
                                            thr=thr, local=(s, i))
        if e:
            e[2].record()
        ild = ops.ild_embedding(i, items, args.ild_kind, check=False)
        if e:
            e[3].record()
            ev["topk0"].append(e[0]); ev["topk1"].append(e[1])
            ev["ild0"].append(e[2]); ev["ild1"].append(e[3])
        return s, i, ild

    for _ in range(args.warmup):
        step(False)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        scores, recs, ild = step(True)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    topk_s = sum(a.elapsed_time(b) for a, b in zip(ev["topk0"], ev["topk1"])) / 1e3 / args.steps
    ild_s = sum(a.elapsed_time(b) for a, b in zip(ev["ild0"], ev["ild1"])) / 1e3 / args.steps
    t = torch.tensor([dt, ild_s, topk_s], dtype=torch.float64,
                     device="cpu" if args.backend == "gloo" else dev)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return {"lay": lay, "S": S, "dt": float(t[0]), "ild_max": float(t[1]),
            "topk_max": float(t[2]), "topk_s": topk_s, "users": users, "items": items,
            "recs": recs if record_recs else None, "scores": scores if record_recs else None,
            "u_lo": u_lo, "u_hi": u_hi, "lo": lo, "hi": hi}


def main():
    args = parse()
    if args.workload in ("catalog", "mmr"):  # the multi-GPU workloads
        rc = maybe_launch(args)
        if rc is not None:
            return rc
    if args.workload == "mmr":
        return mmr_pipeline(args)
    if args.workload != "catalog":
        return secondary(args)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus and rank == 0:
        print(f"note: --gpus {args.gpus} but WORLD_SIZE={world}; using WORLD_SIZE", file=sys.stderr)
    dev_index = 0 if args.same_device else local_rank
    torch.cuda.set_device(dev_index)
    dev = torch.device("cuda", dev_index)
    S = 1
    if world > 1:
        if args.backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group("gloo")
        S = args.item_shards or world
    if rank == 0:
        cold_mfma_probe(dev)  # before any timed work (a cold chip); the hot probe runs after
    r = time_layout(args, world, dev, S)
    U_n, I_n, d, k = args.users, args.items, args.dim, args.k
    step_s = r["dt"] / args.steps
    u_lo, u_hi, lo, hi = r["u_lo"], r["u_hi"], r["lo"], r["hi"]

    cfg_key = f"U{U_n}_I{I_n}_d{d}_k{k}_G{world}"
    idb = r["recs"].element_size() if r["recs"] is not None else 4  # id bytes the ILD reads
    flops = 2.0 * (u_hi - u_lo) * (hi - lo) * d
    achieved = flops / r["topk_s"] / 1e12
    traffic = pmc_traffic("catalog", cfg_key, SCAN_KERNELS, per_step=0) or load_traffic(cfg_key)
    result = {
        "metric": "scored pairs/sec + ILD-eval users/sec, 1M x 10M d=128 at 1/2/4/8 GPU",
        "value": U_n * I_n / step_s,
        "unit": "scored pairs/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": step_s * 1e3,
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "bf16",
        "data": "synthetic (N(0,1/sqrt(d)) bf16 tables, seeded per 1M-row block)",
        "config": {
            "workload": f"score_topk + cosine ILD: {U_n} users x {I_n} items, d={d}, k={k} "
                        f"(BASELINE configs[3]; ranks in a {world // S} x {S} grid: item rows "
                        f"sharded {S} ways, users {world // S} ways)",
            "users": U_n, "items": I_n, "dim": d, "k": k,
            "parallelism": f"item-shard{S}" + (f"+all_to_all(group of {S})" if S > 1 else "")
                           + (f" x user-shard{world // S}" if world // S > 1 else ""),
            "item_shards": S,
        },
        "ild_users_per_s": U_n / r["ild_max"],
        "ild_roofline": dict(_hbm(U_n // world * (k * idb + k * d * 2 + 4), r["ild_max"],
                                  pmc_traffic("catalog", cfg_key, "ild_embedding_stream")),
                             kernel="dr_ild_embedding (cosine; ild_embedding_stream)",
                             per_unit=f"{k * idb + k * d * 2 + 4} B/user = k {8 * idb}-bit ids "
                                      f"+ k bf16 rows + out",
                             # at k=100 report the MFMA side too (upper-triangle Gram)
                             mfma_tflops=U_n // world * k * (k - 1) * d / r["ild_max"] / 1e12,
                             mfma_frac=U_n // world * k * (k - 1) * d / r["ild_max"] / 1e12
                             / MFMA_BF16_PEAK_TFLOPS),
        "score_topk_ms": r["topk_s"] * 1e3,
        "score_topk_ms_max_over_ranks": r["topk_max"] * 1e3,
        "ild_ms": r["ild_max"] * 1e3,
        "roofline": {
            "bound": "mfma",
            "achieved": achieved,
            "peak": MFMA_BF16_PEAK_TFLOPS,
            "unit": "TFLOP/s",
            "frac": achieved / MFMA_BF16_PEAK_TFLOPS,
            "traffic": traffic,
            "kernel": "dr_score_topk = score_scan_kernel (MFMA scan + fused threshold top-k) + topk_finalize_kernel; timed together",
            "flop_per_launch": flops,
            "mfma_counters": pmc_mfma("catalog", cfg_key),
        },
        "cpu_baseline": None,
    }
    result.update(provenance())
    if args.check_users > 0:
        result["check"] = check_lists(args, r["lay"], r["users"], r["items"], r["recs"], u_lo,
                                      U_n, k, world)
    elif world == 1 and args.fp64_check_users > 0:
        # the timed call's own lists on its own tables, against float64
        # (outside the timed region)
        sel = check_user_sample(U_n, I_n, d, k, args.fp64_check_users)
        result["check"] = fp64_gap_check(r["users"], r["items"], r["scores"], r["recs"], sel, k)
        if not result["check"]["ok"]:
            print(f"fp64 list check FAILED: {result['check']}", file=sys.stderr, flush=True)
    if world >= 4 and world % 2 == 0 and S != 2 and not args.no_alt_grid:
        # the (N/2) x 2 grid beside the main layout: same work,
        # 2-way item shards, users split N/2 ways
        del r
        torch.cuda.empty_cache()
        a = time_layout(args, world, dev, 2, record_recs=False)
        a_step = a["dt"] / args.steps
        result["grid_alt"] = {
            "layout": f"{world // 2} x 2 grid (item rows sharded 2 ways, users {world // 2} ways, "
                      f"all_to_all inside each pair)",
            "item_shards": 2, "value": U_n * I_n / a_step, "unit": "scored pairs/s",
            "ms_per_step": a_step * 1e3, "score_topk_ms": a["topk_s"] * 1e3,
            "roofline_frac": 2.0 * (a["u_hi"] - a["u_lo"]) * (a["hi"] - a["lo"]) * d
                             / a["topk_s"] / 1e12 / MFMA_BF16_PEAK_TFLOPS}
        r = None
    if rank == 0:
        with_measured(result["roofline"], dev, "mfma_bf16_tflops")
        # the ILD's gather against the guide's copy rate and this box's own
        # float4 copy probe (HBM rates differ from box to box)
        ild_roof = with_measured(result["ild_roofline"], dev, "hbm_copy_gbs")
        if ild_roof.get("probe_copy_gbs"):
            ild_roof["frac_of_probe_copy"] = ild_roof["achieved"] / ild_roof["probe_copy_gbs"]
    if world == 1 and not args.no_cpu_baseline:
        result["cpu_baseline"] = cpu_baseline(r["users"], r["items"], r["recs"], k,
                                              args.cpu_budget_s)
    if rank == 0:
        print(json.dumps(result), flush=True)
    if world > 1:
        dist.destroy_process_group()


def check_user_sample(U_n: int, I_n: int, d: int, k: int, n: int) -> torch.Tensor:
    """~n users of the call's plan (ops.score_topk_plan), drawn from every
    kind of unit: whole-catalog head blocks, split-tail blocks and the last
    (partial) block; sorted, unique."""
    plan = ops.score_topk_plan(U_n, I_n, torch.bfloat16, d, k)
    upw, head = plan["users_per_wg"], plan["head_blocks"]
    g = torch.Generator().manual_seed(4242)
    head_users = min(head * upw, U_n)
    last0 = max((plan["user_blocks"] - 1) * upw, head_users)
    ranges = [(0, head_users), (head_users, last0), (last0, U_n)]  # head, split tail, last block
    want = [n * 3 // 8, n * 3 // 8, n - 2 * (n * 3 // 8)]
    parts, carry = [], 0
    for (lo, hi), w in zip(reversed(ranges), reversed(want)):  # last block first: it is small
        m = min(w + carry, hi - lo)  # a short range hands its deficit to the next one
        carry = w + carry - m
        if m > 0:
            parts.append(lo + torch.randperm(hi - lo, generator=g)[:m])
    return torch.sort(torch.cat(parts)).values


def fp64_gap_check(users: torch.Tensor, items: torch.Tensor, scores: torch.Tensor,
                   recs: torch.Tensor, sel: torch.Tensor, k: int, chunk: int = 1 << 19,
                   extra: int = 64) -> dict:
    """The rule of tests/test_hip_kernels.py::test_score_topk_float_tolerance
    on the timed call's own lists (bf16 tables: exact products, so only the
    fp32 summation order separates a score from its float64 value):
    every returned score within tol of its float64 value and the list sorted
    within tol; every returned item at or above the exact k-th score - 2 tol;
    every item scoring above the k-th + 2 tol returned. The exact float64
    top-(k + extra) of each selected user over the whole catalog is built on
    the device chunk by chunk (every item above the k-th score is among the
    top k - 1, so it holds the whole must-return set)."""
    dev = users.device
    d = users.shape[1]
    tol = 1e-5 * (d / 64) ** 0.5
    sel = sel.to(dev)
    U = users[sel].double()
    got_i = recs[sel].long()
    got_s = scores[sel].double()
    best_s = torch.full((sel.numel(), k + extra), -float("inf"), dtype=torch.float64, device=dev)
    best_i = torch.zeros((sel.numel(), k + extra), dtype=torch.int64, device=dev)
    t0 = time.perf_counter()
    for c0 in range(0, items.shape[0], chunk):
        S = U @ items[c0:c0 + chunk].double().T
        ts, ti = torch.topk(S, min(k + extra, S.shape[1]), dim=1)
        best_s, pos = torch.topk(torch.cat([best_s, ts], 1), k + extra, dim=1)
        best_i = torch.gather(torch.cat([best_i, ti + c0], 1), 1, pos)
        del S
    exact = (U.unsqueeze(1) * items[got_i.clamp(min=0)].double()).sum(-1)  # float64 score per item
    kth = best_s[:, k - 1:k]
    ok_score = bool(((got_s - exact).abs() <= tol).all())
    ok_sorted = bool((got_s[:, 1:] - got_s[:, :-1] <= 2 * tol).all())
    ok_above = bool((exact >= kth - 2 * tol).all())
    must = best_s > kth + 2 * tol
    hit = (best_i.unsqueeze(2) == got_i.unsqueeze(1)).any(2)
    ok_must = bool((hit | ~must).all())
    ok_valid = bool((got_i >= 0).all())
    exact_order = int((best_i[:, :k] != got_i).any(1).sum())
    return {"users_checked": int(sel.numel()), "rule": "fp64 gap-aware", "tol": tol,
            "ok": ok_score and ok_sorted and ok_above and ok_must and ok_valid,
            "scores_within_tol": ok_score, "sorted_within_tol": ok_sorted,
            "all_above_kth_minus_2tol": ok_above, "all_clear_top_k_returned": ok_must,
            "users_not_in_exact_float64_order": exact_order,
            "max_abs_score_err": float((got_s - exact).abs().max()),
            "check_s": time.perf_counter() - t0}


def check_lists(args, lay, users, items, recs, u_lo, U_n, k, world):
    """Multi-rank parity (outside the timed region): the first --check-users
    users this rank owns after the exchange, rescored over the WHOLE catalog
    by one score_topk call, must give the identical lists (the key order is
    total, so any item partition merges bit-identically)."""
    n_slice = users.shape[0]
    if lay is not None and lay.item_shards > 1:
        f_lo, f_hi = shard_range(n_slice, lay.item_shards, lay.item_shard)
    else:
        f_lo, f_hi = 0, n_slice
    n = min(args.check_users, f_hi - f_lo)
    _, ref = ops.score_topk(users[f_lo:f_lo + n].contiguous(), items, k)
    ok = bool(torch.equal(ref.to(recs.dtype), recs[:n]))
    t = torch.tensor([0 if ok else 1, n], dtype=torch.int64, device=users.device)
    if world > 1:
        if args.backend == "gloo":
            t = t.cpu()
        dist.all_reduce(t)
    if int(t[0]) != 0:
        raise SystemExit(f"multi-rank check FAILED on {int(t[0])} rank(s)")
    return {"users_checked": int(t[1]), "identical": True,
            "first_user": u_lo + f_lo}


# --------------------------------------------------------------------------- secondary workloads
def _timed(fn, steps: int, warmup: int):
    """Run fn() warmup + steps times; return (wall seconds per step, device
    seconds per step from HIP events on the current stream)."""
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    e0.record()
    for _ in range(steps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / steps, e0.elapsed_time(e1) / 1e3 / steps


def _line(metric, value, unit, args, step_s, dtype, config, roofline, cpu, **extra):
    dev = torch.device("cuda", 0)
    if roofline.get("peak") == MFMA_F32_PEAK_TFLOPS:  # fp32 MFMA: the guide's measured rate
        roofline.update(peak_achievable=155.0, frac_of_achievable=roofline["achieved"] / 155.0,
                        achievable_source="MI355X_MICROARCH.md (v_mfma_f32_32x32x2_f32, 155 TF)")
    else:
        with_measured(roofline, dev,
                      "mfma_bf16_tflops" if roofline["bound"] == "mfma" else "hbm_copy_gbs")
    for v in extra.values():
        if isinstance(v, dict) and v.get("bound") == "hbm":
            with_measured(v, dev, "hbm_copy_gbs")
    rec = {"metric": metric, "value": value, "unit": unit, "n_gpus": 1, "steps": args.steps,
           "warmup": args.warmup, "ms_per_step": step_s * 1e3, "higher_is_better": True,
           "scaling": "replicas", "vs_baseline": None, "dtype": dtype,
           "data": "synthetic (seeded)", "config": config, "roofline": roofline,
           "cpu_baseline": cpu}
    rec.update(extra)
    rec.update(provenance())
    print(json.dumps(rec), flush=True)


def _hbm(bytes_per_launch, seconds, traffic=None):
    gbs = bytes_per_launch / seconds / 1e9
    return {"bound": "hbm", "achieved": gbs, "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": gbs / HBM_PEAK_GBS, "traffic": traffic, "bytes_per_launch": bytes_per_launch}


def secondary(args):
    import numpy as np

    sys.path.insert(0, ROOT)
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    cold_mfma_probe(dev)  # before any timed work
    g = torch.Generator(device=dev).manual_seed(1234)
    want_cpu = not args.no_cpu_baseline

    if args.workload == "score1m":
        U_n, I_n, d, k = 1_000_000, 1_000_000, 64, 100
        users, items = gen_table(U_n, d, 1, dev), gen_table(I_n, d, 2, dev)
        wall, dt = _timed(lambda: ops.score_topk(users, items, k), args.steps, args.warmup)
        flops = 2.0 * U_n * I_n * d
        cpu = None
        if want_cpu:
            import oracle

            # the reference's per-user loop restated in torch (as the headline's
            # baseline) on this process's CPU share, users one at a time until
            # the budget (~10 s of CPU work)
            threads, visible, model = host_cpu()
            torch.set_num_threads(threads)
            Uh, Ih = users[:256].float().cpu(), items.float().cpu()
            oracle.reference_loop_topk(Uh, Ih, k, users=[0])  # warm
            n, t0 = 0, time.perf_counter()
            while n < 256 and time.perf_counter() - t0 < args.cpu_budget_s * 2 / 3:
                oracle.reference_loop_topk(Uh, Ih, k, users=[n])
                n += 1
            t = time.perf_counter() - t0
            cpu = {"value": n * I_n / t, "unit": "scored pairs/s", "cores": threads,
                   "kind": "port", "cpu_model": model, "cpus_visible": visible,
                   "sample": f"oracle.reference_loop_topk (the reference get_model_recommendations "
                             f"loop restated in torch), {n} users x {I_n} items, {t:.1f}s on "
                             f"{threads} threads"}
        _line("scored pairs/sec, 1M x 1M d=64 top-100 (BASELINE configs[1])", U_n * I_n / wall,
              "scored pairs/s", args, wall, "bf16",
              {"workload": "score_topk 1M users x 1M items d=64 k=100", "users": U_n,
               "items": I_n, "dim": d, "k": k},
              {"bound": "mfma", "achieved": flops / dt / 1e12, "peak": MFMA_BF16_PEAK_TFLOPS,
               "unit": "TFLOP/s", "frac": flops / dt / 1e12 / MFMA_BF16_PEAK_TFLOPS,
               "traffic": (pmc_traffic("score1m", f"U{U_n}_I{I_n}_d{d}_k{k}_G1", SCAN_KERNELS,
                                       per_step=0)
                           or load_traffic(f"U{U_n}_I{I_n}_d{d}_k{k}_G1")),
               "mfma_counters": pmc_mfma("score1m", f"U{U_n}_I{I_n}_d{d}_k{k}_G1"),
               "kernel": "dr_score_topk (sample scan + thresholds + seeded scan + finalize)"}, cpu)
        return 0

    if args.workload == "ml100k":
        return ml100k(args, dev, g)

    if args.workload == "excl":
        # the headline shape with a 100-items/user exclusion CSR
        # (RankingDataset's frozen items, base_datasets.py:145-151): the
        # compaction and the finalize drop excluded keys by binary search.
        # Timed beside the same call without exclusions, in one process.
        U_n, I_n, d, k, n_ex = args.users, args.items, args.dim, args.k, 100
        users, items = gen_table(U_n, d, 1, dev), gen_table(I_n, d, 2, dev)
        ex = torch.sort(torch.randint(0, I_n, (U_n, n_ex), generator=g, device=dev,
                                      dtype=torch.int32), dim=1).values
        # distinct items per user: a sorted row with repeats bumped past them
        # would need a loop; instead drop the repeats and keep the CSR ragged
        keep = torch.ones_like(ex, dtype=torch.bool)
        keep[:, 1:] = ex[:, 1:] != ex[:, :-1]
        cnt = keep.sum(1).to(torch.int64)
        rowptr = torch.zeros(U_n + 1, dtype=torch.int64, device=dev)
        rowptr[1:] = torch.cumsum(cnt, 0)
        cols = ex[keep].contiguous()
        wall0, dt0 = _timed(lambda: ops.score_topk(users, items, k), args.steps, args.warmup)
        wall, dt = _timed(lambda: ops.score_topk(users, items, k, exclude=(rowptr, cols)),
                          args.steps, args.warmup)
        flops = 2.0 * U_n * I_n * d
        _line("scored pairs/sec with a 100-items/user exclusion CSR, 1M x 10M d=128 top-100 "
              "(SURVEY.md 8d)", U_n * I_n / wall, "scored pairs/s", args, wall, "bf16",
              {"workload": f"score_topk {U_n} users x {I_n} items d={d} k={k}, "
                           f"{int(cols.numel())} excluded (user, item) pairs", "users": U_n,
               "items": I_n, "dim": d, "k": k, "excluded_per_user": n_ex},
              {"bound": "mfma", "achieved": flops / dt / 1e12, "peak": MFMA_BF16_PEAK_TFLOPS,
               "unit": "TFLOP/s", "frac": flops / dt / 1e12 / MFMA_BF16_PEAK_TFLOPS,
               "traffic": None, "kernel": "dr_score_topk with exclusions"}, None,
              no_exclusion_ms=dt0 * 1e3, exclusion_ms=dt * 1e3,
              exclusion_overhead=dt / dt0 - 1.0)
        return 0

    if args.workload == "fp32":
        # MatrixFactorization.score_topk's default (fp32-faithful) mode on the
        # reference experiments' own width, d = 100 (zero-padded to 128 once
        # per parameter version, as the model does): exact fp32 products and
        # fp32 sums on v_mfma_f32_32x32x2_f32
        U_n, I_n, d, k = 262_144, 1_000_000, 100, 100
        w = ops.score_width(torch.float32, d)
        users = ops.pad_columns(torch.randn(U_n, d, generator=g, device=dev), w)
        items = ops.pad_columns(torch.randn(I_n, d, generator=g, device=dev), w)
        wall, dt = _timed(lambda: ops.score_topk(users, items, k), args.steps, args.warmup)
        flops_pad = 2.0 * U_n * I_n * w
        _line("fp32-faithful scored pairs/sec, d=100 (MatrixFactorization default scoring mode)",
              U_n * I_n / wall, "scored pairs/s", args, wall, "f32",
              {"workload": f"score_topk on fp32 tables {U_n} users x {I_n} items, d={d} "
                           f"zero-padded to {w}, k={k}", "users": U_n, "items": I_n, "dim": d,
               "scan_width": w, "k": k},
              {"bound": "mfma", "achieved": flops_pad / dt / 1e12, "peak": MFMA_F32_PEAK_TFLOPS,
               "unit": "TFLOP/s", "frac": flops_pad / dt / 1e12 / MFMA_F32_PEAK_TFLOPS,
               "traffic": pmc_traffic("fp32", f"fp32_U{U_n}_I{I_n}_d{d}_k{k}", SCAN_KERNELS, per_step=0),
               "flop_per_launch": flops_pad,
               "kernel": "dr_score_topk, fp32 scan (v_mfma_f32_32x32x2_f32) + finalize; flops "
                         "counted at the padded width"},
              None, useful_tflops=2.0 * U_n * I_n * d / dt / 1e12)
        return 0

    if args.workload == "gather":
        U_n, I_n, d, n = 1_000_000, 1_000_000, 128, 1 << 23
        Ut = torch.randn(U_n, d, generator=g, device=dev)
        It = torch.randn(I_n, d, generator=g, device=dev)
        uid = torch.randint(0, U_n, (n,), generator=g, device=dev)
        iid = torch.randint(0, I_n, (n,), generator=g, device=dev)
        wall, dt = _timed(lambda: ops.gather_dot(Ut, It, uid, iid, check=False), args.steps,
                          args.warmup)
        per_pair = 2 * d * 4 + 2 * 8 + 4
        cpu = None
        if want_cpu:
            import oracle

            threads, visible, model = host_cpu()
            torch.set_num_threads(threads)
            Uh, Ih = Ut.cpu(), It.cpu()
            m = 1 << 22
            uh, ih = uid[:m].cpu(), iid[:m].cpu()
            oracle.reference_mf_forward(Uh, Ih, uh[:4096], ih[:4096])  # warm
            t0 = time.perf_counter()
            oracle.reference_mf_forward(Uh, Ih, uh, ih)
            t = time.perf_counter() - t0
            cpu = {"value": m / t, "unit": "pairs/s", "cores": threads, "kind": "port",
                   "cpu_model": model, "cpus_visible": visible,
                   "sample": f"oracle.reference_mf_forward (MatrixFactorization.forward restated "
                             f"in torch: two embedding gathers + sum(u * i)), {m} uniform pairs, "
                             f"{t:.2f}s on {threads} threads"}
        # the reference's own call patterns (runs of equal ids, each row read
        # once per run): RankingDataset's (full((n,), u), candidates) over the
        # whole catalog for 8 users, and PairWiseDataset's m x m product
        # (m = 20, the reference config) as model(u, pos) and model(u, neg)
        def run_bytes(u_, i_):
            """ids + outputs + each row once per run of equal user ids (the
            user row and the run's distinct items: what a kernel that keeps a
            run's rows must read)."""
            run = torch.cumsum(torch.cat([torch.ones(1, dtype=torch.int64, device=dev),
                                          (u_[1:] != u_[:-1]).to(torch.int64)]), 0)
            n_runs = int(run[-1])
            n_items_run = torch.unique(run * I_n + i_).numel()
            return u_.numel() * (2 * 8 + 4) + (n_runs + n_items_run) * d * 4
        m_s = 20
        n_mu = n // (m_s * m_s)
        mu = torch.randint(0, U_n, (n_mu,), generator=g, device=dev)
        mpos = torch.randint(0, I_n, (n_mu, m_s), generator=g, device=dev)
        mneg = torch.randint(0, I_n, (n_mu, m_s), generator=g, device=dev)
        pats = {
            "full_u_candidates": (torch.arange(8, device=dev).repeat_interleave(I_n),
                                  torch.arange(I_n, device=dev).repeat(8)),
            "mxm_model_u_pos": (mu.repeat_interleave(m_s * m_s),
                                mpos.repeat_interleave(m_s, dim=1).reshape(-1)),
            "mxm_model_u_neg": (mu.repeat_interleave(m_s * m_s), mneg.repeat(1, m_s).reshape(-1)),
        }
        patterns = {}
        for name, (pu, pi) in pats.items():
            pw, pdt = _timed(lambda: ops.gather_dot(Ut, It, pu, pi, check=False), args.steps,
                             args.warmup)
            nb = run_bytes(pu, pi)
            patterns[name] = dict(_hbm(nb, pdt, pmc_traffic("gather", "gather", "gather_dot_runs",
                                                            group=1 + len(patterns))),
                                  pairs=pu.numel(), pairs_per_s=pu.numel() / pw,
                                  ms=pdt * 1e3, bytes_per_pair=nb / pu.numel(),
                                  per_unit="2 ids x 8 B + 4 B out per pair + d x 4 B per "
                                           "user run for its user row and each distinct item")
            with_measured(patterns[name], dev, "hbm_copy_gbs")
        del pats
        # the autograd backward of MatrixFactorization.forward (dense embedding
        # gradients): two row gathers + two rows of fp32 atomic adds per pair
        gU, gI = torch.zeros_like(Ut), torch.zeros_like(It)
        gout = torch.randn(n, generator=g, device=dev)
        bwall, bdt = _timed(lambda: ops.gather_dot_backward(Ut, It, uid, iid, gout, gU, gI),
                            args.steps, args.warmup)
        added = 2 * d * 4 * n
        backward = {"value": n / bwall, "unit": "pairs/s", "ms": bdt * 1e3,
                    "kernel": "dr_gather_dot_backward",
                    "hbm_roofline": _hbm((2 * d * 4 + 2 * 8 + 4) * n + added, bdt,
                                         pmc_traffic("gather", "gather", "gather_dot_bwd_rows")),
                    "atomic_roofline": {"bound": "fp32 atomics", "added_bytes": added,
                                        "achieved": added / bdt / 1e9, "peak": ATOMIC_F32_GBS,
                                        "unit": "GB/s", "frac": added / bdt / 1e9 / ATOMIC_F32_GBS}}
        _line("MatrixFactorization.forward gathered pairs/sec (fp32 1M x 1M d=128)", n / wall,
              "pairs/s", args, wall, "f32",
              {"workload": f"dr_gather_dot, {n} uniform random (user, item) pairs, fp32 tables "
                           f"{U_n}x{d} and {I_n}x{d}", "pairs": n, "dim": d},
              dict(_hbm(per_pair * n, dt, pmc_traffic("gather", "gather", "gather_dot_runs")),
                   kernel="dr_gather_dot",
                   per_unit=f"{per_pair} B/pair = 2 rows x {d} x 4 B + 2 ids x 8 B + 4 B out"),
              cpu, backward=backward, patterns=patterns)
        return 0

    if args.workload == "bpr":
        U_n, I_n, d, B, npos = 1_000_000, 1_000_000, 128, 1 << 20, 100
        Ut = (torch.randn(U_n, d, generator=g, device=dev) * 0.1).contiguous()
        It = (torch.randn(I_n, d, generator=g, device=dev) * 0.1).contiguous()
        pos = torch.sort(torch.randint(0, I_n, (U_n, npos), generator=g, device=dev), dim=1).values
        uid = torch.randint(0, U_n, (B,), generator=g, device=dev)
        pid = pos[uid, torch.randint(0, npos, (B,), generator=g, device=dev)]
        nid = torch.randint(0, I_n, (B,), generator=g, device=dev)
        clash = (pos[uid] == nid[:, None]).any(dim=1)  # reject negatives that are positives
        nid[clash] = (nid[clash] + 1) % I_n
        gU, gI = torch.zeros_like(Ut), torch.zeros_like(It)
        state = [(torch.zeros_like(Ut), torch.zeros_like(Ut)), (torch.zeros_like(It), torch.zeros_like(It))]
        step_no = [0]
        ev = {"bpr": [], "adam": []}

        def step():
            step_no[0] += 1
            gU.zero_()
            gI.zero_()
            e = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
            e[0].record()
            ops.bpr_fwd_bwd(Ut, It, uid, pid, nid, 1.0 / B, gU, gI, check=False)
            e[1].record()
            for p_, g_, (m_, v_) in ((Ut, gU, state[0]), (It, gI, state[1])):
                ops.adam_dense(p_, g_, m_, v_, 1e-3, 0.9, 0.999, 1e-8, 0.0, step_no[0])
            e[2].record()
            ev["bpr"].append((e[0], e[1]))
            ev["adam"].append((e[1], e[2]))

        wall, dt = _timed(step, args.steps, args.warmup)
        tb = sum(a.elapsed_time(b) for a, b in ev["bpr"][-args.steps:]) / 1e3 / args.steps
        ta = sum(a.elapsed_time(b) for a, b in ev["adam"][-args.steps:]) / 1e3 / args.steps

        # opt-in row-sparse Adam (torch.optim.SparseAdam semantics, SURVEY §8f
        # rank 3): unique touched rows, dr_adam_rows, gradient rows zeroed by
        # the kernel (no full-table memset)
        gU.zero_()
        gI.zero_()
        lev = {"unique": [], "rows": []}
        nrows = [0, 0]

        def lazy_step():
            step_no[0] += 1
            e = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
            ops.bpr_fwd_bwd(Ut, It, uid, pid, nid, 1.0 / B, gU, gI, check=False)
            e[0].record()
            ru, ri = torch.unique(uid), torch.unique(torch.cat([pid, nid]))
            e[1].record()
            ops.adam_rows(Ut, gU, *state[0], ru, 1e-3, 0.9, 0.999, 1e-8, step_no[0])
            ops.adam_rows(It, gI, *state[1], ri, 1e-3, 0.9, 0.999, 1e-8, step_no[0])
            e[2].record()
            lev["unique"].append((e[0], e[1]))
            lev["rows"].append((e[1], e[2]))
            nrows[0], nrows[1] = ru.numel(), ri.numel()

        lwall, _ = _timed(lazy_step, args.steps, args.warmup)

        # device-side PairWiseDataset sampling: m = 20 (the
        # reference config's train_max_sampled), users in order, ~B triples
        m_s = 20
        n_su = B // (m_s * m_s)
        s_rowptr = torch.arange(0, (U_n + 1) * npos, npos, dtype=torch.int64, device=dev)
        s_items = pos.reshape(-1).to(torch.int32)
        s_users = torch.arange(n_su, dtype=torch.int64, device=dev)
        sw, sdt = _timed(lambda: ops.sample_pairwise(s_users, s_rowptr, s_items, I_n, m_s, 11),
                         args.steps, args.warmup)
        sampler = {"value": n_su * m_s * m_s / sw, "unit": "triples/s", "ms_per_call": sw * 1e3,
                   "users": n_su, "max_sampled": m_s,
                   "kernel": "dr_sample_pairwise (draw + pos-major expand, one host read of "
                             "the error counter per call)",
                   "bytes_per_call": n_su * m_s * m_s * 24}
        # the fused step on the reference's own triple layout (PairWiseDataset:
        # users in order, m*m triples each, positive repeated m times in a
        # row), drawn by the device sampler: the kernel sums the gradient of a
        # run of equal ids in registers and adds it with one row of atomics
        _, _, (mu_, mp_, mn_) = ops.sample_pairwise(s_users, s_rowptr, s_items, I_n, m_s, 11)
        nb = mu_.numel()
        mw, mdt = _timed(lambda: ops.bpr_fwd_bwd(Ut, It, mu_, mp_, mn_, 1.0 / nb, gU, gI,
                                                  check=False), args.steps, args.warmup)

        def runs(x):
            return int((x[1:] != x[:-1]).sum()) + 1

        n_runs = runs(mu_) + runs(mp_) + runs(mn_)
        mxm_bytes = nb * (3 * 8 + 8) + n_runs * d * 4 * 2  # ids + loss/hit + per run: row + adds
        mxm = {"value": nb / mw, "unit": "triples/s", "ms": mdt * 1e3, "triples": nb,
               "layout": f"PairWiseDataset m x m (m = {m_s}, {n_su} users in order)",
               "row_runs": n_runs, "atomic_rows_per_triple": n_runs / nb,
               "hbm_roofline": dict(_hbm(mxm_bytes, mdt, pmc_traffic("bpr", "bpr", "bpr_kernel",
                                                                       group=2)),
                                    per_unit="ids + loss/hit per triple, "
                                    "one row read + one row of atomic adds per run of equal ids")}
        gU.zero_()
        gI.zero_()
        tu = sum(a.elapsed_time(b) for a, b in lev["unique"][-args.steps:]) / 1e3 / args.steps
        tr = sum(a.elapsed_time(b) for a, b in lev["rows"][-args.steps:]) / 1e3 / args.steps
        rows_bytes = (nrows[0] + nrows[1]) * (8 * d * 4 + 8)  # p,m,v rw + g read + g zero + id
        lazy = {"value": B / lwall, "unit": "triples/s", "ms_per_step": lwall * 1e3,
                "unique_ms": tu * 1e3, "adam_rows_ms": tr * 1e3,
                "touched_rows": {"users": nrows[0], "items": nrows[1]},
                "adam_rows_roofline": dict(_hbm(rows_bytes, tr, pmc_traffic("bpr", "bpr", "adam_rows_kernel",
                                                                            per_step=2)),
                                           kernel="dr_adam_rows",
                                           per_unit=f"{8 * d * 4 + 8} B/touched row"),
                "note": "torch.optim.SparseAdam semantics over the touched rows; the reference "
                        "trains with dense Adam, which the headline BPR value above reproduces"}
        per_triple = 3 * d * 4 + 3 * 8 + 4 + 4 + 3 * d * 4  # rows + ids + loss/hit + grad adds
        adam_bytes = 2 * (U_n + I_n) * d * 4 * 3 + (U_n + I_n) * d * 4  # p,m,v rw + g read
        cpu = None
        if want_cpu:
            import oracle

            # one pair_wise_train_loop batch restated in torch (two MF forwards,
            # LogSigmoidDifferenceLoss, backward into dense embedding gradients,
            # Adam over both 1M x 128 tables) on this process's CPU share, at
            # two batch sizes: step time = fixed (Adam + zero_grad over the
            # tables) + per-triple part, extrapolated to the batch of B
            threads, visible, model = host_cpu()
            torch.set_num_threads(threads)
            Uh, Ih = Ut.cpu(), It.cpu()
            bs = (1 << 15, 1 << 16)
            ts = []
            for b_ in bs:
                bt = [tuple(t_[:b_].cpu() for t_ in (uid, pid, nid))]
                t0 = time.perf_counter()
                oracle.reference_bpr_steps(Uh, Ih, bt)
                ts.append(time.perf_counter() - t0)
            per = max((ts[1] - ts[0]) / (bs[1] - bs[0]), 0.0)
            fixed = max(ts[0] - per * bs[0], 0.0)
            cpu_step = fixed + per * B
            cpu = {"value": B / cpu_step, "unit": "triples/s", "cores": threads, "kind": "port",
                   "cpu_model": model, "cpus_visible": visible,
                   "sample": f"oracle.reference_bpr_steps (the reference's BPR batch restated in "
                             f"torch: forwards, loss, backward, Adam.step) at {bs[0]} and {bs[1]} "
                             f"triples on the full tables ({ts[0]:.1f}s, {ts[1]:.1f}s) on "
                             f"{threads} threads, extrapolated to {B}: {cpu_step:.1f}s per step"}
        _line("BPR training triples/sec, 1M x 1M d=128 (BASELINE configs[2])", B / wall,
              "triples/s", args, wall, "f32",
              {"workload": f"one BPR step: dr_bpr_fwd_bwd over {B} triples (uniform user, "
                           f"positive from a {npos}-item/user CSR, uniform negative) + "
                           f"dr_adam_dense over both fp32 tables", "users": U_n, "items": I_n,
               "dim": d, "batch": B},
              dict(_hbm(per_triple * B, tb, pmc_traffic("bpr", "bpr", "bpr_kernel")),
                   kernel="dr_bpr_fwd_bwd",
                   per_unit=f"{per_triple} B/triple"),
              cpu, bpr_ms=tb * 1e3, adam_ms=ta * 1e3, lazy_adam_step=lazy, sampler=sampler,
              bpr_mxm_layout=mxm,
              adam_roofline=_hbm(adam_bytes, ta, pmc_traffic("bpr", "bpr", "adam_kernel", per_step=2)),
              # the fused kernel's real ceiling: fp32 atomics execute at the memory
              # side at ~1.3 TB/s of added bytes chip-wide (MI355X_MICROARCH.md,
              # Global float atomics); it adds 3 rows of d fp32 per triple
              bpr_atomic_roofline={"bound": "fp32 atomics", "added_bytes": 3 * d * 4 * B,
                                   "achieved": 3 * d * 4 * B / tb / 1e9,
                                   "peak": ATOMIC_F32_GBS, "unit": "GB/s",
                                   "frac": 3 * d * 4 * B / tb / 1e9 / ATOMIC_F32_GBS})
        return 0

    raise ValueError(args.workload)


def ml100k(args, dev, g):
    """configs[0]: the reference's evaluation step on an ML-100K-shaped
    synthetic set (943 users, 1682 items, ~90.5k train + 10 test interactions
    per user, MatrixFactorization d=32) through the drop-in API:
    recommendations_score_loop = get_model_recommendations (top-10, frozen =
    train items, fp32 scoring) + cosine ILD (the reference's dense D) +
    P@10 / R@10 / MAP@10 / NDCG@10 + Entropy + PRI. The reference runs this on
    the CPU; here the model lives on the GPU (there is no CPU compute path),
    so the line is the whole step's wall time with host-side datasets, as a
    user of the reference would call it. The CPU baseline is the reference
    loop restated in torch (oracle.reference_loop_topk + oracle.ild_sequential)."""
    import numpy as np

    sys.path.insert(0, os.path.join(ROOT, "diversity-recommendations_amd"))
    from divrec import datasets, losses, metrics, models, train

    nu, ni, d, k = 943, 1682, 32, 10
    rng = np.random.default_rng(100)
    tr, te = [], []
    for u in range(nu):  # ~96 train + 10 test items per user, disjoint
        its = rng.choice(ni, 106, replace=False)
        tr += [(u, int(i)) for i in its[10:]]
        te += [(u, int(i)) for i in its[:10]]
    tr_t, te_t = torch.tensor(tr, dtype=torch.int64), torch.tensor(te, dtype=torch.int64)
    train_ds = datasets.UserItemInteractionsDataset(tr_t, number_of_users=nu, number_of_items=ni)
    test_ds = datasets.UserItemInteractionsDataset(te_t, number_of_users=nu, number_of_items=ni)
    full = datasets.UserItemInteractionsDataset(torch.cat([tr_t, te_t]), number_of_users=nu,
                                                number_of_items=ni)
    rds = datasets.RankingDataset(test_ds, frozen=train_ds)
    mf = models.MatrixFactorization(nu, ni, d)  # N(0, 1) fp32 init, as the reference
    It = mf.item_embeddings.weight.detach().clone()
    En = It / It.norm(dim=1, keepdim=True)
    Dc = 1.0 - En @ En.T  # the reference's dense cosine distance matrix
    mf = mf.to(dev)
    scores = [losses.IntraListDiversityScore(distance_matrix=Dc, reduction="none"),
              metrics.PrecisionAtKScore(), metrics.RecallAtKScore(),
              metrics.MeanAveragePrecisionAtKScore(), metrics.NDCGScore(),
              metrics.EntropyDiversityScore(dataset=full), metrics.PRI(dataset=full)]

    def step():
        return train.recommendations_score_loop(rds, mf, scores, k)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        res = step()
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t0) / args.steps
    cpu = None
    if not args.no_cpu_baseline:
        sys.path.insert(0, ROOT)
        import oracle

        threads, visible, model = host_cpu()
        torch.set_num_threads(threads)
        Uh, Ih = mf.user_embeddings.weight.detach().cpu(), It
        frozen = [tr_t[tr_t[:, 0] == u, 1].tolist() for u in range(nu)]
        t0 = time.perf_counter()
        recs = oracle.reference_loop_topk(Uh, Ih, k, users=list(range(nu)), frozen=frozen)
        oracle.ild_sequential(recs.numpy(), Dc.numpy())
        t = time.perf_counter() - t0
        cpu = {"value": nu / t, "unit": "users/s (top-10 + ILD)", "cores": threads, "kind": "port",
               "cpu_model": model, "cpus_visible": visible,
               "sample": f"oracle.reference_loop_topk (the reference get_model_recommendations loop "
                         f"restated in torch) + oracle.ild_sequential (the combinations-order fp32 "
                         f"sum) over all {nu} users, {t:.2f}s on {threads} threads"}
    names = ["ild", "precision", "recall", "map", "ndcg", "entropy", "pri"]
    vals = {n: float(r.float().mean()) if r.dim() else float(r) for n, r in zip(names, res)}
    rec = {"metric": "config 1 evaluation users/sec: ML-100K-shaped MF d=32 top-10 + ILD + 6 metrics "
                     "(BASELINE configs[0])",
           "value": nu / wall, "unit": "users/s", "n_gpus": 1, "steps": args.steps,
           "warmup": args.warmup, "ms_per_step": wall * 1e3, "higher_is_better": True,
           "scaling": "replicas", "vs_baseline": None, "dtype": "f32",
           "data": "synthetic ML-100K-shaped interactions (seeded), N(0,1) fp32 MF weights",
           "config": {"workload": "recommendations_score_loop: get_model_recommendations top-10 "
                                  "(frozen = train) + cosine ILD + P/R/MAP/NDCG@10 + Entropy + PRI",
                      "users": nu, "items": ni, "dim": d, "k": k},
           "roofline": None, "cpu_baseline": cpu, "metric_values": vals,
           "note": "host-side datasets and metric plumbing dominate at this size; the reference "
                   "config runs on the CPU, this build has no CPU compute path (DESIGN.md §1)"}
    rec.update(provenance())
    print(json.dumps(rec), flush=True)
    return 0


def mmr_pipeline(args):
    """configs[4]: per user the top-C candidates of the 10M-item catalog
    (dr_score_topk, k = C), the MMR re-rank of those C to k_out (dr_mmr_rerank)
    and the cosine ILD of the re-ranked lists (dr_ild_embedding). Users are
    sharded over the ranks (torchrun), the item table is replicated; the only
    collective is the all_reduce of the ILD (sum, count). value = users/s of
    the whole pipeline (max over ranks); the three kernels are timed apart."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    dev_index = 0 if args.same_device else int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(dev_index)
    dev = torch.device("cuda", dev_index)
    if world > 1:
        if args.backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group("gloo")
    U_n, I_n, d = args.users, args.items, args.dim
    C, kout, lam = args.candidates, args.mmr_k, args.mmr_lambda
    u_lo, u_hi = shard_range(U_n, world, rank)
    if rank == 0:
        cold_mfma_probe(dev)  # before any timed work
    users = gen_table(U_n, d, 1, dev)[u_lo:u_hi].contiguous()
    items = gen_table(I_n, d, 2, dev)
    torch.cuda.synchronize()
    ev = []
    out = {}

    def step(record):
        e = [torch.cuda.Event(enable_timing=True) for _ in range(4)] if record else None
        if e:
            e[0].record()
        sc, cand = ops.score_topk(users, items, C)
        if e:
            e[1].record()
        picks = ops.mmr_rerank(cand, sc, items, kout, lam)
        if e:
            e[2].record()
        ild = ops.ild_embedding(picks, items, "cosine", check=False)
        mean = global_mean(ild) if world > 1 else torch.sum(ild, 0) / ild.numel()
        if e:
            e[3].record()
            ev.append(e)
        out.update(cand=cand, sc=sc, picks=picks, mean=mean)

    for _ in range(args.warmup):
        step(False)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step(True)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    ph = [sum(e[j].elapsed_time(e[j + 1]) for e in ev) / 1e3 / args.steps for j in range(3)]
    t = torch.tensor([dt] + ph, dtype=torch.float64, device="cpu" if args.backend == "gloo" else dev)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    step_s = float(t[0]) / args.steps
    topk_s, mmr_s, ild_s = ph  # this rank's kernels (rank 0 prints)
    n_r = u_hi - u_lo
    per_user = C * d * 2 + C * 8 + kout * 4  # candidate rows + (id, score) + picks
    flops = 2.0 * n_r * I_n * d
    cpu = None
    if world == 1 and not args.no_cpu_baseline:
        sys.path.insert(0, ROOT)
        import oracle

        threads, visible, model = host_cpu()
        torch.set_num_threads(threads)
        m = 64
        Eh = items.float().cpu()
        ci, cs = out["cand"][:m].cpu(), out["sc"][:m].cpu()
        oracle.mmr_greedy_torch(ci[:1], cs[:1], Eh, kout, lam)  # warm
        t1 = time.perf_counter()
        oracle.mmr_greedy_torch(ci, cs, Eh, kout, lam)
        tm = time.perf_counter() - t1
        cpu = {"value": m / tm, "unit": "users/s (MMR re-rank only)", "cores": threads,
               "kind": "port", "cpu_model": model, "cpus_visible": visible,
               "sample": f"oracle.mmr_greedy_torch (the eager greedy in torch fp32: one C x C "
                         f"cosine GEMM + {kout} argmax rounds per user) on the first {m} users' "
                         f"real top-{C} lists, {tm:.2f}s on {threads} threads"}
    rec = {"metric": f"MMR pipeline users/sec: top-{C} of {I_n} items -> MMR top-{kout} -> ILD, "
                     f"d={d} (BASELINE configs[4])",
           "value": U_n / step_s, "unit": "users/s", "n_gpus": world, "steps": args.steps,
           "warmup": args.warmup, "ms_per_step": step_s * 1e3, "higher_is_better": True,
           "scaling": "strong", "vs_baseline": None, "dtype": "bf16",
           "data": "synthetic (N(0,1/sqrt(d)) bf16 tables, seeded per 1M-row block)",
           "config": {"workload": f"{U_n} users (sharded {world} ways) x {I_n} items, "
                                  f"top-{C} scan -> MMR lambda={lam} -> {kout} -> cosine ILD, "
                                  f"all_reduce of the ILD (sum, count)",
                      "users": U_n, "items": I_n, "dim": d, "candidates": C, "k": kout,
                      "parallelism": f"user-shard{world}"},
           "topk_ms": topk_s * 1e3, "mmr_ms": mmr_s * 1e3, "ild_ms": ild_s * 1e3,
           "mmr_users_per_s": n_r / mmr_s, "mean_ild": float(out["mean"]),
           "roofline": {"bound": "mfma", "achieved": flops / topk_s / 1e12,
                        "peak": MFMA_BF16_PEAK_TFLOPS, "unit": "TFLOP/s",
                        "frac": flops / topk_s / 1e12 / MFMA_BF16_PEAK_TFLOPS,
                        "traffic": pmc_traffic("mmr", f"mmr_U{U_n}_I{I_n}_d{d}_C{C}_k{kout}",
                                               SCAN_KERNELS, per_step=0) if world == 1 else None,
                        "kernel": f"dr_score_topk k={C} (the step's dominant kernel)"},
           "mmr_roofline": dict(_hbm(per_user * n_r, mmr_s,
                                     pmc_traffic("mmr", f"mmr_U{U_n}_I{I_n}_d{d}_C{C}_k{kout}",
                                                 "mmr_pick_kernel") if world == 1 else None),
                                kernel="dr_mmr_rerank",
                                per_unit=f"{per_user} B/user"),
           "cpu_baseline": cpu}
    if rank == 0:
        with_measured(rec["roofline"], dev, "mfma_bf16_tflops")
        with_measured(rec["mmr_roofline"], dev, "hbm_copy_gbs")
        rec.update(provenance())
        print(json.dumps(rec), flush=True)
    if world > 1:
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main() or 0)
