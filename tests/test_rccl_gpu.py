"""The RCCL transport of the multi-GPU path, run once on the GPU box.

Every other multi-rank test exchanges through gloo (host copies) or thread
ranks; the 8-GPU run uses the "nccl" backend (RCCL over xGMI on ROCm) with
device tensors, which no test executed before. Here a spawned child process
initialises a world-size-1 "nccl" process group BEFORE any other GPU call in
that process (as bench.py's ranks do) and runs the product exchange through
``divrec.distributed.Comm(None)`` on device tensors:

  * ``global_thresholds``  - all_gather of the sample sizes and of the strided
    sample rows, dr_sample_thresholds, all_gather of the two tiers;
  * ``thresholded_exchange`` - the first-tier shard scan, exchange_partials
    (all_to_all_single with splits), dr_topk_merge, the failure counts
    (all_gather) and BOTH rescans: a user group whose first tier fails and
    whose safe tier rescues it, and a group that fails both tiers (-inf);
  * ``global_mean`` - the all_reduce of (sum, count) of config 5's ILD.

The lists must equal one dr_score_topk call over the whole catalog and the
exact float64 top-k (integer tables: exact scores) - the reference's
get_model_recommendations (/root/reference/divrec/train/utils.py:53-77) with
the tie order fixed to (score desc, item id asc).
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

from divrec import ops

pytestmark = pytest.mark.gpu

NU, NI, D, K = 3 * 1024 + 77, 300_011, 64, 100
N_TIER2, N_INF = 12, 40  # hot rows seen by each planted group (ks1 = 9 <= 12 < ks = 17 < 40)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _tables(stride):
    """Integer tables. Users [0, 1024): non-negative on the first 32 columns,
    zero on the rest - they see the N_TIER2 rows hot on the first half; users
    [1024, 2048): the same on the last 32 columns - they see the N_INF rows hot
    on the second half; the rest mixed-sign. Hot rows sit at sample positions
    (multiples of the guess stride), so they dominate the sample's top ranks."""
    rng = np.random.default_rng(55)
    U = rng.integers(-3, 4, size=(NU, D)).astype(np.float32)
    U[:1024, :32] = rng.integers(0, 4, size=(1024, 32))
    U[:1024, 32:] = 0
    U[1024:2048, 32:] = rng.integers(0, 4, size=(1024, 32))
    U[1024:2048, :32] = 0
    I = rng.integers(-3, 4, size=(NI, D)).astype(np.float32)
    I[np.arange(N_TIER2) * stride, :32] = 3.0
    I[(np.arange(N_INF) + 100) * stride, 32:] = 3.0
    return U, I


def _child(port, stride, q):
    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    try:
        # the process group first: no GPU call before it in this process
        dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
        from divrec import distributed

        backend = dist.get_backend()
        comm = distributed.Comm(None)
        U, I = _tables(stride)
        users = torch.from_numpy(U).to("cuda").to(torch.bfloat16)
        items = torch.from_numpy(I).to("cuda").to(torch.bfloat16)
        thr = distributed.global_thresholds(users, items, 0, NI, NI, K, comm)
        s, i = distributed.thresholded_exchange(users, items, 0, NI, NI, K, comm, thr=thr)
        ild = ops.ild_embedding(i, items)
        mean = distributed.global_mean(ild, comm)
        torch.cuda.synchronize()
        q.put(dict(backend=backend, thr=thr.cpu().numpy(), s=s.cpu().numpy(), i=i.cpu().numpy(),
                   tiers=distributed.LAST_TIER_FAILURES, mean=float(mean.cpu()),
                   ild=ild.cpu().numpy(), err=None))
        dist.destroy_process_group()
    except Exception as e:  # report, so the parent fails with the message instead of a timeout
        q.put(dict(err=repr(e)))
        raise


def _exact(U, I, k):
    Ud = torch.from_numpy(U).to("cuda").double()
    Id = torch.from_numpy(I).to("cuda").double()
    outi, outs = [], []
    for b in range(0, Ud.shape[0], 256):
        v, o = torch.sort(Ud[b:b + 256] @ Id.T, dim=1, descending=True, stable=True)
        outi.append(o[:, :k].cpu())
        outs.append(v[:, :k].cpu())
    return torch.cat(outi).numpy(), torch.cat(outs).numpy()


def test_rccl_exchange_world1_matches_one_device():
    from divrec.distributed import guess_ranks, sample_stride

    stride = sample_stride(NI, K)
    ks1, ks = guess_ranks(K, (NI // stride) // 32 * 32 / NI)
    assert ks1 <= N_TIER2 < ks < N_INF  # the planted groups fail the tiers they are meant to
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_child, args=(_free_port(), stride, q))
    p.start()
    got = q.get(timeout=300)
    p.join(timeout=60)
    assert got["err"] is None, got["err"]
    assert p.exitcode == 0
    assert got["backend"] == "nccl"
    t1, t2 = got["tiers"]
    assert t1 >= 2048 and 1024 <= t2 < t1  # both rescans ran; the safe tier rescued a group
    U, I = _tables(stride)
    one_s, one_i = ops.score_topk(torch.from_numpy(U).to("cuda").to(torch.bfloat16),
                                  torch.from_numpy(I).to("cuda").to(torch.bfloat16), K)
    ref_i, ref_s = _exact(U, I, K)
    assert np.array_equal(one_i.cpu().numpy().astype(np.int64), ref_i)
    assert np.array_equal(got["i"], one_i.cpu().numpy())
    assert np.array_equal(got["s"], one_s.cpu().numpy())
    assert got["thr"].shape == (2, NU) and (got["thr"][0] >= got["thr"][1]).all()
    ild = got["ild"].astype(np.float64)
    assert abs(got["mean"] - ild.mean()) <= 1e-6 * abs(ild.mean())
