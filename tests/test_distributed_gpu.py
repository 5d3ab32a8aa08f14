"""The default multi-GPU path on the HIP kernels.

bench.py --gpus N runs pure item sharding with global sample thresholds:
divrec.distributed.sharded_score_topk(global_thr=True) -> global_thresholds
(all_gather of a strided sample of the whole catalog, dr_score_topk over it)
-> dr_score_topk_seeded on each shard -> exchange_partials (all_to_all) ->
dr_topk_merge -> verification with the exact fallback. The driver's 8-GPU node
runs it over RCCL; on this one-GPU pool the same code runs with 2 and 4 ranks
that all sit on cuda:0 and exchange through gloo (as bench.py --backend gloo
--same-device does), so every kernel and every collective step of the path
runs for real. The merged lists must equal one dr_score_topk call over the
whole catalog and the exact top-k (integer tables: exact scores), the
reference's get_model_recommendations (/root/reference/divrec/train/utils.py:53-77)
with its tie order fixed to (score desc, item id asc).

Ranks are spawned processes (a fresh HIP context each); at most 4 + the
pytest process use the GPU, well inside the box's process limit.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

from divrec import ops

pytestmark = pytest.mark.gpu


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _tables(nu, ni, d, seed, hot_stride):
    rng = np.random.default_rng(seed)
    half = nu // 2
    U = np.concatenate([rng.integers(0, 4, size=(half, d)),            # non-negative group
                        rng.integers(-3, 4, size=(nu - half, d))]).astype(np.float32)
    I = rng.integers(-3, 4, size=(ni, d)).astype(np.float32)
    if hot_stride:  # 40 hot rows at global sample positions: the sample rank of the guess
        I[np.arange(40) * hot_stride] = 3.0  # is 17 < 40 < k, so the group's guess fails
    return U, I


def _rank_main(rank, world, port, nu, ni, d, k, seed, hot_stride, bounds, q):
    import torch.distributed as dist

    from divrec import distributed
    from divrec.distributed import sharded_score_topk

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    try:
        torch.cuda.set_device(0)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        U, I = _tables(nu, ni, d, seed, hot_stride)
        lo, hi = bounds[rank], bounds[rank + 1]
        users = torch.from_numpy(U).to("cuda").to(torch.bfloat16)
        shard = torch.from_numpy(I[lo:hi]).to("cuda").to(torch.bfloat16)
        (s, i), (ulo, uhi) = sharded_score_topk(users, shard, lo, k, n_items=ni, global_thr=True)
        torch.cuda.synchronize()
        q.put((rank, ulo, uhi, s.cpu().numpy(), i.cpu().numpy(),
               None, distributed.LAST_FALLBACK_USERS))
        dist.destroy_process_group()
    except Exception as e:  # report, so the parent fails with the message instead of a timeout
        q.put((rank, 0, 0, None, None, repr(e), 0))
        raise


def _exact(U, I, k):
    """Exact top-k on the device in float64 (integer tables)."""
    Ud = torch.from_numpy(U).to("cuda").double()
    Id = torch.from_numpy(I).to("cuda").double()
    outi, outs = [], []
    for b in range(0, Ud.shape[0], 256):
        S = Ud[b:b + 256] @ Id.T
        v, o = torch.sort(S, dim=1, descending=True, stable=True)
        outi.append(o[:, :k].cpu())
        outs.append(v[:, :k].cpu())
    return torch.cat(outi).numpy(), torch.cat(outs).numpy()


@pytest.mark.parametrize("world,d,hot,uneven", [(2, 128, False, False), (4, 64, True, True),
                                                (4, 128, True, False), (2, 64, False, True)])
def test_item_sharded_global_thresholds_on_hip(world, d, hot, uneven):
    nu, ni, k, seed = 2 * 2048 + 123, 300_011, 100, 7 * world + d
    from divrec.distributed import sample_stride, shard_range

    stride = sample_stride(ni, k)
    if uneven:  # contiguous but unequal shards (the path accepts any split)
        cuts = np.sort(np.random.default_rng(seed).choice(np.arange(1000, ni - 1000), world - 1,
                                                          replace=False))
        bounds = [0] + [int(c) for c in cuts] + [ni]
    else:
        bounds = [shard_range(ni, world, r)[0] for r in range(world)] + [ni]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank_main,
                         args=(r, world, port, nu, ni, d, k, seed, stride if hot else 0, bounds, q))
             for r in range(world)]
    for p in procs:
        p.start()
    got = [q.get(timeout=240) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
    errs = [g[5] for g in got if g[5]]
    assert not errs, errs
    assert all(p.exitcode == 0 for p in procs)
    fallback = {g[6] for g in got}
    assert len(fallback) == 1  # every rank saw the same all_gathered count
    if hot:  # the non-negative group's guess failed: the exact fallback ran
        assert fallback.pop() >= nu // 2
    U, I = _tables(nu, ni, d, seed, stride if hot else 0)
    one_s, one_i = ops.score_topk(torch.from_numpy(U).to("cuda").to(torch.bfloat16),
                                  torch.from_numpy(I).to("cuda").to(torch.bfloat16), k)
    one_s, one_i = one_s.cpu().numpy(), one_i.cpu().numpy()
    ref_i, ref_s = _exact(U, I, k)
    assert np.array_equal(one_i.astype(np.int64), ref_i)
    seen = np.zeros(nu, dtype=int)
    for rank, ulo, uhi, s, i, _, _ in got:
        assert (ulo, uhi) == shard_range(nu, world, rank)
        assert np.array_equal(i, one_i[ulo:uhi]), f"rank {rank}: lists differ from one device"
        assert np.array_equal(s, one_s[ulo:uhi])
        assert np.array_equal(s, ref_s[ulo:uhi].astype(np.float32))
        seen[ulo:uhi] += 1
    assert (seen == 1).all()
