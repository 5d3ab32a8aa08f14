"""Ranks as threads of one process (test helper).

``divrec.distributed.thresholded_exchange`` / ``exchange_partials`` take any
object with the members of ``divrec.distributed.Comm`` as their group. This
one runs every rank as a thread of the calling process and exchanges tensor
references through shared slots guarded by a barrier, so the PRODUCT exchange
function runs for all ranks at once — on the CPU with a checker top-k, or on
one GPU with the HIP kernels at full configs[3] size (every rank's kernels on
cuda:0's stream, which orders them in enqueue order).
"""
from __future__ import annotations

import threading
from typing import Callable, List

import torch


class ThreadHub:
    def __init__(self, world: int, timeout: float = 600.0):
        self.world = world
        self.barrier = threading.Barrier(world, timeout=timeout)
        self.slots: List = [None] * world

    def comm(self, rank: int) -> "ThreadComm":
        return ThreadComm(self, rank)

    def run(self, fn: Callable[["ThreadComm"], object]) -> list:
        """fn(comm) on every rank, one thread each; returns the results in rank
        order, re-raising the first failure (the barrier is broken so that no
        other rank waits for the failed one)."""
        out, errs = [None] * self.world, []

        def main(r):
            try:
                out[r] = fn(self.comm(r))
            except BaseException as e:  # noqa: BLE001 - reported below
                errs.append((r, e))
                self.barrier.abort()

        ts = [threading.Thread(target=main, args=(r,)) for r in range(self.world)]
        for t in ts:
            t.start()
        for t in ts:
            t.join()
        if errs:
            real = [e for e in errs if not isinstance(e[1], threading.BrokenBarrierError)]
            r, e = (real or errs)[0]
            raise RuntimeError(f"rank {r} failed: {e!r}") from e
        return out


class ThreadComm:
    """divrec.distributed.Comm's members over a ThreadHub."""

    def __init__(self, hub: ThreadHub, rank: int):
        self.hub, self.world, self.rank = hub, hub.world, rank

    def _exchange(self, obj):
        self.hub.slots[self.rank] = obj
        self.hub.barrier.wait()
        got = list(self.hub.slots)
        self.hub.barrier.wait()  # nobody overwrites a slot before every rank read it
        return got

    def all_gather_rows(self, x: torch.Tensor, sizes) -> torch.Tensor:
        assert x.shape[0] == sizes[self.rank]
        got = self._exchange(x)
        return torch.cat([g[: sizes[p]].to(x.device) for p, g in enumerate(got)])

    def all_to_all_rows(self, x: torch.Tensor, in_splits, out_splits) -> torch.Tensor:
        got = self._exchange((x, list(in_splits)))
        parts = []
        for p, (xp, sp) in enumerate(got):
            off = sum(sp[: self.rank])
            assert sp[self.rank] == out_splits[p]
            parts.append(xp[off: off + sp[self.rank]].to(x.device))
        return torch.cat(parts)

    def all_reduce_sum(self, t: torch.Tensor) -> torch.Tensor:
        got = self._exchange(t)
        out = got[0].to(t.device).clone()
        for g in got[1:]:
            out += g.to(t.device)
        return out
