"""Row-sharded search across GPUs: one process per GPU, one all-gather per batch.

A collection of N rows is cut into contiguous shards: rank p of P owns global
rows [p*ceil(N/P), min(N, (p+1)*ceil(N/P))). Every rank scans its shard for the
whole query batch and produces a local top-k key list per query (64-bit keys
that carry the global row, include/vsearch.h "Result key layout"). The only
exchange is an all-gather of those lists over RCCL / xGMI; each rank then
merges the P lists on its own device. Messages are tiny (P x B x k x 8 bytes),
so the step is latency-bound, not link-bandwidth-bound. Two forms:

* ``gather_merge`` given (the product on GPUs): the engine's own communicator
  (vs_comm_init) runs the all-gather and the merge back to back on the
  search's stream (vs_gather_merge_keys), with no cross-stream wait;
* otherwise ``torch.distributed``'s all-gather (the nccl backend runs it on
  its internal stream, which the caller's stream then waits for) and
  vs_merge_keys; the gloo tests use this form.

The orchestration below is written against two callables so the CPU tests can
drive it with gloo and the oracle; the product passes the HIP engine.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Callable, Optional


def shard_range(n_rows: int, world: int, rank: int) -> tuple[int, int]:
    """Contiguous row shard [lo, hi) of `rank`."""
    if world <= 0 or not (0 <= rank < world):
        raise ValueError("bad world/rank")
    per = -(-n_rows // world)
    lo = min(n_rows, rank * per)
    hi = min(n_rows, lo + per)
    return lo, hi


@dataclass
class ShardedSearch:
    """Distributed top-k over a row-sharded collection.

    local_search(queries, k) -> keys tensor [nq, k] (int64 bit patterns)
    merge(gathered [P, nq, k], k) -> keys tensor [nq, k]
    """

    local_search: Callable
    merge: Callable
    group: Optional[object] = None
    # gather even with one rank (tests: the collective path on a one-GPU box)
    always_gather: bool = False
    # gather_merge(local [nq, k], k) -> keys [nq, k]: the engine's all-gather +
    # merge (engine_gather_merge); replaces the torch all-gather and `merge`
    gather_merge: Optional[Callable] = None
    world_size: int = 1  # ranks of gather_merge's communicator
    # (r05) a torch.cuda.Stream for gather_merge: each batch's all-gather +
    # merge then runs on it, after an event on the search's stream, and the
    # next batch's search does not wait for it (the engine orders exchanges
    # among themselves only: vs_gather_merge_keys). The returned keys are
    # ready once that stream is (a device synchronize covers both).
    exchange_stream: Optional[object] = None
    # (r06) with exchange_stream: the result ring R (>= 2) of the
    # callables. Batch i's local keys sit in a pooled buffer the search stream
    # writes again at batch i + R, while batch i's exchange may still read it
    # on the other stream: the search stream waits on that exchange first.
    exchange_ring: int = 0
    _gather_bufs: Optional[dict] = None  # all-gather outputs, reused per shape
    _ev: Optional[object] = None
    _xdone: Optional[list] = None  # the last exchange_ring exchanges' done events

    def search(self, queries, k: int):
        import torch
        import torch.distributed as dist

        overlap = (self.gather_merge is not None and self.exchange_stream is not None and
                   (self.world_size > 1 or self.always_gather))
        if overlap:
            if self.exchange_ring < 2:
                raise ValueError("exchange_stream needs exchange_ring >= 2 (the callables' result "
                                 "ring): a reused local buffer would be overwritten while its "
                                 "exchange still reads it")
            if self._xdone is None:
                self._xdone = []
            if len(self._xdone) >= self.exchange_ring:
                # the exchange that read the buffer this search is about to reuse
                torch.cuda.current_stream().wait_event(self._xdone.pop(0))
        local = self.local_search(queries, k)
        if self.gather_merge is not None:
            if self.world_size == 1 and not self.always_gather:
                return local
            if self.exchange_stream is None:
                return self.gather_merge(local, k)
            if self._ev is None:
                self._ev = torch.cuda.Event()
            self._ev.record()  # the local keys, on the search's stream
            self.exchange_stream.wait_event(self._ev)
            # the exchange reads `local` on its own stream: keep the caching
            # allocator from handing its memory to the search stream before
            # that read is done (a ring-less caller drops `local` right away)
            local.record_stream(self.exchange_stream)
            with torch.cuda.stream(self.exchange_stream):
                out = self.gather_merge(local, k)
                done = torch.cuda.Event()
                done.record()
            self._xdone.append(done)
            # the keys are written on exchange_stream: wait on it (or on a
            # device synchronize) before reading them
            return out
        if not dist.is_available() or not dist.is_initialized():
            return local
        if dist.get_world_size(self.group) == 1 and not self.always_gather:
            return local
        P = dist.get_world_size(self.group)
        local = local.contiguous()
        # concatenated along dim 0 (the form every backend accepts), viewed as [P, nq, k]
        shape = (P * local.shape[0],) + tuple(local.shape[1:])
        if self._gather_bufs is None:
            self._gather_bufs = {}
        key = (shape, local.dtype, str(local.device))
        flat = self._gather_bufs.get(key)
        if flat is None:
            flat = self._gather_bufs[key] = torch.empty(shape, dtype=local.dtype,
                                                        device=local.device)
        if local.is_cuda and dist.get_backend(self.group) == "gloo":
            # gloo moves host memory only: stage through the host (tests that
            # put several ranks on one GPU, where RCCL refuses duplicate devices)
            host = torch.empty(shape, dtype=local.dtype)
            dist.all_gather_into_tensor(host, local.cpu(), group=self.group)
            flat.copy_(host)
        else:
            dist.all_gather_into_tensor(flat, local, group=self.group)
        return self.merge(flat.view((P,) + tuple(local.shape)), k)


class _Ring:
    """Result tensors per (tag, shape, device): one reused tensor (ring = 1),
    or `ring` tensors used in turn, so the last `ring` results stay intact
    (the benchmark keeps every timed step's answer and checks them after the
    timed region); ring = 0: a fresh tensor per call."""

    def __init__(self, ring: int):
        self.ring = ring
        self.cache = {}

    def get(self, tag, shape, device):
        import torch
        if self.ring <= 0:
            return torch.empty(shape, dtype=torch.int64, device=device)
        key = (tag, tuple(shape), str(device))
        ent = self.cache.get(key)
        if ent is None:
            ent = self.cache[key] = [[], 0]
        bufs, i = ent
        if len(bufs) < self.ring:
            bufs.append(torch.empty(shape, dtype=torch.int64, device=device))
            t = bufs[-1]
        else:
            t = bufs[i % self.ring]
        ent[1] = i + 1
        return t


def engine_callables(engine, collection: str, dim: int, stream_fn: Callable[[], int],
                     reuse: bool = False, ring: int = 0):
    """Binds ShardedSearch to the HIP engine (device tensors, caller's stream).

    With ``reuse`` the result tensors are cached per shape and overwritten by
    the next call (a serving loop that consumes each result before issuing
    the next search); ``ring`` = R > 1 keeps R of them in turn (the last R
    results stay valid); otherwise every call returns fresh tensors."""
    pool = _Ring(ring if ring > 1 else (1 if reuse else 0))

    def buf(tag, shape, device):
        return pool.get(tag, shape, device)

    def local_search(queries, k):
        nq = queries.shape[0]
        out = buf("local", (nq, k), queries.device)
        engine.search_keys(collection, queries.data_ptr(), nq, dim, k, out.data_ptr(), stream_fn())
        return out

    def merge(gathered, k):
        P, nq, kin = gathered.shape
        out = buf("merged", (nq, k), gathered.device)
        engine.merge_keys(gathered.data_ptr(), P, nq, kin, k, out.data_ptr(), stream_fn())
        return out

    return local_search, merge


def engine_gather_merge(engine, stream_fn: Callable[[], int], reuse: bool = False,
                        ring: int = 0):
    """ShardedSearch.gather_merge over the engine's communicator (the caller
    ran engine.comm_init on every rank): vs_gather_merge_keys on the search's
    stream. ``reuse`` / ``ring``: as engine_callables."""
    pool = _Ring(ring if ring > 1 else (1 if reuse else 0))

    def gather_merge(local, k):
        local = local.contiguous()
        nq, kin = local.shape
        out = pool.get("gathered", (nq, k), local.device)
        engine.gather_merge_keys(local.data_ptr(), nq, kin, k, out.data_ptr(), stream_fn())
        return out

    return gather_merge
