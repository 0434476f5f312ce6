"""Query-tile sharding across GPUs.

One process per GPU; every rank holds the full index (replicated: each rank upserts the
same batches into its own dk_ctx); query records are split into contiguous tiles, one per
rank, so a query's candidates, scores and decisions are computed on exactly one rank.  The
only exchange is the result gather: all-gather the per-rank match counts, then gather
every rank's match list (first / candidate / prob / kind) to rank 0, which owns the
MatchListener replay.  Two ways to move the lists:

* ``SharedRegionGather`` (default): every rank's dk_match copies its tile's list over its own
  GPU's PCIe link into its slice of ONE node-wide shared host mapping (dk_set_result_region,
  overlapped with scoring as on one GPU); the exchange is an all-gather of the per-rank
  counts, after which rank 0 reads the whole node list in place.  The listener runs on the
  host, so this is the shortest path: no list crosses xGMI and then funnels through GPU 0's
  single host link.
* ``gather_matches``: device-resident lists gathered to GPU 0 over RCCL/xGMI, then moved to
  the host by rank 0.  With the "nccl" backend (RCCL on ROCm) the tensors are device
  tensors; the same code runs on CPU tensors with "gloo" (tests).
"""
from __future__ import annotations

import mmap
import os
import tempfile

import numpy as np

from . import _abi as A

PAGE = mmap.PAGESIZE


def tile(n, rank, world):
    """Contiguous query tile [q0, q1) of `rank`."""
    return n * rank // world, n * (rank + 1) // world


def max_tile(n, world):
    return max(tile(n, r, world)[1] - tile(n, r, world)[0] for r in range(world))


def gather_matches(dist, torch, device, nq, n, scored, fill, world, rank, nq_max):
    """Gather every rank's match list to rank 0.

    fill(first, cand, prob, kind) writes this rank's entries into the given tensors
    (first: nq+1 int64, then n entries each).  Returns (per-rank lists, total scored) on
    rank 0, (None, total scored) elsewhere."""
    cnt = torch.tensor([n, scored, nq], dtype=torch.int64, device=device)
    allc = [torch.zeros_like(cnt) for _ in range(world)]
    dist.all_gather(allc, cnt)
    mx = max(1, int(max(int(c[0]) for c in allc)))
    first = torch.zeros(nq_max + 1, dtype=torch.int64, device=device)
    cand = torch.zeros(mx, dtype=torch.int32, device=device)
    prob = torch.zeros(mx, dtype=torch.float64, device=device)
    kind = torch.zeros(mx, dtype=torch.uint8, device=device)
    fill(first, cand, prob, kind)
    out = [] if rank == 0 else None
    for t in (first, cand, prob, kind):
        lst = [torch.empty_like(t) for _ in range(world)] if rank == 0 else None
        dist.gather(t, lst, dst=0)
        if rank == 0:
            out.append(lst)
    total = int(sum(int(c[1]) for c in allc))
    if rank != 0:
        return None, total
    ranks = []
    for r in range(world):
        nr, nqr = int(allc[r][0]), int(allc[r][2])
        ranks.append({"first": out[0][r][: nqr + 1].cpu().numpy(),
                      "candidate": out[1][r][:nr].cpu().numpy().astype(np.uint32),
                      "prob": out[2][r][:nr].cpu().numpy(),
                      "kind": out[3][r][:nr].cpu().numpy()})
    return ranks, total


def concat_ranks(ranks):
    """Node-level match list in query order from the per-rank tiles (a concatenation,
    since tiles are contiguous in query order)."""
    firsts, base = [], 0
    for i, r in enumerate(ranks):
        f = r["first"].astype(np.int64) + base
        firsts.append(f if i == len(ranks) - 1 else f[:-1])
        base += len(r["candidate"])
    return {"first": np.concatenate(firsts) if firsts else np.zeros(1, np.int64),
            "candidate": np.concatenate([r["candidate"] for r in ranks]),
            "prob": np.concatenate([r["prob"] for r in ranks]),
            "kind": np.concatenate([r["kind"] for r in ranks])}


class RegionUnavailable(RuntimeError):
    """Raised on every rank when some rank cannot use the shared mapping."""


class SharedRegionGather:
    """Node-wide shared host mapping with one result region per rank (SURVEY §8e exchange).

    Collective: every rank constructs it with the same (nq_max, capacity).  Rank 0 creates
    the file under /dev/shm, every rank maps it and hands its page-aligned slice to its
    engine (dk_set_result_region registers it with HIP); the file is unlinked as soon as all
    ranks hold the mapping, so nothing is left behind.  After :meth:`exchange` of a step,
    rank 0 reads every rank's list in place (:meth:`rank_lists`).  A rank must not start its
    next dk_match while rank 0 still reads the previous lists (callers barrier between
    replay and the next batch)."""

    def __init__(self, dist, torch, device, engine, nq_max, capacity, world, rank,
                 shm_dir="/dev/shm"):
        self.dist, self.torch, self.device = dist, torch, device
        self.world, self.rank, self.nq_max = world, rank, int(nq_max)
        self.slice_bytes = -(-A.region_bytes(nq_max, capacity) // PAGE) * PAGE
        total = self.slice_bytes * world
        name = [None]
        if rank == 0:
            d = shm_dir if os.path.isdir(shm_dir) else None
            if d is not None:
                st = os.statvfs(d)   # a small /dev/shm (container default) would SIGBUS
                if st.f_bavail * st.f_frsize < total + (64 << 20):
                    d = None         # page-cache-backed file in the default temp dir
            fd, path = tempfile.mkstemp(prefix="dukehip_results_", dir=d)
            os.ftruncate(fd, total)
            os.close(fd)
            name = [path]
        dist.broadcast_object_list(name, src=0)
        self.path = name[0]
        with open(self.path, "r+b") as f:
            self.map = mmap.mmap(f.fileno(), total)
        dist.barrier()
        if rank == 0:
            os.unlink(self.path)
        self.slices = [memoryview(self.map)[r * self.slice_bytes:(r + 1) * self.slice_bytes]
                       for r in range(world)]
        self.engine = engine
        ok = 1
        if engine is not None:
            try:
                engine.set_result_region(self.slices[rank], self.nq_max)
            except A.DukeHipError:
                ok = 0
        flag = torch.tensor([ok], dtype=torch.int64, device=device)
        dist.all_reduce(flag, op=dist.ReduceOp.MIN)   # every rank takes the same path
        if int(flag.item()) == 0:
            self.close()
            raise RegionUnavailable("a rank could not register its result region")
        self.counts = None

    def exchange(self, nq, n, scored):
        """All-gather of (entries, pairs scored, queries) per rank: after it every rank's
        list is complete in the mapping.  Returns the node's pairs scored."""
        torch = self.torch
        cnt = torch.tensor([n, scored, nq], dtype=torch.int64, device=self.device)
        allc = [torch.zeros_like(cnt) for _ in range(self.world)]
        self.dist.all_gather(allc, cnt)
        self.counts = [tuple(int(v) for v in c.cpu()) for c in allc]
        return sum(c[1] for c in self.counts)

    def rank_lists(self):
        """Rank 0: every rank's {first, candidate, prob, kind} views, in rank (= query) order
        (concat_ranks joins them)."""
        return [A.region_views(self.slices[r], self.nq_max, nqr, nr)
                for r, (nr, _, nqr) in enumerate(self.counts)]

    def close(self):
        if self.engine is not None and self.engine.ctx:
            self.engine.set_result_region(None, 0)
        self.engine = None
        for mv in self.slices:
            mv.release()
        self.slices = []
        try:
            self.map.close()
        except BufferError:  # a caller still holds views of the lists; GC unmaps
            pass
