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
    """Contiguous query tile [q0, q1) of `rank` (equal query counts)."""
    return n * rank // world, n * (rank + 1) // world


def max_tile(n, world):
    return max(tile(n, r, world)[1] - tile(n, r, world)[0] for r in range(world))


# A query's fixed cost beside its candidates, in candidate units: one wave's worth of
# padding on average plus its per-wave tables (the score kernel pads a query to 64 slots)
QUERY_COST = 32


def cost_bounds(counts, world):
    """Tile boundaries b[0..world] balancing the estimated cost -- the query's candidate
    count (dk_candidate_counts) plus QUERY_COST -- over contiguous tiles (tiles
    weighted by their blocks' sizes; Zipfian surname blocks make equal query counts
    unbalanced).  Every rank computes the same boundaries from its replica of the index."""
    c = np.asarray(counts, dtype=np.float64) + QUERY_COST
    pre = np.concatenate([[0.0], np.cumsum(c)])
    total = pre[-1]
    b = [0]
    for r in range(1, world):
        b.append(int(np.searchsorted(pre, total * r / world, side="left")))
    b.append(len(c))
    for r in range(1, world + 1):       # monotone (empty tiles allowed)
        b[r] = max(b[r], b[r - 1])
    return b


def cost_tile(counts, rank, world):
    b = cost_bounds(counts, world)
    return b[rank], b[rank + 1]


class SharedBatch:
    """One batch packed once into SoA columns and shared by every rank of the node (SURVEY
    §8e: the index is replicated, so every rank upserts the same records).  Rank 0 packs
    and writes the arrays into one file under /dev/shm; the others map it read-only and
    wrap zero-copy views, instead of re-packing the strings per rank.  Collective."""

    def __init__(self, dist, rank, arrays=None, shm_dir="/dev/shm"):
        """arrays (rank 0): {name: numpy array}; the other ranks pass None."""
        import json
        meta = [None]
        if rank == 0:
            d = shm_dir if os.path.isdir(shm_dir) else None
            layout, off = {}, 0
            for k, a in arrays.items():
                a = np.ascontiguousarray(a)
                off = -(-off // 64) * 64
                layout[k] = (off, str(a.dtype), list(a.shape))
                off += a.nbytes
            fd, path = tempfile.mkstemp(prefix="dukehip_batch_", dir=d)
            os.ftruncate(fd, max(off, 1))
            with os.fdopen(fd, "r+b") as f:
                mm = mmap.mmap(f.fileno(), max(off, 1))
                for k, a in arrays.items():
                    o, dt, shp = layout[k]
                    a = np.ascontiguousarray(a)
                    mm[o:o + a.nbytes] = a.tobytes()
                mm.flush()
            meta = [json.dumps({"path": path, "size": max(off, 1), "layout": layout})]
        dist.broadcast_object_list(meta, src=0)
        m = json.loads(meta[0])
        with open(m["path"], "rb") as f:
            self.map = mmap.mmap(f.fileno(), m["size"], access=mmap.ACCESS_READ)
        dist.barrier()
        if rank == 0:
            os.unlink(m["path"])
        self.arrays = {}
        for k, (o, dt, shp) in m["layout"].items():
            n = int(np.prod(shp)) if shp else 1
            self.arrays[k] = np.frombuffer(self.map, dtype=np.dtype(dt), count=n, offset=o).reshape(shp)

    def close(self):
        self.arrays = {}
        try:
            self.map.close()
        except BufferError:
            pass


def columns_to_arrays(prefix, columns):
    """A list of Column -> flat {name: array} (for SharedBatch)."""
    out = {}
    for i, c in enumerate(columns):
        out[f"{prefix}{i}.offsets"] = c.offsets
        out[f"{prefix}{i}.units"] = c.units
        if c.present is not None:
            out[f"{prefix}{i}.present"] = c.present
    return out


def arrays_to_columns(prefix, arrays):
    cols, i = [], 0
    while f"{prefix}{i}.offsets" in arrays:
        cols.append(A.Column(arrays[f"{prefix}{i}.offsets"], arrays[f"{prefix}{i}.units"],
                             arrays.get(f"{prefix}{i}.present")))
        i += 1
    return cols


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


class RegionOverflow(RuntimeError):
    """Raised on every rank when some rank's match list did not fit its region."""


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
        self.shm_dir = shm_dir
        self._setup(engine, capacity)

    def _setup(self, engine, capacity):
        dist, torch, device, world, rank = self.dist, self.torch, self.device, self.world, self.rank
        shm_dir, nq_max = self.shm_dir, self.nq_max
        self.capacity = int(capacity)
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

    def exchange(self, nq, n, scored, ok=True):
        """All-gather of (entries, pairs scored, queries, ok) per rank: after it every
        rank's list is complete in the mapping.  Returns the node's pairs scored.  A rank
        whose dk_match failed with DK_E_NOMEM (its list did not fit its region) still calls
        this with ok=False, so no rank blocks: every rank then raises RegionOverflow."""
        torch = self.torch
        cnt = torch.tensor([n, scored, nq, 1 if ok else 0], dtype=torch.int64, device=self.device)
        allc = [torch.zeros_like(cnt) for _ in range(self.world)]
        self.dist.all_gather(allc, cnt)
        got = [tuple(int(v) for v in c.cpu()) for c in allc]
        if not all(c[3] for c in got):
            raise RegionOverflow("a rank's match list did not fit its result region")
        self.counts = [c[:3] for c in got]
        return sum(c[1] for c in self.counts)

    def match(self, engine, queries):
        """dk_match into this rank's region + exchange, collective and overflow-safe: when a
        list does not fit, every rank learns it in the exchange, the regions are re-made
        (collectively) with room for the largest list, and the match runs again."""
        while True:
            try:
                res, ok = engine.match(queries), True
            except A.DukeHipError as e:
                if e.code != A.DK_E_NOMEM:
                    raise
                res, ok = None, False
            try:
                total = self.exchange(len(queries), res.n if ok else 0,
                                      res.pairs_scored if ok else 0, ok)
                return res, total
            except RegionOverflow:
                if res is not None:
                    res.close()
                probe = engine.match(queries, on_device=True)
                need = self.torch.tensor([probe.n], dtype=self.torch.int64, device=self.device)
                probe.close()
                self.dist.all_reduce(need, op=self.dist.ReduceOp.MAX)
                self.resize(engine, int(need.item() * 1.25) + 4096)

    def resize(self, engine, capacity):
        """Collective: a new shared mapping with `capacity` entries per rank."""
        self.close()
        self._setup(engine, capacity)

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
        self.counts = None
