"""Query-tile sharding across GPUs.

One process per GPU; every rank holds the full index (replicated: each rank upserts the
same batches into its own dk_ctx); query records are split into contiguous tiles, one per
rank, so a query's candidates, scores and decisions are computed on exactly one rank.  The
only exchange is the result gather: all-gather the per-rank match counts, then gather
every rank's match list (first / candidate / prob / kind) to rank 0, which owns the
MatchListener replay.  With the "nccl" backend (RCCL on ROCm) the tensors are device
tensors and travel over xGMI; the same code runs on CPU tensors with "gloo" (tests).
"""
from __future__ import annotations

import numpy as np


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
