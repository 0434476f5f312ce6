"""CPU, world_size 2 (gloo): the query-tile sharding and the rank-0 match gather that
bench.py runs over RCCL.  Each rank fabricates the match list of its tile from a
deterministic rule; rank 0 must reassemble exactly the single-rank list."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from dukehip import _abi as A
from dukehip import dist as dshard

N = 1003


def full_list(n):
    """The node-level list: query i has (i % 4) entries, candidate = 7*i + e."""
    first = [0]
    cand, prob, kind = [], [], []
    for i in range(n):
        for e in range(i % 4):
            cand.append(7 * i + e)
            prob.append(0.5 + 1e-3 * e + 1e-9 * i)
            kind.append(1 + (e % 2))
        first.append(len(cand))
    return (np.array(first, np.int64), np.array(cand, np.uint32), np.array(prob, np.float64),
            np.array(kind, np.uint8))


def _worker(rank, world, port, out):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    q0, q1 = dshard.tile(N, rank, world)
    first, cand, prob, kind = full_list(N)
    a, b = int(first[q0]), int(first[q1])
    my_first = first[q0:q1 + 1] - a

    def fill(f, c, p, k):
        f[: len(my_first)] = torch.from_numpy(my_first)
        c[: b - a] = torch.from_numpy(cand[a:b].astype(np.int32))
        p[: b - a] = torch.from_numpy(prob[a:b])
        k[: b - a] = torch.from_numpy(kind[a:b])

    ranks, total = dshard.gather_matches(dist, torch, torch.device("cpu"), q1 - q0, b - a,
                                         10 * (q1 - q0), fill, world, rank,
                                         dshard.max_tile(N, world))
    if rank == 0:
        got = dshard.concat_ranks(ranks)
        ok = (np.array_equal(got["first"], first) and np.array_equal(got["candidate"], cand)
              and np.array_equal(got["prob"], prob) and np.array_equal(got["kind"], kind)
              and total == 10 * N)
        out.put(bool(ok))
    dist.barrier()
    dist.destroy_process_group()


def _region_worker(rank, world, port, out):
    """SharedRegionGather: each rank writes its tile into its slice of the shared mapping
    (what dk_match does through dk_set_result_region); rank 0 reads the node list in place."""
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    q0, q1 = dshard.tile(N, rank, world)
    first, cand, prob, kind = full_list(N)
    a, b = int(first[q0]), int(first[q1])
    nq_max = dshard.max_tile(N, world)
    g = dshard.SharedRegionGather(dist, torch, torch.device("cpu"), None, nq_max, 800, world, rank)
    ok = True
    for step in range(2):  # the mapping is reused across batches
        v = A.region_views(g.slices[rank], nq_max, q1 - q0, b - a)
        v["first"][:] = (first[q0:q1 + 1] - a).astype(np.uint64)
        v["candidate"][:] = cand[a:b]
        v["prob"][:] = prob[a:b] + step
        v["kind"][:] = kind[a:b]
        total = g.exchange(q1 - q0, b - a, 10 * (q1 - q0))
        if rank == 0:
            got = dshard.concat_ranks(g.rank_lists())
            ok = ok and (np.array_equal(got["first"], first) and np.array_equal(got["candidate"], cand)
                         and np.array_equal(got["prob"], prob + step)
                         and np.array_equal(got["kind"], kind) and total == 10 * N)
        dist.barrier()
    if rank == 0:
        out.put(bool(ok and not os.path.exists(g.path)))
    g.close()
    dist.barrier()
    dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_tiles_partition_queries():
    for n in (0, 1, 7, 1000, 1003):
        for w in (1, 2, 3, 8):
            spans = [dshard.tile(n, r, w) for r in range(w)]
            assert spans[0][0] == 0 and spans[-1][1] == n
            assert all(spans[i][1] == spans[i + 1][0] for i in range(w - 1))


@pytest.mark.parametrize("world", [2])
def test_gather_world2_gloo(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q))
             for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(120)
    assert all(p.exitcode == 0 for p in procs)
    assert q.get(timeout=5) is True



def test_shared_region_gather_world2_gloo():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_region_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(120)
    assert all(p.exitcode == 0 for p in procs)
    assert q.get(timeout=5) is True
