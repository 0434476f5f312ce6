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


# ---------------------------------------------------------------------------------------
# cost-weighted tiles, the pack-once shared batch and the overflow-safe region exchange;
# a gather of REAL match lists (the CPU oracle's, per cost tile) against one full run
# ---------------------------------------------------------------------------------------
def test_cost_bounds_balance():
    rng = np.random.default_rng(5)
    counts = (rng.zipf(1.3, 5000) * 10).clip(0, 100000)
    for w in (1, 2, 3, 8):
        b = dshard.cost_bounds(counts, w)
        assert b[0] == 0 and b[-1] == len(counts) and all(b[i] <= b[i + 1] for i in range(w))
        cost = np.asarray(counts, float) + dshard.QUERY_COST
        per = [cost[b[r]:b[r + 1]].sum() for r in range(w)]
        assert max(per) - min(per) <= 2 * cost.max() + 1e-9
    assert dshard.cost_bounds([], 3) == [0, 0, 0, 0]


def _batch_worker(rank, world, port, out):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    vals = [["abc", None, "ł\U0001F600", ""], ["x", "y", "z", "w"]]
    cols = [A.Column.from_strings(v) for v in vals]
    arrays = None
    if rank == 0:
        arrays = dshard.columns_to_arrays("p", cols)
        arrays["ident"] = np.arange(4, dtype=np.uint64)
    sb = dshard.SharedBatch(dist, rank, arrays)
    got = dshard.arrays_to_columns("p", sb.arrays)
    ok = len(got) == 2 and np.array_equal(sb.arrays["ident"], np.arange(4))
    for g, c in zip(got, cols):
        ok = ok and np.array_equal(g.offsets, c.offsets) and np.array_equal(g.units, c.units)
        ok = ok and ((g.present is None and c.present is None) or np.array_equal(g.present, c.present))
    out.put((rank, bool(ok)))
    sb.close()
    dist.barrier()
    dist.destroy_process_group()


def _overflow_worker(rank, world, port, out):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    g = dshard.SharedRegionGather(dist, torch, torch.device("cpu"), None, 10, 100, world, rank)
    raised = False
    try:
        g.exchange(10, 0 if rank else 5, 7, ok=(rank == 0))   # rank 1's list did not fit
    except dshard.RegionOverflow:
        raised = True
    g.resize(None, 1000)
    total = g.exchange(10, 5, 7)
    out.put((rank, raised and total == 14 and g.capacity == 1000))
    g.close()
    dist.barrier()
    dist.destroy_process_group()


def _oracle_case():
    import oracle as O
    from dukehip import synth
    p = synth.persons(1200, 400, seed=17)
    props = [{"comparator": A.CMP_JAROWINKLER, "low": 0.1, "high": 0.95},
             {"comparator": A.CMP_LEVENSHTEIN, "low": 0.2, "high": 0.8},
             {"comparator": A.CMP_LEVENSHTEIN, "low": 0.1, "high": 0.85}]
    keys = synth.keys_config2(p)
    ot = O.OracleTable(props, [p["name"], p["address"], p["dob"]], keys=keys,
                       threshold=0.9, maybe=0.7)
    n = len(p["name"])
    # candidate counts per query (its bucket sizes), as dk_candidate_counts reports them
    sizes = []
    for k in keys:
        from collections import Counter
        cnt = Counter(k)
        sizes.append([cnt[v] for v in k])
    counts = np.sum(np.array(sizes), axis=0)
    return ot, n, counts


def _oracle_worker(rank, world, port, out):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    ot, n, counts = _oracle_case()
    q0, q1 = dshard.cost_tile(counts, rank, world)
    r = ot.match(np.arange(q0, q1, dtype=np.uint32))
    qidx = r["query"].astype(np.int64) - q0
    my_first = np.searchsorted(qidx, np.arange(q1 - q0 + 1), side="left").astype(np.int64)
    m = len(r["candidate"])

    def fill(f, c, p, k):
        f[: len(my_first)] = torch.from_numpy(my_first)
        c[:m] = torch.from_numpy(r["candidate"].astype(np.int32))
        p[:m] = torch.from_numpy(r["prob"])
        k[:m] = torch.from_numpy(r["kind"])

    nq_max = max(b - a for a, b in (dshard.cost_tile(counts, x, world) for x in range(world)))
    ranks, total = dshard.gather_matches(dist, torch, torch.device("cpu"), q1 - q0, m,
                                         r["pairs_scored"], fill, world, rank, nq_max)
    if rank == 0:
        full = ot.match()
        got = dshard.concat_ranks(ranks)
        fq = np.repeat(np.arange(n), np.diff(got["first"]))
        ok = (np.array_equal(fq, full["query"]) and np.array_equal(got["candidate"], full["candidate"])
              and np.array_equal(got["prob"], full["prob"]) and np.array_equal(got["kind"], full["kind"])
              and total == full["pairs_scored"] and len(full["candidate"]) > 0)
        out.put(bool(ok))
    dist.barrier()
    dist.destroy_process_group()


def _spawn(target, world=2):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=target, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(180)
    assert all(p.exitcode == 0 for p in procs)
    return q


def test_shared_batch_world2_gloo():
    q = _spawn(_batch_worker)
    got = sorted(q.get(timeout=5) for _ in range(2))
    assert got == [(0, True), (1, True)]


def test_region_overflow_is_collective_world2_gloo():
    q = _spawn(_overflow_worker)
    got = sorted(q.get(timeout=5) for _ in range(2))
    assert got == [(0, True), (1, True)]


def test_oracle_lists_cost_tiles_world2_gloo():
    q = _spawn(_oracle_worker)
    assert q.get(timeout=5) is True
