"""GPU parity of the incremental blocking index: sorted base + sorted delta.

After a full sort, later upserts re-sort only the rows added since (the delta segments) and
retire superseded base rows in place; `dk_match` must return exactly what a full re-sort
returns -- Duke's candidate order (key function, then (group, row) in the bucket), the
delete-by-ID visibility of IncrementalLuceneDatabase.java:516-517 and the deleted-flag
exclusion of :478 -- for contiguous batches (the symmetric dedup schedule), strided query
sets (the direct schedule), linkage, and transient (httptransform) rows on top of a delta.
Checked against the oracle and against DK_DELTA=0 (every index change fully re-sorted).

Oracle: oracle/duke_oracle.c, PARITY UNPINNED against Duke 1.2 itself.
"""
import numpy as np
import pytest

import oracle as O
import dukehip as dh
from test_gpu_parity import schema_of, assert_same, persons_case

pytestmark = pytest.mark.gpu


def alive_of(ident, upto):
    alive = np.ones(upto, np.uint8)
    last = {}
    for r in range(upto):
        i = int(ident[r])
        if i in last:
            alive[last[i]] = 0
        last[i] = r
    return alive


def upsert(eng, vals, keys, ident, a, b, deleted=None, group=None, transient=False):
    eng.upsert(b - a, ident[a:b], [dh.Column.from_strings(v[a:b]) for v in vals],
               deleted=None if deleted is None else deleted[a:b],
               group=None if group is None else group[a:b],
               key_columns=[dh.Column.from_strings(k[a:b]) for k in keys], transient=transient)


def batch_plan(n, rng, nb):
    cuts = np.sort(rng.choice(np.arange(50, n - 20), nb - 1, replace=False))
    edges = [0] + [int(c) for c in cuts] + [n]
    return list(zip(edges[:-1], edges[1:]))


@pytest.mark.parametrize("mode", ["dedup", "linkage"])
@pytest.mark.parametrize("delta_min", ["64", "100000"])
def test_delta_index_equals_oracle(mode, delta_min, monkeypatch):
    """A stream of upserts (new rows, IDs re-posted from base and delta rows, deleted
    flags): each match sees exactly the oracle's index.  delta_min 64 forces periodic full
    re-sorts between delta builds; 100000 keeps every later batch in the delta."""
    monkeypatch.setenv("DK_DELTA_MIN", delta_min)
    p, props, vals, keys = persons_case(1400, 600, 11 if mode == "dedup" else 12)
    n = len(vals[0])
    rng = np.random.default_rng(5)
    deleted = (rng.random(n) < 0.04).astype(np.uint8)
    ident = np.arange(n, dtype=np.uint64)
    plan = batch_plan(n, rng, 9)
    # re-post IDs: every later batch supersedes some rows of earlier batches (base and delta)
    for a, b in plan[1:]:
        k = max(1, (b - a) // 8)
        dst = rng.choice(np.arange(a, b), k, replace=False)
        ident[dst] = ident[rng.choice(np.arange(0, a), k, replace=False)]
    group = None
    if mode == "linkage":
        group = np.where(rng.random(n) < 0.5, 1, 2).astype(np.uint8)
    eng = dh.GpuEngine(schema_of(props, 0.9, 0.7, mode, len(keys)))
    eng.reset_profile()
    for a, b in plan:
        upsert(eng, vals, keys, ident, a, b, deleted=deleted, group=group)
        ot = O.OracleTable(props, [v[:b] for v in vals], keys=[k[:b] for k in keys],
                           ident=ident[:b], deleted=deleted[:b], alive=alive_of(ident, b),
                           group=None if group is None else group[:b], threshold=0.9, maybe=0.7,
                           mode=mode)
        for q in (np.arange(a, b, dtype=np.uint32),          # the batch (symmetric schedule)
                  np.arange(0, b, dtype=np.uint32),          # base + delta rows, contiguous
                  np.arange(1, b, 3, dtype=np.uint32)):      # strided (direct schedule)
            res = eng.match(q)
            assert_same(res, ot.match(q))
            res.close()
    prof = eng.profile()
    eng.close()
    assert prof["delta_builds"] > 0, prof
    if delta_min == "64":
        assert prof["full_builds"] > 1, prof
    else:   # full sorts only when a longer value changes the replica layout
        assert prof["delta_builds"] >= 5 and prof["full_builds"] <= 3, prof


def test_delta_equals_full_resort(monkeypatch):
    """Bit-identical match lists with and without the delta (DK_DELTA=0 re-sorts fully)."""
    p, props, vals, keys = persons_case(1200, 500, 21)
    n = len(vals[0])
    ident = np.arange(n, dtype=np.uint64)
    ident[1500:1560] = ident[100:160]
    plan = [(0, 900), (900, 1300), (1300, 1500), (1500, n)]
    out = {}
    for flag in ("1", "0"):
        monkeypatch.setenv("DK_DELTA", flag)
        eng = dh.GpuEngine(schema_of(props, 0.9, 0.7, "dedup", len(keys)))
        lists = []
        for a, b in plan:
            upsert(eng, vals, keys, ident, a, b)
            for q in (np.arange(a, b, dtype=np.uint32), np.arange(0, b, 2, dtype=np.uint32)):
                res = eng.match(q)
                lists.append((res.first.copy(), res.candidate.copy(), res.prob.copy(), res.kind.copy(),
                              res.pairs_scored))
                res.close()
        out[flag] = (lists, eng.profile())
        eng.close()
    assert out["1"][1]["delta_builds"] >= 1   # a longer value may force a full sort
    assert out["0"][1]["delta_builds"] == 0
    for x, y in zip(out["1"][0], out["0"][0]):
        for u, v in zip(x[:4], y[:4]):
            assert np.array_equal(u, v)
        assert x[4] == y[4]


def test_transient_rows_on_a_delta():
    """httptransform batches (query-only rows) over an index with a delta, then more
    indexing: the transient rows are never candidates and vanish with dk_drop_transient."""
    p, props, vals, keys = persons_case(900, 400, 31)
    n = len(vals[0])
    ident = np.arange(n, dtype=np.uint64)
    eng = dh.GpuEngine(schema_of(props, 0.9, 0.7, "dedup", len(keys)))
    upsert(eng, vals, keys, ident, 0, 800)
    eng.match(np.arange(0, 800, dtype=np.uint32)).close()      # full sort
    upsert(eng, vals, keys, ident, 800, 1000)                   # delta
    # transient rows 1000..1100 (query-only): matched against rows < 1000
    upsert(eng, vals, keys, ident, 1000, 1100, transient=True)
    ot = O.OracleTable(props, [v[:1100] for v in vals], keys=[k[:1100] for k in keys],
                       ident=ident[:1100], alive=np.r_[np.ones(1000, np.uint8), np.zeros(100, np.uint8)],
                       threshold=0.9, maybe=0.7)
    q = np.arange(1000, 1100, dtype=np.uint32)
    res = eng.match(q)
    assert_same(res, ot.match(q))
    res.close()
    eng.drop_transient()
    upsert(eng, vals, keys, ident, 1000, n)                      # the same rows, indexed now
    ot = O.OracleTable(props, vals, keys=list(keys), ident=ident, alive=np.ones(n, np.uint8),
                       threshold=0.9, maybe=0.7)
    for q in (np.arange(1000, n, dtype=np.uint32), np.arange(0, n, 5, dtype=np.uint32)):
        res = eng.match(q)
        assert_same(res, ot.match(q))
        res.close()
    prof = eng.profile()
    eng.close()
    assert prof["delta_builds"] >= 2, prof


def test_delta_grows_replica_layout():
    """A delta row longer than every base value changes the replica layout (units per
    value): the next build is a full sort, and the results stay exact."""
    p, props, vals, keys = persons_case(500, 200, 41)
    n = len(vals[0])
    vals = [list(v) for v in vals]
    vals[1][650] = ("12 a much longer street name " * 3)[:60]
    assert max(len(v or "") for v in vals[1][:600]) <= 56   # replica rows 56 -> 60
    ident = np.arange(n, dtype=np.uint64)
    eng = dh.GpuEngine(schema_of(props, 0.9, 0.7, "dedup", len(keys)))
    upsert(eng, vals, keys, ident, 0, 600)
    eng.match(np.arange(600, dtype=np.uint32)).close()
    eng.reset_profile()
    upsert(eng, vals, keys, ident, 600, n)
    ot = O.OracleTable(props, vals, keys=list(keys), ident=ident, alive=np.ones(n, np.uint8),
                       threshold=0.9, maybe=0.7)
    q = np.arange(600, n, dtype=np.uint32)
    res = eng.match(q)
    assert_same(res, ot.match(q))
    res.close()
    prof = eng.profile()
    eng.close()
    assert prof["full_builds"] == 1 and prof["delta_builds"] == 0, prof
