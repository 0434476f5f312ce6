"""GPU, full size: configs[2]'s north-star path on a replica whose key-word rows pass 4 GiB.

VERDICT r4 item 4.  The 10M x 10M run's layout -- one QGram property's key-word rows larger
than a 32-bit buffer offset, read by k_score_gq through its head / tail buffer resources --
with no environment override: 18M records (synth.linkage_columns: column-wise numpy, the set
tiled 9 times with the year moved per copy; every 4000th ADDRESS up to 65 units, so the rows
hold 15-16 key words), indexed on the device, 3,000 group-2 queries spread over the whole
replica matched, and checked bit-exactly against the C oracle (oracle/duke_oracle.c, PARITY
UNPINNED against Duke itself) run on the records sharing a key with them (the candidate sets
are exactly those rows, in the same relative order).
"""
import numpy as np
import pytest

import oracle as O
import dukehip as dh
from dukehip import _abi as A
from dukehip import synth
from test_gpu_parity import schema_of

pytestmark = pytest.mark.gpu

QG, NUM = A.CMP_QGRAM, A.CMP_NUMERIC
# bench.py's configs[2] schema
PROPS = [{"comparator": QG, "low": 0.1, "high": 0.9, "q": 2, "formula": A.QGRAM_DICE},
         {"comparator": QG, "low": 0.05, "high": 0.8, "q": 2, "formula": A.QGRAM_JACCARD},
         {"comparator": NUM, "low": 0.2, "high": 0.6, "min_ratio": 0.9996},
         {"comparator": NUM, "low": 0.4, "high": 0.75, "min_ratio": 0.9}]
NAMES = ["NAME", "ADDRESS", "BIRTHYEAR", "ZIP"]


def _subset(col, rows):
    """(offsets, UTF-16 units) of rows `rows` of a Latin-1 Column."""
    o = col.offsets.astype(np.int64)
    lens = o[rows + 1] - o[rows]
    no = np.zeros(len(rows) + 1, np.int64)
    np.cumsum(lens, out=no[1:])
    src = np.repeat(o[rows] - no[:-1], lens) + np.arange(int(no[-1]))
    return no.astype(np.uint32), col.units[src].astype(np.uint16)


def test_config2_full_size_replica_past_4gib():
    cols, kcols, group, k1, k2 = synth.linkage_columns(9_000_000, copies=9, long_every=4000)
    n = len(group)
    ident = np.arange(n, dtype=np.uint64)
    eng = dh.GpuEngine(schema_of(PROPS, 0.9, 0.7, "linkage", 2))
    try:
        eng.upsert(n, ident, [cols[k] for k in NAMES], group=group, key_columns=kcols)
        rng = np.random.default_rng(5)
        q = np.sort(rng.choice(np.nonzero(group == 2)[0], 3000, replace=False)).astype(np.uint32)
        res = eng.match(q)
        prof = eng.profile()
    finally:
        eng.close()
    # the layout: the largest QGram property's key-word rows past a 32-bit offset
    print("replica positions", prof["replica_positions"], "largest key-word rows", prof["gram_row_bytes"], "B")
    assert prof["gram_row_bytes"] > (1 << 32), prof
    assert prof["replica_positions"] >= 2 * n, prof
    # the oracle on the rows sharing a key with a query (global row order kept)
    rows = np.union1d(q.astype(np.int64), np.nonzero(np.isin(k1, k1[q]) | np.isin(k2, k2[q]))[0])
    ot = O.OracleTable.from_packed(PROPS, [_subset(cols[k], rows) for k in NAMES],
                                   [_subset(c, rows) for c in kcols], ident=rows.astype(np.uint64),
                                   group=group[rows], threshold=0.9, maybe=0.7, mode="linkage")
    ref = ot.match(np.searchsorted(rows, q).astype(np.uint32), nthreads=16)
    assert res.pairs_scored == ref["pairs_scored"] and res.pairs_scored > 1_000_000
    assert np.array_equal(res.query, rows[ref["query"]])
    assert np.array_equal(res.candidate, rows[ref["candidate"]])
    assert np.array_equal(res.kind, ref["kind"])
    assert np.array_equal(res.prob, ref["prob"])
    assert res.n > 300   # the perturbed copies among the queries (~0.28 per query)
