"""CPU: the opt-in bulk writer of the H2 link database (dukehip.jdbc_links, the Python mirror
of integration/java/.../GpuJdbcLinkDatabase.java) against the per-callback stream it
replaces -- LinkDatabaseMatchListener driving JDBCLinkDatabase one statement per link
(oracle/linkdb_ref.py: LinkDBListener over SqlLinkDB) -- over the same table layout, on
sqlite3.  PARITY UNPINNED against Duke's JDBCLinkDatabase table (absent jar; recalled)."""
import sqlite3

import numpy as np
import pytest

import linkdb_ref as R
from dukehip import jdbc_links as J
from test_linkdb import random_batches


def table(conn):
    return conn.execute("select id1, id2, kind, status, perhaps, timestamp from links "
                        "order by id1, id2").fetchall()


def per_callback(batches):
    conn = sqlite3.connect(":memory:")
    db = R.SqlLinkDB(conn, J.CREATE)
    for t, (qs, entries) in enumerate(batches):
        ts = 1000 + 10 * t
        L = R.LinkDBListener(db, lambda ts=ts: ts)
        L.batch_ready(len(qs))
        for i, (q, lst) in enumerate(zip(qs, entries)):
            if not lst:
                L.no_match_for((i, q))
            for c, p, kind in lst:
                (L.matches if kind == 1 else L.matches_perhaps)((i, q), c, p)
        L.batch_done()
        db.commit()
    return conn, db.statements


def bulk(batches):
    conn = sqlite3.connect(":memory:")
    w = J.JdbcBulkLinkWriter(conn)
    stmts = 0
    for t, (qs, entries) in enumerate(batches):
        first = np.zeros(len(qs) + 1, np.uint64)
        first[1:] = np.cumsum([len(x) for x in entries])
        flat = [e for lst in entries for e in lst]
        w.apply(qs, first, [c for c, _, _ in flat], [p for _, p, _ in flat], [k for _, _, k in flat],
                1000 + 10 * t)
        stmts += w.statements
    return conn, stmts


@pytest.mark.parametrize("seed", [1, 2, 3, 4, 5])
def test_bulk_writer_equals_per_callback_stream(seed):
    batches = random_batches(seed, nids=80, nbatches=15)
    a, n_cb = per_callback(batches)
    b, n_bulk = bulk(batches)
    want = table(a)
    assert table(b) == want
    assert any(r[3] == J.RETRACTED for r in want) and any(r[3] == J.INFERRED for r in want)
    assert n_bulk == 6 * len(batches) < n_cb


def test_retraction_by_a_later_record_of_the_batch():
    """Record b retracts the link a asserted earlier in the same batch when b's own list
    does not hold it (the per-record order the bulk writer replays)."""
    batches = [(["a", "b"], [[("b", 0.95, 1)], [("c", 0.8, 2)]])]
    a, _ = per_callback(batches)
    b, _ = bulk(batches)
    assert table(a) == table(b)
    rows = {(r[0], r[1]): r for r in table(b)}
    assert rows[("a", "b")][3] == J.RETRACTED and rows[("b", "c")][3] == J.INFERRED
