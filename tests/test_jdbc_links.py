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


def per_callback(batches, conn=None):
    conn = conn or sqlite3.connect(":memory:")
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


def bulk(batches, conn=None):
    conn = conn or sqlite3.connect(":memory:")
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


def test_asserted_links_are_kept():
    """a manual ASSERTED link is neither retracted nor overwritten by the batch's
    INFERRED links (JDBCLinkDatabase.assertLink keeps it, recalled Link.overrides)."""
    batches = [(["a", "b", "c"], [[("b", 0.95, 1)], [("c", 0.8, 2)], []]),
               (["a", "c"], [[("c", 0.9, 1)], [("b", 0.75, 2)]])]
    seed = [("a", "b", 1, R.ASSERTED, 1.0, 5), ("a", "c", 2, R.ASSERTED, 0.5, 5)]

    def run(fn):
        conn = sqlite3.connect(":memory:")
        conn.execute(J.CREATE)
        conn.executemany("insert into links values (?, ?, ?, ?, ?, ?)", seed)
        conn.commit()
        return fn(batches, conn)

    a, _ = run(per_callback)
    b, _ = run(bulk)
    assert table(a) == table(b)
    rows = {(r[0], r[1]): r for r in table(b)}
    assert rows[("a", "b")][3] == R.ASSERTED and rows[("a", "c")][3] == R.ASSERTED
    assert rows[("b", "c")][3] == J.INFERRED


@pytest.mark.parametrize("window_commits", [True, False])
def test_retraction_between_batches_two_connections(tmp_path, window_commits):
    """the route retracts a deleted record's links through the link
    database's own connection (App.java:994-999) before deduplicate; the bulk writer runs on
    a second connection (WAL).  Opening the listener window commits those writes, so the
    writer's SELECT sees them and its upsert of a link the next batch re-asserts does not
    wait on their row locks; the final table equals the one-connection per-callback stream.
    Without that commit the second connection cannot write (or reads stale rows)."""
    b1 = (["a", "b", "c"], [[("b", 0.95, 1), ("c", 0.8, 2)], [("c", 0.85, 2)], []])
    b2 = (["a", "c"], [[("b", 0.93, 1)], [("a", 0.82, 2)]])

    # one connection, stock Duke's per-callback stream
    ref = sqlite3.connect(":memory:")
    db = R.SqlLinkDB(ref, J.CREATE)
    for t, step in enumerate((b1, None, b2)):
        if step is None:
            db.retract("b", 1005)       # record "b" deleted between the batches
            continue
        qs, entries = step
        L = R.LinkDBListener(db, lambda ts=1000 + 10 * t: ts)
        L.batch_ready(len(qs))
        for i, (q, lst) in enumerate(zip(qs, entries)):
            if not lst:
                L.no_match_for((i, q))
            for c, p, kind in lst:
                (L.matches if kind == 1 else L.matches_perhaps)((i, q), c, p)
        L.batch_done()
        db.commit()

    path = str(tmp_path / "links.db")
    primary = sqlite3.connect(path, timeout=0.2)
    primary.execute("pragma journal_mode=wal")
    sdb = R.SqlLinkDB(primary, J.CREATE)
    primary.commit()
    w = J.JdbcBulkLinkWriter(sqlite3.connect(path, timeout=0.2), primary=primary if window_commits else None)

    def batch(t, qs, entries):
        w.set_listener_window(True)
        first = np.zeros(len(qs) + 1, np.uint64)
        first[1:] = np.cumsum([len(x) for x in entries])
        flat = [e for lst in entries for e in lst]
        w.apply(qs, first, [c for c, _, _ in flat], [p for _, p, _ in flat], [k for _, _, k in flat],
                1000 + 10 * t)
        w.set_listener_window(False)

    batch(0, *b1)
    sdb.retract("b", 1005)              # uncommitted on the primary connection
    if window_commits:
        batch(2, *b2)
        primary.commit()
        assert table(w.conn) == table(ref)
        assert {(r[0], r[1]): r[3] for r in table(ref)}[("a", "b")] == J.INFERRED  # re-asserted
    else:
        with pytest.raises(sqlite3.OperationalError):   # the retraction's write lock
            batch(2, *b2)
