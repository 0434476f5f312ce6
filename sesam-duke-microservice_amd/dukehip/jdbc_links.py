"""Bulk writes of a batch's links into a SQL link table: the Python mirror of
integration/java/.../GpuJdbcLinkDatabase.java (the H2 `link-database-type`, App.java:567-570,
597-602), opt-in.

The reference's H2 path is Duke's JDBCLinkDatabase driven per callback by
LinkDatabaseMatchListener (BaseLinkDatabaseMatchListener.java:53-109): for each query record,
its stored INFERRED links it did not produce again are retracted (status RETRACTED, the
batch's time) and its new links asserted -- one SQL statement per link, the database read
once per record (getAllLinksFor).  This writer gives the table the same final state with one
SELECT of the batch's records' INFERRED links, the per-record rules replayed in memory (in
batch order, so a later record sees what an earlier one wrote), and one executemany of the
final row per touched link, in ONE transaction per batch (deduplicate).

Transactions: the writer holds a connection of its own beside the link database's (Duke's
JDBCLinkDatabase, `primary` here), through which the routes keep writing outside a batch --
the deleted records' link retractions (App.java:994-999) go through it before deduplicate
runs.  Opening the listener window (set_listener_window(True), GpuProcessor before
batchReady) commits the primary connection's pending writes first, so this connection's
SELECT sees them and its upserts never wait on their row locks; inside the window the
primary connection writes nothing (the listener's writes are dropped).

A stored ASSERTED link (a manual one) is never overwritten by the batch's INFERRED links or
retractions: [Duke 1.2, recalled] JDBCLinkDatabase.assertLink keeps a row whose status is
ASSERTED when the new link's is not (Link.overrides), and the listener retracts only
INFERRED links.

PARITY UNPINNED against Duke's table: JDBCLinkDatabase is in the absent Duke 1.2 jar, so the
layout below (table `links`, columns id1 / id2 / kind / status / perhaps / timestamp, key
(id1, id2), assertLink = update-or-insert of that row unless the stored one is ASSERTED) is
recalled.  Tested against the per-callback stream over the same layout
(tests/test_jdbc_links.py, oracle/linkdb_ref.py).  The statements are SQLite's (`insert or
ignore`, `create temp table`, `on conflict ... do update`): this module drives sqlite3
connections; the Java writer uses H2's `merge ... key` forms for the same steps.
"""
from __future__ import annotations

from . import _abi as A

# [Duke 1.2 JDBCLinkDatabase, recalled]
TABLE = "links"
CREATE = (f"create table if not exists {TABLE} (id1 varchar(200) not null, id2 varchar(200) not null, "
          "kind int not null, status int not null, perhaps float, timestamp bigint not null, "
          "primary key (id1, id2))")
INFERRED, RETRACTED, ASSERTED = 1, 2, 3   # the sink's codes (dukehip.links); Java: Duke's ids
SAME, MAYBE = 1, 2


def _u16(s):
    return s.encode("utf-16-be", "surrogatepass")   # String.compareTo order


def link_key(a, b):
    """Link(id1, id2): the smaller ID (UTF-16 code units) first."""
    return (a, b) if _u16(a) <= _u16(b) else (b, a)


class JdbcBulkLinkWriter:
    def __init__(self, conn, primary=None, upsert=None):
        """conn: this writer's sqlite3 connection to the link table (created if missing).
        primary: the link database's own connection, whose pending writes the listener window
        commits when it opens.  upsert: the update-or-insert statement."""
        self.conn, self.primary = conn, primary
        conn.execute(CREATE)
        conn.commit()
        self.upsert = upsert or (f"insert into {TABLE} (id1, id2, kind, status, perhaps, timestamp) "
                                 "values (?, ?, ?, ?, ?, ?) on conflict (id1, id2) do update set "
                                 "kind = excluded.kind, status = excluded.status, "
                                 "perhaps = excluded.perhaps, timestamp = excluded.timestamp")
        self.statements = 0     # SQL statements of the last batch (bulk: a handful)
        self.window = False

    def set_listener_window(self, open_):
        """GpuProcessor around a batch (GpuJdbcLinkDatabase.setListenerWindow): opening it
        commits the link database's pending writes (the routes' retractions)."""
        if open_ and self.primary is not None:
            self.primary.commit()
        self.window = open_

    def _links_of(self, ids):
        """The stored links touching any of `ids`: {key: [kind, status, perhaps, ts]}."""
        cur = self.conn.cursor()
        cur.execute("create temp table if not exists dk_batch_ids (id varchar(200) primary key)")
        cur.execute("delete from dk_batch_ids")
        cur.executemany("insert or ignore into dk_batch_ids values (?)", [(i,) for i in ids])
        cur.execute(f"select id1, id2, kind, status, perhaps, timestamp from {TABLE} where "
                    "id1 in (select id from dk_batch_ids) or id2 in (select id from dk_batch_ids)")
        out = {(a, b): [k, s, p, t] for a, b, k, s, p, t in cur.fetchall()}
        self.statements = 4
        return out

    def apply(self, query_ids, first, candidate_ids, prob, kind, timestamp):
        """One batch's match list: query record i (ID query_ids[i]) has entries
        first[i] .. first[i+1]-1 (candidate ID, probability, SAME / MAYBE), in batch order."""
        state = self._links_of(set(query_ids))
        by_id = {}
        for k in state:
            by_id.setdefault(k[0], set()).add(k)
            by_id.setdefault(k[1], set()).add(k)
        final = {}
        for i, q in enumerate(query_ids):
            cur = {}
            for e in range(int(first[i]), int(first[i + 1])):
                k = link_key(q, candidate_ids[e])
                cur[k] = [int(kind[e]), INFERRED, float(prob[e]), int(timestamp)]
            # the record's stored INFERRED links it did not produce again: retracted
            for k in list(by_id.get(q, ())):
                row = state[k]
                if k in cur or row[1] != INFERRED:
                    continue
                row = [row[0], RETRACTED, row[2], int(timestamp)]
                state[k] = row
                final[k] = row
            for k, row in cur.items():
                if k in state and state[k][1] == ASSERTED:
                    continue    # a manual link stays (Link.overrides)
                state[k] = row
                final[k] = row
                by_id.setdefault(k[0], set()).add(k)
                by_id.setdefault(k[1], set()).add(k)
        cur = self.conn.cursor()
        cur.executemany(self.upsert, [(a, b, r[0], r[1], r[2], r[3]) for (a, b), r in final.items()])
        self.conn.commit()
        self.statements += 2
        return len(final)

    def apply_result(self, res, query_ids, row_ids, timestamp):
        """A MatchResult (dukehip.processor) of queries with IDs query_ids; row_ids[row] is
        the ID of candidate row `row`."""
        cand = [row_ids[int(r)] for r in res.candidate]
        return self.apply(query_ids, res.first, cand, res.prob,
                          [SAME if int(k) == A.KIND_MATCH else MAYBE for k in res.kind], timestamp)
