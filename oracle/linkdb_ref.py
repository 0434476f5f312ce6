"""Per-callback restatement of the link sink (TEST INFRASTRUCTURE: the checker of
dk_linkdb_apply / dukehip.links.LinkDatabase; never imported by the product).

* ``SinceAwareLinkDB``   <- SinceAwareInMemoryLinkDatabase.java:12-41 (assertLink's identical-
  link skip within 1e-6, getChangesSince) over [Duke 1.2, recalled] InMemoryLinkDatabase (one
  link per ID pair, assertLink replaces it).
* ``SqlLinkDB``          <- [Duke 1.2, recalled] JDBCLinkDatabase over a SQL table (the H2
  link-database-type, App.java:567-570, 597-602): getAllLinksFor = one SELECT, assertLink =
  one update-or-insert of the (id1, id2) row -- the per-callback stream the bulk writer
  (dukehip.jdbc_links) is checked against; table layout recalled (unpinned).
* ``LinkDBListener``     <- [Duke 1.2, recalled] LinkDatabaseMatchListener as
  BaseLinkDatabaseMatchListener.java:53-109 drives it: per record, its matches /
  matchesPerhaps collected; when the next record starts (or noMatchFor / batchDone) the
  record's stored INFERRED links it did not produce again are retracted and its new links
  asserted.  Link(id1, id2) keeps the smaller ID (String.compareTo, UTF-16 code units) first.
PARITY UNPINNED: Duke 1.2's LinkDatabaseMatchListener / Link / InMemoryLinkDatabase sources are
absent from /root/reference; the reference's own SinceAware rules are followed exactly.
"""
from __future__ import annotations

INFERRED, RETRACTED, ASSERTED = 1, 2, 3
SAME, MAYBE = 1, 2


def _u16(s):
    return s.encode("utf-16-be", "surrogatepass")   # big-endian bytes order = code-unit order


class Link:
    __slots__ = ("id1", "id2", "status", "kind", "confidence", "timestamp")

    def __init__(self, a, b, status, kind, confidence, timestamp):
        if _u16(a) > _u16(b):
            a, b = b, a
        self.id1, self.id2 = a, b
        self.status, self.kind = status, kind
        self.confidence, self.timestamp = confidence, timestamp

    def key(self):
        return (self.id1, self.id2)

    def copy(self):
        return Link(self.id1, self.id2, self.status, self.kind, self.confidence, self.timestamp)


class SinceAwareLinkDB:
    def __init__(self):
        self.links = {}    # (id1, id2) -> Link
        self.order = {}    # (id1, id2) -> assertion sequence number
        self.seq = 0

    def all_links_for(self, rid):
        return [l for k, l in self.links.items() if rid in k]

    def assert_link(self, link):                    # SinceAwareInMemoryLinkDatabase.java:12-30
        old = self.links.get(link.key())
        if old is not None and link.status == old.status and link.kind == old.kind:
            if abs(link.confidence - old.confidence) < 0.000001:
                return False
        self.links[link.key()] = link               # InMemoryLinkDatabase.assertLink
        self.order[link.key()] = self.seq
        self.seq += 1
        return True

    def retract(self, rid, timestamp, other=None):  # App.java:994-999 (deleted records)
        # getAllLinksFor(id), link.retract() [recalled: status RETRACTED, timestamp now] on the
        # stored Link itself, then assertLink (which then finds it unchanged)
        for l in self.all_links_for(rid):
            if other is not None and other not in l.key():
                continue
            l.status, l.timestamp = RETRACTED, timestamp
            self.order[l.key()] = self.seq
            self.seq += 1

    def changes_since(self, since):                 # :32-40
        out = [l for l in self.links.values() if l.timestamp > since]
        return sorted(out, key=lambda l: (l.timestamp, self.order[l.key()]))


class SqlLinkDB:
    """One SQL statement per call, on a DB-API (qmark) connection; the table layout of
    dukehip.jdbc_links (created if missing)."""

    def __init__(self, conn, create, table="links"):
        self.conn, self.table = conn, table
        conn.execute(create)
        self.statements = 0

    def all_links_for(self, rid):
        self.statements += 1
        rows = self.conn.execute(f"select id1, id2, kind, status, perhaps, timestamp from {self.table} "
                                 "where id1 = ? or id2 = ?", (rid, rid)).fetchall()
        return [Link(a, b, s, k, p, t) for a, b, k, s, p, t in rows]

    def assert_link(self, link):
        # [Duke 1.2, recalled] JDBCLinkDatabase.assertLink reads the stored row first and
        # keeps it when it is ASSERTED and the new link is not (Link.overrides: asserted
        # information overrides inferred)
        self.statements += 1
        old = self.conn.execute(f"select status from {self.table} where id1 = ? and id2 = ?",
                                (link.id1, link.id2)).fetchone()
        if old is not None and old[0] == ASSERTED and link.status != ASSERTED:
            return False
        self.conn.execute(f"insert into {self.table} (id1, id2, kind, status, perhaps, timestamp) "
                          "values (?, ?, ?, ?, ?, ?) on conflict (id1, id2) do update set "
                          "kind = excluded.kind, status = excluded.status, perhaps = excluded.perhaps, "
                          "timestamp = excluded.timestamp",
                          (link.id1, link.id2, link.kind, link.status, link.confidence, link.timestamp))
        return True

    def retract(self, rid, timestamp):
        """App.java:994-999 (a deleted record): getAllLinksFor(id), link.retract() [recalled:
        status RETRACTED, timestamp now], assertLink -- outside the listener, so uncommitted
        until the next commit on this connection."""
        for l in self.all_links_for(rid):
            l.status, l.timestamp = RETRACTED, timestamp
            self.assert_link(l)

    def commit(self):   # JDBCLinkDatabase.commit at batchDone
        self.conn.commit()


class LinkDBListener:
    """The MatchListener callbacks, one by one.  A query record is passed as (position in
    the batch, ID) -- Duke compares Record objects, so two records of one ID stay apart."""

    def __init__(self, db: SinceAwareLinkDB, clock):
        self.db, self.clock = db, clock
        self.current, self.cur = None, None

    def batch_ready(self, size):
        self.current = None

    def _start(self, rec):
        self.current, self.cur = rec, {}

    def _end(self):
        if self.current is None:
            return
        rid, cur = self.current[1], self.cur
        for l in self.db.all_links_for(rid):
            if l.key() in cur or l.status != INFERRED:
                continue
            r = l.copy()
            r.status, r.timestamp = RETRACTED, self.clock()
            self.db.assert_link(r)
        for l in cur.values():
            self.db.assert_link(l)
        self.current = None

    def _add(self, r1, r2, conf, kind):
        if self.current != r1:
            self._end()
            self._start(r1)
        l = Link(r1[1], r2, INFERRED, kind, conf, self.clock())
        self.cur[l.key()] = l

    def matches(self, r1, r2, conf):
        self._add(r1, r2, conf, SAME)

    def matches_perhaps(self, r1, r2, conf):
        self._add(r1, r2, conf, MAYBE)

    def no_match_for(self, r):
        self._end()
        self._start(r)
        self._end()

    def batch_done(self):
        self._end()
