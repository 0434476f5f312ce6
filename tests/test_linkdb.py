"""Link sink: dk_linkdb_apply (bulk, native) against the per-callback
restatement of LinkDatabaseMatchListener + SinceAwareInMemoryLinkDatabase
(oracle/linkdb_ref.py), and the GET ?since= body shape (App.java:846-874).  CPU only: the link
database is host code.  PARITY UNPINNED for Duke's own listener / Link classes (absent)."""
import json
import random

import numpy as np
import pytest

import linkdb_ref as R
from dukehip.ingest import Interner
from dukehip.links import LinkDatabase, interned_string, LINK_RETRACTED


def random_batches(seed, nids=60, nbatches=12):
    """Batches of (query IDs, per query [(candidate ID, prob, kind)]) with links that recur,
    change confidence by < 1e-6 / more, change kind, and disappear (retractions)."""
    rng = random.Random(seed)
    ids = [f"ds__{i}" for i in range(nids)] + ["ds__ä", "ds__\U0001F600", "ds__Z", "ds__a:b"]
    rng.shuffle(ids)
    base = {}
    out = []
    for _ in range(nbatches):
        qs = rng.sample(ids, rng.randint(1, 14))
        if rng.random() < 0.3:
            qs.append(qs[0])          # one ID twice in a batch (two records)
        entries = []
        for q in qs:
            lst = []
            for c in rng.sample([x for x in ids if x != q], rng.randint(0, 5)):
                k = tuple(sorted((q, c)))
                p = base.setdefault(k, rng.uniform(0.7, 1.0))
                r = rng.random()
                if r < 0.2:
                    p += rng.choice([3e-7, -4e-7])      # within the 1e-6 rule
                elif r < 0.35:
                    p = rng.uniform(0.7, 1.0)
                    base[k] = p
                kind = 1 if (p > 0.9) != (rng.random() < 0.1) else 2
                lst.append((c, p, kind))
            entries.append(lst)
        out.append((qs, entries))
    return out


def run_reference(batches):
    db = R.SinceAwareLinkDB()
    stamps = []
    for t, (qs, entries) in enumerate(batches):
        ts = 1000 + 10 * t
        stamps.append(ts)
        L = R.LinkDBListener(db, lambda ts=ts: ts)
        L.batch_ready(len(qs))
        for i, (q, lst) in enumerate(zip(qs, entries)):
            if not lst:
                L.no_match_for((i, q))
            for c, p, kind in lst:
                (L.matches if kind == 1 else L.matches_perhaps)((i, q), c, p)
        L.batch_done()
    return db, stamps


def run_bulk(batches):
    ids = Interner()
    ldb = LinkDatabase(ids)
    for t, (qs, entries) in enumerate(batches):
        qid = ids.intern(qs)
        first = np.zeros(len(qs) + 1, np.uint64)
        first[1:] = np.cumsum([len(x) for x in entries])
        flat = [e for lst in entries for e in lst]
        cid = ids.intern([c for c, _, _ in flat]) if flat else np.zeros(0, np.uint64)
        ldb.apply(qid, first, cid, [p for _, p, _ in flat], [k for _, _, k in flat], timestamp=1000 + 10 * t)
    return ids, ldb


@pytest.mark.parametrize("seed", [1, 2, 3, 4])
def test_bulk_link_sink_equals_per_callback(seed):
    batches = random_batches(seed)
    ref, stamps = run_reference(batches)
    ids, ldb = run_bulk(batches)
    assert len(ldb) == len(ref.links)
    for since in [0] + stamps:
        ch = ldb.changes_since(since)
        want = ref.changes_since(since)
        got = [(interned_string(ids, a), interned_string(ids, b), int(s), int(k), float(c), int(t))
               for a, b, s, k, c, t in zip(ch["id1"], ch["id2"], ch["status"], ch["kind"],
                                           ch["confidence"], ch["timestamp"])]
        assert got == [(l.id1, l.id2, l.status, l.kind, l.confidence, l.timestamp) for l in want]
    assert any(l.status == R.RETRACTED for l in ref.links.values())
    ldb.close()
    ids.close()


def test_identical_link_keeps_timestamp():
    """SinceAwareInMemoryLinkDatabase.java:18-24: same status + kind, |dconf| < 1e-6 -> skipped."""
    ids = Interner()
    ldb = LinkDatabase(ids)
    q, c = ids.intern(["ds__1", "ds__2"])
    one = np.array([0, 1], np.uint64)
    st = ldb.apply([q], one, [c], [0.95], [1], timestamp=100)
    assert st == {"asserted": 1, "unchanged": 0, "retracted": 0}
    st = ldb.apply([c], one, [q], [0.95 + 5e-7], [1], timestamp=200)    # reverse direction too
    assert st["unchanged"] == 1
    assert ldb.changes_since(100)["id1"].size == 0
    st = ldb.apply([q], one, [c], [0.95], [2], timestamp=300)           # kind changed
    assert st["asserted"] == 1 and ldb.changes_since(200)["kind"][0] == 2
    st = ldb.apply([q], np.array([0, 0], np.uint64), [], [], [], timestamp=400)   # noMatchFor
    ch = ldb.changes_since(300)
    assert st["retracted"] == 1 and ch["status"][0] == LINK_RETRACTED and ch["timestamp"][0] == 400
    st = ldb.apply([q], np.array([0, 0], np.uint64), [], [], [], timestamp=500)   # stays retracted
    assert st == {"asserted": 0, "unchanged": 0, "retracted": 0}
    with pytest.raises(Exception):
        ldb.apply([q], one, [c], [0.9], [0], timestamp=600)              # kind must be MATCH/MAYBE
    ldb.close()
    ids.close()


class _Rec:
    def __init__(self, d):
        self.d = d

    def get_value(self, k):
        return self.d.get(k)


def test_since_feed_shape():
    """App.java:846-874: `_id` = id1 + "_" + id2 with ':' -> '_', `_updated`, `_deleted`,
    entity/dataset ids (null when the record is gone), confidence; JsonObject.toString."""
    ids = Interner()
    ldb = LinkDatabase(ids)
    a, b, c = ids.intern(["ds:x__1", "ds:x__2", "ds:x__<3>"])
    ldb.apply([a, c], np.array([0, 1, 1], np.uint64), [b], [0.975], [1], timestamp=1234)
    recs = {"ds:x__1": _Rec({"dukeOriginalEntityId": "1", "dukeDatasetId": "ds:x"})}
    body = ldb.since_feed(0, recs.get)
    assert body == ('[{"_id":"ds_x__1_ds_x__2","_updated":1234,"_deleted":false,"entity1":"1",'
                    '"entity2":null,"dataset1":"ds:x","dataset2":null,"confidence":0.975}]')
    assert json.loads(body)[0]["confidence"] == 0.975
    assert ldb.since_feed(1234, recs.get) == "[]"
    ldb.close()
    ids.close()


@pytest.mark.parametrize("seed", [5, 6])
def test_deleted_record_retraction_and_links_for(seed):
    """The POST route's deleted-record branch (App.java:994-999: getAllLinksFor, retract,
    assertLink) natively (dk_linkdb_retract_all) between bulk batches, and getAllLinksFor
    (dk_linkdb_links_for), against the per-callback restatement."""
    batches = random_batches(seed)
    rng = random.Random(seed)
    ref = R.SinceAwareLinkDB()
    ids = Interner()
    ldb = LinkDatabase(ids)
    for t, (qs, entries) in enumerate(batches):
        ts = 1000 + 10 * t
        L = R.LinkDBListener(ref, lambda ts=ts: ts)
        L.batch_ready(len(qs))
        for i, (q, lst) in enumerate(zip(qs, entries)):
            if not lst:
                L.no_match_for((i, q))
            for c, p, kind in lst:
                (L.matches if kind == 1 else L.matches_perhaps)((i, q), c, p)
        L.batch_done()
        qid = ids.intern(qs)
        first = np.zeros(len(qs) + 1, np.uint64)
        first[1:] = np.cumsum([len(x) for x in entries])
        flat = [e for lst in entries for e in lst]
        cid = ids.intern([c for c, _, _ in flat]) if flat else np.zeros(0, np.uint64)
        ldb.apply(qid, first, cid, [p for _, p, _ in flat], [k for _, _, k in flat], timestamp=ts)
        for q in rng.sample(qs, min(2, len(qs))):        # deleted records of the next POST
            links = ref.all_links_for(q)
            if links and rng.random() < 0.5:              # one link of the record
                o = links[0].id2 if links[0].id1 == q else links[0].id1
                ref.retract(q, ts + 5, other=o)
                assert ldb.retract(ids.intern([q])[0], ids.intern([o])[0], ts + 5) == 1
            else:                                         # all of them
                ref.retract(q, ts + 5)
                assert ldb.retract(ids.intern([q])[0], timestamp=ts + 5) == len(links)
    for since in (0, 1050, 1100):
        ch = ldb.changes_since(since)
        got = [(interned_string(ids, a), interned_string(ids, b), int(s), int(k), float(c), int(t))
               for a, b, s, k, c, t in zip(ch["id1"], ch["id2"], ch["status"], ch["kind"],
                                           ch["confidence"], ch["timestamp"])]
        assert got == [(l.id1, l.id2, l.status, l.kind, l.confidence, l.timestamp)
                       for l in ref.changes_since(since)]
    some = batches[0][0][0]
    lf = ldb.links_for(ids.intern([some])[0])
    got = [(interned_string(ids, a), interned_string(ids, b), int(s)) for a, b, s in
           zip(lf["id1"], lf["id2"], lf["status"])]
    assert got == [(l.id1, l.id2, l.status) for l in ref.all_links_for(some)] and got
    ldb.close()
    ids.close()


class _JavaWiring:
    """GpuLinkDatabase + GpuProcessor as wired in integration/java: the unchanged per-callback
    listener (linkdb_ref.LinkDBListener, the reference's LinkDatabaseMatchListener) writes into
    this database, which drops every write while GpuProcessor's listener window is open
    (batchReady .. batchDone) and forwards a RETRACTED link outside it (the deleted-record
    branch, App.java:994-999) to dk_linkdb_retract; getAllLinksFor reads the native links."""

    def __init__(self, ids, ldb):
        self.ids, self.ldb, self.window = ids, ldb, False

    def all_links_for(self, rid):
        lf = self.ldb.links_for(self.ids.intern([rid])[0])
        return [R.Link(interned_string(self.ids, a), interned_string(self.ids, b), int(s), int(k),
                       float(c), int(t))
                for a, b, s, k, c, t in zip(lf["id1"], lf["id2"], lf["status"], lf["kind"],
                                            lf["confidence"], lf["timestamp"])]

    def assert_link(self, link):
        if self.window:
            return False
        if link.status == R.RETRACTED:
            a, b = self.ids.intern([link.id1, link.id2])
            self.ldb.retract(a, b, link.timestamp)
        return True


@pytest.mark.parametrize("seed", [7, 8, 9])
def test_java_wiring_listener_plus_bulk_equals_per_callback(seed):
    """the Java drop-in's link wiring -- listener replay into the window-
    dropping GpuLinkDatabase, the bulk applyBatch inside the window (after the replay, before
    batchDone), deleted-record retractions between batches through assertLink -- gives the
    same links and ?since= feed as the reference's per-callback listener on a plain
    SinceAwareInMemoryLinkDatabase, on batches that re-assert, change and retract links."""
    batches = random_batches(seed)
    rng = random.Random(seed)
    ref = R.SinceAwareLinkDB()
    ids = Interner()
    ldb = LinkDatabase(ids)
    wired = _JavaWiring(ids, ldb)
    for t, (qs, entries) in enumerate(batches):
        ts = 1000 + 10 * t
        for db in (ref, wired):
            if db is wired:
                wired.window = True                              # GpuProcessor.deduplicate
            L = R.LinkDBListener(db, lambda ts=ts: ts)
            L.batch_ready(len(qs))
            for i, (q, lst) in enumerate(zip(qs, entries)):
                if not lst:
                    L.no_match_for((i, q))
                for c, p, kind in lst:
                    (L.matches if kind == 1 else L.matches_perhaps)((i, q), c, p)
            if db is wired:                                      # matchAndReplay's applyBatch
                qid = ids.intern(qs)
                first = np.zeros(len(qs) + 1, np.uint64)
                first[1:] = np.cumsum([len(x) for x in entries])
                flat = [e for lst in entries for e in lst]
                cid = ids.intern([c for c, _, _ in flat]) if flat else np.zeros(0, np.uint64)
                ldb.apply(qid, first, cid, [p for _, p, _ in flat], [k for _, _, k in flat], timestamp=ts)
            L.batch_done()
            wired.window = False
        # the next POST's deleted records (App.java:994-999), per link through assertLink
        for q in rng.sample(qs, min(2, len(qs))):
            ref.retract(q, ts + 5)
            for link in wired.all_links_for(q):
                link.status, link.timestamp = R.RETRACTED, ts + 5    # Link.retract()
                wired.assert_link(link)
    for since in [0] + [1000 + 10 * t for t in range(len(batches))]:
        ch = ldb.changes_since(since)
        got = [(interned_string(ids, a), interned_string(ids, b), int(s), int(k), float(c), int(t))
               for a, b, s, k, c, t in zip(ch["id1"], ch["id2"], ch["status"], ch["kind"],
                                           ch["confidence"], ch["timestamp"])]
        assert got == [(l.id1, l.id2, l.status, l.kind, l.confidence, l.timestamp)
                       for l in ref.changes_since(since)]
    assert any(l.status == R.RETRACTED for l in ref.links.values())
    ldb.close()
    ids.close()


def test_java_wiring_without_window_diverges():
    """The wiring the window replaced (listener retractions forwarded during the replay,
    before applyBatch) is observably different: the retracted links carry the listener's
    writes first, so the check above is not vacuous."""
    ids = Interner()
    ldb = LinkDatabase(ids)
    wired = _JavaWiring(ids, ldb)
    q, c = ids.intern(["ds__1", "ds__2"])
    ldb.apply([q], np.array([0, 1], np.uint64), [c], [0.95], [1], timestamp=100)
    L = R.LinkDBListener(wired, lambda: 150)                      # window left closed
    L.batch_ready(1)
    L.no_match_for((0, "ds__1"))                                  # retracts via assertLink now
    ldb.apply([q], np.array([0, 0], np.uint64), [], [], [], timestamp=200)
    L.batch_done()
    ch = ldb.changes_since(0)
    assert int(ch["status"][0]) == LINK_RETRACTED and int(ch["timestamp"][0]) == 150   # not 200
    ldb.close()
    ids.close()
