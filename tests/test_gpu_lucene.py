"""GPU parity of the Lucene-compatible candidate source: the reference's own
IncrementalLuceneDatabase.findCandidateMatches semantics on the device (postings, TF-IDF
top-k, min-relevance), then Processor.compare over the hits in hit order -- against the
Python restatement of the query (oracle/lucene_ref.py) and the C oracle's compare_rows.

PARITY UNPINNED: Lucene and Duke are absent from /root/reference (see lucene_ref.py)."""
import json
import os

import numpy as np
import pytest

import lucene_ref as R
import oracle as O
import dukehip as dh
from dukehip import _abi as A
from dukehip import synth
from test_gpu_parity import schema_of

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


def expected(props, vals, lookup, ident, in_index, deleted, group, queries, thr, maybe, max_hits,
             min_rel, mode):
    ref = R.LuceneIndexRef([f"f{i}" for i in lookup], max_hits, min_rel, linkage=mode == "linkage")
    ref.set_docs([vals[i] for i in lookup], in_index, deleted, group)
    return expected_with(ref, props, vals, lookup, ident, queries, thr, maybe)


def expected_with(ref, props, vals, lookup, ident, queries, thr=0.9, maybe=0.7):
    """The pair list of Processor.compare over `ref`'s hits (isSameAs dropped)."""
    ot = O.OracleTable(props, vals, ident=ident, threshold=thr, maybe=maybe)
    out = {"query": [], "candidate": [], "prob": [], "kind": []}
    scored = 0
    for q in queries:
        for c in ref.candidates(int(q)):
            if ident[c] == ident[q]:          # Processor.isSameAs
                continue
            scored += 1
            p = ot.compare_rows(int(q), int(c))
            kind = 1 if p > thr else (2 if maybe != 0.0 and p > maybe else 0)
            if kind:
                out["query"].append(int(q))
                out["candidate"].append(int(c))
                out["prob"].append(p)
                out["kind"].append(kind)
    return out, scored


def check(res, want, scored):
    assert res.pairs_scored == scored
    assert list(res.query) == want["query"]
    assert list(res.candidate) == want["candidate"]
    assert list(res.kind) == want["kind"]
    assert list(res.prob) == want["prob"]


def upsert(eng, vals, ident, a, b, deleted=None, group=None, transient=False):
    eng.upsert(b - a, ident[a:b], [dh.Column.from_strings(v[a:b]) for v in vals],
               deleted=None if deleted is None else deleted[a:b],
               group=None if group is None else group[a:b], transient=transient)


PROPS = [{"comparator": A.CMP_JAROWINKLER, "low": 0.1, "high": 0.95},
         {"comparator": A.CMP_LEVENSHTEIN, "low": 0.2, "high": 0.8},
         {"comparator": A.CMP_LEVENSHTEIN, "low": 0.1, "high": 0.85}]


@pytest.mark.parametrize("mode", ["dedup", "linkage"])
@pytest.mark.parametrize("lookup,max_hits,min_rel", [([0], 10, 0.9), ([1, 2, 0], 10, 0.9),
                                                     ([0, 1], 5, 0.3)])
def test_lucene_candidates_equal_restatement(mode, lookup, max_hits, min_rel):
    p = synth.persons(1200, 500, seed=61)
    vals = [p["name"], p["address"], p["dob"]]
    n = len(vals[0])
    rng = np.random.default_rng(61)
    ident = np.arange(n, dtype=np.uint64)
    ident[1500:1580] = ident[100:180]               # re-posted IDs: delete-by-ID
    deleted = (rng.random(n) < 0.03).astype(np.uint8)
    group = np.where(rng.random(n) < 0.5, 1, 2).astype(np.uint8) if mode == "linkage" else None
    sch = schema_of(PROPS, 0.9, 0.7, mode, 0)
    A.lucene_source(sch, lookup, max_hits, min_rel)
    eng = dh.GpuEngine(sch)
    plan = [(0, 1000), (1000, 1500), (1500, n)]
    for a, b in plan:
        upsert(eng, vals, ident, a, b, deleted, group)
        alive = np.ones(b, bool)
        last = {}
        for r in range(b):
            if int(ident[r]) in last:
                alive[last[int(ident[r])]] = False
            last[int(ident[r])] = r
        for q in (np.arange(a, b, dtype=np.uint32), np.arange(0, b, 7, dtype=np.uint32)):
            res = eng.match(q)
            want, scored = expected(PROPS, [v[:b] for v in vals], lookup, ident[:b], alive,
                                    deleted[:b], None if group is None else group[:b], q, 0.9, 0.7,
                                    max_hits, min_rel, mode)
            check(res, want, scored)
            assert res.pairs_scored > 0
            res.close()
    counts = eng.candidate_counts(np.arange(0, n, 11, dtype=np.uint32))
    assert counts.max() <= max_hits
    eng.close()


def test_lucene_transient_queries():
    """httptransform: query-only rows are matched against the index, never hits themselves."""
    p = synth.persons(600, 300, seed=62)
    vals = [p["name"], p["address"], p["dob"]]
    n = len(vals[0])
    ident = np.arange(n, dtype=np.uint64)
    sch = schema_of(PROPS, 0.9, 0.7, "dedup", 0)
    A.lucene_source(sch, [1, 2, 0], 10, 0.9)
    eng = dh.GpuEngine(sch)
    upsert(eng, vals, ident, 0, 700)
    upsert(eng, vals, ident, 700, n, transient=True)
    q = np.arange(700, n, dtype=np.uint32)
    res = eng.match(q)
    in_index = np.r_[np.ones(700, bool), np.zeros(n - 700, bool)]
    want, scored = expected(PROPS, vals, [1, 2, 0], ident, in_index, np.zeros(n, np.uint8), None, q,
                            0.9, 0.7, 10, 0.9, "dedup")
    check(res, want, scored)
    res.close()
    eng.drop_transient()
    eng.close()


def test_reference_pipeline_on_lucene_semantics():
    """The reference's own pipeline (testdukeconfig.xml, no key functions: the GPU runs its
    Lucene candidate semantics, lookup property NAME) over the stress-test entities, posted in
    batches through GpuProcessor.deduplicate -- no reconfiguration needed."""
    from test_gpu_configs import stress_entities, alive_after, oracle_props
    from dukehip.config import DukeConfig
    with open(os.path.join(HERE, "golden", "testdukeconfig_schema.json")) as f:
        cfg = DukeConfig.from_dict(json.load(f)["pipelines"]["Deduplication/countries-dbpedia-mondial"])
    dbpedia, mondial = cfg.data_sources
    db = dh.GpuBlockingDatabase(cfg)                # no key functions -> Lucene semantics
    assert db.lookup == ["NAME"]
    proc = dh.GpuProcessor(cfg, db)
    batches = []
    for src, seed in ((dbpedia, 1234), (mondial, 4321)):
        ents = stress_entities(3000, seed)
        for a in range(0, len(ents), 1000):
            batches.append(dh.records_from_entities(ents[a:a + 1000], src))
    allrecs, ids, results = [], {}, []
    for recs in batches:
        res = proc.deduplicate(recs)
        results.append((len(allrecs), len(allrecs) + len(recs), res))
        allrecs += recs
    props = oracle_props(db.props)
    vals = [[r.get_value(p.name) for r in allrecs] for p in db.props]
    ident = np.array([ids.setdefault(r.get_value("ID"), len(ids)) for r in allrecs], np.uint64)
    deleted = np.array([r.get_value("dukeDeleted") == "true" for r in allrecs], np.uint8)
    lookup = [i for i, p in enumerate(db.props) if p.name == "NAME"]
    total = 0
    for a, e, res in results:
        alive = alive_after(list(ident), e).astype(bool)
        want, scored = expected(props, [v[:e] for v in vals], lookup, ident[:e], alive, deleted[:e],
                                None, np.arange(a, e), cfg.threshold, cfg.maybe_threshold, 10, 0.9,
                                "dedup")
        check(res, want, scored)
        total += res.n
    assert total > 100
    db.close()


@pytest.mark.parametrize("defect", ["nonmonotone", "null_offsets"])
def test_malformed_large_batch_rejected(defect):
    """A batch of >= 8192 rows stages its columns and the Lucene source on concurrent
    threads; a malformed lookup column (offsets running backwards, or no offsets at all) must
    be DK_E_INVALID with the index unchanged -- not a crash in the Lucene task."""
    p = synth.persons(9000, 1000, seed=63)
    vals = [p["name"], p["address"], p["dob"]]
    n = len(vals[0])
    ident = np.arange(n, dtype=np.uint64)
    sch = schema_of(PROPS, 0.9, 0.7, "dedup", 0)
    A.lucene_source(sch, [0, 1], 10, 0.9)
    eng = dh.GpuEngine(sch)
    upsert(eng, vals, ident, 0, 500)
    cols = [dh.Column.from_strings(v) for v in vals]
    bad = cols[0]
    if defect == "nonmonotone":
        bad.offsets = bad.offsets.copy()
        bad.offsets[5000] = bad.offsets[5001] + 7    # offsets[5001] < offsets[5000]
        raw = [c.c() for c in cols]
    else:
        raw = [c.c() for c in cols]
        raw[0].offsets = None
    arr = (A.dk_column * len(raw))(*raw)
    b = A.dk_batch()
    b.n = n
    b.ident = ident.ctypes.data
    b.columns = arr
    rc = eng.lib.dk_upsert(eng.ctx, A.C.byref(b), None)
    assert rc == A.DK_E_INVALID, (rc, eng.lib.dk_last_error())
    assert eng.num_rows == 500
    q = np.arange(500, dtype=np.uint32)
    in_index = np.ones(500, bool)
    want, scored = expected(PROPS, [v[:500] for v in vals], [0, 1], ident[:500], in_index,
                            np.zeros(500, np.uint8), None, q, 0.9, 0.7, 10, 0.9, "dedup")
    res = eng.match(q)
    check(res, want, scored)
    res.close()
    eng.close()


def indexed_versions(ident, b):
    """(alive, in_stats) after rows [0, b): the live version of each ID, and every version."""
    alive = np.ones(b, bool)
    last = {}
    for r in range(b):
        if int(ident[r]) in last:
            alive[last[int(ident[r])]] = False
        last[int(ident[r])] = r
    return alive, np.ones(b, bool)


@pytest.mark.parametrize("devices", [None, [0, 0]])
def test_lucene_unmerged_statistics_after_reposts(devices):
    """Re-posted IDs under both statistics modes.  Every re-post deletes the older version and
    adds the new one (IncrementalLuceneDatabase.java:516-517, 578-590); DK_LUCENE_STATS_MERGED
    (the default, checked with re-posts by test_lucene_candidates_equal_restatement) counts only
    live versions in maxDoc / docFreq, DK_LUCENE_STATS_UNMERGED keeps the superseded versions in
    both (Lucene 4's deleted-but-unmerged documents) until dk_lucene_merge -- never as hits."""
    p = synth.persons(1300, 600, seed=64)
    vals = [p["name"], p["address"], p["dob"]]
    n = len(vals[0])
    ident = np.arange(n, dtype=np.uint64)
    ident[1300:1600] = ident[0:300]                 # 300 re-posts of the first batch's IDs
    ident[1700:1750] = ident[1300:1350]             # re-posts of re-posts
    deleted = np.zeros(n, np.uint8)
    lookup, max_hits, min_rel = [1, 2, 0], 5, 0.3
    sch = schema_of(PROPS, 0.9, 0.7, "dedup", 0)
    A.lucene_source(sch, lookup, max_hits, min_rel)
    eng = dh.GpuEngine(sch, devices=devices)
    eng.lucene_stats(unmerged=True)
    differs = 0
    for a, b in [(0, 1000), (1000, 1500), (1500, n)]:
        upsert(eng, vals, ident, a, b)
        alive, every = indexed_versions(ident, b)
        q = np.arange(0, b, 3, dtype=np.uint32)
        args = (PROPS, [v[:b] for v in vals], lookup, ident[:b])
        res = eng.match(q)
        ref = R.LuceneIndexRef([f"f{i}" for i in lookup], max_hits, min_rel)
        ref.set_docs([vals[i][:b] for i in lookup], alive, deleted[:b], None, in_stats=every)
        want = expected_with(ref, *args, q)
        check(res, *want)
        res.close()
        merged = expected(*args, alive, deleted[:b], None, q, 0.9, 0.7, max_hits, min_rel, "dedup")
        differs += merged != want
    assert differs >= 1      # the superseded versions do move the scores
    eng.lucene_merge()       # forceMerge: back to the merged statistics
    alive, _ = indexed_versions(ident, n)
    q = np.arange(0, n, 3, dtype=np.uint32)
    res = eng.match(q)
    check(res, *expected(PROPS, vals, lookup, ident, alive, deleted, None, q, 0.9, 0.7, max_hits,
                         min_rel, "dedup"))
    res.close()
    eng.lucene_stats(unmerged=False)
    res = eng.match(q)
    check(res, *expected(PROPS, vals, lookup, ident, alive, deleted, None, q, 0.9, 0.7, max_hits,
                         min_rel, "dedup"))
    res.close()
    eng.close()


def test_lucene_stats_needs_lucene_source():
    sch = schema_of(PROPS, 0.9, 0.7, "dedup", 1)
    eng = dh.GpuEngine(sch)
    assert eng.lib.dk_lucene_set_stats(eng.ctx, A.LUCENE_STATS_UNMERGED) == A.DK_E_STATE
    assert eng.lib.dk_lucene_merge(eng.ctx) == A.DK_E_STATE
    assert eng.lib.dk_lucene_set_stats(eng.ctx, 7) == A.DK_E_INVALID
    eng.close()


def test_reposted_id_ranks_differently_merged_vs_unmerged():
    """tests/test_lucene.py's re-post case through the device: under MERGED (the
    default) Q's second hit is A, under UNMERGED it is B -- the superseded "anna" versions
    count in docFreq -- each equal to the restatement's pair list.  Which mode matches the
    reference depends on when its IndexWriter merges: both are approximations (INTEGRATION.md
    §5, parity unpinned)."""
    from test_lucene import REPOST_NAMES, REPOST_CITY, REPOST_ALIVE
    props = [{"comparator": A.CMP_EXACT, "low": 0.3, "high": 0.9},
             {"comparator": A.CMP_EXACT, "low": 0.3, "high": 0.9}]
    vals = [REPOST_NAMES, REPOST_CITY]
    ident = np.array(list(range(9)) + [5, 6, 7, 8], np.uint64)
    sch = schema_of(props, 0.01, 0.0, "dedup", 0)
    A.lucene_source(sch, [0, 1], 2, 0.0)
    eng = dh.GpuEngine(sch)
    upsert(eng, vals, ident, 0, 9)
    upsert(eng, vals, ident, 9, 13)
    q = np.array([0], np.uint32)
    got = {}
    for unmerged in (False, True):
        eng.lucene_stats(unmerged=unmerged)
        ref = R.LuceneIndexRef(["f0", "f1"], 2, 0.0)
        ref.set_docs(vals, REPOST_ALIVE, in_stats=[True] * 13 if unmerged else None)
        res = eng.match(q)
        check(res, *expected_with(ref, props, vals, [0, 1], ident, q, 0.01, 0.0))
        got[unmerged] = list(res.candidate)
        res.close()
    assert got == {False: [1], True: [2]}
    eng.close()
