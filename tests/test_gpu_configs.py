"""GPU parity on BASELINE.json's configurations and the reference's own schema, the
committed golden fixtures pushed through the production kernel, and the C-ABI boundary
contracts (failure-atomic upsert, single-pair compares that leave the index alone).

Oracle: oracle/duke_oracle.c (PARITY UNPINNED against Duke 1.2 itself, see its header);
fixtures: tests/golden/*.jsonl (tests/gen_golden.py) and testdukeconfig_schema.json
(tests/gen_reference_schema.py, the reference's src/main/resources/testdukeconfig.xml).
"""
import json
import math
import os
import random
import struct

import numpy as np
import pytest

import oracle as O
import dukehip as dh
from dukehip import _abi as A
from dukehip import dist as dshard
from dukehip import synth
from dukehip.config import DukeConfig, DUKE_CMP
from test_gpu_parity import schema_of, run_both, assert_same, persons_case

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
GOLDEN = os.path.join(HERE, "golden")
LEV, JW, QG, EX, NUM = A.CMP_LEVENSHTEIN, A.CMP_JAROWINKLER, A.CMP_QGRAM, A.CMP_EXACT, A.CMP_NUMERIC
WL, DICE_T, JACC_T = A.CMP_WEIGHTED_LEVENSHTEIN, A.CMP_DICE_TOKENS, A.CMP_JACCARD_TOKENS


def oracle_props(props):
    """dukehip.config.Property list (schema order) -> oracle property dicts."""
    out = []
    for p in props:
        c = p.comparator.to_c(p.low, p.high)
        out.append({"comparator": c.comparator, "low": c.low, "high": c.high, "q": c.qgram_q,
                    "formula": c.qgram_formula, "tokenizer": c.qgram_tokenizer,
                    "min_ratio": c.min_ratio})
    return out


def alive_after(ident, upto):
    alive = np.ones(upto, np.uint8)
    last = {}
    for r in range(upto):
        if ident[r] in last:
            alive[last[ident[r]]] = 0
        last[ident[r]] = r
    return alive


# ---------------------------------------------------------------------------------------
# configs[0]: the reference's Deduplication pipeline (testdukeconfig.xml) over the stress
# test's shape (sesam_node_deduplication_stresstest_config.conf.json:18-71: 2 x 10,000
# fake entities, country = first name, capital = last name, area in 1..10, ids drawn from
# a 1..1,000,000 pool), posted in HTTP batches through GpuProcessor.deduplicate.
# Blocking contract (stated; the reference itself uses Lucene): key = NAME[0:3].
# ---------------------------------------------------------------------------------------
def stress_entities(n, seed):
    return synth.stress_entities(n, seed)


def test_reference_schema_dedup_gpu():
    with open(os.path.join(GOLDEN, "testdukeconfig_schema.json")) as f:
        cfg = DukeConfig.from_dict(json.load(f)["pipelines"]["Deduplication/countries-dbpedia-mondial"])
    dbpedia, mondial = cfg.data_sources
    kf = dh.PartsKey(("NAME", None, 0, 3))
    db = dh.GpuBlockingDatabase(cfg, [kf])
    proc = dh.GpuProcessor(cfg, db)
    assert [p.name for p in db.props] == ["AREA", "CAPITAL", "NAME"]
    batches = []
    for src, seed in ((dbpedia, 1234), (mondial, 4321)):
        ents = stress_entities(10_000, seed)
        for a in range(0, len(ents), 2500):
            batches.append(dh.records_from_entities(ents[a:a + 2500], src))
    allrecs, ids, results = [], {}, []
    for recs in batches:
        res = proc.deduplicate(recs)
        results.append((len(allrecs), len(allrecs) + len(recs), res))
        allrecs += recs
    props = oracle_props(db.props)
    vals = [[r.get_value(p.name) for r in allrecs] for p in db.props]
    ident = np.array([ids.setdefault(r.get_value("ID"), len(ids)) for r in allrecs], np.uint64)
    deleted = np.array([r.get_value("dukeDeleted") == "true" for r in allrecs], np.uint8)
    keys = [kf.make_key(r) for r in allrecs]
    assert sum(r.get_value("CAPITAL") is None for r in allrecs) == 10_000   # "capical"
    total = 0
    for a, e, res in results:
        ot = O.OracleTable(props, [v[:e] for v in vals], keys=[keys[:e]], ident=ident[:e],
                           deleted=deleted[:e], alive=alive_after(list(ident), e),
                           threshold=cfg.threshold, maybe=cfg.maybe_threshold)
        assert_same(res, ot.match(np.arange(a, e, dtype=np.uint32)))
        total += res.n
    assert total > 1000
    db.close()


# ---------------------------------------------------------------------------------------
# configs[2] (QGram DICE/JACCARD + Numeric min-ratio 0.9, cross-group key blocking) and
# configs[4] (WeightedLevenshtein + QGram q=3 JACCARD, key = first two tokens) in linkage
# ---------------------------------------------------------------------------------------
@pytest.mark.parametrize("variant", ["default", "gq_defer1", "gq_nodefer", "gq_noscreen",
                                     "legacy_grouped", "tail_resource", "row_resources",
                                     "no_grouped", "host_grams"])
def test_config2_linkage_qgram_numeric(variant, monkeypatch):
    """configs[2]'s schema through each of its device paths, bit-exact against the oracle:
    k_score_gq (default: the screen with QGram role 0 deferred to the exact pass; role 1
    deferred; no role deferred; no screen -- every valid pair takes the exact pass; its head /
    tail row resources are the layout a 10M x 10M replica takes, at any size),
    k_score_grouped (DK_GQ=0) with one buffer resource per
    property, with head and tail resources (DK_GROUPED_ROW=1) or a resource per tail row
    (DK_GROUPED_ROW=2: replicas past k_score_gq's resources), k_score_nodp (DK_GROUPED=0),
    and q-gram sets built on the host instead of the device (DK_DEV_GRAMS=0)."""
    env = {"gq_defer1": [("DK_GQ_DEFER", "1")],
           "gq_nodefer": [("DK_GQ_DEFER", "-1")],
           "gq_noscreen": [("DK_GQ_SCREEN", "0")],
           "legacy_grouped": [("DK_GQ", "0")],
           "tail_resource": [("DK_GQ", "0"), ("DK_GROUPED_ROW", "1")],
           "row_resources": [("DK_GQ", "0"), ("DK_GROUPED_ROW", "2")],
           "no_grouped": [("DK_GROUPED", "0")],
           "host_grams": [("DK_DEV_GRAMS", "0")]}.get(variant, [])
    for kv in env:
        monkeypatch.setenv(*kv)
    p, group = synth.linkage_persons(2500)
    props = [{"comparator": QG, "low": 0.1, "high": 0.95, "q": 2, "formula": A.QGRAM_DICE},
             {"comparator": QG, "low": 0.2, "high": 0.8, "q": 2, "formula": A.QGRAM_JACCARD},
             {"comparator": NUM, "low": 0.3, "high": 0.7, "min_ratio": 0.9},
             {"comparator": NUM, "low": 0.4, "high": 0.75, "min_ratio": 0.9}]
    vals = [p["name"], p["address"], p["birthyear"], p["zip"]]
    res, ref = run_both(props, vals, synth.keys_config2(p), mode="linkage", group=group,
                        threshold=0.9, maybe=0.7, queries=np.arange(2500, len(group)))
    assert res.n > 100
    assert_same(res, ref)


@pytest.mark.parametrize("case", ["bench", "low_maybe", "match_only", "zero_low", "overlap", "wide_high"])
def test_config2_screen_edges(case, monkeypatch):
    """k_score_gq's single-precision screen only drops pairs whose exact probability cannot
    reach the list: bit-exact lists against the oracle where the bound is tight (the bench's
    configuration, thresholds that put many pairs near the bound), where it must give up
    (low = 0: the zero factor; high = 0.995: a role bound past kScreenHi), and for the
    OVERLAP formula; with the role deferred or not."""
    monkeypatch.setenv("DK_GQ_DEFER", "1" if case in ("zero_low", "overlap") else "0")
    p, group = synth.linkage_persons(2000)
    qlow, qhigh, formula, th, mb = 0.1, 0.9, A.QGRAM_DICE, 0.9, 0.7
    if case == "low_maybe":
        th, mb = 0.8, 0.35
    elif case == "match_only":
        th, mb = 0.6, 0.0
    elif case == "zero_low":
        qlow = 0.0
    elif case == "overlap":
        formula = A.QGRAM_OVERLAP
    elif case == "wide_high":
        qhigh = 0.995
    props = [{"comparator": QG, "low": qlow, "high": qhigh, "q": 2, "formula": formula},
             {"comparator": QG, "low": 0.1, "high": 0.8, "q": 2, "formula": A.QGRAM_JACCARD},
             {"comparator": NUM, "low": 0.2, "high": 0.6, "min_ratio": 0.9996},
             {"comparator": NUM, "low": 0.4, "high": 0.75, "min_ratio": 0.9}]
    vals = [p["name"], p["address"], p["birthyear"], p["zip"]]
    res, ref = run_both(props, vals, synth.keys_config2(p), mode="linkage", group=group,
                        threshold=th, maybe=mb, queries=np.arange(2000, len(group)))
    assert res.n > 50
    assert_same(res, ref)


def test_config4_linkage_long_text():
    texts, group = synth.long_texts(1000)
    props = [{"comparator": WL, "low": 0.2, "high": 0.9},
             {"comparator": QG, "low": 0.3, "high": 0.8, "q": 3, "formula": A.QGRAM_JACCARD}]
    res, ref = run_both(props, [texts, texts], synth.keys_first_two_tokens(texts), mode="linkage",
                        group=group, threshold=0.9, maybe=0.7, queries=np.arange(1000, len(group)))
    assert res.n > 10
    assert_same(res, ref)


# ---------------------------------------------------------------------------------------
# golden fixtures through the production kernel (dk_property_similarity)
# ---------------------------------------------------------------------------------------
def fx(v):
    if v is None:
        return None
    return float.fromhex(v["hex"])


GOLDEN_PROPS = {
    "levenshtein": {"comparator": LEV},
    "jarowinkler": {"comparator": JW},
    "exact": {"comparator": EX},
    "weighted_levenshtein": {"comparator": WL},
    "dice_tokens": {"comparator": DICE_T},
    "jaccard_tokens": {"comparator": JACC_T},
    "qgram_q2_f1_ends": {"comparator": QG, "q": 2, "formula": 1, "tokenizer": A.QGRAM_ENDS},
    "qgram_q3_f2_ends": {"comparator": QG, "q": 3, "formula": 2, "tokenizer": A.QGRAM_ENDS},
    "qgram_q2_f1_positional": {"comparator": QG, "q": 2, "formula": 1, "tokenizer": A.QGRAM_POSITIONAL},
}
for _q in (1, 2, 3):
    for _f in (0, 1, 2):
        GOLDEN_PROPS[f"qgram_q{_q}_f{_f}"] = {"comparator": QG, "q": _q, "formula": _f}


def load_jsonl(name):
    with open(os.path.join(GOLDEN, name)) as f:
        return [json.loads(l) for l in f]


def units_str(u):
    return struct.pack(f"<{len(u)}H", *u).decode("utf-16-le", "surrogatepass")


@pytest.mark.parametrize("fixture", ["comparators.jsonl", "long_values.jsonl"])
def test_golden_fixtures_through_kernel(fixture):
    rows = load_jsonl(fixture)
    strs = []
    for r in rows:
        strs += [units_str(r["s1"]), units_str(r["s2"])]
    keys = [k for k in GOLDEN_PROPS if k in rows[0]]
    assert keys
    checked = 0
    for key in keys:
        prop = dict(GOLDEN_PROPS[key], low=0.1, high=0.9)
        eng = dh.GpuEngine(schema_of([prop], 0.9, 0.0, "allpairs", 0))
        eng.upsert(len(strs), np.arange(len(strs)), [dh.Column.from_strings(strs)])
        for i, r in enumerate(rows):
            want = fx(r[key])
            got = eng.property_similarity(0, 2 * i, 2 * i + 1)
            if not r["s1"] or not r["s2"]:
                assert math.isnan(got), (key, i)   # Processor never compares empty values
                continue
            if key == "levenshtein":
                n1, n2 = len(r["s1"]), len(r["s2"])
                ln = min(n1, n2)
                if 2 * ln > max(n1, n2) and got != 1.0:
                    # the integer distance, bit-exact also where Duke's early exit fired
                    # (Comparator.compare returns its column minimum): dist = len * (1 - sim)
                    assert round((1.0 - got) * ln) == min(r["compact_distance"], ln), (i, got)
            assert got == want or (math.isnan(got) and want is not None and math.isnan(want)), \
                (key, i, got, want)
            checked += 1
        eng.close()
    assert checked > len(rows)


def java_div(a, b):
    """Java's double division (IEEE: x/0 is +-Infinity, 0/0 and NaN operands give NaN)."""
    if b == 0.0:
        if a == 0.0 or math.isnan(a):
            return math.nan
        return math.copysign(math.inf, a) * math.copysign(1.0, b)
    return a / b


def java_numeric(d1, ok1, d2, ok2, min_ratio):
    if not ok1 or not ok2:
        return 0.5
    if d1 == 0.0 and d2 == 0.0:
        return 1.0
    if d2 < d1:
        d1, d2 = d2, d1
    ratio = java_div(d1, d2)
    return 0.0 if ratio < min_ratio else ratio


def test_golden_numeric_through_kernel():
    allrows = load_jsonl("numeric.jsonl")
    # fixture pairs: NumericComparator.compare(s1, s2) at the row's min-ratio
    pairs = [r for r in allrows if "s1" in r]
    assert pairs
    for mr in sorted({r["min_ratio"] for r in pairs}):
        sel = [r for r in pairs if r["min_ratio"] == mr]
        strs = []
        for r in sel:
            strs += [units_str(r["s1"]), units_str(r["s2"])]
        eng = dh.GpuEngine(schema_of([{"comparator": NUM, "low": 0.1, "high": 0.9, "min_ratio": mr}],
                                     0.9, 0.0, "allpairs", 0))
        eng.upsert(len(strs), np.arange(len(strs)), [dh.Column.from_strings(strs)])
        for i, r in enumerate(sel):
            got = eng.property_similarity(0, 2 * i, 2 * i + 1)
            if not r["s1"] or not r["s2"]:
                assert math.isnan(got)
                continue
            want = fx(r["numeric"])
            assert got == want or (math.isnan(got) and math.isnan(want)), (r, got)
            assert math.copysign(1.0, got) == math.copysign(1.0, want) or math.isnan(got)
        eng.close()
    # parsed values (Double.parseDouble fixture) crossed at random
    rows = [r for r in allrows if "parse" in r]
    strs = [units_str(r["parse"]) for r in rows]
    parsed = [(fx(r["value"]) if r["value"] is not None else 0.0, r["value"] is not None) for r in rows]
    eng = dh.GpuEngine(schema_of([{"comparator": NUM, "low": 0.1, "high": 0.9, "min_ratio": 0.7}],
                                 0.9, 0.0, "allpairs", 0))
    eng.upsert(len(strs), np.arange(len(strs)), [dh.Column.from_strings(strs)])
    rng = random.Random(3)
    pairs = [(i, i + 1) for i in range(len(rows) - 1)] + [
        (rng.randrange(len(rows)), rng.randrange(len(rows))) for _ in range(2000)]
    for a, b in pairs:
        got = eng.property_similarity(0, a, b)
        if not strs[a] or not strs[b]:
            assert math.isnan(got)
            continue
        want = java_numeric(parsed[a][0], parsed[a][1], parsed[b][0], parsed[b][1], 0.7)
        assert got == want or (math.isnan(got) and math.isnan(want)), (strs[a], strs[b], got, want)
    eng.close()


# ---------------------------------------------------------------------------------------
# boundary contracts
# ---------------------------------------------------------------------------------------
def upsert_slice(eng, vals, keys, ident, a, b, deleted=None):
    return eng.upsert(b - a, ident[a:b], [dh.Column.from_strings(v[a:b]) for v in vals],
                      deleted=None if deleted is None else deleted[a:b],
                      key_columns=[dh.Column.from_strings(k[a:b]) for k in keys])


@pytest.mark.parametrize("sparse", [False, True])
def test_failed_upsert_leaves_index_unchanged(sparse):
    """A batch rejected by dk_upsert (a Levenshtein value over 256 units) that re-posts
    already indexed IDs must not tombstone them; a valid re-post of those IDs in shuffled
    positions afterwards supersedes them exactly once (Lucene delete-then-add).  sparse:
    64-bit identities far above the row count (the ID map's hash side and its undo log)."""
    p, props, vals, keys = persons_case(600, 200, 31)
    n = len(vals[0])
    eng = dh.GpuEngine(schema_of(props, 0.9, 0.7, "dedup", 2))
    big = np.random.default_rng(5).choice(2 ** 62, size=n, replace=False).astype(np.uint64) + 2 ** 40
    idmap = (lambda a: big[np.asarray(a, dtype=np.int64)]) if sparse else (lambda a: np.asarray(a, np.uint64))
    ident = idmap(np.arange(n))
    upsert_slice(eng, vals, keys, ident, 0, 500)
    # batch 2: IDs 0..59 again + new ones, and one over-long ADDRESS value
    perm = np.random.default_rng(1).permutation(60)
    b_ident = idmap(np.r_[perm, np.arange(500, n)])
    b_vals = [[v[i] for i in perm] + v[500:] for v in vals]
    b_keys = [[k[i] for i in perm] + k[500:] for k in keys]
    bad = [list(col) for col in b_vals]
    bad[1][7] = "x" * 300
    with pytest.raises(dh.DukeHipError) as e:
        eng.upsert(len(b_ident), b_ident, [dh.Column.from_strings(v) for v in bad],
                   key_columns=[dh.Column.from_strings(k) for k in b_keys])
    assert e.value.code == A.DK_E_UNSUPPORTED
    assert eng.num_rows == 500
    # the index is as before: compare with the oracle over the first batch
    q = np.arange(500, dtype=np.uint32)
    ot = O.OracleTable(props, [v[:500] for v in vals], keys=[k[:500] for k in keys],
                       threshold=0.9, maybe=0.7)
    assert_same(eng.match(q), ot.match(q))
    # the valid batch: rows 500.. hold IDs perm + 500..n-1
    eng.upsert(len(b_ident), b_ident, [dh.Column.from_strings(v) for v in b_vals],
               key_columns=[dh.Column.from_strings(k) for k in b_keys])
    full_vals = [v[:500] + bv for v, bv in zip(vals, b_vals)]
    full_keys = [k[:500] + bk for k, bk in zip(keys, b_keys)]
    full_ident = np.r_[ident[:500], b_ident].astype(np.uint64)
    m = len(full_ident)
    ot = O.OracleTable(props, full_vals, keys=full_keys, ident=full_ident,
                       alive=alive_after(list(full_ident), m), threshold=0.9, maybe=0.7)
    q = np.arange(m, dtype=np.uint32)
    assert_same(eng.match(q), ot.match(q))
    eng.close()


def test_compare_rows_then_match_then_compare_rows():
    """dk_compare_rows uses private scratch: the cached blocking tables stay valid."""
    p, props, vals, keys = persons_case(700, 300, 32)
    n = len(vals[0])
    eng = dh.GpuEngine(schema_of(props, 0.9, 0.7, "dedup", 2))
    ident = np.arange(n, dtype=np.uint64)
    upsert_slice(eng, vals, keys, ident, 0, n)
    ot = O.OracleTable(props, vals, keys=keys, threshold=0.9, maybe=0.7)
    q = np.arange(n, dtype=np.uint32)
    ref = ot.match(q)
    assert_same(eng.match(q), ref)             # builds the tables
    pairs = [(0, 1), (5, 9), (17, 17), (n - 1, 3), (42, 400)]
    for a, b in pairs:
        assert eng.compare_rows(a, b) == ot.compare_rows(a, b)
    assert_same(eng.match(q), ref)             # reuses the tables
    for a, b in pairs:
        assert eng.compare_rows(b, a) == ot.compare_rows(b, a)
    assert_same(eng.match(q[::3]), ot.match(q[::3]))
    eng.close()


def test_compare_values_unindexed_records():
    rng = random.Random(33)
    props = [{"comparator": JW, "low": 0.1, "high": 0.95},
             {"comparator": LEV, "low": 0.2, "high": 0.8},
             {"comparator": WL, "low": 0.1, "high": 0.9},
             {"comparator": QG, "low": 0.2, "high": 0.8, "q": 3, "formula": 1},
             {"comparator": NUM, "low": 0.3, "high": 0.7, "min_ratio": 0.5}]
    eng = dh.GpuEngine(schema_of(props, 0.9, 0.7, "dedup", 1))
    eng.upsert(2, [0, 1], [dh.Column.from_strings(["zz", "zy"]) for _ in props],
               key_columns=[dh.Column.from_strings(["k", "k"])])
    alpha = "abcdeł\U0001F600 "
    for t in range(60):
        def val(i):
            if rng.random() < 0.1:
                return None
            if i == 4:
                return str(rng.randint(0, 30))
            return "".join(rng.choice(alpha) for _ in range(rng.randint(1, 90 if i == 2 else 20)))
        r1 = [val(i) for i in range(len(props))]
        r2 = [v if (v is not None and rng.random() < 0.4) else val(i) for i, v in enumerate(r1)]
        got = eng.compare_values([dh.Column.from_strings([a, b]) for a, b in zip(r1, r2)])
        ot = O.OracleTable(props, [[a, b] for a, b in zip(r1, r2)], keys=[["k", "k"]])
        want = ot.compare_rows(0, 1)
        assert got == want or (math.isnan(got) and math.isnan(want)), (t, r1, r2, got, want)
    assert eng.num_rows == 2                      # the ctx's index is untouched
    eng.close()


def test_processor_compare_and_deduplicate_flush_pending():
    """GpuProcessor.compare on unindexed records; records handed to Database.index()
    before deduplicate (App.java:988-1001) are committed with the batch."""
    cfg = dh.DukeConfig([dh.Property("NAME", dh.Comparator(DUKE_CMP + "Levenshtein"), 0.1, 0.9)],
                        threshold=0.6, maybe_threshold=0.5)
    db = dh.GpuBlockingDatabase(cfg, [dh.PartsKey(("NAME", None, 0, 1))])
    proc = dh.GpuProcessor(cfg, db)
    a = dh.Record({"ID": "d__1", "NAME": "anna"})
    b = dh.Record({"ID": "d__2", "NAME": "anne"})
    ot = O.OracleTable([{"comparator": LEV, "low": 0.1, "high": 0.9}], [["anna", "anne"]],
                       keys=[["a", "a"]])
    assert proc.compare(a, b) == ot.compare_rows(0, 1)
    proc.deduplicate([a, b])
    lis = dh.CollectingListener()
    proc.add_match_listener(lis)
    gone = dh.Record({"ID": "d__2", "NAME": "anne", "dukeDeleted": "true"})
    db.index(gone)                                # deleted version of d__2
    proc.deduplicate([dh.Record({"ID": "d__3", "NAME": "annu"})])
    assert db.pending == []
    hits = [e for e in lis.events if e[0] in ("matches", "matchesPerhaps")]
    assert hits and all(e[2] != "d__2" for e in hits)   # d__2 is deleted: not a candidate
    assert any(e[2] == "d__1" for e in hits)
    db.close()


def test_overwrite_keeps_older_versions():
    p, props, vals, keys = persons_case(300, 100, 34)
    n = len(vals[0])
    ident = np.arange(n, dtype=np.uint64)
    ident[350:] = ident[:50]
    eng = dh.GpuEngine(schema_of(props, 0.9, 0.7, "dedup", 2))
    eng.set_overwrite(True)
    upsert_slice(eng, vals, keys, ident, 0, 300)
    upsert_slice(eng, vals, keys, ident, 300, n)
    ot = O.OracleTable(props, vals, keys=keys, ident=ident, threshold=0.9, maybe=0.7)
    q = np.arange(n, dtype=np.uint32)
    assert_same(eng.match(q), ot.match(q))
    eng.close()


def test_linkage_group_validated():
    cfg = dh.DukeConfig([dh.Property("NAME", dh.Comparator(DUKE_CMP + "Levenshtein"), 0.1, 0.9)],
                        threshold=0.6, linkage=True)
    db = dh.GpuBlockingDatabase(cfg, [dh.PartsKey(("NAME", None, 0, 1))])
    with pytest.raises(ValueError):
        db.index_batch([dh.Record({"ID": "1__a__1", "NAME": "x"})])
    eng = db.engine
    with pytest.raises(dh.DukeHipError) as e:
        eng.upsert(2, [0, 1], [dh.Column.from_strings(["a", "b"])], group=[1, 3],
                   key_columns=[dh.Column.from_strings(["a", "b"])])
    assert e.value.code == A.DK_E_INVALID and eng.num_rows == 0
    db.close()


def test_two_engines_tiles_equal_single_engine():
    """Two dk_ctx on one device, each matching its query tile of a replicated index:
    concat_ranks of their lists equals the single-engine list bit for bit."""
    p, props, vals, keys = persons_case(1500, 500, 35)
    n = len(vals[0])
    ident = np.arange(n, dtype=np.uint64)
    engs = [dh.GpuEngine(schema_of(props, 0.9, 0.7, "dedup", 2)) for _ in range(3)]
    for e in engs:
        upsert_slice(e, vals, keys, ident, 0, n)
    q = np.arange(n, dtype=np.uint32)
    full = engs[0].match(q)
    lists = []
    for r, e in enumerate(engs[1:]):
        a, b = dshard.tile(n, r, 2)
        res = e.match(q[a:b])
        lists.append({"first": res.first.copy(), "candidate": res.candidate.copy(),
                      "prob": res.prob.copy(), "kind": res.kind.copy()})
        res.close()
    cat = dshard.concat_ranks(lists)
    assert np.array_equal(cat["first"], full.first.astype(np.int64))
    for k in ("candidate", "prob", "kind"):
        assert np.array_equal(cat[k], getattr(full, k))
    for e in engs:
        e.close()


@pytest.mark.parametrize("mode,ndev", [("dedup", 2), ("dedup", 3), ("linkage", 2)])
def test_multi_device_ctx_equals_single_ctx(mode, ndev):
    _multi_device_case(mode, [0] * ndev)


@pytest.mark.parametrize("mode", ["dedup", "linkage"])
def test_multi_device_distinct_gpus(mode):
    """The same over two physically different GPUs: the group's pinned match list
    (hipHostMallocPortable) is filled by copies from both devices' streams, and the
    cost-balanced tiles run on separate devices.  Runs only where two GPUs are visible (the
    round-end 8-GPU node; the 1-GPU box skips it)."""
    import torch
    if torch.cuda.device_count() < 2:
        pytest.skip("needs two visible GPUs")
    _multi_device_case(mode, [0, 1])


def _multi_device_case(mode, devices):
    """dk_create_multi over `devices` (one stream set each; repeated entries of device 0 on a
    one-GPU box): the replicated
    index takes the same batches (re-posted IDs, deleted rows, a rejected batch, transient
    query rows), and every match -- its queries split into cost-balanced tiles matched
    concurrently -- equals the single-ctx list bit for bit, as do candidate counts, compare
    and property similarity (SURVEY §8b/§8e in one process)."""
    p, props, vals, keys = persons_case(1500, 500, 41)
    n = len(vals[0])
    rng = np.random.default_rng(41)
    ident = np.arange(n, dtype=np.uint64)
    ident[1700:1760] = ident[100:160]
    deleted = (rng.random(n) < 0.03).astype(np.uint8)
    group = np.where(np.arange(n) % 3 == 0, 1, 2).astype(np.uint8) if mode == "linkage" else None
    sch = schema_of(props, 0.9, 0.7, mode, 2)
    one = dh.GpuEngine(sch)
    many = dh.GpuEngine(sch, devices=list(devices))
    assert many.num_devices == len(devices) and one.num_devices == 1

    def up(e, a, b, transient=False, bad=False):
        cols = [dh.Column.from_strings(v[a:b]) for v in vals]
        if bad:
            cols[1] = dh.Column.from_strings(["x" * 300] + list(vals[1][a + 1:b]))
        return e.upsert(b - a, ident[a:b], cols, deleted=deleted[a:b],
                        group=None if group is None else group[a:b],
                        key_columns=[dh.Column.from_strings(k[a:b]) for k in keys], transient=transient)

    def same(q):
        r1, r2 = one.match(q), many.match(q)
        assert r1.pairs_scored == r2.pairs_scored and r1.n == r2.n
        for k in ("first", "candidate", "prob", "kind"):
            assert np.array_equal(getattr(r1, k), getattr(r2, k)), k
        r1.close()
        r2.close()

    for a, b in ((0, 1200), (1200, 1700), (1700, n)):
        for e in (one, many):
            up(e, a, b)
        q = np.arange(a, b, dtype=np.uint32) if mode == "dedup" else \
            np.array([i for i in range(a, b) if group[i] == 2], dtype=np.uint32)
        same(q)
    for e in (one, many):                      # a rejected batch changes neither index
        with pytest.raises(dh.DukeHipError):
            up(e, 0, 50, bad=True)
    assert many.num_rows == one.num_rows == n
    allq = np.arange(n, dtype=np.uint32)[::3]
    same(allq)
    assert np.array_equal(one.candidate_counts(allq), many.candidate_counts(allq))
    for r1, r2 in ((0, 1), (5, 900), (1701, 101)):
        assert one.compare_rows(r1, r2) == many.compare_rows(r1, r2)
        assert one.property_similarity(1, r1, r2) == many.property_similarity(1, r1, r2)
    if mode == "dedup":                        # httptransform: query-only rows on every device
        rows = [up(e, 0, 200, transient=True) for e in (one, many)]
        assert np.array_equal(rows[0], rows[1])
        same(np.asarray(rows[0], np.uint32))
        one.drop_transient()
        many.drop_transient()
        assert many.num_rows == one.num_rows == n
    with pytest.raises(dh.DukeHipError) as e:  # the list is handed over in host memory
        many.match(allq, on_device=True)
    assert e.value.code == A.DK_E_UNSUPPORTED
    one.close()
    many.close()


# ---------------------------------------------------------------------------------------
# the symmetric dedup schedule (owner slots + emission pass) against the direct schedule
# (DK_SYM=0) and the oracle
# ---------------------------------------------------------------------------------------
def sym_case(seed, n=2400):
    rng = random.Random(seed)
    alpha = "abcdeł"
    fixed = ["".join(rng.choice("abc") for _ in range(6)) for _ in range(n)]   # equal-length JW
    name = [("".join(rng.choice(alpha) for _ in range(rng.randint(3, 9))) if rng.random() > 0.05 else None)
            for _ in range(n)]
    num = [str(rng.randint(1, 9)) if rng.random() > 0.1 else None for _ in range(n)]
    props = [{"comparator": JW, "low": 0.2, "high": 0.9},
             {"comparator": LEV, "low": 0.1, "high": 0.8},
             {"comparator": QG, "low": 0.3, "high": 0.7, "q": 2, "formula": A.QGRAM_DICE},
             {"comparator": NUM, "low": 0.3, "high": 0.7, "min_ratio": 0.5},
             {"comparator": EX, "low": 0.4, "high": 0.6}]
    vals = [fixed, name, name, num, fixed]
    keys = [[f[:1] for f in fixed], [(v or "")[:1] for v in name]]
    return props, vals, keys


@pytest.mark.parametrize("seed", [41, 42])
def test_symmetric_schedule_equals_direct(seed, monkeypatch):
    props, vals, keys = sym_case(seed)
    n = len(vals[0])
    rng = np.random.default_rng(seed)
    ident = np.arange(n, dtype=np.uint64)
    ident[2000:2100] = ident[100:200]                # superseded rows (not in the tables)
    ident[2100:2110] = ident[2110:2120]              # superseded inside the query range
    deleted = (rng.random(n) < 0.03).astype(np.uint8)
    eng = dh.GpuEngine(schema_of(props, 0.75, 0.55, "dedup", 2))
    upsert_slice(eng, vals, keys, ident, 0, 1500, deleted)
    upsert_slice(eng, vals, keys, ident, 1500, n, deleted)
    ot = O.OracleTable(props, vals, keys=keys, ident=ident, deleted=deleted,
                       alive=alive_after(list(ident), n), threshold=0.75, maybe=0.55)
    # the mirror decision bytes are cleared per call: shrinking then growing query sets on
    # one engine, one chunk or many (every chunk's write pass sets its queries' first[])
    for q in (np.arange(n, dtype=np.uint32), np.arange(700, 1900, dtype=np.uint32),
              np.arange(1500, n, dtype=np.uint32), np.arange(n, dtype=np.uint32)):
        for chunk in (None, "3000", "512"):
            if chunk:
                monkeypatch.setenv("DK_CHUNK_SLOTS", chunk)
            else:
                monkeypatch.delenv("DK_CHUNK_SLOTS", raising=False)
            # the bucket lookup index (SymIndex) on the 3000-slot chunks, binary searches else
            monkeypatch.setenv("DK_SYMIDX", "1" if chunk == "3000" else "0")
            eng.reset_profile()
            eng.set_profiling(True)
            res = eng.match(q)
            assert eng.profile()["sym_matches"] == 1
            ref = ot.match(q)
            assert res.n > 0
            assert_same(res, ref)
            res_dev = eng.match(q, on_device=True)
            assert res_dev.n == res.n and res_dev.pairs_scored == res.pairs_scored
            res_dev.close()
            monkeypatch.setenv("DK_SYM", "0")
            direct = eng.match(q)
            monkeypatch.delenv("DK_SYM")
            assert_same(direct, ref)
            eng.set_profiling(False)
            res.close()
            direct.close()
    eng.close()


def sym2_case(seed, n=3000):
    """Latin-1 JaroWinkler / Levenshtein / Exact / Numeric values for k_score_sym2: lengths
    from 1 to 40 units (the two half-waves' queries pick different row buckets), missing
    values on both sides, small key buckets (most owned lists under 32: many waves hold two
    queries)."""
    rng = random.Random(seed)
    alpha = "abcdeé"
    def word(lo, hi):
        return "".join(rng.choice(alpha) for _ in range(rng.randint(lo, hi)))
    name = [word(1, 14) if rng.random() > 0.05 else None for _ in range(n)]
    addr = [word(3, 40) if rng.random() > 0.08 else None for _ in range(n)]
    code = [word(2, 3) if rng.random() > 0.1 else None for _ in range(n)]
    num = [str(rng.randint(1, 9)) if rng.random() > 0.1 else None for _ in range(n)]
    props = [{"comparator": JW, "low": 0.2, "high": 0.9},
             {"comparator": LEV, "low": 0.1, "high": 0.8},
             {"comparator": LEV, "low": 0.15, "high": 0.85},
             {"comparator": NUM, "low": 0.3, "high": 0.7, "min_ratio": 0.5},
             {"comparator": EX, "low": 0.4, "high": 0.6}]
    vals = [name, addr, code, num, code]
    keys = [[(v or "")[:2] for v in name], [(v or "")[:2] for v in addr]]
    return props, vals, keys


@pytest.mark.parametrize("seed", [43, 44])
def test_sym2_two_queries_per_wave(seed, monkeypatch):
    """k_score_sym2 (owner slots padded to 32, a query per half-wave) bit-exact against the
    oracle, against one query per wave (DK_SYM2=0), against the direct schedule (DK_SYM=0) and
    with the bucket lookup index of large batches (DK_SYMIDX=1: SymIndex instead of binary
    searches), with the owner slots in query order instead of by length within each tile
    (DK_SYM_ORDER=0), with superseded and deleted rows, a delta segment, one chunk and many."""
    props, vals, keys = sym2_case(seed)
    n = len(vals[0])
    rng = np.random.default_rng(seed)
    ident = np.arange(n, dtype=np.uint64)
    ident[2500:2600] = ident[100:200]
    deleted = (rng.random(n) < 0.03).astype(np.uint8)
    eng = dh.GpuEngine(schema_of(props, 0.75, 0.55, "dedup", 2))
    upsert_slice(eng, vals, keys, ident, 0, 2000, deleted)
    upsert_slice(eng, vals, keys, ident, 2000, n, deleted)
    ot = O.OracleTable(props, vals, keys=keys, ident=ident, deleted=deleted,
                       alive=alive_after(list(ident), n), threshold=0.75, maybe=0.55)
    for q in (np.arange(n, dtype=np.uint32), np.arange(900, 2700, dtype=np.uint32)):
        ref = ot.match(q)
        assert len(ref["query"]) > 100
        for chunk in (None, "640"):
            if chunk:
                monkeypatch.setenv("DK_CHUNK_SLOTS", chunk)
            else:
                monkeypatch.delenv("DK_CHUNK_SLOTS", raising=False)
            for env in ({}, {"DK_SYM2": "0"}, {"DK_SYM": "0"}, {"DK_SYMIDX": "1"}, {"DK_SYM_ORDER": "0"}):
                for k, v in env.items():
                    monkeypatch.setenv(k, v)
                eng.reset_profile()
                res = eng.match(q)
                prof = eng.profile()
                assert prof["sym_matches"] == (0 if env.get("DK_SYM") == "0" else 1)
                assert prof["sym2_matches"] == (0 if env.get("DK_SYM") == "0" or env.get("DK_SYM2") == "0" else 1)
                assert_same(res, ref)
                res.close()
                for k in env:
                    monkeypatch.delenv(k)
    eng.close()


def test_symmetric_schedule_overwrite_duplicates():
    """overwrite: several alive rows of one ID; isSameAs filters them from each other."""
    props, vals, keys = sym_case(43, n=900)
    n = len(vals[0])
    ident = np.arange(n, dtype=np.uint64) % 700
    eng = dh.GpuEngine(schema_of(props, 0.75, 0.55, "dedup", 2))
    eng.set_overwrite(True)
    upsert_slice(eng, vals, keys, ident, 0, n)
    ot = O.OracleTable(props, vals, keys=keys, ident=ident, threshold=0.75, maybe=0.55)
    q = np.arange(n, dtype=np.uint32)
    eng.set_profiling(True)
    assert_same(eng.match(q), ot.match(q))
    assert eng.profile()["sym_matches"] == 1
    eng.close()


# ---------------------------------------------------------------------------------------
# native ingestion (dk_pack_json) through the processor == the Record path
# ---------------------------------------------------------------------------------------
@pytest.mark.parametrize("linkage", [False, True])
def test_deduplicate_json_equals_record_path(linkage):
    with open(os.path.join(GOLDEN, "testdukeconfig_schema.json")) as f:
        key = "RecordLinkage/countries-dbpedia-mondial" if linkage else "Deduplication/countries-dbpedia-mondial"
        cfg_d = json.load(f)["pipelines"][key]
    kf = [dh.PartsKey(("NAME", None, 0, 3))]
    procs, lis = [], []
    for _ in range(2):
        cfg = DukeConfig.from_dict(cfg_d)
        db = dh.GpuBlockingDatabase(cfg, kf)
        p = dh.GpuProcessor(cfg, db)
        l = dh.CollectingListener()
        p.add_match_listener(l)
        procs.append(p)
        lis.append(l)
    srcs = procs[0].config.data_sources
    for si, (seed, src_i) in enumerate(((11, 0), (12, 1), (13, 0))):
        ents = stress_entities(1500, seed)
        for e in ents[::50]:
            e["country"] = "  The " + e["country"].upper() + "  "   # the cleaners at work
        body = json.dumps(ents)
        src0, src1 = procs[0].config.data_sources[src_i], procs[1].config.data_sources[src_i]
        ref = procs[0].deduplicate(dh.records_from_entities(dh.parse_entities(body)[0], src0))
        got = procs[1].deduplicate_json(body, src1)
        assert got.n == ref.n and got.pairs_scored == ref.pairs_scored
        for k in ("first", "candidate", "prob", "kind"):
            assert np.array_equal(getattr(got, k), getattr(ref, k)), k
    assert lis[0].events == lis[1].events and len(lis[0].events) > 100
    # findRecordById through the native rows
    db0, db1 = procs[0].database, procs[1].database
    some = [e for e in lis[0].events if e[0] == "matches"][:20]
    for ev in some:
        r0, r1 = db0.find_record_by_id(ev[2]), db1.find_record_by_id(ev[2])
        assert r1 is not None and r1.get_values("NAME") == r0.get_values("NAME")
        assert r1.get_value("dukeOriginalEntityId") == r0.get_value("dukeOriginalEntityId")
    for p in procs:
        p.database.close()


def test_find_record_by_id_across_packing_paths():
    """An ID indexed through the Record path and re-posted through the native JSON path:
    findRecordById returns the live (re-posted) version -- the index's ID map is the one
    source of truth -- and a natively packed record's dukeDatasetId is its source's dataset
    id, also when that id contains "__" (IncrementalDataSource.java:90)."""
    with open(os.path.join(GOLDEN, "testdukeconfig_schema.json")) as f:
        cfg_d = json.load(f)["pipelines"]["Deduplication/countries-dbpedia-mondial"]
    cfg_d = json.loads(json.dumps(cfg_d))
    cfg_d["data_sources"][0]["dataset_id"] = "db__pedia"
    cfg = DukeConfig.from_dict(cfg_d)
    db = dh.GpuBlockingDatabase(cfg, [dh.PartsKey(("NAME", None, 0, 3))])
    proc = dh.GpuProcessor(cfg, db)
    src = cfg.data_sources[0]
    ents = stress_entities(200, 5)
    proc.deduplicate(dh.records_from_entities(ents, src))
    rid = db.find_record_by_id(f"db__pedia__{ents[7]['_id']}")
    assert rid is not None and rid.get_value("dukeDatasetId") == "db__pedia"
    changed = dict(ents[7])
    name_col = next(c for c in src.columns if c.property == "NAME")
    changed[name_col.name] = "Reposted Name"
    proc.deduplicate_json(json.dumps([changed]), src)
    r = db.find_record_by_id(f"db__pedia__{ents[7]['_id']}")
    want = dh.records_from_entities([changed], src)[0]
    assert r.get_value("NAME") == want.get_value("NAME") != rid.get_value("NAME")
    assert r.get_value("dukeDatasetId") == "db__pedia"
    assert r.get_value("dukeOriginalEntityId") == ents[7]["_id"]
    db.close()


class _LinkAdapter(dh.MatchListener):
    """Feeds the per-callback link-sink checker (oracle/linkdb_ref.py) from the replay."""

    def __init__(self, L):
        self.L, self.pos = L, {}

    def batch_ready(self, size):
        self.pos = {}
        self.L.batch_ready(size)

    def _q(self, r):
        return (self.pos.setdefault(id(r), len(self.pos)), r.get_value("ID"))

    def matches(self, r1, r2, c):
        self.L.matches(self._q(r1), r2.get_value("ID"), c)

    def matches_perhaps(self, r1, r2, c):
        self.L.matches_perhaps(self._q(r1), r2.get_value("ID"), c)

    def no_match_for(self, r):
        self.L.no_match_for(self._q(r))

    def batch_done(self):
        self.L.batch_done()


def test_link_database_written_in_bulk_equals_callbacks():
    """GpuProcessor with a LinkDatabase: after each deduplicate batch the bulk-written link
    database equals the per-callback LinkDatabaseMatchListener over the same replay."""
    import time
    import linkdb_ref as R
    from dukehip.links import LinkDatabase, interned_string
    p, props, vals, keys = persons_case(500, 250, 44)
    n = len(vals[0])
    cfg = dh.DukeConfig([dh.Property("NAME", dh.Comparator(DUKE_CMP + "JaroWinkler"), 0.1, 0.95),
                         dh.Property("ADDRESS", dh.Comparator(DUKE_CMP + "Levenshtein"), 0.2, 0.8),
                         dh.Property("DOB", dh.Comparator(DUKE_CMP + "Levenshtein"), 0.1, 0.85)],
                        threshold=0.9, maybe_threshold=0.7)
    kfs = [dh.PartsKey(("NAME", -1, 0, 3), ("DOB", None, 0, 4)),
           dh.PartsKey(("NAME", 0, 0, 2), ("DOB", None, 5, 10))]
    db = dh.GpuBlockingDatabase(cfg, kfs)
    proc = dh.GpuProcessor(cfg, db)
    ldb = LinkDatabase(db.ids)
    proc.set_link_database(ldb)
    ref = R.SinceAwareLinkDB()
    clock = {"t": 0}
    adapter = _LinkAdapter(R.LinkDBListener(ref, lambda: clock["t"]))
    proc.add_match_listener(adapter)
    rng = np.random.default_rng(44)
    ids = [f"ds__{i}" for i in range(n)]
    for bi, (a, b) in enumerate([(0, 300), (300, 600), (600, n), (0, 200)]):
        recs = []
        for i in range(a, b):
            j = i if bi < 3 else int(rng.integers(0, n))   # last batch re-posts, changed values
            recs.append(dh.Record({"ID": ids[i], "NAME": p["name"][j], "ADDRESS": p["address"][j],
                                   "DOB": p["dob"][j]}))
        clock["t"] = int(time.time() * 1000) + bi * 10   # timestamps are not compared
        before = len(ref.links)
        proc.deduplicate(recs)
        assert len(ref.links) >= before
    ch = ldb.changes_since(0)
    got = {(interned_string(db.ids, x), interned_string(db.ids, y)): (int(s), int(k), float(c))
           for x, y, s, k, c in zip(ch["id1"], ch["id2"], ch["status"], ch["kind"], ch["confidence"])}
    want = {l.key(): (l.status, l.kind, l.confidence) for l in ref.links.values()}
    assert got == want
    assert any(v[0] == R.RETRACTED for v in want.values())
    db.close()


@pytest.mark.gpu
def test_deduplicate_json_parallel_host_paths(monkeypatch):
    """Batches large enough for every parallel host path (chunked split, slice parse, merge,
    shard-parallel ID and key interning, parallel upsert staging): the POSTed-body path
    equals the Record path, including a second batch that re-posts half the IDs."""
    monkeypatch.setenv("DK_INGEST_THREADS", "8")
    with open(os.path.join(GOLDEN, "testdukeconfig_schema.json")) as f:
        cfg_d = json.load(f)["pipelines"]["Deduplication/countries-dbpedia-mondial"]
    kf = [dh.PartsKey(("NAME", None, 0, 4)), dh.PartsKey(("CAPITAL", None, 0, 3))]
    procs = []
    for _ in range(2):
        cfg = DukeConfig.from_dict(cfg_d)
        procs.append(dh.GpuProcessor(cfg, dh.GpuBlockingDatabase(cfg, kf)))
    first = stress_entities(36000, 21)
    second = stress_entities(36000, 22)
    for i, e in enumerate(second):
        if i % 2 == 0:
            e["_id"] = first[(i * 7) % len(first)]["_id"]   # re-posted IDs
    for ents in (first, second):
        body = json.dumps(ents)
        src0 = procs[0].config.data_sources[0]
        src1 = procs[1].config.data_sources[0]
        ref = procs[0].deduplicate(dh.records_from_entities(dh.parse_entities(body)[0], src0))
        got = procs[1].deduplicate_json(body, src1)
        assert got.n == ref.n and got.pairs_scored == ref.pairs_scored and got.n > 0
        for k in ("first", "candidate", "prob", "kind"):
            assert np.array_equal(getattr(got, k), getattr(ref, k)), k
    for p in procs:
        p.database.close()
