"""GPU parity: libdukehip.so (through its C-ABI) against the CPU oracle on the same
seeded inputs.  Integers / decisions / candidate sets bit-exact; probabilities compared
bit-exact as well (same operation order, no FMA) — the north star allows 1e-12 relative.

Oracle: oracle/duke_oracle.c, PARITY UNPINNED against Duke 1.2 itself (see its header).
"""
import ctypes as C
import random

import numpy as np
import pytest

import oracle as O
import dukehip as dh
from dukehip import _abi as A
from dukehip import synth

pytestmark = pytest.mark.gpu

LEV, JW, QG, EX, NUM = A.CMP_LEVENSHTEIN, A.CMP_JAROWINKLER, A.CMP_QGRAM, A.CMP_EXACT, A.CMP_NUMERIC
WL, DICE_T, JACC_T = A.CMP_WEIGHTED_LEVENSHTEIN, A.CMP_DICE_TOKENS, A.CMP_JACCARD_TOKENS
MODES = {"dedup": A.MODE_DEDUP, "linkage": A.MODE_LINKAGE, "allpairs": A.MODE_ALLPAIRS}


def schema_of(props, threshold, maybe, mode, nkeys):
    arr = (A.dk_property * max(1, len(props)))()
    for i, p in enumerate(props):
        arr[i] = A.dk_property(p["comparator"], p.get("q", 2), p.get("formula", 0),
                               p.get("tokenizer", 0), p["low"], p["high"], p.get("min_ratio", 0.0))
    s = A.dk_schema(len(props), arr, threshold, maybe, MODES[mode], nkeys)
    s._keep = arr
    return s


def run_both(props, values, keys=(), mode="dedup", group=None, deleted=None, ident=None,
             threshold=0.9, maybe=0.0, queries=None, batches=None):
    n = len(values[0])
    ident = np.arange(n, dtype=np.uint64) if ident is None else np.asarray(ident, np.uint64)
    eng = dh.GpuEngine(schema_of(props, threshold, maybe, mode, len(keys)))
    bounds = batches or [(0, n)]
    for a, b in bounds:
        eng.upsert(b - a, ident[a:b], [dh.Column.from_strings(v[a:b]) for v in values],
                   group=None if group is None else np.asarray(group[a:b], np.uint8),
                   deleted=None if deleted is None else np.asarray(deleted[a:b], np.uint8),
                   key_columns=[dh.Column.from_strings(k[a:b]) for k in keys] if keys else None)
    q = np.arange(n, dtype=np.uint32) if queries is None else np.asarray(queries, np.uint32)
    res = eng.match(q)
    # oracle: rows superseded by a later upsert of the same identity are not alive
    alive = np.ones(n, np.uint8)
    last = {}
    for r in range(n):
        if int(ident[r]) in last:
            alive[last[int(ident[r])]] = 0
        last[int(ident[r])] = r
    ot = O.OracleTable(props, values, keys=list(keys), ident=ident, group=group, deleted=deleted,
                       alive=alive, threshold=threshold, maybe=maybe, mode=mode)
    ref = ot.match(q)
    eng.close()
    return res, ref


def assert_same(res, ref):
    assert res.pairs_scored == ref["pairs_scored"]
    assert res.n == len(ref["query"])
    assert np.array_equal(res.query, ref["query"])
    assert np.array_equal(res.candidate, ref["candidate"])
    assert np.array_equal(res.kind, ref["kind"])
    a, b = res.prob, ref["prob"]
    same = (a == b) | (np.isnan(a) & np.isnan(b))
    if not same.all():
        i = int(np.argmin(same))
        raise AssertionError(f"prob differs at {i}: {a[i]!r} vs {b[i]!r}")


def rand_strings(rng, n, alpha, lo, hi, none_frac=0.0, empty_frac=0.0):
    out = []
    for _ in range(n):
        r = rng.random()
        if r < none_frac:
            out.append(None)
        elif r < none_frac + empty_frac:
            out.append("")
        else:
            out.append("".join(rng.choice(alpha) for _ in range(rng.randint(lo, hi))))
    return out


def allpairs_single(prop, vals):
    """Every ordered pair through the fused kernel with one property; threshold -1 so
    every non-NaN probability comes back."""
    return run_both([prop], [vals], mode="allpairs", threshold=-1.0)


@pytest.mark.parametrize("lo,hi", [(1, 3), (1, 16), (10, 32), (30, 64)])
def test_levenshtein_allpairs(lo, hi):
    rng = random.Random(lo * 100 + hi)
    vals = rand_strings(rng, 160, "abcd", lo, hi)
    res, ref = allpairs_single({"comparator": LEV, "low": 0.1, "high": 0.9}, vals)
    assert_same(res, ref)


def test_levenshtein_quirks():
    vals = ["a", "b", "ab", "aab", "kitten", "sitting", "x" * 64, "x" * 63 + "y", "abcdefgh",
            "badcfehg", "zz", "ba"]
    res, ref = allpairs_single({"comparator": LEV, "low": 0.0, "high": 1.0}, vals)
    assert_same(res, ref)


@pytest.mark.parametrize("alpha", ["ab", "abcdefgh", "abcdefghijklmnopqrstuvwxyz"])
def test_jarowinkler_allpairs(alpha):
    rng = random.Random(len(alpha))
    vals = rand_strings(rng, 150, alpha, 1, 24)
    res, ref = allpairs_single({"comparator": JW, "low": 0.1, "high": 0.95}, vals)
    assert_same(res, ref)


@pytest.mark.parametrize("q,formula,tok", [(2, 0, 0), (2, 1, 0), (2, 2, 0), (3, 1, 0), (1, 2, 0),
                                           (4, 0, 0), (2, 0, 1), (3, 2, 1)])
def test_qgram_allpairs(q, formula, tok):
    rng = random.Random(q * 10 + formula + 100 * tok)
    vals = rand_strings(rng, 120, "abc", 0, 12)
    vals = [v for v in vals if v] + ["a"]
    res, ref = allpairs_single({"comparator": QG, "low": 0.2, "high": 0.8, "q": q,
                                "formula": formula, "tokenizer": tok}, vals)
    assert_same(res, ref)


def test_numeric_and_exact():
    nums = ["1", "2", "0", "-0", "0.0", "-3", "-4.5", "1e3", "1000", "abc", " 7 ", "7f", "NaN",
            "Infinity", "-Infinity", "0x1p3", "8", "1e", "", "1.", ".5", "0.5d", "3.3", "3.30"]
    res, ref = allpairs_single({"comparator": NUM, "low": 0.04, "high": 0.73, "min_ratio": 0.0}, nums)
    assert_same(res, ref)
    res, ref = allpairs_single({"comparator": NUM, "low": 0.04, "high": 0.73, "min_ratio": 0.7}, nums)
    assert_same(res, ref)
    res, ref = allpairs_single({"comparator": EX, "low": 0.3, "high": 0.9}, nums)
    assert_same(res, ref)


def test_utf16_and_surrogates():
    rng = random.Random(5)
    alpha = ["a", "b", "ł", "\U0001F600", "é"]
    vals = ["".join(rng.choice(alpha) for _ in range(rng.randint(1, 10))) for _ in range(80)]
    for prop in ({"comparator": LEV, "low": 0.1, "high": 0.9},
                 {"comparator": JW, "low": 0.1, "high": 0.9},
                 {"comparator": QG, "low": 0.1, "high": 0.9, "q": 2, "formula": 1}):
        res, ref = allpairs_single(prop, vals)
        assert_same(res, ref)


def test_missing_and_empty_values():
    rng = random.Random(9)
    props = [{"comparator": LEV, "low": 0.1, "high": 0.9},
             {"comparator": JW, "low": 0.2, "high": 0.8},
             {"comparator": NUM, "low": 0.3, "high": 0.7}]
    n = 120
    vals = [rand_strings(rng, n, "ab", 1, 6, none_frac=0.2, empty_frac=0.1),
            rand_strings(rng, n, "ab", 1, 6, none_frac=0.2, empty_frac=0.1),
            [None if rng.random() < 0.2 else str(rng.randint(0, 5)) for _ in range(n)]]
    res, ref = run_both(props, vals, mode="allpairs", threshold=0.6, maybe=0.4)
    assert_same(res, ref)


def persons_case(n_orig, n_dup, seed):
    p = synth.persons(n_orig, n_dup, seed=seed)
    props = [{"comparator": JW, "low": 0.1, "high": 0.95},
             {"comparator": LEV, "low": 0.2, "high": 0.8},
             {"comparator": LEV, "low": 0.1, "high": 0.85}]
    return p, props, [p["name"], p["address"], p["dob"]], synth.keys_config2(p)


@pytest.mark.parametrize("seed", [1, 2])
def test_dedup_blocking_persons(seed):
    p, props, vals, keys = persons_case(1500, 500, seed)
    res, ref = run_both(props, vals, keys, threshold=0.9, maybe=0.7)
    assert res.n > 0
    assert_same(res, ref)


def test_dedup_deleted_and_upsert_batches():
    p, props, vals, keys = persons_case(700, 300, 3)
    n = len(vals[0])
    rng = np.random.default_rng(3)
    deleted = (rng.random(n) < 0.05).astype(np.uint8)
    ident = np.arange(n, dtype=np.uint64)
    ident[-50:] = ident[:50]   # later batch re-upserts 50 IDs (delete-then-add)
    res, ref = run_both(props, vals, keys, deleted=deleted, ident=ident, threshold=0.9,
                        maybe=0.7, batches=[(0, 400), (400, 750), (750, n)],
                        queries=np.arange(750, n))
    assert_same(res, ref)


def test_linkage_blocking():
    p, props, vals, keys = persons_case(800, 400, 4)
    n = len(vals[0])
    group = np.where(np.arange(n) % 3 == 0, 1, 2).astype(np.uint8)
    res, ref = run_both(props, vals, keys, mode="linkage", group=group, threshold=0.9, maybe=0.7)
    assert res.n > 0
    assert_same(res, ref)


def test_allpairs_short_strings():
    rng = random.Random(11)
    vals = rand_strings(rng, 400, "abcdefghij", 4, 16)
    res, ref = run_both([{"comparator": LEV, "low": 0.05, "high": 0.95}], [vals],
                        mode="allpairs", threshold=0.85)
    assert_same(res, ref)


def test_small_chunks_match_single_chunk(monkeypatch):
    p, props, vals, keys = persons_case(600, 200, 5)
    monkeypatch.setenv("DK_CHUNK_SLOTS", "1000")
    res, ref = run_both(props, vals, keys, threshold=0.9, maybe=0.7)
    assert_same(res, ref)


def test_empty_batch_and_no_candidates():
    props = [{"comparator": LEV, "low": 0.1, "high": 0.9}]
    res, ref = run_both(props, [["abc", "abd", "xyz"]], [["k1", "k2", "k3"]])
    assert res.pairs_scored == 0 and res.n == 0
    assert_same(res, ref)


def test_compare_rows_matches_oracle():
    p, props, vals, keys = persons_case(50, 20, 6)
    eng = dh.GpuEngine(schema_of(props, 0.9, 0.7, "dedup", 2))
    n = len(vals[0])
    eng.upsert(n, np.arange(n), [dh.Column.from_strings(v) for v in vals],
               key_columns=[dh.Column.from_strings(k) for k in keys])
    ot = O.OracleTable(props, vals, keys=keys)
    for a, b in [(0, 1), (3, 7), (10, 10), (60, 2)]:
        assert eng.compare_rows(a, b) == ot.compare_rows(a, b)
    eng.close()


def test_processor_replay_order():
    """GpuProcessor.deduplicate replays batchReady / per-record callbacks / batchDone."""
    cfg = dh.DukeConfig([dh.Property("NAME", dh.Comparator("no.priv.garshol.duke.comparators.Levenshtein"), 0.1, 0.9)],
                        threshold=0.6, maybe_threshold=0.5)
    recs = [dh.Record({"ID": f"d__{i}", "NAME": v}) for i, v in
            enumerate(["anna", "anne", "bob", "anna", "annie"])]
    db = dh.GpuBlockingDatabase(cfg, [dh.PartsKey(("NAME", None, 0, 1))])
    proc = dh.GpuProcessor(cfg, db)
    lis = dh.CollectingListener()
    proc.add_match_listener(lis)
    proc.deduplicate(recs)
    ev = lis.events
    assert ev[0] == ("batchReady", 5) and ev[-1] == ("batchDone",)
    assert ("noMatchFor", "d__2") in ev
    qs = [e[1] for e in ev[1:-1]]
    assert qs == sorted(qs, key=lambda x: int(x.split("__")[1]))  # grouped in batch order
    db.close()


def mutate(rng, s, k, alpha):
    b = list(s)
    for _ in range(k):
        r = rng.random()
        if b and r < 0.35:
            del b[rng.randrange(len(b))]
        elif b and r < 0.7:
            b[rng.randrange(len(b))] = rng.choice(alpha)
        else:
            b.insert(rng.randrange(len(b) + 1), rng.choice(alpha))
    return "".join(b)


def families(rng, nbase, per, alpha, lo, hi, edits, cap):
    """Base strings plus edited copies, so that many pairs are similar enough to reach
    the DP (and the >= 0.5 similarity branch of PropertyImpl)."""
    out = []
    for _ in range(nbase):
        base = "".join(rng.choice(alpha) for _ in range(rng.randint(lo, hi)))
        out.append(base[:cap])
        for _ in range(per):
            out.append((mutate(rng, base, rng.randint(0, edits), alpha) or "z")[:cap])
    return out


WL_ALPHA = "abcdef 01.-/'" + '"\\,'


@pytest.mark.parametrize("lo,hi", [(1, 3), (1, 16), (10, 40), (30, 64), (60, 130), (120, 256)])
def test_weighted_levenshtein_allpairs(lo, hi):
    rng = random.Random(lo * 1000 + hi)
    vals = families(rng, 20, 5, WL_ALPHA, lo, hi, max(2, hi // 8), 256)
    res, ref = allpairs_single({"comparator": WL, "low": 0.1, "high": 0.9}, vals)
    assert_same(res, ref)


def test_weighted_levenshtein_quirks_and_utf16():
    vals = ["a", "b", "ab", "ba", "a.", "1", "12", "x" * 256, "x" * 255 + "y", "é", "\U0001F600a",
            "a\U0001F600", "o'neil-smith", "oneil smith", "a b", "ab ", " ", "\\", "/"]
    res, ref = allpairs_single({"comparator": WL, "low": 0.0, "high": 1.0}, vals)
    assert_same(res, ref)


@pytest.mark.parametrize("lo,hi", [(60, 100), (65, 128), (120, 256)])
def test_levenshtein_long_allpairs(lo, hi):
    """Query values over 64 units take the long-value DP (no cutoff replay)."""
    rng = random.Random(hi)
    vals = families(rng, 16, 6, "abcd", lo, hi, hi // 6, 256)
    res, ref = allpairs_single({"comparator": LEV, "low": 0.1, "high": 0.9}, vals)
    assert_same(res, ref)


def test_long_and_short_properties_fused():
    """WeightedLevenshtein + long Levenshtein + JaroWinkler + QGram in one kernel, with
    missing values, under blocking."""
    rng = random.Random(77)
    n = 600
    text = families(rng, 60, 9, WL_ALPHA, 20, 200, 12, 256)[:n]
    lev = families(rng, 60, 9, "abc", 50, 120, 10, 256)[:n]
    name = families(rng, 60, 9, "abcdefg", 3, 12, 2, 64)[:n]
    for col in (text, lev):
        for i in range(0, n, 17):
            col[i] = None
    keys = [[("k%d" % (i % 40)) for i in range(n)]]
    props = [{"comparator": WL, "low": 0.2, "high": 0.9},
             {"comparator": LEV, "low": 0.1, "high": 0.8},
             {"comparator": JW, "low": 0.3, "high": 0.7},
             {"comparator": QG, "low": 0.4, "high": 0.6, "q": 3, "formula": 1}]
    res, ref = run_both(props, [text, lev, name, text], keys, threshold=0.6, maybe=0.3)
    assert res.n > 0
    assert_same(res, ref)


@pytest.mark.parametrize("long_cmp", [WL, LEV])
def test_long_dp_variants_blocked(long_cmp):
    """One long-DP property under blocking, query values of 1 to 256 units (every one of the
    twelve DP variants), with missing values, beside a short Levenshtein / JaroWinkler / QGram
    property; bit-exact against the oracle."""
    rng = random.Random(long_cmp * 7 + 3)
    n = 900
    lo = 1 if long_cmp == WL else 40
    text = families(rng, 90, 9, WL_ALPHA if long_cmp == WL else "abcd", lo, 256, 14, 256)[:n]
    short = families(rng, 90, 9, "abcdefg", 3, 30, 3, 64)[:n]
    for i in range(0, n, 19):
        text[i] = None
    keys = [[("k%d" % (i % 45)) for i in range(n)]]
    props = [{"comparator": long_cmp, "low": 0.2, "high": 0.9},
             {"comparator": LEV if long_cmp == WL else JW, "low": 0.3, "high": 0.7},
             {"comparator": QG, "low": 0.4, "high": 0.6, "q": 3, "formula": 1}]
    res, ref = run_both(props, [text, short, text], keys, threshold=0.6, maybe=0.3)
    assert res.n > 0
    assert_same(res, ref)


@pytest.mark.parametrize("cmp", [DICE_T, JACC_T])
def test_token_comparators_allpairs(cmp):
    rng = random.Random(cmp)
    words = ["oslo", "bergen", "a", "b", "gate", "vei", "ø", "\U0001F600"]
    vals = []
    for _ in range(140):
        k = rng.randint(0, 6)
        sep = [" ", "  ", " "][rng.randint(0, 2)]
        v = sep.join(rng.choice(words) for _ in range(k))
        if rng.random() < 0.2:
            v = " " + v + " "
        vals.append(v if v else " ")
    vals += ["a a b", "a b", "b a", " ", "  "]
    res, ref = allpairs_single({"comparator": cmp, "low": 0.1, "high": 0.9}, vals)
    assert_same(res, ref)


@pytest.mark.parametrize("q,formula", [(1, 0), (2, 1), (3, 2), (4, 0)])
def test_qgram_ends_allpairs(q, formula):
    rng = random.Random(q * 7 + formula)
    vals = [v for v in rand_strings(rng, 120, "ab^$", 1, 10) if v]
    res, ref = allpairs_single({"comparator": QG, "low": 0.2, "high": 0.8, "q": q,
                                "formula": formula, "tokenizer": A.QGRAM_ENDS}, vals)
    assert_same(res, ref)


@pytest.mark.parametrize("cmp", [LEV, WL])
def test_unsupported_value_length(cmp):
    eng = dh.GpuEngine(schema_of([{"comparator": cmp, "low": 0.1, "high": 0.9}], 0.9, 0.0, "dedup", 1))
    eng.upsert(1, [0], [dh.Column.from_strings(["x" * 256])], key_columns=[dh.Column.from_strings(["k"])])
    with pytest.raises(dh.DukeHipError):
        eng.upsert(1, [1], [dh.Column.from_strings(["x" * 257])], key_columns=[dh.Column.from_strings(["k"])])
    eng.close()


def test_transient_rows_httptransform_mode():
    """dk_upsert_transient (setIndexingIsDisabled(true), App.java:1130-1132): the batch is
    matched against the index without entering it, then dropped; the index is unchanged."""
    p, props, vals, keys = persons_case(900, 300, 12)
    n = len(vals[0])
    n1, m = 800, n - 800
    group = np.where(np.arange(n) % 2 == 0, 1, 2).astype(np.uint8)
    ident = np.arange(n, dtype=np.uint64)
    ident[n1:n1 + 40] = ident[:40]        # posted again: isSameAs skips the indexed version
    eng = dh.GpuEngine(schema_of(props, 0.9, 0.7, "linkage", len(keys)))

    def up(a, b, transient=False):
        return eng.upsert(b - a, ident[a:b], [dh.Column.from_strings(v[a:b]) for v in vals],
                          group=group[a:b], key_columns=[dh.Column.from_strings(k[a:b]) for k in keys],
                          transient=transient)

    up(0, n1)
    rows = up(n1, n, transient=True)
    assert list(rows) == list(range(n1, n))
    with pytest.raises(dh.DukeHipError):
        up(0, 10)                         # indexing refused while transient rows exist
    res = eng.match(rows)
    alive = np.r_[np.ones(n1, np.uint8), np.zeros(m, np.uint8)]
    ot = O.OracleTable(props, vals, keys=list(keys), ident=ident, group=group, alive=alive,
                       threshold=0.9, maybe=0.7, mode="linkage")
    ref = ot.match(rows)
    assert res.n > 0
    assert_same(res, ref)
    res.close()
    # queries from the index itself never see the transient rows
    q = np.arange(0, n1, 7, dtype=np.uint32)
    assert_same(eng.match(q), ot.match(q))
    eng.drop_transient()
    assert eng.num_rows == n1
    # the arenas are reused: a normal batch after the drop scores like a fresh index
    up(n1, n)
    alive2 = np.ones(n, np.uint8)
    alive2[:40] = 0                       # superseded by the re-posted IDs
    ot2 = O.OracleTable(props, vals, keys=list(keys), ident=ident, group=group, alive=alive2,
                        threshold=0.9, maybe=0.7, mode="linkage")
    q = np.arange(n, dtype=np.uint32)
    assert_same(eng.match(q), ot2.match(q))
    eng.close()


def test_httptransform_duke_links_bulk_equals_listener():
    """GpuProcessor with indexing disabled -> entity_links from the match arrays equals
    BaseLinkDatabaseMatchListener's per-callback map; the index is left unchanged."""
    from dukehip import links as L
    from dukehip.config import DataSource, DataSourceColumn
    cfg = dh.DukeConfig([dh.Property("NAME", dh.Comparator("no.priv.garshol.duke.comparators.JaroWinkler"), 0.1, 0.95),
                         dh.Property("ADDRESS", dh.Comparator("no.priv.garshol.duke.comparators.Levenshtein"), 0.2, 0.8)],
                        threshold=0.85, maybe_threshold=0.6, linkage=True)
    p = synth.persons(300, 150, seed=21)
    n = len(p["name"])
    ents = [{"_id": str(i), "name": p["name"][i], "address": p["address"][i], "extra": None}
            for i in range(n)]
    cols = [DataSourceColumn("name", "NAME", None), DataSourceColumn("address", "ADDRESS", None)]
    src1 = DataSource("crm", cols, 1)
    src2 = DataSource("erp", cols, 2)
    db = dh.GpuBlockingDatabase(cfg, [dh.PartsKey(("NAME", None, 0, 2))])
    proc = dh.GpuProcessor(cfg, db)
    proc.deduplicate(dh.records_from_entities(ents[:300], src1))
    before = db.engine.num_rows
    lis = L.EntityLinksListener()
    proc.add_match_listener(lis)
    db.set_indexing_is_disabled(True)
    recs = dh.records_from_entities(ents[300:], src2)
    res = proc.deduplicate(recs)
    db.set_indexing_is_disabled(False)
    assert db.engine.num_rows == before and len(db.rows) == before
    bulk = L.entity_links(res, recs, db.rows)
    assert bulk == lis.links() and len(bulk) > 0
    body = L.http_transform_response(ents[300:], False, bulk)
    assert '"duke_links":[{"datasetId":"crm"' in body and '"extra"' not in body
    db.close()


def test_result_region_matches_pool(monkeypatch):
    """dk_set_result_region: the list lands in caller memory (here an anonymous mmap, as a
    rank's slice of the node-wide shared mapping is) identical to the pooled host result;
    a list that does not fit fails with DK_E_NOMEM, too many queries with DK_E_INVALID."""
    import mmap
    p, props, vals, keys = persons_case(900, 300, 8)
    monkeypatch.setenv("DK_CHUNK_SLOTS", "4096")   # several overlapped chunk copies
    n = len(vals[0])
    eng = dh.GpuEngine(schema_of(props, 0.9, 0.7, "dedup", 2))
    eng.upsert(n, np.arange(n), [dh.Column.from_strings(v) for v in vals],
               key_columns=[dh.Column.from_strings(k) for k in keys])
    q = np.arange(n, dtype=np.uint32)
    ref = eng.match(q)
    ref_arrays = [ref.first.copy(), ref.candidate.copy(), ref.prob.copy(), ref.kind.copy()]
    ref.close()
    assert len(ref_arrays[1]) > 0
    buf = mmap.mmap(-1, A.region_bytes(n, len(ref_arrays[1]) + 100))
    eng.set_result_region(buf, n)
    for _ in range(2):
        res = eng.match(q)
        v = A.region_views(buf, n, n, res.n)
        for got, want in zip((res.first, res.candidate, res.prob, res.kind), ref_arrays):
            assert np.array_equal(got, want)
        for got, want in zip((v["first"], v["candidate"], v["prob"], v["kind"]), ref_arrays):
            assert np.array_equal(got, want)
        res.close()
    with pytest.raises(A.DukeHipError) as e:
        eng.match(np.arange(n + 1, dtype=np.uint32) % n)
    assert e.value.code == A.DK_E_INVALID
    small = mmap.mmap(-1, A.region_bytes(n, 10))
    eng.set_result_region(small, n)
    with pytest.raises(A.DukeHipError) as e:
        eng.match(q)
    assert e.value.code == A.DK_E_NOMEM
    eng.set_result_region(None, 0)
    res = eng.match(q)
    assert np.array_equal(res.prob, ref_arrays[2])
    res.close()
    eng.close()


def test_tables_rebuilt_after_each_upsert():
    """The blocking tables are index state reused across dk_match calls; every upsert
    (incl. re-upserted IDs and deleted rows) must be visible to the next match."""
    p, props, vals, keys = persons_case(600, 300, 9)
    n = len(vals[0])
    rng = np.random.default_rng(9)
    deleted = (rng.random(n) < 0.05).astype(np.uint8)
    ident = np.arange(n, dtype=np.uint64)
    ident[700:740] = ident[:40]
    eng = dh.GpuEngine(schema_of(props, 0.9, 0.7, "dedup", len(keys)))
    for a, b in [(0, 500), (500, 800), (800, n)]:
        eng.upsert(b - a, ident[a:b], [dh.Column.from_strings(v[a:b]) for v in vals],
                   deleted=deleted[a:b],
                   key_columns=[dh.Column.from_strings(k[a:b]) for k in keys])
        alive = np.ones(b, np.uint8)
        last = {}
        for r in range(b):
            if int(ident[r]) in last:
                alive[last[int(ident[r])]] = 0
            last[int(ident[r])] = r
        ot = O.OracleTable(props, [v[:b] for v in vals], keys=[k[:b] for k in keys],
                           ident=ident[:b], deleted=deleted[:b], alive=alive,
                           threshold=0.9, maybe=0.7)
        for q in (np.arange(a, b, dtype=np.uint32), np.arange(0, b, 3, dtype=np.uint32)):
            res = eng.match(q)   # the second match reuses the tables the first one built
            assert_same(res, ot.match(q))
            res.close()
    eng.close()


LATIN1 = "abcdefghijklmnopqrstuvwxyz éßÿ0123"


@pytest.mark.parametrize("formula,tok", [(0, A.QGRAM_BASIC), (1, A.QGRAM_BASIC), (2, A.QGRAM_BASIC),
                                         (1, A.QGRAM_ENDS)])
def test_qgram_bigram_keys_allpairs(formula, tok):
    """Latin-1 bigrams take the 16-bit-key replica and the per-row perfect hash (tables of
    256 and 512 slots: sets of up to 64 grams), including the key-0 bigram U+00FF U+00FF
    (its rows get no seed and read the candidate sets in place), one-gram and empty sets."""
    rng = random.Random(formula * 3 + tok)
    vals = [v for v in rand_strings(rng, 140, LATIN1, 1, 66) if v]
    vals += ["ÿÿ", "aÿÿb", "ÿÿÿÿ", "ab", "a", "ÿ", "ba", "aba", "é" * 40, LATIN1 * 2]
    res, ref = allpairs_single({"comparator": QG, "low": 0.2, "high": 0.8, "q": 2,
                                "formula": formula, "tokenizer": tok}, vals)
    assert_same(res, ref)


def test_qgram_bigram_keys_widened_arena():
    """A UTF-16 value arriving in a later batch widens the property's arena: the bigram-key
    replica and its seeds are then no longer used (the next match rebuilds the replica with
    u32 codes); both matches equal the oracle."""
    rng = random.Random(77)
    vals = [v for v in rand_strings(rng, 300, LATIN1, 2, 30) if v]
    keys = [v[:1] for v in vals]
    n = len(vals)
    prop = {"comparator": QG, "low": 0.2, "high": 0.8, "q": 2, "formula": 2}
    res, ref = run_both([prop], [vals], keys=[keys], threshold=0.5, maybe=0.3)
    assert_same(res, ref)
    vals2 = vals + ["Ā" + v for v in vals[:40]]
    keys2 = keys + keys[:40]
    res, ref = run_both([prop], [vals2], keys=[keys2], threshold=0.5, maybe=0.3,
                        batches=[(0, n), (n, len(vals2))])
    assert_same(res, ref)


@pytest.mark.parametrize("mode", ["dedup", "linkage"])
def test_order_classes_wide_schema(mode):
    """Past 12 record keys: 14 scored properties, rows missing values,
    each row in the order class of its HashMap capacity (16 for <= 12 keys, 32 past that);
    Processor.compare visits the QUERY record's order, so the kernels must pick the order
    per query row.  Compared bit-exact with the oracle fed the same per-row classes, and
    shown to matter: the same rows all in class 0 give different probabilities."""
    from dukehip import config as cfgmod
    rng = random.Random(14)
    n = 700
    kinds = [LEV, JW, EX, NUM, QG, LEV, JW, LEV, EX, QG, LEV, JW, NUM, LEV]
    props = [{"comparator": c, "low": 0.2 + 0.01 * i, "high": 0.8 + 0.01 * i} for i, c in enumerate(kinds)]
    pool = rand_strings(rng, 40, "abcde", 2, 9)
    vals = []
    for p in props:
        col = []
        for _ in range(n):
            if rng.random() < 0.3:
                col.append(None)
            elif p["comparator"] == NUM:
                col.append(str(rng.randint(1, 60)))
            else:
                col.append(rng.choice(pool))
        vals.append(col)
    names = [f"P{i}" for i in range(len(props))]
    extra = [cfgmod.ID_PROPERTY, cfgmod.ORIGINAL_ENTITY_ID_PROPERTY_NAME, cfgmod.DATASET_ID_PROPERTY_NAME]
    orders = []
    for cap in (16, 32):
        o = cfgmod.java_hashmap_order(names + extra + [cfgmod.DELETED_PROPERTY_NAME], cap)
        orders.append([names.index(k) for k in o if k in names])
    assert orders[0] != orders[1]
    nvals = np.array([sum(v[r] is not None for v in vals) for r in range(n)])
    oclass = (nvals + len(extra) > 12).astype(np.uint8)
    assert 0 < oclass.sum() < n
    keys = [[rng.choice("xyz") for _ in range(n)]]
    group = [1 + (r % 2) for r in range(n)] if mode == "linkage" else None
    ident = np.arange(n, dtype=np.uint64)

    def run(oc):
        s = schema_of(props, 0.7, 0.4, mode, len(keys))
        flat = (C.c_int * (2 * len(props)))(*[x for o in orders for x in o])
        s.norders, s.orders, s._orders = 2, flat, flat
        eng = dh.GpuEngine(s)
        eng.upsert(n, ident, [dh.Column.from_strings(v) for v in vals],
                   group=None if group is None else np.asarray(group, np.uint8),
                   key_columns=[dh.Column.from_strings(k) for k in keys], order_class=oc)
        res = eng.match(np.arange(n, dtype=np.uint32))
        cv = [eng.compare_values([dh.Column.from_strings([v[a], v[b]]) for v in vals],
                                 order_class=(int(oc[a]), int(oc[b]))) for a, b in ((0, 1), (5, 9), (17, 3))]
        eng.close()
        return res, cv

    res, cv = run(oclass)
    ot = O.OracleTable(props, vals, keys=keys, ident=ident, group=group, threshold=0.7, maybe=0.4,
                       mode=mode, orders=orders, oclass=oclass)
    ref = ot.match(np.arange(n, dtype=np.uint32))
    assert len(ref["query"]) > 50
    assert_same(res, ref)
    for (a, b), got in zip(((0, 1), (5, 9), (17, 3)), cv):
        want = ot.compare_rows(a, b)
        assert got == want or (np.isnan(got) and np.isnan(want))
    flat, _ = run(np.zeros(n, np.uint8))
    assert not (np.array_equal(flat.candidate, res.candidate) and np.array_equal(flat.prob, res.prob))


@pytest.mark.parametrize("variant", ["gq", "grouped", "grouped_row1", "grouped_row2"])
def test_order_classes_grouped(variant, monkeypatch):
    """the order classes through the grouped kernels -- two bigram QGram and three
    Numeric properties (k_score_gq's roles; k_score_grouped with DK_GQ=0, its head / tail
    and per-row resources with DK_GROUPED_ROW=1 / 2) in records of
    more than 12 keys (the unscored columns count), each row in its HashMap capacity's class,
    bit-exact against the oracle fed the same classes; the two classes' orders differ."""
    from dukehip import config as cfgmod
    env = {"grouped": [("DK_GQ", "0")], "grouped_row1": [("DK_GQ", "0"), ("DK_GROUPED_ROW", "1")],
           "grouped_row2": [("DK_GQ", "0"), ("DK_GROUPED_ROW", "2")]}.get(variant, [])
    for kv in env:
        monkeypatch.setenv(*kv)
    rng = random.Random(23)
    n = 1200
    props = [{"comparator": QG, "low": 0.15, "high": 0.92, "q": 2, "formula": A.QGRAM_DICE},
             {"comparator": QG, "low": 0.1, "high": 0.85, "q": 2, "formula": A.QGRAM_JACCARD},
             {"comparator": NUM, "low": 0.3, "high": 0.7, "min_ratio": 0.8},
             {"comparator": NUM, "low": 0.35, "high": 0.65, "min_ratio": 0.5},
             {"comparator": NUM, "low": 0.4, "high": 0.75, "min_ratio": 0.9}]
    names = ["NAME", "ADDRESS", "AGE", "ZIP", "SCORE"]
    unscored = [f"COL{i}" for i in range(8)]   # columns no property scores: record keys only
    extra = [cfgmod.ID_PROPERTY, cfgmod.ORIGINAL_ENTITY_ID_PROPERTY_NAME, cfgmod.DATASET_ID_PROPERTY_NAME]
    allkeys = names + unscored + extra + [cfgmod.DELETED_PROPERTY_NAME]
    orders = []
    for cap in (16, 32):
        o = cfgmod.java_hashmap_order(allkeys, cap)
        orders.append([names.index(k) for k in o if k in names])
    assert orders[0] != orders[1]
    pool = rand_strings(rng, 60, "abcdefgh", 3, 12)
    vals = []
    for p in props:
        col = []
        for _ in range(n):
            if rng.random() < 0.2:
                col.append(None)
            elif p["comparator"] == NUM:
                col.append(str(rng.randint(20, 40)))
            else:
                col.append(rng.choice(pool))
        vals.append(col)
    # a record's keys: its values, 0-8 unscored columns, the synthetic ones
    nun = np.array([rng.randint(0, 8) for _ in range(n)])
    nvals = np.array([sum(v[r] is not None for v in vals) for r in range(n)])
    oclass = (nvals + nun + len(extra) > 12).astype(np.uint8)
    assert 0 < oclass.sum() < n
    keys = [[rng.choice("pqrs") for _ in range(n)]]
    group = [1 + (r % 2) for r in range(n)]
    ident = np.arange(n, dtype=np.uint64)
    s = schema_of(props, 0.8, 0.5, "linkage", len(keys))
    flat = (C.c_int * (2 * len(props)))(*[x for o in orders for x in o])
    s.norders, s.orders, s._orders = 2, flat, flat
    eng = dh.GpuEngine(s)
    eng.upsert(n, ident, [dh.Column.from_strings(v) for v in vals], group=np.asarray(group, np.uint8),
               key_columns=[dh.Column.from_strings(k) for k in keys], order_class=oclass)
    res = eng.match(np.arange(n, dtype=np.uint32))
    eng.close()
    ot = O.OracleTable(props, vals, keys=keys, ident=ident, group=group, threshold=0.8, maybe=0.5,
                       mode="linkage", orders=orders, oclass=oclass)
    ref = ot.match(np.arange(n, dtype=np.uint32))
    assert len(ref["query"]) > 50
    assert_same(res, ref)


def assert_close(res, ref, thresholds, rel=1e-12, edge=1e-9):
    """The north star's floating-point bar for comparators on sin / cos / atan2: candidate
    sets equal, probabilities within 1e-12 relative, decisions equal except for pairs within
    1e-9 of a threshold."""
    got = {(int(q), int(c)): (float(p), int(k)) for q, c, p, k in zip(res.query, res.candidate, res.prob, res.kind)}
    want = {(int(q), int(c)): (float(p), int(k)) for q, c, p, k in
            zip(ref["query"], ref["candidate"], ref["prob"], ref["kind"])}
    assert res.pairs_scored == ref["pairs_scored"]
    near = lambda p: any(abs(p - t) <= edge for t in thresholds)
    for key in set(got) | set(want):
        if key not in got or key not in want:
            p = (got.get(key) or want.get(key))[0]
            assert near(p), (key, got.get(key), want.get(key))
            continue
        (a, ka), (b, kb) = got[key], want[key]
        assert abs(a - b) <= rel * abs(b), (key, a, b)
        assert ka == kb or near(b), (key, ka, kb)


@pytest.mark.parametrize("mode", ["dedup", "allpairs"])
def test_geoposition(mode):
    """GeopositionComparator (parity unpinned: the formula is recalled,
    see oracle/duke_oracle.c dko_geoposition): positions scattered within a few km, some
    unparsable ("x,1" -> 0.5) and some missing, next to a Levenshtein name; the GPU path
    against the oracle at the north star's tolerance, and each similarity through
    dk_property_similarity.  A value without ',' is accepted; comparing it fails the call
    (stock Duke raises there)."""
    rng = random.Random(31)
    n = 600
    pos = []
    for _ in range(n):
        r = rng.random()
        if r < 0.1:
            pos.append(None)
        elif r < 0.15:
            pos.append(f"x{rng.randint(0, 9)},{rng.uniform(0, 1):.4f}")
        else:
            base = rng.choice([(59.91, 10.75), (60.39, 5.32), (-33.86, 151.2)])
            pos.append(f"{base[0] + rng.uniform(-0.03, 0.03):.6f},{base[1] + rng.uniform(-0.03, 0.03):.6f}")
    names = rand_strings(rng, n, "abc", 3, 6, none_frac=0.05)
    props = [{"comparator": A.CMP_GEOPOSITION, "low": 0.1, "high": 0.95, "min_ratio": 4000.0},
             {"comparator": LEV, "low": 0.3, "high": 0.8}]
    keys = [[rng.choice("pq") for _ in range(n)]] if mode == "dedup" else []
    res, ref = run_both(props, [pos, names], keys=keys, mode=mode, threshold=0.8, maybe=0.6)
    assert len(ref["query"]) > 100
    assert_close(res, ref, (0.8, 0.6))
    eng = dh.GpuEngine(schema_of(props, 0.8, 0.6, "allpairs", 0))
    eng.upsert(60, np.arange(60, dtype=np.uint64), [dh.Column.from_strings(v[:60]) for v in (pos, names)])
    for a, b in [(i, j) for i in range(0, 60, 7) for j in range(1, 60, 5)]:
        got = eng.property_similarity(0, a, b)
        if pos[a] is None or pos[b] is None:
            assert got != got
            continue
        want = O.geoposition(pos[a], pos[b], 4000.0)
        assert abs(got - want) <= 1e-12 * abs(want), (pos[a], pos[b], got, want)
    # a value without ',' (ADVICE r4): accepted at upsert; stock Duke raises only when it
    # compares it (Geoposition.parse), so does the GPU path -- here every pair is compared
    rows = eng.upsert(1, np.array([99], np.uint64), [dh.Column.from_strings(["59.9"]), dh.Column.from_strings(["a"])])
    with pytest.raises(dh.DukeHipError) as e:
        eng.property_similarity(0, int(rows[0]), 1)
    assert e.value.code == A.DK_E_UNSUPPORTED
    with pytest.raises(dh.DukeHipError) as e:
        eng.match(np.arange(61, dtype=np.uint32))
    assert e.value.code == A.DK_E_UNSUPPORTED
    a, b = [i for i in range(60) if pos[i] is not None][:2]   # others still fine
    got, want = eng.property_similarity(0, a, b), O.geoposition(pos[a], pos[b], 4000.0)
    assert abs(got - want) <= 1e-12 * abs(want), (got, want)
    eng.close()
    # key blocking: the record's key is its own, it is never compared, the batch scores as
    # without it (bit-exact against the oracle on the rest)
    if mode == "dedup":
        eng = dh.GpuEngine(schema_of(props, 0.8, 0.6, "dedup", 1))
        eng.upsert(n + 1, np.arange(n + 1, dtype=np.uint64),
                   [dh.Column.from_strings(pos + ["59.9"]), dh.Column.from_strings(names + ["a"])],
                   key_columns=[dh.Column.from_strings(keys[0] + ["zzz"])])
        res2 = eng.match(np.arange(n + 1, dtype=np.uint32))
        assert res2.pairs_scored == res.pairs_scored
        assert np.array_equal(res2.candidate, res.candidate) and np.array_equal(res2.prob, res.prob)
        eng.close()


@pytest.mark.parametrize("dups", [False, True])
def test_large_batch_identity_map(dups):
    """dk_upsert resolves a batch of >= 65536 dense identities on parallel ranges when none
    repeats inside the batch (identities re-posted from an earlier batch become tombstones),
    and falls back to the serial loop when one does: the match list against the oracle's
    alive rows either way."""
    rng = random.Random(70 + int(dups))
    n1 = n2 = 70000
    n = n1 + n2
    vals = ["".join(rng.choice("abcdefghij") for _ in range(3)) for _ in range(n)]
    ident = np.arange(n, dtype=np.uint64)
    npr = np.random.default_rng(70 + int(dups))
    ident[n1:n1 + n2 // 2] = npr.choice(n1, n2 // 2, replace=False)   # re-posted in batch 2
    if dups:
        ident[100:200] = ident[5000:5100]                            # repeats inside batch 1
        ident[n1 + 10:n1 + 20] = ident[n1 + 30:n1 + 40]              # and inside batch 2
    q = np.concatenate([np.arange(0, 1000), np.arange(4950, 5150), np.arange(n1, n1 + 1000)]).astype(np.uint32)
    res, ref = run_both([{"comparator": EX, "low": 0.1, "high": 0.9}], [vals], keys=[vals], ident=ident,
                        threshold=0.8, queries=q, batches=[(0, n1), (n1, n)])
    assert res.n > 0
    assert_same(res, ref)
