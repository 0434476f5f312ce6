"""CPU: native ingestion (dk_pack_json, host code of libdukehip.so) against the Python
restatement of IncrementalDataSource.java:50-101 (dukehip.records.records_from_entities +
Column packing + PartsKey) on the same JSON bodies, and its error contract."""
import json
import random

import numpy as np
import pytest

import dukehip as dh
from dukehip import _abi as A
from dukehip import ingest as I
from dukehip.config import DataSource, DataSourceColumn

CLEAN = {"lc": "no.priv.garshol.duke.cleaners.LowerCaseNormalizeCleaner",
         "country": "no.priv.garshol.duke.examples.CountryNameCleaner",
         "capital": "no.priv.garshol.duke.examples.CapitalCleaner"}


def source(group=None):
    cols = [DataSourceColumn("name", "NAME", CLEAN["country"]),
            DataSourceColumn("city", "CITY", CLEAN["capital"]),
            DataSourceColumn("note", "NOTE", CLEAN["lc"]),
            DataSourceColumn("area", "AREA", None),
            DataSourceColumn("raw", "RAW", None),
            DataSourceColumn("extra", "UNSCORED", None)]
    return DataSource("ds-1", cols, group)


PROPS = ["AREA", "NAME", "CITY", "NOTE", "RAW"]
KEYS = [dh.PartsKey(("NAME", None, 0, 3), ("AREA", None, None, None)),
        dh.PartsKey(("NOTE", -1, -2, None)), dh.PartsKey(("RAW", 0, 1, 5), ("CITY", 1, None, 2))]


def rand_text(rng, alpha, lo, hi):
    return "".join(rng.choice(alpha) for _ in range(rng.randint(lo, hi)))


def rand_entities(rng, n):
    latin = list("abcdeABCDE  \t\xa0\n,()") + ["é", "Ø", "ñ", "ß", "Å", "́", "the ", ", the"]
    wide = latin + ["ł", "€", "\U0001F600", " "]
    ents = []
    for i in range(n):
        e = {"_id": rng.choice([str(i), i, f"x{i}"])}
        if rng.random() < 0.9:
            e["name"] = rand_text(rng, latin, 0, 14)
        if rng.random() < 0.8:
            e["city"] = [rand_text(rng, latin, 1, 10)] if rng.random() < 0.2 else rand_text(rng, latin, 0, 12)
        if rng.random() < 0.8:
            e["note"] = rand_text(rng, latin, 0, 20)
        if rng.random() < 0.8:
            e["area"] = rng.choice([rng.randint(-5, 50), rng.random() * 100, "7", True, False, [3], []])
        if rng.random() < 0.8:
            e["raw"] = rand_text(rng, wide, 0, 12)
        if rng.random() < 0.3:
            e["extra"] = rand_text(rng, wide, 0, 5)
        if rng.random() < 0.2:
            e["_deleted"] = rng.choice([True, False, "TRUE", "no", 1, [True]])
        ents.append(e)
    return ents


def reference(body, src):
    ents, _ = dh.parse_entities(body)
    recs = dh.records_from_entities(ents, src)
    vals = [[r.get_value(p) for r in recs] for p in PROPS]
    keys = [[kf.make_key(r) for r in recs] for kf in KEYS]
    return recs, vals, keys


@pytest.mark.parametrize("seed", range(6))
def test_pack_json_matches_python_path(seed):
    rng = random.Random(seed)
    src = source(group=None if seed % 2 == 0 else 1 + seed % 2)
    ns = I.NativeSource(src, PROPS, KEYS)
    it = I.Interner()
    ents = rand_entities(rng, 300)
    body = json.dumps(ents, ensure_ascii=bool(seed % 3 == 0))
    recs, vals, keys = reference(body, src)
    pk = ns.pack(body, it)
    assert pk.n == len(recs)
    for p in range(len(PROPS)):
        assert pk.values(p) == vals[p], PROPS[p]
    for k in range(len(KEYS)):
        assert pk.keys(k) == keys[k]
    assert pk.ids() == [r.get_value("ID") for r in recs]
    assert pk.entity_ids() == [r.get_value("dukeOriginalEntityId") for r in recs]
    assert list(pk.deleted) == [r.get_value("dukeDeleted") == "true" for r in recs]
    # exact interning: equal IDs <=> equal idents, stable across batches
    ids = [r.get_value("ID") for r in recs]
    ident = list(pk.ident)
    assert len(set(ident)) == len(set(ids))
    for a, b in zip(ids, ident):
        assert it.find(a) == b
    pk2 = ns.pack(body, it)
    assert list(pk2.ident) == ident
    # the columns are what Column.from_strings builds (layout the GPU path takes)
    for p in range(len(PROPS)):
        ref_col = A.Column.from_strings(vals[p])
        c = pk.ptr.contents.columns[p]
        off = np.ctypeslib.as_array(C_u32(c.offsets), (pk.n + 1,))
        assert np.array_equal(off, ref_col.offsets)
        assert c.width == ref_col.units.itemsize


@pytest.mark.parametrize("seed", range(3))
def test_pack_json_key_only_property(seed):
    """A key function may read a column no property scores ("extra" -> UNSCORED): its value
    is kept for the key parts (dk_source_column.prop = nprops + j) and not packed (the
    configs[2] json leg's DOB)."""
    rng = random.Random(100 + seed)
    src = source()
    kfs = KEYS + [dh.PartsKey(("UNSCORED", None, 0, 3), ("AREA", None, None, None)),
                  dh.PartsKey(("NAME", 0, 0, 2), ("UNSCORED", None, 1, 4))]
    ns = I.NativeSource(src, PROPS, kfs)
    ents = rand_entities(rng, 300)
    body = json.dumps(ents)
    recs = dh.records_from_entities(dh.parse_entities(body)[0], src)
    pk = ns.pack(body, I.Interner())
    assert pk.n == len(recs) and ns.nprops == len(PROPS)
    for p in range(len(PROPS)):
        assert pk.values(p) == [r.get_value(PROPS[p]) for r in recs]
    for k, kf in enumerate(kfs):
        assert pk.keys(k) == [kf.make_key(r) for r in recs]
    assert any(r.get_value("UNSCORED") for r in recs)
    with pytest.raises(I.UnsupportedComparator):   # no column fills it
        I.NativeSource(src, PROPS, [dh.PartsKey(("NOWHERE", None, 0, 2))])


def plain_source(group=None):
    """No column cleans: plain entities take dk_pack_json's ASCII fast path."""
    cols = [DataSourceColumn("name", "NAME", None), DataSourceColumn("city", "CITY", None),
            DataSourceColumn("note", "NOTE", None), DataSourceColumn("area", "AREA", None),
            DataSourceColumn("raw", "RAW", None), DataSourceColumn("extra", "UNSCORED", None)]
    return DataSource("ds-1", cols, group)


def plain_entities(rng, n):
    """Mostly plain ASCII entities (the fast path), every few one the general path takes:
    escapes, UTF-8, arrays, a JSON null, a string `_deleted`."""
    ascii_ = list("abcdeXYZ019 -\t")
    odd = ["é", "\U0001F600", "\\", '"', "\n", "€"]
    ents = []
    for i in range(n):
        e = {"_id": rng.choice([str(i), i, f"x {i}", True])}
        for k in ("name", "city", "note", "raw", "extra"):
            if rng.random() < 0.85:
                e[k] = rand_text(rng, ascii_, 0, 16)
        if rng.random() < 0.5:
            e["area"] = rng.choice([rng.randint(-5, 50), rng.random() * 100, "7", True, False, ""])
        if rng.random() < 0.1:
            e["_deleted"] = rng.choice([True, False])
        r = rng.random()
        if r < 0.05:
            e["note"] = rand_text(rng, ascii_ + odd, 1, 10)
        elif r < 0.08:
            e["city"] = [rand_text(rng, ascii_, 1, 6)]
        elif r < 0.10:
            e["_deleted"] = rng.choice(["TRUE", "no", [True]])
        elif r < 0.11:
            e["extra"] = None
        ents.append(e)
    return ents


@pytest.mark.parametrize("seed", range(4))
def test_pack_json_ascii_fast_path(seed, monkeypatch):
    """dk_pack_json's ASCII fast path (plain entities, no cleaners) gives the Python path's
    values, keys, IDs and flags, and exactly the general path's columns (DK_INGEST_NOFAST)."""
    rng = random.Random(200 + seed)
    src = plain_source(group=None if seed % 2 == 0 else 1 + (seed // 2) % 2)
    kfs = [dh.PartsKey(("NAME", -1, 0, 3), ("AREA", None, 0, 4)), dh.PartsKey(("NAME", 0, 0, 2),
           ("UNSCORED", None, 5, 10)), dh.PartsKey(("NOTE", -2, -3, None)), dh.PartsKey(("RAW", 1, None, None))]
    ents = [e for e in plain_entities(rng, 400) if e.get("extra", "") is not None]   # null: an error
    body = json.dumps(ents, ensure_ascii=bool(seed % 2))
    if seed == 3:
        monkeypatch.setenv("DK_INGEST_THREADS", "4")
    recs = dh.records_from_entities(dh.parse_entities(body)[0], src)
    ns = I.NativeSource(src, PROPS, kfs)
    packs = []
    for nofast in (False, True):
        if nofast:
            monkeypatch.setenv("DK_INGEST_NOFAST", "1")
        pk = ns.pack(body, I.Interner())
        assert pk.n == len(recs)
        for p in range(len(PROPS)):
            assert pk.values(p) == [r.get_value(PROPS[p]) for r in recs], PROPS[p]
        for k, kf in enumerate(kfs):
            assert pk.keys(k) == [kf.make_key(r) for r in recs]
        assert pk.ids() == [r.get_value("ID") for r in recs]
        assert pk.entity_ids() == [r.get_value("dukeOriginalEntityId") for r in recs]
        assert list(pk.deleted) == [r.get_value("dukeDeleted") == "true" for r in recs]
        packs.append(pk)
    a, b = packs
    assert list(a.ident) == list(b.ident)
    for p in range(len(PROPS)):
        ca, cb = a.ptr.contents.columns[p], b.ptr.contents.columns[p]
        assert ca.width == cb.width and bool(ca.present) == bool(cb.present)


def C_u32(p):
    import ctypes as C
    return C.cast(p, C.POINTER(C.c_uint32))


def test_single_entity_body_and_duplicate_members():
    src = source()
    ns = I.NativeSource(src, PROPS, KEYS)
    it = I.Interner()
    body = '{"_id": "a1", "name": "X", "name": "The Gambia", "area": 1e3, "raw": "\\u00e9\\ud83d\\ude00"}'
    pk = ns.pack(body, it)
    recs, vals, keys = reference(body, src)
    assert pk.n == 1 and pk.values(1) == ["gambia"] == vals[1]
    assert pk.values(0) == ["1e3"] and pk.values(4) == ["é\U0001F600"]
    assert pk.ids() == ["ds-1__a1"]


@pytest.mark.parametrize("body,code", [
    ('[{"name": "x"}]', A.DK_E_INVALID),                  # no _id
    ('[{"_id": ""}]', A.DK_E_INVALID),                    # empty _id
    ('[{"_id": null}]', A.DK_E_INVALID),                  # JsonNull.getAsString
    ('[{"_id": "1", "name": null}]', A.DK_E_INVALID),
    ('[{"_id": "1", "name": ["a", "b"]}]', A.DK_E_INVALID),  # JsonArray.getAsString
    ('[{"_id": "1", "name": {"a": 1}}]', A.DK_E_INVALID),
    ('[{"_id": "1", "_deleted": null}]', A.DK_E_INVALID),
    ('[1, 2]', A.DK_E_INVALID),                           # entities must be objects
])
@pytest.mark.parametrize("plain", [False, True])
def test_pack_json_errors(body, code, plain):
    # plain: a source without cleaners (its plain entities take the ASCII fast path)
    ns = I.NativeSource(plain_source() if plain else source(), PROPS, KEYS)
    with pytest.raises(A.DukeHipError) as e:
        ns.pack(body, I.Interner())
    assert e.value.code == code
    if body in ('[{"name": "x"}]', '[{"_id": ""}]'):
        assert "Got an entity with no '_id' attribute!" in A.load().dk_last_error().decode()
    with pytest.raises(ValueError):   # the Python restatement rejects the same batches
        ents, _ = dh.parse_entities(body)
        dh.records_from_entities(ents, source())


@pytest.mark.parametrize("body", [
    "[{'_id': 'a'}]",                                      # lenient (Gson) JSON
    '[{"_id": "a", "name": "€"}]',                    # outside the cleaner table
    '[{"_id": "a", "raw": "x"}] junk',
])
def test_pack_json_declines(body):
    ns = I.NativeSource(source(), PROPS, KEYS)
    with pytest.raises(I.NativeUnsupported):
        ns.pack(body, I.Interner())


def test_second_value_for_a_property_declines():
    src = DataSource("d", [DataSourceColumn("a", "NAME", None), DataSourceColumn("b", "NAME", None)])
    ns = I.NativeSource(src, ["NAME"], [])
    with pytest.raises(I.NativeUnsupported):
        ns.pack('[{"_id": "1", "a": "x", "b": "y"}]', I.Interner())
    pk = ns.pack('[{"_id": "1", "a": "x", "b": ""}]', I.Interner())   # empty: skipped
    assert pk.values(0) == ["x"]


def tricky_entities(rng, n):
    """Values full of JSON structure characters (brackets, quotes, backslashes) and ignored
    members holding nested containers: the chunk-parallel split must see them as data."""
    alpha = list('ab {}[]",\\:') + ["\\u005d", "é", "\U0001F600"]
    ents = []
    for i in range(n):
        e = {"_id": str(i) + rng.choice(["", "{", "]", '"', "\\"]),
             "raw": "".join(rng.choice(alpha) for _ in range(rng.randint(0, 12))),
             "nested": {"x": [1, {"y": "]}"}], "z": "[{"} if rng.random() < 0.5 else ["}", "]"]}
        if rng.random() < 0.7:
            e["area"] = rng.choice([[3], rng.randint(0, 9), "4"])
        ents.append(e)
    return ents


@pytest.mark.parametrize("threads", [1, 3, 8])
def test_pack_json_parallel_split_matches_python_path(threads, monkeypatch):
    monkeypatch.setenv("DK_INGEST_THREADS", str(threads))
    rng = random.Random(100 + threads)
    src = source()
    ns = I.NativeSource(src, PROPS, KEYS)
    body = json.dumps(tricky_entities(rng, 400), ensure_ascii=threads == 3)
    # odd whitespace between entities and around the array
    body = "\n [ " + body[1:-1].replace("}, {", "} ,\n\t{") + " ] \n"
    recs, vals, keys = reference(body, src)
    pk = ns.pack(body, I.Interner())
    assert pk.n == len(recs)
    for p in range(len(PROPS)):
        assert pk.values(p) == vals[p], PROPS[p]
    for k in range(len(KEYS)):
        assert pk.keys(k) == keys[k]
    assert pk.ids() == [r.get_value("ID") for r in recs]


@pytest.mark.parametrize("threads", [1, 4])
@pytest.mark.parametrize("body,code", [
    ('[{"_id": "1"}, {"_id": "2"},]', A.DK_E_INVALID),      # trailing comma: not an object
    ('[{"_id": "1"} {"_id": "2"}]', A.DK_E_UNSUPPORTED),    # missing comma
    ('[{"_id": "1"}, {"_id": "2"]', A.DK_E_UNSUPPORTED),    # mismatched bracket
    ('[{"_id": "1"}, {"_id": "2}]', A.DK_E_UNSUPPORTED),    # unterminated string
    ('[{"_id": "1"}, 7, {"_id": "3"}]', A.DK_E_INVALID),    # a non-object element
    ('[{"_id": "1"}, {"name": "x"}, {"_id": "3"', A.DK_E_INVALID),  # entity 1 fails first
    ('[{"_id": "1"}] x', A.DK_E_UNSUPPORTED),              # trailing characters
    ('  ', A.DK_E_UNSUPPORTED),
    ('5', A.DK_E_INVALID),
    ('[ , ]', A.DK_E_INVALID),
    ('[{"_id": "1"}, "x"]', A.DK_E_INVALID),
    ('[{"_id": "1"} "x"]', A.DK_E_UNSUPPORTED),
    ('[ ', A.DK_E_UNSUPPORTED),
    ('[{"_id": "1"},', A.DK_E_UNSUPPORTED),
    ('[{"_id": "1"}, 5', A.DK_E_INVALID),
    ('[[1]]', A.DK_E_INVALID),
    ('[{"_id": "1"}, [1]]', A.DK_E_INVALID),
    ('[{"_id": "1"} [1]]', A.DK_E_UNSUPPORTED),
    ('[}', A.DK_E_INVALID),
    ('[{"_id": "1"}}]', A.DK_E_UNSUPPORTED),
])
def test_pack_json_errors_parallel(body, code, threads, monkeypatch):
    monkeypatch.setenv("DK_INGEST_THREADS", str(threads))
    ns = I.NativeSource(source(), PROPS, KEYS)
    if code == A.DK_E_UNSUPPORTED:   # declined: the caller's own packing path takes it
        with pytest.raises(I.NativeUnsupported):
            ns.pack(body, I.Interner())
        return
    with pytest.raises(A.DukeHipError) as e:
        ns.pack(body, I.Interner())
    assert e.value.code == code


def test_pack_json_empty_array():
    ns = I.NativeSource(source(), PROPS, KEYS)
    pk = ns.pack(" [ \n ] ", I.Interner())
    assert pk.n == 0


def test_parallel_interning_equals_sequential(monkeypatch):
    """Record IDs interned shard-parallel (large batches) get the ids sequential interning
    gives: dense, in first-appearance order, re-posted IDs keep theirs; across batches that
    grow the table and batches that only look up."""
    rng = random.Random(7)
    src = DataSource("ds", [DataSourceColumn("raw", "RAW", None)])
    ns = I.NativeSource(src, ["RAW"], [])
    bodies = []
    for b, (n, span) in enumerate([(9000, 6000), (20000, 30000), (12000, 30000), (9000, 40000)]):
        ents = [{"_id": f"id{rng.randrange(span)}" + ("é" if rng.random() < 0.05 else ""), "raw": "x"}
                for _ in range(n)]
        bodies.append(json.dumps(ents))
    got = {}
    for threads in ("1", "8"):
        monkeypatch.setenv("DK_INGEST_THREADS", threads)
        it = I.Interner()
        packs = [ns.pack(body, it) for body in bodies]   # the idents live in their batches
        got[threads] = [[int(x) for x in pk.ident] for pk in packs]
        ids = [r for body in bodies for r in (f"ds__{e['_id']}" for e in json.loads(body))]
        flat = [x for batch in got[threads] for x in batch]
        assert [it.find(r) for r in ids] == flat
        assert len(it) == len(set(ids))
    assert got["1"] == got["8"]
    # first-appearance numbering
    seen = {}
    for r in (f"ds__{e['_id']}" for body in bodies for e in json.loads(body)):
        seen.setdefault(r, len(seen))
    assert [x for batch in got["8"] for x in batch] == [seen[f"ds__{e['_id']}"] for body in bodies
                                                        for e in json.loads(body)]


def _pack_or_error(ns, body):
    try:
        pk = ns.pack(body, I.Interner())
    except I.NativeUnsupported:
        return ("unsupported",)
    except A.DukeHipError as e:
        return ("error", e.code)
    return ("ok", pk.n, [pk.values(p) for p in range(len(PROPS))],
            [pk.keys(k) for k in range(len(KEYS))], pk.ids())


@pytest.mark.parametrize("threads", [1, 5])
def test_split_simd_equals_scalar(threads, monkeypatch):
    """The 64-byte-block split (escape runs carried across blocks, prefix-XOR string mask)
    against the byte-at-a-time split: values with backslash / quote / bracket runs of every
    length at every offset, valid and corrupted bodies."""
    monkeypatch.setenv("DK_INGEST_THREADS", str(threads))
    rng = random.Random(7 + threads)
    ns = I.NativeSource(source(), PROPS, KEYS)
    pieces = ["\\", "\\\\", '"', '\\"', "{", "}", "[", "]", "a", " ", ",", ":", "é"]
    for trial in range(40):
        ents = []
        for i in range(rng.randint(0, 120)):
            v = "".join(rng.choice(pieces) * rng.randint(1, 70 if rng.random() < 0.1 else 3)
                        for _ in range(rng.randint(0, 12)))
            ents.append({"_id": f"{i}{v[:5]}", "raw": v, "area": rng.choice(["1", [2], 3]),
                         "nested": {"k": [v, {"x": v}]}})
        body = json.dumps(ents, ensure_ascii=rng.random() < 0.5)
        if trial % 4 == 3 and body:   # corrupt one byte: both splits must fail the same way
            k = rng.randrange(len(body))
            body = body[:k] + rng.choice(['"', "\\", "}", "]", "{", ","]) + body[k + 1:]
        monkeypatch.setenv("DK_INGEST_SCALAR", "1")
        want = _pack_or_error(ns, body)
        monkeypatch.setenv("DK_INGEST_SCALAR", "0")
        got = _pack_or_error(ns, body)
        assert got == want, (trial, body[:200])
