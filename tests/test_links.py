"""CPU: the httptransform response (App.writeHttpTransformResponse, App.java:1180-1200) and
the bulk duke_links map against BaseLinkDatabaseMatchListener's per-callback bookkeeping
(BaseLinkDatabaseMatchListener.java:84-88, 115-135), on match arrays shaped like a
dk_result (no GPU needed: the arrays are built here)."""
import types

import numpy as np

import dukehip as dh
from dukehip import _abi as A
from dukehip import links as L
from dukehip.records import parse_entities


def test_java_double_to_string():
    cases = {0.9726578958815478: "0.9726578958815478", 1.0: "1.0", 0.5: "0.5", 1e-5: "1.0E-5",
             1.5e-5: "1.5E-5", 0.001: "0.001", 0.0009: "9.0E-4", 1e7: "1.0E7",
             123456789.0: "1.23456789E8", 9999999.0: "9999999.0", -2.5: "-2.5", 0.0: "0.0",
             float("nan"): "NaN", float("inf"): "Infinity"}
    for x, s in list(cases.items()) + [(-0.0, "-0.0")]:
        assert L.java_double(x) == s, (x, L.java_double(x))


def test_gson_writer_escaping_nulls_and_numbers():
    ents, single = parse_entities('{"_id": 7, "a": null, "n": [1.50, null, -0], "s": "<a href=\'x\'>&\\u2028\\t\\u0001é"}')
    assert single
    out = L.gson_dumps(ents[0])
    # compact; numbers keep their literal text; null members dropped, null array items kept
    assert out == ('{"_id":7,"n":[1.50,null,-0],"s":"\\u003ca href\\u003d\\u0027x\\u0027\\u003e'
                   '\\u0026\\u2028\\t\\u0001é"}')


def _records(prefix, n, dataset):
    return [dh.Record({"ID": f"{dataset}__{prefix}{i}", "dukeOriginalEntityId": f"{prefix}{i}",
                       "dukeDatasetId": dataset}) for i in range(n)]


def _fake_result(rng, nq, nrows):
    cnt = rng.integers(0, 4, nq)
    cnt[rng.random(nq) < 0.3] = 0
    first = np.zeros(nq + 1, np.uint64)
    np.cumsum(cnt, out=first[1:])
    n = int(first[-1])
    return types.SimpleNamespace(
        n=n, nqueries=nq, on_device=False, first=first,
        candidate=rng.integers(0, nrows, n).astype(np.uint32),
        prob=rng.random(n), kind=np.where(rng.random(n) < 0.5, A.KIND_MATCH, A.KIND_MAYBE).astype(np.uint8))


def test_entity_links_bulk_equals_listener_replay():
    rng = np.random.default_rng(4)
    rows = _records("r", 50, "crm")
    queries = _records("q", 40, "erp")
    queries += [queries[3], queries[7]]            # same _id posted twice: lists concatenate
    res = _fake_result(rng, len(queries), len(rows))
    lis = L.EntityLinksListener()
    proc = dh.GpuProcessor.__new__(dh.GpuProcessor)
    proc.listeners = [lis]
    proc.database = types.SimpleNamespace(rows=rows)
    lis.batch_ready(len(queries))
    proc._replay(queries, res)
    bulk = L.entity_links(res, queries, rows)
    assert bulk == lis.links()
    assert all(k.startswith("q") for k in bulk)
    no_match = {q.get_value("dukeOriginalEntityId") for i, q in enumerate(queries)
                if res.first[i] == res.first[i + 1]} - set(bulk)
    assert no_match                               # computeIfAbsent only on a callback


def test_http_transform_response_shapes():
    ents, single = parse_entities('[{"_id": "a", "x": 1}, {"_id": "b", "gone": null}]')
    links = {"a": [{"datasetId": "crm", "entityId": "r1", "confidence": 0.95}]}
    body = L.http_transform_response(ents, single, links)
    assert body == ('[{"_id":"a","x":1,"duke_links":[{"datasetId":"crm","entityId":"r1",'
                    '"confidence":0.95}]},{"_id":"b","duke_links":[]}]')
    ents, single = parse_entities('{"_id": "a", "duke_links": 5}')
    body = L.http_transform_response(ents, single, links)
    assert body.startswith('{"_id":"a","duke_links":[{')   # replaced in place, one object
    # a one-element array request answers with an array
    ents, single = parse_entities('[{"_id": "b"}]')
    assert L.http_transform_response(ents, single, {}) == '[{"_id":"b","duke_links":[]}]'
