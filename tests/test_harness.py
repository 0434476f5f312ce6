"""The plain-C client (integration/c/dk_harness.c) against the C-ABI: it builds with
-std=c99 -pedantic against include/dukehip.h, links libdukehip.so, and on a GPU its match
list equals the oracle's (same data, batches, deleted flags and re-posted IDs).

Oracle: oracle/duke_oracle.c, PARITY UNPINNED against Duke 1.2 itself."""
import os
import subprocess

import numpy as np
import pytest

import oracle as O
from dukehip import _abi as A
from dukehip import synth

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HARNESS = os.path.join(ROOT, "integration", "c", "build", "dk_harness")


def ensure_built():
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "integration", "c")], check=True,
                   capture_output=True)
    assert os.path.exists(HARNESS)


def write_input(path, props, vals, keys, ident, deleted, threshold, maybe):
    with open(path, "w", encoding="utf-8") as f:
        f.write(f"{len(props)} {len(keys)} {A.MODE_DEDUP} {threshold!r} {maybe!r}\n")
        for p in props:
            f.write(f"{p['comparator']} {p.get('q', 2)} {p.get('formula', 0)} {p.get('tokenizer', 0)} "
                    f"{p['low']!r} {p['high']!r} {p.get('min_ratio', 0.0)!r}\n")
        for i in range(len(ident)):
            cells = [str(int(ident[i])), str(int(deleted[i])), "0"]
            cells += ["\\N" if v[i] is None else v[i] for v in vals]
            cells += [k[i] for k in keys]
            f.write("\t".join(cells) + "\n")


def test_harness_builds_and_reports_no_device(tmp_path):
    """C99 + -pedantic build; without a GPU dk_create fails with DK_E_DEVICE, reported
    through dk_last_error (the product has no CPU fallback)."""
    ensure_built()
    try:
        import torch
        if torch.cuda.is_available():
            pytest.skip("a GPU is present: the -m gpu test runs the harness")
    except ImportError:
        pass
    inp = tmp_path / "in.txt"
    write_input(inp, [{"comparator": A.CMP_LEVENSHTEIN, "low": 0.1, "high": 0.9}], [["a", "b"]],
                [["k", "k"]], [0, 1], [0, 0], 0.9, 0.0)
    r = subprocess.run([HARNESS, str(inp)], capture_output=True, text=True)
    assert r.returncode == 2, (r.returncode, r.stdout, r.stderr)
    assert f"dk_create failed ({A.DK_E_DEVICE})" in r.stderr


@pytest.mark.gpu
def test_harness_match_list_equals_oracle(tmp_path):
    ensure_built()
    p = synth.persons(700, 300, seed=17)
    rng = np.random.default_rng(17)
    n = len(p["name"])
    # the reference's schema shape (testdukeconfig.xml): Levenshtein / Numeric / Levenshtein
    area = [None if rng.random() < 0.05 else str(int(x)) for x in rng.integers(1, 11, n)]
    props = [{"comparator": A.CMP_NUMERIC, "low": 0.04, "high": 0.73},
             {"comparator": A.CMP_LEVENSHTEIN, "low": 0.12, "high": 0.61},
             {"comparator": A.CMP_LEVENSHTEIN, "low": 0.09, "high": 0.93}]
    vals = [area, p["address"], p["name"]]
    keys = synth.keys_config2(p)
    ident = np.arange(n, dtype=np.uint64)
    ident[900:940] = ident[10:50]
    deleted = (rng.random(n) < 0.03).astype(np.uint8)
    inp = tmp_path / "in.txt"
    write_input(inp, props, vals, keys, ident, deleted, 0.9, 0.7)
    r = subprocess.run([HARNESS, str(inp), "600,250,150"], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    alive = np.ones(n, np.uint8)
    last = {}
    for i in range(n):
        if int(ident[i]) in last:
            alive[last[int(ident[i])]] = 0
        last[int(ident[i])] = i
    ot = O.OracleTable(props, vals, keys=keys, ident=ident, deleted=deleted, alive=alive,
                       threshold=0.9, maybe=0.7)
    ref = ot.match(np.arange(n, dtype=np.uint32))
    lines = r.stdout.splitlines()
    got = {"query": [], "candidate": [], "kind": [], "prob": []}
    for ln in lines:
        parts = ln.split()
        if parts[0] == "q":
            qrow = int(parts[1])
            for j in range(2, len(parts), 3):
                got["query"].append(qrow)
                got["candidate"].append(int(parts[j]))
                got["kind"].append(int(parts[j + 1]))
                got["prob"].append(float.fromhex(parts[j + 2]))
        elif parts[0] == "scored":
            assert int(parts[1]) == ref["pairs_scored"]
        elif parts[0] == "compare":
            assert float.fromhex(parts[1]) == ot.compare_rows(0, 1)
    assert got["query"] == list(ref["query"]) and got["candidate"] == list(ref["candidate"])
    assert got["kind"] == list(ref["kind"]) and got["prob"] == list(ref["prob"])
    assert len(got["query"]) > 50


def run_harness(args, timeout=180):
    r = subprocess.run([HARNESS] + [str(a) for a in args], capture_output=True, text=True, timeout=timeout)
    assert r.returncode == 0, r.stderr
    return r.stdout


def parse_lists(out):
    """harness stdout -> ([per batch {query, candidate, kind, prob, scored}], links, compare)"""
    batches, links, compare, cur = [], [], None, None
    for ln in out.splitlines():
        parts = ln.split()
        if parts[0] == "batch" or (parts[0] == "q" and cur is None):
            cur = {"query": [], "candidate": [], "kind": [], "prob": [], "scored": None}
            batches.append(cur)
            if parts[0] == "batch":
                continue
        if parts[0] == "q":
            qrow = int(parts[1])
            for j in range(2, len(parts), 3):
                cur["query"].append(qrow)
                cur["candidate"].append(int(parts[j]))
                cur["kind"].append(int(parts[j + 1]))
                cur["prob"].append(float.fromhex(parts[j + 2]))
        elif parts[0] == "scored":
            cur["scored"] = int(parts[1])
        elif parts[0] == "compare":
            compare = float.fromhex(parts[1])
        elif parts[0] == "link":
            links.append((parts[1], parts[2], int(parts[3]), int(parts[4]), float.fromhex(parts[5]),
                          int(parts[6])))
    return batches, links, compare


@pytest.mark.gpu
def test_harness_multi_device_equals_single(tmp_path):
    """The multi-device entry (dk_create_multi over two / three entries of device 0) through
    the plain-C client: the same output, byte for byte, as the single-device ctx -- per-batch
    lists and the final full match."""
    ensure_built()
    p = synth.persons(1400, 600, seed=23)
    rng = np.random.default_rng(23)
    n = len(p["name"])
    props = [{"comparator": A.CMP_JAROWINKLER, "low": 0.1, "high": 0.95},
             {"comparator": A.CMP_LEVENSHTEIN, "low": 0.2, "high": 0.8},
             {"comparator": A.CMP_LEVENSHTEIN, "low": 0.1, "high": 0.85}]
    vals = [p["name"], p["address"], p["dob"]]
    keys = synth.keys_config2(p)
    ident = np.arange(n, dtype=np.uint64)
    ident[1500:1560] = ident[20:80]
    deleted = (rng.random(n) < 0.02).astype(np.uint8)
    inp = tmp_path / "in.txt"
    write_input(inp, props, vals, keys, ident, deleted, 0.9, 0.7)
    for extra in ([], ["--per-batch"]):
        want = run_harness([inp, "900,700,400"] + extra)
        assert want.count("\nq ") > 100
        for devs in ("0,0", "0,0,0"):
            assert run_harness([inp, "900,700,400", "--devices", devs] + extra) == want, (devs, extra)


@pytest.mark.gpu
def test_harness_reference_pipeline_lucene_and_link_feed(tmp_path):
    """The reference's own pipeline (testdukeconfig.xml: no key functions, so its Lucene
    candidate semantics; lookup property NAME) driven through the plain-C client batch by
    batch as Processor.deduplicate runs it, with the bulk link sink: every batch's list equals
    the restated Lucene query + the oracle's Processor.compare (oracle/lucene_ref.py), and the
    ?since= feed equals the per-callback LinkDatabaseMatchListener replay into a
    SinceAwareInMemoryLinkDatabase (oracle/linkdb_ref.py).  PARITY UNPINNED (Lucene / Duke)."""
    import json
    import linkdb_ref as LR
    import dukehip as dh
    from dukehip.config import DukeConfig
    from dukehip.lucene import lookup_properties
    from test_gpu_lucene import expected
    from test_gpu_configs import alive_after, oracle_props
    ensure_built()
    with open(os.path.join(ROOT, "tests", "golden", "testdukeconfig_schema.json")) as f:
        cfg = DukeConfig.from_dict(json.load(f)["pipelines"]["Deduplication/countries-dbpedia-mondial"])
    _, props = cfg.to_schema(A.MODE_DEDUP, 0)
    recs = []
    for src, seed in zip(cfg.data_sources, (1234, 4321)):
        recs += dh.records_from_entities(synth.stress_entities(1200, seed), src)
    n = len(recs)
    ids = {}
    ident = np.array([ids.setdefault(r.get_value("ID"), len(ids)) for r in recs], np.uint64)
    deleted = np.array([r.get_value("dukeDeleted") == "true" for r in recs], np.uint8)
    vals = [[r.get_value(p.name) for r in recs] for p in props]
    lookup = [i for i, p in enumerate(props) if p.name in lookup_properties(cfg, props)]
    assert [props[i].name for i in lookup] == ["NAME"]
    oprops = oracle_props(props)
    inp = tmp_path / "ref.txt"
    write_input(inp, oprops, vals, [], ident, deleted, cfg.threshold, cfg.maybe_threshold)
    sizes = [600, 600, 600, 600]
    out = run_harness([inp, ",".join(map(str, sizes)), "--lucene",
                       ",".join(map(str, lookup)) + ":10:0.9", "--per-batch", "--linkdb"])
    got, links, compare = parse_lists(out)
    assert len(got) == len(sizes)
    db = LR.SinceAwareLinkDB()
    a = 0
    total = 0
    for t, (sz, g) in enumerate(zip(sizes, got)):
        e = a + sz
        alive = alive_after(list(ident), e).astype(bool)
        want, scored = expected(oprops, [v[:e] for v in vals], lookup, ident[:e], alive, deleted[:e],
                                None, np.arange(a, e), cfg.threshold, cfg.maybe_threshold, 10, 0.9, "dedup")
        assert g["scored"] == scored
        for k in ("query", "candidate", "kind", "prob"):
            assert g[k] == want[k], (t, k)
        total += len(g["query"])
        # the batch's callbacks in batch order into the per-callback link sink
        L = LR.LinkDBListener(db, lambda ts=t + 1: ts)
        L.batch_ready(sz)
        by_q = {}
        for q, c, k, pr in zip(want["query"], want["candidate"], want["kind"], want["prob"]):
            by_q.setdefault(q, []).append((c, k, pr))
        for i, q in enumerate(range(a, e)):
            lst = by_q.get(q, [])
            if not lst:
                L.no_match_for((i, str(int(ident[q]))))
            for c, k, pr in lst:
                (L.matches if k == 1 else L.matches_perhaps)((i, str(int(ident[q]))), str(int(ident[c])), pr)
        L.batch_done()
        a = e
    assert total > 50
    feed = [(l.id1, l.id2, l.status, l.kind, l.confidence, l.timestamp) for l in db.changes_since(0)]
    assert links == feed and len(links) > 20
    ot = O.OracleTable(oprops, vals, ident=ident, threshold=cfg.threshold, maybe=cfg.maybe_threshold)
    assert compare == ot.compare_rows(0, 1)
