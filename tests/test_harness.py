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
