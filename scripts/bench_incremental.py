"""Incremental index latency: small HTTP-sized batches
upserted into a large resident index, each followed by the dk_match of that batch -- the
microservice's POST /dedup path per batch (App.java:924-1028: index + commit + match).

For each index size N (configs[1] person records, two key functions): one full upsert of N
records and the table build (the full sort), then R batches of B new records (10 % of them re-post
IDs already indexed: delete-by-ID of a base row), each timed as upsert + first match after it
(the table build included).  Run with the delta index (default) and with DK_DELTA=0 (every
index change re-sorts all rows), to show the per-batch cost is independent of N with it.

  python scripts/bench_incremental.py --sizes 1000000,10000000 --batch 1000 --rounds 20
prints one JSON line per (N, mode).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "sesam-duke-microservice_amd"))

import numpy as np  # noqa: E402

from dukehip import _abi as A  # noqa: E402
from dukehip import synth  # noqa: E402
import dukehip as dh  # noqa: E402


def schema():
    props = [(A.CMP_JAROWINKLER, 0.1, 0.95), (A.CMP_LEVENSHTEIN, 0.2, 0.8), (A.CMP_LEVENSHTEIN, 0.1, 0.85)]
    arr = (A.dk_property * 3)()
    for i, (op, lo, hi) in enumerate(props):
        arr[i] = A.dk_property(op, 2, 0, 0, lo, hi, 0.0)
    s = A.dk_schema(3, arr, 0.9, 0.7, A.MODE_DEDUP, 2)
    s._keep = arr
    return s


def columns(p, a, b):
    cols = [synth.column(p[f][a:b]) for f in ("name", "address", "dob")]
    keys = synth.keys_config2({f: p[f][a:b] for f in ("name", "given", "surname", "dob") if f in p})
    return cols, [synth.column(k) for k in keys]


def run(n, batch, rounds, p, delta):
    os.environ["DK_DELTA"] = "1" if delta else "0"
    import torch
    eng = dh.GpuEngine(schema(), device=0)
    cols, kcols = columns(p, 0, n)
    eng.upsert(n, np.arange(n, dtype=np.uint64), cols, key_columns=kcols)
    eng.candidate_counts(np.arange(1, dtype=np.uint32))   # builds the tables: the full sort
    torch.cuda.synchronize()
    rng = np.random.default_rng(7)
    lat, ups, mat, idx = [], [], [], []
    row = n
    for r in range(rounds):
        a = n + r * batch
        cols, kcols = columns(p, a, a + batch)
        ident = np.arange(a, a + batch, dtype=np.uint64)
        repost = rng.choice(batch, batch // 10, replace=False)
        ident[repost] = rng.choice(n, batch // 10, replace=False).astype(np.uint64)
        eng.reset_profile()
        eng.set_profiling(True)
        t0 = time.perf_counter()
        rows = eng.upsert(batch, ident, cols, key_columns=kcols)
        t1 = time.perf_counter()
        res = eng.match(rows)
        t2 = time.perf_counter()
        eng.set_profiling(False)
        prof = eng.profile()
        res.close()
        row += batch
        if r == 0:
            continue   # first batch also sizes the small-batch pools
        ups.append((t1 - t0) * 1e3)
        mat.append((t2 - t1) * 1e3)
        lat.append((t2 - t0) * 1e3)
        idx.append(prof["ms_index"])
    prof = eng.profile()
    eng.close()
    med = lambda v: float(np.median(v))  # noqa: E731
    return {"index_records": n, "batch": batch, "batches_timed": len(lat),
            "delta_index": delta, "ms_batch_median": med(lat), "ms_batch_p90": float(np.percentile(lat, 90)),
            "ms_upsert_median": med(ups), "ms_match_median": med(mat), "ms_table_build_median": med(idx),
            "last_batch_profile": {k: prof[k] for k in ("full_builds", "delta_builds")}}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sizes", default="1000000,10000000")
    ap.add_argument("--batch", type=int, default=1000)
    ap.add_argument("--rounds", type=int, default=20)
    args = ap.parse_args()
    sizes = [int(x) for x in args.sizes.split(",")]
    extra = args.batch * args.rounds
    t = time.time()
    p = synth.persons(int((max(sizes) + extra) * 0.9), (max(sizes) + extra) - int((max(sizes) + extra) * 0.9))
    print(f"synth {time.time() - t:.1f}s", file=sys.stderr, flush=True)
    for n in sizes:
        for delta in (True, False):
            out = run(n, args.batch, args.rounds, p, delta)
            print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
