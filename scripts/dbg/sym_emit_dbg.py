"""Debug: per-query entry counts of the symmetric schedule vs the oracle (sym_case)."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "sesam-duke-microservice_amd"), os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")]
import numpy as np
import dukehip as dh
import oracle as O
from test_gpu_configs import sym_case, upsert_slice, alive_after
from test_gpu_parity import schema_of

def counts(first):
    f = np.asarray(first, dtype=np.int64)
    return f[1:] - f[:-1]

for seed, split, dele, prof in ((41, True, True, True), (41, True, True, False), (41, False, False, True)):
    props, vals, keys = sym_case(seed)
    n = len(vals[0])
    rng = np.random.default_rng(seed)
    ident = np.arange(n, dtype=np.uint64)
    if dele:
        ident[2000:2100] = ident[100:200]
        ident[2100:2110] = ident[2110:2120]
    deleted = ((rng.random(n) < 0.03) if dele else np.zeros(n, bool)).astype(np.uint8)
    eng = dh.GpuEngine(schema_of(props, 0.75, 0.55, "dedup", 2))
    if split:
        upsert_slice(eng, vals, keys, ident, 0, 1500, deleted)
        upsert_slice(eng, vals, keys, ident, 1500, n, deleted)
    else:
        upsert_slice(eng, vals, keys, ident, 0, n, deleted)
    ot = O.OracleTable(props, vals, keys=keys, ident=ident, deleted=deleted,
                       alive=alive_after(list(ident), n), threshold=0.75, maybe=0.55)
    q = np.arange(n, dtype=np.uint32)
    eng.set_profiling(prof)
    ref = ot.match(q)
    rc = np.bincount(ref["query"], minlength=n)
    for dev in (False, True):
        res = eng.match(q, on_device=dev)
        if dev:
            print("device n", res.n, "ref", len(ref["query"]))
            res.close()
            continue
        gc = counts(res.first)
        bad = np.nonzero(gc != rc)[0]
        print(f"seed {seed} split {split} del {dele} prof {prof}: n {res.n} ref {len(ref['query'])} bad queries {len(bad)} "
              f"first {bad[:10].tolist()} gpu {gc[bad[:10]].tolist()} ref {rc[bad[:10]].tolist()}")
        print("  sum gpu", gc.sum(), "ratio per bad", (gc[bad] / np.maximum(rc[bad], 1))[:10].round(2).tolist())
        res.close()
    os.environ["DK_SYM"] = "0"
    res = eng.match(q)
    print("  direct n", res.n)
    res.close()
    del os.environ["DK_SYM"]
    eng.close()
