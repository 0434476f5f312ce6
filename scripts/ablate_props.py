"""Per-property cost of the fused scoring kernel on the bench workload (1M persons):
times dk_match with single-property schemas.  Diagnostic only (not the bench)."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "sesam-duke-microservice_amd"))
import numpy as np  # noqa: E402
import dukehip as dh  # noqa: E402
from dukehip import _abi as A, synth  # noqa: E402

n = int(os.environ.get("N", "1000000"))
p = synth.persons(n - n // 10, n // 10)
keys = [synth.column(k) for k in synth.keys_config2(p)]
spec = {"NAME": (A.CMP_JAROWINKLER, 0.1, 0.95, "name"), "ADDRESS": (A.CMP_LEVENSHTEIN, 0.2, 0.8, "address"),
        "DOB": (A.CMP_LEVENSHTEIN, 0.1, 0.85, "dob")}
cols = {k: synth.column(p[v[3]]) for k, v in spec.items()}
SETS = (["DOB", "ADDRESS", "NAME"], ["DOB"], ["ADDRESS"], ["NAME"], [])
if os.environ.get("PROPS") is not None:   # e.g. PROPS=ADDRESS (one schema, for PMC passes)
    SETS = ([x for x in os.environ["PROPS"].split(",") if x],)
for names in SETS:
    arr = (A.dk_property * max(1, len(names)))()
    for i, k in enumerate(names):
        c, lo, hi, _ = spec[k]
        arr[i] = A.dk_property(c, 2, 0, 0, lo, hi, 0.0)
    s = A.dk_schema(len(names), arr, 0.9, 0.7, A.MODE_DEDUP, 2)
    eng = dh.GpuEngine(s)
    eng.upsert(n, np.arange(n), [cols[k] for k in names], key_columns=keys)
    q = np.arange(n, dtype=np.uint32)
    eng.match(q).close()
    eng.set_profiling(True)
    t = time.perf_counter()
    for _ in range(3):
        r = eng.match(q)
        r.close()
    el = (time.perf_counter() - t) / 3
    pr = eng.profile()
    print(f"{'+'.join(names) or 'none':20s} step {el*1e3:8.1f} ms  score {pr['ms_score']/3:8.1f} ms  "
          f"gen {pr['ms_generate']/3:6.1f}  emit {pr['ms_emit']/3:6.2f}  gather {pr['ms_gather']/3:6.1f}  pairs {r.pairs_scored}", flush=True)
    eng.close()
